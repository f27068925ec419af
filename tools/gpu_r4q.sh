# Kernel timelines of C3 fp32 with the collision term: default schedule (packed
# batch + trajectory continuation) and pair records-in-batch with a raised budget
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
for v in default pairrec; do
  O=$ROOT/gpurun_out/r4q/$v; mkdir -p $O
  E=""; [ $v = pairrec ] && E="IKG_REC_BUDGET_MB=8192 IKG_REC_PREFER_PAIR=1"
  (cd /tmp && env $E timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
    python3 $ROOT/bench.py --collision --dtype f32 --batch 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > $O/bench.json) || exit $?
done
