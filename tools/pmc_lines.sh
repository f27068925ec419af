#!/bin/bash
# Counter profiles for the bench lines that lacked them (round 5): HBM bytes of
# c2_yaw and c4_strong, executed FP ops of the multi-start (medium-range)
# pair kernel in fp64 and fp32.  One rocprofv3 --pmc pass per counter group,
# each under its own time limit; then the summaries into profiles/.
#   TAG=r5pmc tools/pmc_lines.sh        (GPU box, repo root)
ROOT=$(pwd); O=$ROOT/gpurun_out/${TAG:-pmc_lines}; mkdir -p $O/pmc $O/flops; cd /tmp; export TMPDIR=/tmp
P="python3 $ROOT/tools/pmc_probe.py"
pass() { dir=$1; shift; cnt=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d $dir -o run -- $P "$@" > $dir.log 2>&1
  rc=$?; echo "$(basename $dir) rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
YAW=0.7853981633974483
pass $O/pmc/fetch_b4096_f64_yaw FETCH_SIZE 4096 f64 32 3 --yaw $YAW
pass $O/pmc/write_b4096_f64_yaw WRITE_SIZE 4096 f64 32 3 --yaw $YAW
pass $O/pmc/fetch_b1048576_f64 FETCH_SIZE 1048576 f64 32 2 --seed 7
pass $O/pmc/write_b1048576_f64 WRITE_SIZE 1048576 f64 32 2 --seed 7
pass $O/pmc/fetch_b131072_f64 FETCH_SIZE 131072 f64 32 3 --seed 7
pass $O/pmc/write_b131072_f64 WRITE_SIZE 131072 f64 32 3 --seed 7
for DT in f64 f32; do SFX=$([ "$DT" = f64 ] && echo F64 || echo F32)
  mkdir -p $O/flops/${DT}_med
  pass $O/flops/${DT}_med/ops "SQ_INSTS_VALU_FMA_$SFX SQ_INSTS_VALU_MUL_$SFX SQ_INSTS_VALU_ADD_$SFX SQ_INSTS_VALU_TRANS_$SFX" \
    131072 $DT 32 2 --randq0 --variant 1 --save-iters $O/flops/${DT}_med/iters.npy
done
cd $ROOT
python tools/pmc_summary.py $O/pmc f64 4096 r05 --sfx=yaw && python tools/pmc_summary.py $O/pmc f64 1048576 r05 && \
python tools/pmc_summary.py $O/pmc f64 131072 r05 && \
python tools/pmc_flops.py $O/flops/f64_med 131072 f64 r05 --med && python tools/pmc_flops.py $O/flops/f32_med 131072 f32 r05 --med
echo ALLDONE
