# kernel trace of the --collision c2 bench at several stretch-wave packings
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ppw; mkdir -p $O
for v in 1 4 16 32; do
  IKG_STRETCH_PPW=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b$v.json 2>/dev/null || exit 1
done
