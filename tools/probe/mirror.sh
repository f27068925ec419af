# stretch kernel per-update speed: one problem per wave on 2 lanes (1), mirrored on all 64 lanes (-1), packed (32)
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/mirror; mkdir -p $O
for v in 1 -1 32; do
IKG_STRETCH_PPW=$v IKG_HANDOFF_ROUNDS=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b$v.json 2>/dev/null || exit 1
done
