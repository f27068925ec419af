# kernel split of the C5 multi-start solve with the collision term
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c5prof; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench.py --no-cpu-baseline --collision --dtype f32 --batch 512 --multistart 256 --steps 5 --warmup 1 > $O/b.json 2>/dev/null
