set -o pipefail
O=gpurun_out/col_r01c; mkdir -p $O
timeout -k 10 240 python bench.py --collision --no-cpu-baseline > $O/c2_f64.json 2>$O/err.txt &&
timeout -k 10 240 python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline > $O/c3_f32.json 2>>$O/err.txt &&
timeout -k 10 240 python bench.py --collision --dtype f64 --batch 65536 --no-cpu-baseline > $O/c3_f64.json 2>>$O/err.txt &&
timeout -k 10 240 python bench.py --collision --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline > $O/c5_f32.json 2>>$O/err.txt &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --collision --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.json 2>>$GRAFT_REPO_ROOT/$O/err.txt
