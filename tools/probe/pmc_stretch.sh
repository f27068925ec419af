cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_st; mkdir -p $O
timeout -k 10 60 python3 $R/tools/probe/iters_c2.py > $O/iters.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b.json 2>$O/p1.err || exit 1
