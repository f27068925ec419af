# instruction-cache counters: batch kernel and the stretch kernel packed (32) vs spread (1)
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/icache; mkdir -p $O
for v in 1 32; do
IKG_STRETCH_PPW=$v IKG_HANDOFF_ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b$v.json 2>$O/p$v.err || exit 1
done
