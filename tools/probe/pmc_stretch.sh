# instruction / cycle counters of the continuation and stretch kernels (c2 --collision)
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmc_st; mkdir -p $O
for v in ${ROUNDS:-0 2}; do
IKG_HANDOFF_ROUNDS=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $O/r$v -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b$v.json 2>$O/r$v.err || exit 1
done
