# GPU clock during the stretch kernel: GRBM_GUI_ACTIVE / duration, packed vs spread waves
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/clock; mkdir -p $O
for v in 1 32; do
IKG_STRETCH_PPW=$v IKG_HANDOFF_ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --no-cpu-baseline --collision --steps 2 --warmup 1 > $O/b$v.json 2>$O/p$v.err || exit 1
done
