# c2 / c3 --collision kernel time per solve vs hand-off rounds (and continuation groups per wave)
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/rounds; mkdir -p $O
for v in ${ROUNDS:-0 2}; do for g in ${GROUPS_:-4}; do
  for cfg in "c2 --collision" "c3 --collision --dtype f32 --batch 65536"; do set -- $cfg; t=$1; shift
    IKG_CONT_G=$g IKG_HANDOFF_ROUNDS=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r${v}g${g}_$t -o run -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" > $O/r${v}g${g}_$t.json 2>/dev/null || exit 1
  done
done; done
