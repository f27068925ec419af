#!/bin/bash
# rocprofv3 kernel-trace summary of one bench.py configuration:
#   OUT=gpurun_out/x/c3col [ENV="IKG_REC_BUDGET_MB=8192"] tools/kernel_trace.sh <bench.py args>
# writes $OUT/run_kernel_stats.csv (+ trace) and $OUT/bench.json.
ROOT=$(pwd); O=${OUT:?OUT=dir}; case $O in /*) ;; *) O=$ROOT/$O;; esac
mkdir -p $O; export TMPDIR=/tmp; cd /tmp
env $ENV timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 $ROOT/bench.py --no-cpu-baseline --no-extra "$@" > $O/bench.json 2> $O/bench.err
rc=$?; echo "kernel trace rc=$rc"; exit $rc
