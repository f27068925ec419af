#!/bin/bash
# One rocprofv3 --pmc pass over tools/pmc_probe.py (counters only with
# --kernel-trace; one counter group per pass -- MI355X_MICROARCH.md).
#   tools/pmc_pass.sh OUTDIR "COUNTERS" B dtype ppw reps [pmc_probe.py options]
# e.g. tools/pmc_pass.sh gpurun_out/x/pmc/fetch_b65536_f32_col FETCH_SIZE 65536 f32 32 3 --collision
# then tools/pmc_summary.py / tools/pmc_flops.py turn the passes into profiles/*.json.
ROOT=$(pwd); dir=$1; cnt=$2; shift 2
case $dir in /*) ;; *) dir=$ROOT/$dir;; esac
mkdir -p $(dirname $dir); cd /tmp; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d $dir -o run -- \
  python3 $ROOT/tools/pmc_probe.py "$@" > $dir.log 2>&1
rc=$?; echo "$(basename $dir) rc=$rc"; exit $rc
