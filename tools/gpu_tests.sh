#!/bin/bash
# One GPU call: a named subset of the GPU tests with parity reports, then
# (SUITE=1) the rest of the GPU suite, then (BENCH=1) the default bench line.
#   TAG=r5a FIRST="tests/test_gpu_memory.py tests/test_gpu_fullbatch.py" SUITE=1 BENCH=1 tools/gpu_tests.sh
# Outputs under gpurun_out/$TAG: pytest_first.log, pytest_gpu.log, bench.json,
# reports/*_vs_oracle.json (IKG_REPORT_DIR).  Every GPU step has its own time
# limit; a step that times out, aborts or faults ends the call.
TAG=${TAG:?TAG=name}
O=gpurun_out/$TAG
mkdir -p $O
export IKG_REPORT_DIR=$O/reports
stop() { case $1 in 0|1) return 0;; *) echo "FATAL $2 rc=$1"; exit $1;; esac; }
if [ -n "$FIRST" ]; then
  timeout -k 10 ${FIRST_TIMEOUT:-600} python -u -m pytest $FIRST -m gpu ${XFLAG--x} -v -s --timeout 300 --timeout-method thread \
    > $O/pytest_first.log 2>&1
  rc=$?; echo "first rc=$rc"; grep -E "passed|failed" $O/pytest_first.log | tail -1; stop $rc first
fi
if [ "${SUITE:-0}" = 1 ]; then
  DESEL=""
  for f in $FIRST; do DESEL="$DESEL --deselect $f"; done
  timeout -k 10 ${SUITE_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $DESEL \
    > $O/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" $O/pytest_gpu.log | tail -1; stop $rc suite
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('$O/bench.json')); print('C2', round(d['ms_per_step'], 4), 'ms', round(d['value'] / 1e6, 3), 'M/s')"
fi
echo ALLDONE
