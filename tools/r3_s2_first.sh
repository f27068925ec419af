#!/bin/bash
# Round 3 (session 2) first GPU pass: GPU tests, default bench line, C2 rocprof.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/s2a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
cat $OUT/bench.json
