#!/bin/bash
# Interleaved A/B of ab_libs/*.so (tools/ablate.py): C2 fp64 (real eps and forced 1000
# updates), C3 fp32 packed, random-seed fp64; then the GPU tests on the in-tree library.
ROOT=$(pwd); O=$ROOT/gpurun_out/${ABTAG:-ab}; mkdir -p $O
L="$ROOT/ab_libs/*.so"
ABL_EPS=1e-3 ABL_ROUNDS=12 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2_f64.txt 2>&1 || exit 3
ABL_ROUNDS=8 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2_f64_forced.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=8 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" > $O/c3_f32.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_RANDQ0=1 ABL_ROUNDS=6 timeout -k 10 300 python tools/ablate.py 131072 f64 "$L" > $O/rand_f64.txt 2>&1 || exit 3
cat $O/*.txt
if [ -n "$ABTESTS" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -8
  exit $rc
fi
