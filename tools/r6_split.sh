#!/bin/bash
# Split records scan (several waves per listed problem, IKG_SCAN_SPLIT), one
# GPU call: its equality test, the collision and full-batch oracle tests, then
# an interleaved A/B of the wave target on the collision lines.
#   TAG=name [VARIANTS=...] [CONFIGS=...] tools/r6_split.sh
TAG=${TAG:?TAG=name}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_collision.py -m gpu -k split -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1 || { tail -30 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_fullbatch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_col.log 2>&1 || { tail -30 $O/pytest_col.log; exit 1; }
tail -1 $O/pytest_col.log
ABTAG=$TAG/ab CONFIGS="${CONFIGS:-c2col c3col c5col}" VARIANTS="${VARIANTS:-IKG_SCAN_SPLIT=0 base IKG_SCAN_SPLIT=8192}" REPS=${REPS:-2} timeout -k 10 600 bash tools/bench_env_ab.sh || exit 1
cat $O/ab/summary.txt
