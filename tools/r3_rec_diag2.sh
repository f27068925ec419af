#!/bin/bash
# Round 3: replays of a captured REC solve after the collision tests, with the
# records in stream-ordered (graph) memory and in a persistent hipMalloc buffer.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r3diag
for p in 0 1; do
  IKG_GRAPH_DIAG=1 IKG_TRAJ_REC=1 IKG_REC_PERSIST=$p timeout -k 10 300 python -u -m pytest -v -s --timeout 120 \
    --timeout-method thread tests/test_gpu_collision.py tests/test_gpu_graph.py > gpurun_out/r3diag/rec_diag_persist$p.log 2>&1
  rc=$?
  echo "persist=$p rc=$rc"; grep -E "FAILED|passed|failed|\[diag\]" gpurun_out/r3diag/rec_diag_persist$p.log | head -40
  [ $rc -le 1 ] || exit $rc
done
