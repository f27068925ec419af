#!/bin/bash
# Round 3: the REC=1 graph-replay failure with every workspace allocation traced.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r3diag
IKG_TRAJ_REC=1 IKG_WS_TRACE=1 timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_collision.py tests/test_gpu_graph.py > gpurun_out/r3diag/rec_trace.log 2>&1
rc=$?
echo "rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r3diag/rec_trace.log | head
exit $((rc > 1 ? rc : 0))
