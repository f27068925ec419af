#!/bin/bash
# Round 3: captured solves take hipMalloc scratch (ws_alloc): the REC=1 and
# PRESCREEN=0 schedules through the collision + graph tests in one process,
# then C2 with the collision term, default vs records-in-batch-kernel.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r3verify
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_bridge.py > gpurun_out/r3verify/bridge.log 2>&1; rc=$?; echo "bridge rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/r3verify/bridge.log | head; [ $rc -le 1 ] || exit $rc
for cfg in "IKG_TRAJ_REC=1" "IKG_TRAJ_PRESCREEN=0" "X=1"; do
  env $cfg IKG_GRAPH_DIAG=1 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_collision.py tests/test_gpu_graph.py > gpurun_out/r3verify/tests_${cfg%%=*}.log 2>&1
  rc=$?
  echo "$cfg rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r3verify/tests_${cfg%%=*}.log | head
  [ $rc -le 1 ] || exit $rc
done
for k in 1 2; do
  for cfg in "IKG_TRAJ_REC=0" "IKG_TRAJ_REC=1"; do
    env $cfg timeout -k 10 120 python bench.py --collision --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/r3verify/bench_${cfg}_$k.json 2>gpurun_out/r3verify/bench.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],3), round(d['value']/1e6,3))" gpurun_out/r3verify/bench_${cfg}_$k.json
  done
done
