#!/bin/bash
# Graph-replay tests under IKG_POISON=1 for each opt-in collision schedule.
mkdir -p gpurun_out/modes
for env in "IKG_TRAJ_PRESCREEN=0" "IKG_TRAJ_REC=0" "IKG_CONT_TRAJ=0"; do
  env IKG_POISON=1 $env timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_graph.py > gpurun_out/modes/graph_$env.log 2>&1
  rc=$?; echo "$env rc=$rc $(tail -1 gpurun_out/modes/graph_$env.log)"; [ $rc -le 1 ] || exit $rc
done
