#!/bin/bash
# Round 3: the round-2 failure of IKG_TRAJ_REC=1 (collision + graph tests in
# one pytest process), rerun once as recorded and once with poisoned workspaces.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r3diag
for v in 0 1; do
  IKG_TRAJ_REC=1 IKG_POISON=$v timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
    tests/test_gpu_collision.py tests/test_gpu_graph.py > gpurun_out/r3diag/rec_both_poison$v.log 2>&1
  rc=$?
  echo "poison=$v rc=$rc"; grep -E "FAILED|passed|failed|rows differ" gpurun_out/r3diag/rec_both_poison$v.log | head -20
  [ $rc -le 1 ] || exit $rc
done
