#!/bin/bash
# Round 3: window-exhaustion fix + poisoned workspaces + graph replay of the
# opt-in continuation schedules, one pytest process per step.  A step that
# faults, aborts or times out (exit > 1) ends the script.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r3diag
run() {  # name, env..., -- pytest args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/r3diag/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 gpurun_out/r3diag/$name.log
  [ $rc -le 1 ] || exit $rc
}
run collision X=1 -- tests/test_gpu_collision.py
run graph X=1 -- tests/test_gpu_graph.py
run graph_rec_poison IKG_TRAJ_REC=1 IKG_POISON=1 -- tests/test_gpu_graph.py
run graph_noprescreen_poison IKG_TRAJ_PRESCREEN=0 IKG_POISON=1 -- tests/test_gpu_graph.py
run graph_poison IKG_POISON=1 -- tests/test_gpu_graph.py
