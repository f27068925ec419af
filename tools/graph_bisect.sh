# GPU collision + graph tests repeated under the default and opt-in schedules
for env in "X=1" "IKG_TRAJ_PRESCREEN=0" "IKG_TRAJ_REC=1"; do
  for k in 1 2; do
    env $env timeout -k 10 200 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_collision.py -x -q --timeout 60 --timeout-method thread -k "not multistart_with_collision" > /tmp/g.log 2>&1
    rc=$?; echo "$env run $k rc=$rc $(tail -1 /tmp/g.log)"; grep "^FAILED" /tmp/g.log | cut -c1-200
    case $rc in 0|1) ;; *) exit $rc ;; esac
  done
done
