# GPU collision + graph tests repeated; $1: extra environment (e.g. IKG_TRAJ_REC=1)
for k in 1 2 3 4; do
  env ${1:-X=1} timeout -k 10 200 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_graph.py -q --timeout 60 --timeout-method thread > /tmp/g.log 2>&1
  echo "run $k rc=$? $(tail -1 /tmp/g.log)"; grep "AssertionError: " /tmp/g.log | cut -c1-600
done
