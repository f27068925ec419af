# round-end check: full GPU suite, smoke, default bench; then the opt-in records' failing tests (diagnostic)
O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cut -c1-300 $O/bench.json
IKG_TRAJ_REC=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_graph.py -q --timeout 60 --timeout-method thread > $O/rec_pytest.log 2>&1
grep -E "^FAILED|AssertionError" $O/rec_pytest.log | cut -c1-300
exit 0
