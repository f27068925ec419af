# Round-4 GPU check: the full-batch parity tests (reports -> gpurun_out/r4b/reports),
# the graph / binding tests, then the whole -m gpu suite.
mkdir -p gpurun_out/r4b
export IKG_REPORT_DIR=gpurun_out/r4b/reports
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_graph.py tests/test_gpu_bridge.py -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/r4b/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4b/pytest_gpu.log 2>&1
echo "suite rc=$?"
