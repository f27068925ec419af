mkdir -p gpurun_out/r4a
export IKG_REPORT_DIR=gpurun_out/r4a/reports
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r4a/pytest_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_fullbatch.py > gpurun_out/r4a/pytest_gpu.log 2>&1
echo "suite rc=$?"
timeout -k 10 200 python bench.py > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err
echo "bench rc=$?"
