# Generic-model bench (tools/generic_bench.py) at both dtypes, plus the
# specialisation and plain-C caller GPU tests -> gpurun_out/generic/
set -o pipefail
mkdir -p gpurun_out/generic
timeout -k 10 300 python -u -m pytest tests/test_gpu_jit.py tests/test_c_demo.py -m gpu -x -v --timeout 120 --timeout-method thread --tb=short > gpurun_out/generic/pytest.log 2>&1 && \
timeout -k 10 200 python tools/generic_bench.py --dtype f64 > gpurun_out/generic/generic_bench_f64.json 2> gpurun_out/generic/err.log && \
timeout -k 10 200 python tools/generic_bench.py --dtype f32 > gpurun_out/generic/generic_bench_f32.json 2>> gpurun_out/generic/err.log
rc=$?; tail -3 gpurun_out/generic/pytest.log; cat gpurun_out/generic/*.json; exit $rc
