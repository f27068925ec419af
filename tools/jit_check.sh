set -o pipefail
mkdir -p gpurun_out/jit
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --tb=short > gpurun_out/jit/pytest.log 2>&1 && \
timeout -k 10 200 python tools/generic_bench.py --dtype f64 > gpurun_out/jit/generic_bench_f64.json 2>gpurun_out/jit/gb.err && \
timeout -k 10 200 python tools/generic_bench.py --dtype f32 > gpurun_out/jit/generic_bench_f32.json 2>>gpurun_out/jit/gb.err
rc=$?; tail -3 gpurun_out/jit/pytest.log; cat gpurun_out/jit/generic_bench_*.json; exit $rc
