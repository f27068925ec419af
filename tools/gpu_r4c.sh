# duo layout: A/B against pair (fp64/fp32, q0 = 0 and random seeds), then the parity tests
mkdir -p gpurun_out/r4c
timeout -k 10 240 python tools/layout_ab.py --variants 1,4 --out gpurun_out/r4c/ab_q0.json > gpurun_out/r4c/ab_q0.log 2>&1
echo "ab rc=$?"
timeout -k 10 240 python tools/layout_ab.py --variants 1,4 --seeds --sizes 4096,16384 --out gpurun_out/r4c/ab_seeds.json > gpurun_out/r4c/ab_seeds.log 2>&1
echo "ab seeds rc=$?"
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r4c/pytest_parity.log 2>&1
echo "parity rc=$?"
