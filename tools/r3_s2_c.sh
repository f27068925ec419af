#!/bin/bash
# Round 3 (session 2): the whole GPU suite, then bench --gpus 2 on the 1-GPU box (gloo rehearsal).
ROOT=$(pwd); O=$ROOT/gpurun_out/s2c; mkdir -p $O
IKG_REPORT_DIR=$O/reports timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err; rc=$?
echo "bench g2 rc=$rc"; tail -c 1500 $O/bench_g2.json; tail -5 $O/bench_g2.err
