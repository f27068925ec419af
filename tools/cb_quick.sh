# quick controller-row check: parity tests + bench lines
ROOT=$(pwd); O=$ROOT/gpurun_out/cb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_control.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "all f64" "task f64" "jac f64" "all f32"; do set -- $cfg
  timeout -k 10 120 python tools/control_bench.py --outputs $1 --dtype $2 --no-cpu > $O/b_$1_$2.json || exit 1
  python -c "import json,sys; d=json.load(open('$O/b_$1_$2.json')); print('  $1 $2', round(d['ms_per_launch'],3), 'ms', round(d['roofline']['frac'],3))"
done
