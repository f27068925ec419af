# collision row quick check: parity tests + the --collision bench lines
ROOT=$(pwd); O=$ROOT/gpurun_out/colq; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_planner.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $O/$n.json || exit 1
  python -c "import json; d=json.load(open('$O/$n.json')); print('$n', round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,3), 'M/s')"; }
run c2_f64 --collision
run c3_f32 --collision --dtype f32 --batch 65536
run c5_f32 --collision --dtype f32 --batch 512 --multistart 256
