#!/bin/bash
# Round 3: full GPU test suite, then the bench configurations (C2 fp64, C3
# fp32, C4 per-GPU share fp64/fp32, C2 with the collision term, C5 share).
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/${R3TAG:-r3run}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|error" $OUT/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit $rc
b() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $OUT/bench_$n.json 2>$OUT/bench_$n.err || { echo "bench $n failed"; tail -5 $OUT/bench_$n.err; exit 3; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms', round(d['ms_per_step'],3), 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'value', round(d['value']/1e6,3))" $OUT/bench_$n.json $n
}
b c2 --steps 20 --warmup 3
b c3 --batch 65536 --dtype f32 --steps 10 --warmup 2
b c4f64 --batch 131072 --steps 5 --warmup 2
b c4f32 --batch 131072 --dtype f32 --steps 5 --warmup 2
b c2col --collision --steps 20 --warmup 3
b c5f32 --multistart 256 --batch 512 --dtype f32 --steps 5 --warmup 2
