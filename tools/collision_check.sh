#!/bin/bash
# GPU session for the collision term: benches with/without it and a kernel
# trace of the collision run.  Usage (GPU box, repo root): bash tools/collision_check.sh [tag]
TAG=${1:-r01}
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; cat "$OUT/$name.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.err"; exit $rc; fi
}
timeout -k 10 600 python -m pytest tests/test_gpu_collision.py -q -p no:cacheprovider > "$OUT/col_pytest_$TAG.log" 2>&1
rc=$?; tail -3 "$OUT/col_pytest_$TAG.log"; [ $rc -gt 1 ] && exit $rc
run cq_uniform_$TAG 120 python tools/collision_bench.py
run cq_solutions_$TAG 120 python tools/collision_bench.py --batch 4096 --converged
run col_f64_b4096_$TAG 300 python bench.py --collision --no-cpu-baseline
run col_f32_b65536_$TAG 300 python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline
run col_ms256_$TAG 300 python bench.py --collision --dtype f32 --multistart 256 --batch 512 --steps 3 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_col_$TAG" -o run -- python3 bench.py --collision --no-cpu-baseline --steps 5 > "$OUT/prof_col_$TAG.log" 2>&1
rc=$?; echo "== rocprof rc=$rc"; exit $rc
