#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
# Usage (from the repo root on the GPU box): bash tools/gpu_check.sh [tag]
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

stop_if_fatal() {  # $1 = exit code, $2 = step name
  case $1 in
    0|1) return 0 ;;
    *) echo "FATAL: step $2 exited $1 — stopping" | tee -a "$OUT/summary.txt"; exit "$1" ;;
  esac
}

echo "== pytest -m gpu" | tee "$OUT/summary.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu_$TAG.log" | tee -a "$OUT/summary.txt"; stop_if_fatal $rc pytest

echo "== smoke" | tee -a "$OUT/summary.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -3 "$OUT/smoke_$TAG.log" | tee -a "$OUT/summary.txt"; stop_if_fatal $rc smoke

echo "== bench" | tee -a "$OUT/summary.txt"
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_$TAG.json" | tee -a "$OUT/summary.txt"; stop_if_fatal $rc bench
timeout -k 10 300 python bench.py --dtype f32 --batch 65536 --no-cpu-baseline > "$OUT/bench_f32_$TAG.json" 2>> "$OUT/bench_$TAG.err"
rc=$?; cat "$OUT/bench_f32_$TAG.json" | tee -a "$OUT/summary.txt"; stop_if_fatal $rc bench_f32

echo "== rocprofv3 kernel trace" | tee -a "$OUT/summary.txt"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
  python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_bench_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; stop_if_fatal $rc rocprof
cd "$ROOT"
find "$OUT/prof_$TAG" -name "*stats*" | head -5 | tee -a "$OUT/summary.txt"
echo "done" | tee -a "$OUT/summary.txt"
