# Kernel timeline of the --collision bench (C2 fp64 by default; BENCH_ARGS
# adds bench.py options): rocprofv3 kernel trace -> gpurun_out/coltrace/run/
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p "$ROOT/gpurun_out/coltrace/run"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/coltrace/run" -o run -- \
  python3 "$ROOT/bench.py" --collision --steps 3 --warmup 1 ${BENCH_ARGS:-} > "$ROOT/gpurun_out/coltrace/run/bench.json" || exit $?
cd "$ROOT"
python3 tools/trace_timeline.py gpurun_out/coltrace --last 8
