# Continuation stretch speed by layout (C2 fp64 --collision): default; one
# problem per continuation wave (IKG_CONT_G=1); hand-off to the pair-layout
# stretch kernel (1 round) with 32 problems per wave and with one mirrored
# problem per wave (IKG_STRETCH_PPW=-1) -> gpurun_out/contlayout/
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
run() {  # name, env...
  local n=$1; shift
  mkdir -p "$ROOT/gpurun_out/contlayout/$n"
  cd /tmp
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/contlayout/$n" -o run -- \
    python3 "$ROOT/bench.py" --collision --steps 3 --warmup 1 > "$ROOT/gpurun_out/contlayout/$n/bench.json" || exit $?
  cd "$ROOT"
}
run a_default IKG_HANDOFF_ROUNDS=0
run b_g1 IKG_CONT_G=1
run c_ho1 IKG_HANDOFF_ROUNDS=1
run d_ho1_mirror IKG_HANDOFF_ROUNDS=1 IKG_STRETCH_PPW=-1
python3 tools/trace_timeline.py gpurun_out/contlayout --last 6
