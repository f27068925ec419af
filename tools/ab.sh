#!/bin/bash
# Interleaved A/B of the libraries in ab_libs/*.so (tools/ablate.py, one process,
# every library in turn per round).  Replaces round 3's one-off r3_ab*.sh.
#   ABTAG=<dir under gpurun_out>  CONFIGS="c2_f64 c2_f64_forced c3_f32 rand_f64 c2col_f64 c4s_f64"
#   ABTESTS=1: then the GPU tests on the in-tree library
ROOT=$(pwd); O=$ROOT/gpurun_out/${ABTAG:-ab}; mkdir -p $O
L=${ABLIBS:-"$ROOT/ab_libs/*.so"}  # ABLIBS: space-separated library paths or globs
run() {  # name rounds batch dtype [env...]
  n=$1 r=$2 b=$3 d=$4; shift 4
  env ABL_ROUNDS=$r "$@" timeout -k 10 300 python tools/ablate.py $b $d "$L" > $O/$n.txt 2>&1 || exit 3
}
for c in ${CONFIGS:-c2_f64 c2_f64_forced c3_f32 rand_f64}; do
  case $c in
    c2_f64) run $c 12 4096 f64 ABL_EPS=1e-3 ;;
    c2_f64_forced) run $c 8 4096 f64 ;;                      # every problem runs 1,000 updates
    c2_f32) run $c 10 4096 f32 ABL_EPS=1e-3 ;;
    c3_f32) run $c 8 65536 f32 ABL_EPS=1e-3 ;;
    c4s_f64) run $c 6 131072 f64 ABL_EPS=1e-3 ;;
    c4s_f32) run $c 6 131072 f32 ABL_EPS=1e-3 ;;
    rand_f64) run $c 6 131072 f64 ABL_EPS=1e-3 ABL_RANDQ0=1 ;;
    rand_f32) run $c 6 131072 f32 ABL_EPS=1e-3 ABL_RANDQ0=1 ;;
    big_f32) run $c 3 1048576 f32 ABL_EPS=1e-3 ABL_RANDQ0=1 ;;     # C5-sized launch (3+ waves per SIMD)
    c2col_f64) run $c 10 4096 f64 ABL_EPS=1e-3 ABL_COLLISION=1 ;;
    c3col_f32) run $c 6 65536 f32 ABL_EPS=1e-3 ABL_COLLISION=1 ;;
    c3colrec_f32) run $c 6 65536 f32 ABL_EPS=1e-3 ABL_COLLISION=1 IKG_REC_BUDGET_MB=8192 IKG_REC_PREFER_PAIR=1 ;;
    c4scol_f64) run $c 4 131072 f64 ABL_EPS=1e-3 ABL_COLLISION=1 ;;
    c3colbig_f32) run $c 6 65536 f32 ABL_EPS=1e-3 ABL_COLLISION=1 IKG_REC_BUDGET_MB=8192 ;;  # records if the layout writes them
    c2col_f64_nopool) run $c 10 4096 f64 ABL_EPS=1e-3 ABL_COLLISION=1 IKG_WS_POOL=0 ;;
    c3col_f32_nopool) run $c 6 65536 f32 ABL_EPS=1e-3 ABL_COLLISION=1 IKG_WS_POOL=0 ;;
    c3colbig_f32_nopool) run $c 6 65536 f32 ABL_EPS=1e-3 ABL_COLLISION=1 IKG_REC_BUDGET_MB=8192 IKG_WS_POOL=0 ;;
    c5col_f32) run $c 3 512 f32 ABL_EPS=1e-3 ABL_COLLISION=1 ABL_MS=256 ;;                  # C5 share: 256 seeds x 512 targets
    c2col_f32) run $c 10 4096 f32 ABL_EPS=1e-3 ABL_COLLISION=1 ;;
    c2colpk_f32) run $c 10 4096 f32 ABL_EPS=1e-3 ABL_COLLISION=1 ABL_VARIANT=2 ;;           # packed layout at C2
    *) echo "unknown config $c"; exit 2 ;;
  esac
done
grep -H median $O/*.txt
if [ -n "$ABTESTS" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest_gpu.log 2>&1
  echo "pytest rc=$?"; tail -2 $O/pytest_gpu.log
fi
