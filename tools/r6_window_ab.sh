#!/bin/bash
# Round-6 window checkpoints, one GPU call:
#  1. the collision / full-batch / graph tests (SUITE=1: then the rest);
#  2. interleaved A/B of the collision lines: head, IKG_BOX_COVER=0, and the
#     baseline build ab_libs/r6base.so (round 5's records, built from the
#     previous commit);
#  3. rocprofv3 kernel traces of c2col / c3col, head and baseline;
#  4. FETCH_SIZE / WRITE_SIZE passes of the C2 and C3 collision solves, head
#     and baseline (tools/pmc_summary.py --collision turns them into traffic).
# TAG=name [CONFIGS=...] [NOPMC=1] tools/r6_window_ab.sh
TAG=${TAG:?TAG=name}
TAG=$TAG FIRST="tests/test_gpu_collision.py tests/test_gpu_fullbatch.py tests/test_gpu_graph.py" SUITE=${SUITE:-0} bash tools/gpu_tests.sh || exit $?
ABTAG=$TAG/ab REPS=${REPS:-2} CONFIGS="${CONFIGS:-c2col c3col c5col c4scol}" VARIANTS="${VARIANTS:-base IKG_BOX_COVER=0 IKGRASP_LIB=/root/repo/ab_libs/r6base.so}" timeout -k 10 600 bash tools/bench_env_ab.sh || exit $?
TAG=$TAG/trace LIBS="head r6base" CONFIGS="c2col c3col" bash tools/r6_abl_trace.sh || exit $?
[ "${NOPMC:-0}" = 1 ] && exit 0
for lib in head r6base; do
  L=/root/repo/ab_libs/$lib.so; [ $lib = head ] && L=$PWD/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/libikgrasp.so
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    IKGRASP_LIB=$L bash tools/pmc_pass.sh gpurun_out/$TAG/pmc_$lib/${n}_b4096_f64_col $c 4096 f64 32 3 --collision || exit $?
    IKGRASP_LIB=$L bash tools/pmc_pass.sh gpurun_out/$TAG/pmc_$lib/${n}_b65536_f32_col $c 65536 f32 32 3 --collision || exit $?
  done
done
echo ALLDONE
