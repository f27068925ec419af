#!/bin/bash
# VERDICT r5 item 3 (fp64 throughput regime) and item 5 (multi-start traffic):
# SQ occupancy/issue counters of the fp64 pair kernel at the C4 share
# (131,072 problems) and the C5 share (256 seeds x 512 targets) for the product
# library and a 3-wave build (csrc EXTRA=-DIKG_PAIR_MINW64=3 -> ab_libs/w3.so),
# an interleaved timing A/B of the two, and FETCH/WRITE passes of the
# multi-start lines.  Outputs under gpurun_out/$TAG.
TAG=${TAG:?TAG=name}; O=gpurun_out/$TAG; mkdir -p $O
P=motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/libikgrasp.so
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY"
stop() { [ $1 -eq 0 ] || { echo "FATAL $2 rc=$1"; exit $1; }; }
ABTAG=$TAG/ab ABLIBS="$PWD/$P $PWD/ab_libs/w3.so" CONFIGS="c4s_f64 rand_f64 c2_f64" timeout -k 10 300 bash tools/ab.sh; stop $? ab
for lib in prod w3; do
  [ $lib = prod ] && L=$PWD/$P || L=$PWD/ab_libs/w3.so
  IKGRASP_LIB=$L bash tools/pmc_pass.sh $O/pmc/sq_b131072_f64_$lib "$SQ" 131072 f64 32 2; stop $? sq1
  IKGRASP_LIB=$L bash tools/pmc_pass.sh $O/pmc/sq_b512_f64_s256_$lib "$SQ" 512 f64 32 2 --multistart 256; stop $? sq2
done
bash tools/pmc_pass.sh $O/pmc/fetch_b512_f64_s256 FETCH_SIZE 512 f64 32 3 --multistart 256; stop $? f1
bash tools/pmc_pass.sh $O/pmc/write_b512_f64_s256 WRITE_SIZE 512 f64 32 3 --multistart 256; stop $? w1
bash tools/pmc_pass.sh $O/pmc/fetch_b512_f32_s256 FETCH_SIZE 512 f32 32 3 --multistart 256; stop $? f2
bash tools/pmc_pass.sh $O/pmc/write_b512_f32_s256 WRITE_SIZE 512 f32 32 3 --multistart 256; stop $? w2
bash tools/pmc_pass.sh $O/pmc/fetch_b512_f32_s256_col FETCH_SIZE 512 f32 32 3 --multistart 256 --collision; stop $? f3
bash tools/pmc_pass.sh $O/pmc/write_b512_f32_s256_col WRITE_SIZE 512 f32 32 3 --multistart 256 --collision; stop $? w3
ABTAG=$TAG/budget REPS=2 CONFIGS="c4scol c5col" VARIANTS="IKG_REC_BUDGET_MB=12288,IKG_WS_KEEP_MB=1280 IKG_REC_BUDGET_MB=24576,IKG_WS_KEEP_MB=1280" timeout -k 10 400 bash tools/bench_env_ab.sh; stop $? budget
echo ALLDONE
