#!/bin/bash
# Instruction-mix counters of the packed fp32 kernel per guard variant
# (ab_libs/lib_<name>.so, tools/build_variants.sh): where the guard's cost goes.
# usage: bash tools/guard_pmc.sh TAG B "name..." [randq0 ignored]
TAG=$1 B=$2
for n in $3; do
  IKGRASP_LIB=$(pwd)/ab_libs/lib_$n.so PMC_PASSES="p1 p3 p5" bash tools/pmc_mix.sh ${TAG}_$n $B f32 0 3 || exit $?
  python3 tools/pmc_agg.py gpurun_out/pmc_${TAG}_$n packed > gpurun_out/pmc_${TAG}_$n/agg.txt
done
