#!/bin/bash
# rocprofv3 kernel traces of the collision lines, the head library against a
# baseline build (ab_libs/r6base.so): TAG=name tools/r6_trace.sh
TAG=${TAG:?TAG=name}
for cfg in c2col c3col; do
  case $cfg in c2col) A="--collision --steps 20 --warmup 3";; c3col) A="--collision --dtype f32 --batch 65536 --steps 10 --warmup 2";; esac
  OUT=gpurun_out/$TAG/${cfg}_head bash tools/kernel_trace.sh $A || exit $?
  OUT=gpurun_out/$TAG/${cfg}_base ENV="IKGRASP_LIB=/root/repo/ab_libs/r6base.so" bash tools/kernel_trace.sh $A || exit $?
done
echo ALLDONE
