#!/bin/bash
# kernel traces of the collision lines for timing-only library variants
# (ab_libs/<name>.so): TAG=name LIBS="a b" tools/r6_abl_trace.sh
TAG=${TAG:?TAG=name}
for lib in ${LIBS:?LIBS=names}; do
  for cfg in ${CONFIGS:-c2col c3col}; do
    case $cfg in c2col) A="--collision --steps 20 --warmup 3";; c3col) A="--collision --dtype f32 --batch 65536 --steps 10 --warmup 2";;
      c4scol) A="--collision --batch 131072 --steps 5 --warmup 1";; c5col) A="--collision --multistart 256 --batch 512 --dtype f32 --steps 5 --warmup 1";; esac
    L=/root/repo/ab_libs/$lib.so; [ $lib = head ] && L=/root/repo/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/libikgrasp.so
    OUT=gpurun_out/$TAG/${cfg}_$lib ENV="IKGRASP_LIB=$L" bash tools/kernel_trace.sh $A || exit $?
  done
done
echo ALLDONE
