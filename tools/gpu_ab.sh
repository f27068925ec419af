#!/bin/bash
# GPU parity tests + interleaved per-iteration timing of the built library and
# any variant builds (tools/build_variants.sh).  usage: bash tools/gpu_ab.sh TAG
TAG=${1:-ab}; OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
N=motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/ablate.py 4096 f64 "$N/libikgrasp.so $N/var/*.so" > $OUT/t_f64.txt 2>&1 || exit $?
timeout -k 10 200 python tools/ablate.py 65536 f32 "$N/libikgrasp.so $N/var/*.so" > $OUT/t_f32.txt 2>&1 || exit $?
grep -h "B=" $OUT/t_*.txt
exit $rc
