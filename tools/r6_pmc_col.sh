#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the C2 and C3 collision solves for one
# library and environment: TAG=name [LIB=path] [ENVV="K=V ..."] tools/r6_pmc_col.sh
TAG=${TAG:?TAG=name}
L=${LIB:-$PWD/motion-planning-and-control-for-dual-manipulator-robot_amd/ikgrasp/_native/libikgrasp.so}
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  env $ENVV IKGRASP_LIB=$L bash tools/pmc_pass.sh gpurun_out/$TAG/${n}_b4096_f64_col $c 4096 f64 32 3 --collision || exit $?
  env $ENVV IKGRASP_LIB=$L bash tools/pmc_pass.sh gpurun_out/$TAG/${n}_b65536_f32_col $c 65536 f32 32 3 --collision || exit $?
done
echo ALLDONE
