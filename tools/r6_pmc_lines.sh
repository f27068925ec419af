#!/bin/bash
# HBM counter passes for the bench lines whose `traffic` had no profile at the
# end of round 6 (C3 fp64, C4 share fp32), one GPU call:
#   gpurun -- bash tools/r6_pmc_lines.sh
# then locally: python tools/pmc_summary.py gpurun_out/r6pmc/pmc f64 65536 r06
#               python tools/pmc_summary.py gpurun_out/r6pmc/pmc f32 131072 r06
set -o pipefail
O=gpurun_out/r6pmc
for cfg in "65536 f64" "131072 f32"; do set -- $cfg
  for c in FETCH_SIZE WRITE_SIZE; do
    n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
    bash tools/pmc_pass.sh $O/pmc/${n}_b$1_$2 $c $1 $2 32 3 || exit $?
  done
done
echo ALLDONE
