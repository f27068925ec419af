#!/bin/bash
# Round-6 evidence at the round's last code commit, one GPU call:
#   RTAG=r6final tools/refresh.sh  (GPU suite with oracle reports, smoke, every
#   bench line, kernel-trace summaries of C2 / C3 / C2 + collision, HBM and FP-op
#   counter passes), then the collision counter passes of C3 and C5 (the
#   window-checkpoint solves) and a kernel trace of C3 + collision.
# Locally after the call: tools/pmc_summary.py turns the passes into
# profiles/pmc_*_col.json, then the collision bench lines are re-run.
set -o pipefail
RTAG=${RTAG:-r6final} bash tools/refresh.sh || exit $?
O=gpurun_out/${RTAG:-r6final}
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  bash tools/pmc_pass.sh $O/pmc/${n}_b65536_f32_col $c 65536 f32 32 3 --collision || exit $?
  bash tools/pmc_pass.sh $O/pmc/${n}_b512_f32_s256_col $c 512 f32 32 3 --multistart 256 --collision || exit $?
done
OUT=$O/prof_c3col bash tools/kernel_trace.sh --collision --dtype f32 --batch 65536 --steps 10 --warmup 2 || exit $?
echo ALLDONE
