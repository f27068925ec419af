#!/bin/bash
# Collision continuation A/B: trajectory-first (default) against the
# interleaved continuation (IKG_CONT_TRAJ=0); collision and graph GPU tests first.
# Usage on the GPU box: bash tools/traj_ab.sh [outdir]
O=${1:-gpurun_out/traj}; mkdir -p $O; export TMPDIR=/tmp
fatal() { case $1 in 0) return 0;; *) echo "FATAL $2 rc=$1" | tee -a $O/summary.txt; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_graph.py tests/test_gpu_generic.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log | tee $O/summary.txt; fatal $rc pytest
for mode in 1 0; do
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --no-cpu-baseline > $O/c2_m$mode.json 2>>$O/bench.err; fatal $? c2
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline > $O/c3_m$mode.json 2>>$O/bench.err; fatal $? c3
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline > $O/c5_m$mode.json 2>>$O/bench.err; fatal $? c5
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_c2 -o run -- python3 $OLDPWD/bench.py --collision --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>>$OLDPWD/$O/bench.err; fatal $? prof
cd $OLDPWD
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']))"; done | tee -a $O/summary.txt
