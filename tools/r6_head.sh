#!/bin/bash
# Head check at the round's last commit, one GPU call: the GPU suite, smoke and
# the default bench line with the in-tree library the driver will load.
#   TAG=name bash tools/r6_head.sh
TAG=${TAG:?TAG=name}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench.err || exit 1
python -c "import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('value_with_collision'))"
echo ALLDONE
