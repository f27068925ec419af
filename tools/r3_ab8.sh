#!/bin/bash
# Compacted collision sweep: C2 / C3 with the collision term and the plain query, then GPU tests.
ROOT=$(pwd); O=$ROOT/gpurun_out/ab8; mkdir -p $O
L="$ROOT/ab_libs/*.so"
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2col_f64.txt 2>&1 || exit 3
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=6 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" > $O/c3col_f32.txt 2>&1 || exit 3
grep -H median $O/*.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $ROOT/bench.py --collision --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/prof_c2col.json 2> $O/prof.err || exit 3
cd $ROOT
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 $O/pytest.log
python -c "
import csv
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'ikg' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')"
