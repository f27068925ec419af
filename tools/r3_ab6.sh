#!/bin/bash
ROOT=$(pwd); O=$ROOT/gpurun_out/ab6; mkdir -p $O
L="$ROOT/ab_libs/*.so"
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2col_f64.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2_f64.txt 2>&1 || exit 3
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=6 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" > $O/c3col_f32.txt 2>&1 || exit 3
grep -H median $O/*.txt
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $ROOT/tools/ablate.py 4096 f64 "$ROOT/ab_libs/lib_cur.so" > $O/prof.log 2>&1 || exit 3
