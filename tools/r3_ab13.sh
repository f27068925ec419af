#!/bin/bash
ROOT=$(pwd); O=$ROOT/gpurun_out/ab13; mkdir -p $O
L="$ROOT/ab_libs/lib_jc*.so $ROOT/ab_libs/lib_r2.so"
ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 65536 f32 "$L" > $O/c3_f32.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=8 timeout -k 10 300 python tools/ablate.py 131072 f32 "$L" > $O/c4s_f32.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_MS=256 ABL_ROUNDS=8 timeout -k 10 300 python tools/ablate.py 512 f32 "$L" > $O/c5_f32.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f32 "$L" > $O/c2_f32.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2_f64.txt 2>&1 || exit 3
ABL_COLLISION=1 ABL_EPS=1e-3 ABL_ROUNDS=10 timeout -k 10 300 python tools/ablate.py 4096 f64 "$L" > $O/c2col_f64.txt 2>&1 || exit 3
grep -H median $O/*.txt
