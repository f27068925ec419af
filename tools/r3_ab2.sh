#!/bin/bash
# Random-seed (C5-like) and C4-share timing across round-2 / current / no-guard /
# uniform-branch libraries, then bench.py C5 share lines.
ROOT=$(pwd); O=$ROOT/gpurun_out/ab2; mkdir -p $O
L="$ROOT/ab_libs/*.so"
ABL_RANDQ0=1 ABL_ROUNDS=5 timeout -k 10 300 python tools/ablate.py 131072 f64 "$L" > $O/rand_f64_forced.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_RANDQ0=1 ABL_ROUNDS=5 timeout -k 10 300 python tools/ablate.py 131072 f64 "$L" > $O/rand_f64.txt 2>&1 || exit 3
ABL_RANDQ0=1 ABL_ROUNDS=5 timeout -k 10 300 python tools/ablate.py 131072 f32 "$L" > $O/rand_f32_forced.txt 2>&1 || exit 3
ABL_EPS=1e-3 ABL_ROUNDS=5 timeout -k 10 300 python tools/ablate.py 131072 f64 "$L" > $O/c4share_f64.txt 2>&1 || exit 3
grep -H median $O/*.txt
timeout -k 10 300 python bench.py --multistart 256 --batch 512 --dtype f64 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_f64.json 2>$O/c5.err || exit 3
timeout -k 10 300 python bench.py --multistart 256 --batch 512 --dtype f32 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5_f32.json 2>>$O/c5.err || exit 3
python -c "
import json
for n in ('c5_f64','c5_f32'):
    d=json.load(open('$O/'+n+'.json')); print(n, round(d['ms_per_step'],3), 'ms', round(d['value']))"
