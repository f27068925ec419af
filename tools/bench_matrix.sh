#!/bin/bash
# Bench every BASELINE config that fits one GPU (per-GPU shares of the 8-GPU configs).
TAG=${1:-r01}
OUT=gpurun_out/matrix_$TAG
mkdir -p $OUT
run() { name=$1; shift; timeout -k 10 240 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err; rc=$?;
        echo "$name rc=$rc $(python -c "import json,sys; d=json.load(open('$OUT/$name.json')); print(f\"value={d['value']:.4g} problems/s={d['problems_per_s']:.4g} ms/step={d['ms_per_step']:.3f} conv={d['converged_fraction']:.3f}\")" 2>/dev/null)";
        [ $rc -le 1 ] || exit $rc; }
run c2_b4096_f64
run c3_b65536_f32 --dtype f32 --batch 65536 --no-cpu-baseline
run c3_b65536_f64 --dtype f64 --batch 65536 --no-cpu-baseline
run c4share_b131072_f64 --dtype f64 --batch 131072 --no-cpu-baseline
run c4share_b131072_f32 --dtype f32 --batch 131072 --no-cpu-baseline
run c5share_ms256x512_f32 --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline
run c5share_ms256x512_f64 --dtype f64 --batch 512 --multistart 256 --no-cpu-baseline
run c2_yaw_b4096_f64 --yaw 0.785398 --no-cpu-baseline
