#!/bin/bash
# Round 3: guard trip counts on the GPU (lib_cnt.so), then bench.py smoke
# runs: N=1 default line (extras + CPU legs) and the --gpus 2 gloo rehearsal.
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/r3cb; mkdir -p $OUT
for a in "131072 f64 randq0" "8192 f64 randq0" "4096 f64 zero" "8192 f32 randq0" "8192 f64 randq0 1e-3"; do
  timeout -k 10 120 python tools/sing_count.py $a || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench1.json')); print({k: d[k] for k in ('value','ms_per_step','n_gpus')}); print(json.dumps(d['extra'])[:1500]); print(json.dumps(d['cpu_baseline'])[:1200]); print(json.dumps(d['roofline'])[:800]); print(json.dumps(d['roofline_hbm']))"
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench2.json 2> $OUT/bench2.err || { tail -20 $OUT/bench2.err; exit 3; }
python -c "import json; d=json.load(open('$OUT/bench2.json')); print({k: d[k] for k in ('value','ms_per_step','n_gpus')}, d['config']); print(json.dumps(d['extra']['c4_strong']))"
