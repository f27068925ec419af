# C3 fp32 with the collision term: packed + trajectory continuation (default) vs
# the pair kernel recording in-batch (budget raised), and C4-share fp64 likewise
mkdir -p gpurun_out/r4f
b() { n=$1; shift; timeout -k 10 200 "$@" > gpurun_out/r4f/$n.json 2>> gpurun_out/r4f/err.log; echo "$n rc=$?"; }
b c3col_default python bench.py --collision --dtype f32 --batch 65536 --steps 10 --warmup 2
b c3col_pairrec env IKG_REC_BUDGET_MB=8192 IKG_REC_PREFER_PAIR=1 python bench.py --collision --dtype f32 --batch 65536 --steps 10 --warmup 2
b c3_plain python bench.py --no-cpu-baseline --no-extra --dtype f32 --batch 65536 --steps 10 --warmup 2
b c3_pair python bench.py --no-cpu-baseline --no-extra --dtype f32 --batch 65536 --steps 10 --warmup 2 --variant 1
b c2col python bench.py --collision --steps 20 --warmup 3
b c4scol_default python bench.py --collision --batch 131072 --steps 5 --warmup 1
b c4scol_rec env IKG_REC_BUDGET_MB=32768 python bench.py --collision --batch 131072 --steps 5 --warmup 1
python - <<PY
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4f/*.json")):
    try:
        d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 3), "M/s")
    except Exception as e: print(f, e)
PY
