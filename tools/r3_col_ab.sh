#!/bin/bash
# Collision schedules at C2 / C3: default (records in the batch kernel + pre-screen) against
# IKG_TRAJ_PRESCREEN=0 (first checks inside the record scan), twice each, interleaved.
ROOT=$(pwd); O=$ROOT/gpurun_out/colab; mkdir -p $O
for r in 1 2; do
  for m in default noprescreen; do
    E=""; [ $m = noprescreen ] && E="IKG_TRAJ_PRESCREEN=0"
    env $E timeout -k 10 200 python bench.py --collision --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/c2_${m}_$r.json 2>>$O/err.log || exit 3
    env $E timeout -k 10 200 python bench.py --collision --dtype f32 --batch 65536 --steps 10 --warmup 2 --no-cpu-baseline --no-extra > $O/c3_${m}_$r.json 2>>$O/err.log || exit 3
  done
done
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$O/*.json")):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 3), "M/s")
PY
