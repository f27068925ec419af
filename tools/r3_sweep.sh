#!/bin/bash
tools/batch_sweep.sh || exit 3
python - <<PY
import json, glob, os
fs = glob.glob("gpurun_out/sweep/b*.json")
for f in sorted(fs, key=lambda f: (f.rsplit("_", 1)[-1], int(os.path.basename(f)[1:].split("_")[0]))):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 3), "M/s", d["roofline"]["kernel"])
PY
