#!/bin/bash
# Interleaved A/B of environment knobs on bench.py configurations, one process
# per run (a knob read once per process, e.g. IKG_SCAN_CERT, IKG_REC_BUDGET_MB).
#   ABTAG=r5cert CONFIGS="c2col c3col" VARIANTS="IKG_SCAN_CERT=0 IKG_SCAN_CERT=1" REPS=3 tools/bench_env_ab.sh
# A variant is NAME=VALUE[,NAME=VALUE...] or "base" (no change).
# Writes gpurun_out/$ABTAG/<config>__<variant>__<rep>.json and a summary table
# (ms per step, kernel ms) to gpurun_out/$ABTAG/summary.txt.
ABTAG=${ABTAG:?ABTAG=name}
O=gpurun_out/$ABTAG
mkdir -p $O
declare -A ARGS=(
  [c2]="--steps 20 --warmup 3"
  [c2f32]="--dtype f32 --steps 20 --warmup 3"
  [c2col]="--collision --steps 20 --warmup 3"
  [c3]="--dtype f32 --batch 65536 --steps 10 --warmup 2"
  [c3col]="--collision --dtype f32 --batch 65536 --steps 10 --warmup 2"
  [c3col64]="--collision --dtype f64 --batch 65536 --steps 5 --warmup 2"
  [c4s]="--batch 131072 --steps 5 --warmup 1"
  [c4scol]="--collision --batch 131072 --steps 5 --warmup 1"
  [c2col32]="--collision --dtype f32 --steps 20 --warmup 3"
  [c5col]="--collision --multistart 256 --batch 512 --dtype f32 --steps 5 --warmup 1"
)
for rep in $(seq 1 ${REPS:-3}); do
  for cfg in $CONFIGS; do
    for v in $VARIANTS; do
      f=$O/${cfg}__${v//[=,\/]/_}__$rep.json
      env $( [ "$v" = base ] || echo $v | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra ${ARGS[$cfg]} > $f 2>> $O/bench.err
      rc=$?; [ $rc -eq 0 ] || { echo "FATAL $cfg $v rc=$rc"; exit $rc; }
    done
  done
done
python - <<PY | tee $O/summary.txt
import json, glob, os, collections
rows = collections.defaultdict(list)
for f in sorted(glob.glob("$O/*.json")):
    parts = os.path.basename(f)[:-5].split("__")
    cfg, v, rep = parts[0], "__".join(parts[1:-1]), parts[-1]
    d = json.load(open(f))
    rows[(cfg, v)].append((d["ms_per_step"], d["roofline"]["kernel_ms"]))
for (cfg, v), r in sorted(rows.items()):
    ms = sorted(x[0] for x in r); km = sorted(x[1] for x in r)
    print(f"{cfg:10s} {v:28s} ms/step median {ms[len(ms)//2]:.4f} (min {ms[0]:.4f})  kernel median {km[len(km)//2]:.4f}  n={len(r)}")
PY
echo ALLDONE
