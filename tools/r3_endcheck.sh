#!/bin/bash
# End-of-session check: smoke, the default bench line, the 2-rank rehearsal.
ROOT=$(pwd); O=$ROOT/gpurun_out/endcheck; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err || { tail -5 $O/bench_g2.err; exit 3; }
python - <<PY
import json
d = json.load(open("$O/bench.json"))
print("N=1", round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 3), "M/s", "cpu", round(d["cpu_baseline"]["value"]), "col", round(d["extra"]["c2_collision"]["ms_per_step"], 3), "c4", round(d["extra"]["c4_strong"]["ms_per_step"], 2))
e = json.load(open("$O/bench_g2.json"))
print("N=2 rehearsal", e["n_gpus"], e["config"]["parallelism"], round(e["ms_per_step"], 3))
PY
