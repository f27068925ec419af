# Multi-start fp32 (C5 share: 256 seeds x 512 targets) under the pair and the
# packed layout, alternating, 3 runs each -> gpurun_out/mslayout/
set -o pipefail
mkdir -p gpurun_out/mslayout
for r in 1 2 3; do
  for v in 1 2; do
    timeout -k 10 120 python bench.py --dtype f32 --batch 512 --multistart 256 --variant $v --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/mslayout/v${v}_$r.json || exit $?
  done
done
python3 - <<'PY'
import json
for v, name in ((1, "pair"), (2, "packed")):
    ms = [json.load(open(f"gpurun_out/mslayout/v{v}_{r}.json"))["ms_per_step"] for r in (1, 2, 3)]
    print(name, [round(x, 3) for x in ms])
PY
