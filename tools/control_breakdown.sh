set -o pipefail
mkdir -p gpurun_out/cb
for o in task jac J pv pvj err; do
  timeout -k 10 120 python tools/control_bench.py --outputs $o --no-cpu > gpurun_out/cb/$o.json || exit $?
done
python3 - <<'PY'
import json
for o in "task jac J pv pvj err".split():
    d = json.load(open(f"gpurun_out/cb/{o}.json")); r = d["roofline"]
    print(o, round(d["ms_per_launch"], 3), r["algorithmic_bytes_per_state"], round(r["achieved"]), round(r["frac"], 3))
PY
