# Multi-rank rehearsal on the one-GPU box: bench.py --gpus 2
# spawns 2 ranks on 1 GPU, so it runs as a gloo rehearsal (ranks share the
# device; not a throughput number) and prints the `ranks` block
mkdir -p gpurun_out/r4cc
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r4cc/bench_gpus2_gloo.json 2> gpurun_out/r4cc/bench_gpus2_gloo.err || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r4cc/bench_gpus2_gloo.json"))
print(json.dumps(d["ranks"]), d["n_gpus"], d["config"].get("backend"))
print(json.dumps(d["extra"]["c4_strong"].get("ranks")))
PY
