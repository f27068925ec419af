# records for any q0 layout, packed always medium-range trig: the GPU suite, then
# bench lines (C2 f64/f32, C3) and random-seed / multistart / collision configs
mkdir -p gpurun_out/r4i
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4i/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r4i/pytest_gpu.log; grep -E "^FAILED|Error" gpurun_out/r4i/pytest_gpu.log | head -10
[ $rc -le 1 ] || exit $rc
b() { n=$1; shift; timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra "$@" > gpurun_out/r4i/$n.json 2>> gpurun_out/r4i/err.log || exit 3; }
for rep in 1 2; do
  b c2_$rep --steps 20 --warmup 3
  b c2f32_$rep --steps 20 --warmup 3 --dtype f32
  b c3_$rep --steps 10 --warmup 2 --dtype f32 --batch 65536
done
b c2col --collision --steps 20 --warmup 3
b c5_f64 --multistart 256 --batch 512 --steps 5 --warmup 1
b c5_f32 --multistart 256 --batch 512 --steps 5 --warmup 1 --dtype f32
b c5col_f32 --collision --multistart 256 --batch 512 --dtype f32 --steps 5 --warmup 1
b c3col_f32 --collision --dtype f32 --batch 65536 --steps 10 --warmup 2
python - <<PY
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4i/*.json")):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 4), "ms kernel", round(d["roofline"]["kernel_ms"], 4), round(d["value"]/1e6, 4), "M/s")
PY
