# cost of the medium-range trig series (MED) where per-problem seeds are not used:
# IKG_FORCE_MED=1 against the default, interleaved by repetition
mkdir -p gpurun_out/r4g
for rep in 1 2; do
  for med in 0 1; do
    for cfg in "c2 --batch 4096" "c2f32 --batch 4096 --dtype f32" "c3 --batch 65536 --dtype f32"; do
      set -- $cfg; n=$1; shift
      IKG_FORCE_MED=$med timeout -k 10 120 python bench.py --no-cpu-baseline --no-extra --steps 20 --warmup 3 "$@" > gpurun_out/r4g/${n}_med${med}_$rep.json 2>> gpurun_out/r4g/err.log || exit 3
    done
  done
done
python - <<PY
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r4g/*.json")):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 4), "ms kernel", round(d["roofline"]["kernel_ms"], 4))
PY
