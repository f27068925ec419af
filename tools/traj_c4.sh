O=gpurun_out/c4; mkdir -p $O
for mode in 1 0; do
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f64 --batch 131072 --no-cpu-baseline > $O/c4_f64_m$mode.json 2>>$O/err || exit 1
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f32 --batch 131072 --no-cpu-baseline > $O/c4_f32_m$mode.json 2>>$O/err || exit 1
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f64 --batch 512 --multistart 256 --no-cpu-baseline > $O/c5_f64_m$mode.json 2>>$O/err || exit 1
done
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']))"; done
