# full GPU test suite + smoke + collision benches (C2, C3, C4 share, C5 share), both continuations
O=gpurun_out/full; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/graph_bisect.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for mode in 1 0; do
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --no-cpu-baseline > $O/c2_f64_m$mode.json 2>>$O/err || exit 1
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline > $O/c3_f32_m$mode.json 2>>$O/err || exit 1
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline > $O/c5_f32_m$mode.json 2>>$O/err || exit 1
  IKG_CONT_TRAJ=$mode timeout -k 10 200 python bench.py --collision --dtype f64 --batch 131072 --no-cpu-baseline > $O/c4_f64_m$mode.json 2>>$O/err || exit 1
done
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']))"; done
