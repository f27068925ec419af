# records in the batch kernel (default) vs the trajectory kernel (IKG_TRAJ_REC=0) vs interleaved
O=gpurun_out/rec; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_collision.py tests/test_gpu_graph.py tests/test_gpu_jit.py tests/test_gpu_generic.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "IKG_TRAJ_REC=1" "X=1" "IKG_CONT_TRAJ=0"; do
  n=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 200 python bench.py --collision --no-cpu-baseline > $O/c2_$n.json 2>>$O/err || exit 1
  env $cfg timeout -k 10 200 python bench.py --collision --dtype f32 --batch 16384 --no-cpu-baseline > $O/b16k_f32_$n.json 2>>$O/err || exit 1
done
env timeout -k 10 200 python bench.py --no-cpu-baseline > $O/c2_nocol.json 2>>$O/err || exit 1
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), round(d['value']))"; done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_c2 -o run -- python3 $OLDPWD/bench.py --collision --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>>$OLDPWD/$O/err
