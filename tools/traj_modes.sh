# trajectory continuation: tests (default, separate launches, pre-screen on), timing by mode
O=gpurun_out/traj4; mkdir -p $O; export TMPDIR=/tmp
run() { n=$1; shift; timeout -k 10 200 env "$@" python bench.py --collision --no-cpu-baseline > $O/$n.json 2>>$O/err || exit 1
        python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3))"; }
run3() { n=$1; shift; timeout -k 10 200 env "$@" python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline > $O/$n.json 2>>$O/err || exit 1
        python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3))"; }
PT="python -u -m pytest tests/test_gpu_collision.py -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
IKG_TRAJ_FUSE=0 timeout -k 10 400 $PT -k "traj or fp64" > $O/pytest_sep.log 2>&1 || { tail -30 $O/pytest_sep.log; exit 1; }
IKG_TRAJ_PRESCREEN=1 timeout -k 10 400 $PT -k "traj or fp64" > $O/pytest_pre.log 2>&1 || { tail -30 $O/pytest_pre.log; exit 1; }
tail -1 $O/pytest.log; tail -1 $O/pytest_sep.log; tail -1 $O/pytest_pre.log
run c2_old IKG_CONT_TRAJ=0
run c2_def
run c2_sep IKG_TRAJ_FUSE=0 IKG_TRAJ_WINDOW=1001
run c2_pre IKG_TRAJ_PRESCREEN=1
run c2_w64 IKG_TRAJ_WINDOW=64
run3 c3_old IKG_CONT_TRAJ=0
run3 c3_def
run3 c3_nopre IKG_TRAJ_PRESCREEN=0
run3 c3_sep IKG_TRAJ_FUSE=0 IKG_TRAJ_WINDOW=1001
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_c2 -o run -- python3 $OLDPWD/bench.py --collision --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2>>$OLDPWD/$O/err
