#!/bin/bash
# Controller row on the GPU: parity tests, benches, kernel trace.
ROOT=$(pwd); O=$ROOT/gpurun_out/control; mkdir -p $O; export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 0;; *) echo "FATAL $2 rc=$1" | tee -a $O/summary.txt; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_control.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; fatal $rc pytest; [ $rc = 0 ] || exit 1
for cfg in "all f64" "task f64" "jac f64" "all f32"; do set -- $cfg
  timeout -k 10 180 python tools/control_bench.py --outputs $1 --dtype $2 > $O/bench_$1_$2.json 2>> $O/bench.err; fatal $? bench_$1_$2
  cat $O/bench_$1_$2.json
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $ROOT/tools/control_bench.py --no-cpu --steps 10 > $O/prof_bench.json 2>> $O/bench.err; fatal $? prof
echo done
