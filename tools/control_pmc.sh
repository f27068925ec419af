#!/bin/bash
# HBM traffic of the controller kernel: FETCH_SIZE / WRITE_SIZE in separate passes
ROOT=$(pwd); OUT=$ROOT/gpurun_out/control_pmc; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 $ROOT/tools/control_bench.py --no-cpu --steps 3 --warmup 1 > $OUT/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
