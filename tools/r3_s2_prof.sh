#!/bin/bash
# Round 3 (session 2): C3/C5 config tests against the oracle, rocprofv3
# kernel-trace summaries (C2 fp64, C3 fp32), packed-kernel FP counters,
# collision-solve HBM counters.
ROOT=$(pwd); O=$ROOT/gpurun_out/s2b; mkdir -p $O; export TMPDIR=/tmp
fatal() { case $1 in 0) return 0;; *) echo "FATAL $2 rc=$1"; exit $1;; esac; }
IKG_REPORT_DIR=$O/reports timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -v -s --timeout 300 --timeout-method thread > $O/pytest_configs.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|c3_vs|c5_share" $O/pytest_configs.log | tail -20
[ $rc -le 1 ] || exit $rc
cd /tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1; fatal $? list
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
  python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/prof_c2.json 2> $O/prof_c2.err; fatal $? profc2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --dtype f32 --batch 65536 --no-cpu-baseline --no-extra > $O/prof_c3.json 2> $O/prof_c3.err; fatal $? profc3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2col -o run -- \
  python3 $ROOT/bench.py --collision --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/prof_c2col.json 2> $O/prof_c2col.err; fatal $? profcol
P="python3 $ROOT/tools/pmc_probe.py"
mkdir -p $O/flops/f32_b65536
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
  SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/flops/f32_b65536/ops -o run -- $P 65536 f32 32 3 \
  --save-iters $O/flops/f32_b65536/iters.npy > $O/flops_f32.log 2>&1; fatal $? flops32
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch_b4096_f64_col -o run -- $P 4096 f64 32 3 --collision > $O/pmc_fetch_col.log 2>&1; fatal $? fcol
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc/write_b4096_f64_col -o run -- $P 4096 f64 32 3 --collision > $O/pmc_write_col.log 2>&1; fatal $? wcol
echo ALLDONE
