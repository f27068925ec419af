#!/bin/bash
# Evidence refresh (round 3 on; RTAG names the output dir): GPU tests, smoke, bench lines (C2 default with extras and CPU
# legs, C3, C4 share, C5 share, collision), rocprofv3 kernel-trace summaries, PMC passes.
ROOT=$(pwd); O=$ROOT/gpurun_out/${RTAG:-refresh3}; mkdir -p $O; export TMPDIR=/tmp
fatal() { case $1 in 0) return 0;; *) echo "FATAL $2 rc=$1" | tee -a $O/summary.txt; exit $1;; esac; }
IKG_REPORT_DIR=$O/reports timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" $O/pytest_gpu.log | tail -1 | tee -a $O/summary.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; fatal $? smoke
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench.err; fatal $? bench
b() { n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra "$@" > $O/bench_$n.json 2>> $O/bench.err; fatal $? $n; }
b c3_f32 --dtype f32 --batch 65536
b c3_f64 --dtype f64 --batch 65536
b c4s_f64 --batch 131072 --steps 5
b c4s_f32 --dtype f32 --batch 131072 --steps 5
b c5_f64 --multistart 256 --batch 512 --steps 5
b c5_f32 --multistart 256 --batch 512 --dtype f32 --steps 5
b c2col --collision --steps 20
b c3col_f32 --collision --dtype f32 --batch 65536
b c5col_f32 --collision --multistart 256 --batch 512 --dtype f32 --steps 5
python - <<PY >> $O/summary.txt
import json, glob, os
for f in sorted(glob.glob("$O/bench_*.json")):
    d = json.load(open(f)); print(os.path.basename(f), round(d["ms_per_step"], 3), "ms", round(d["value"] / 1e6, 3), "M/s", "kernel", round(d["roofline"]["kernel_ms"], 3))
PY
cd /tmp
P="python3 $ROOT/tools/pmc_probe.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/prof_c2.json 2>> $O/bench.err; fatal $? profc2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $ROOT/bench.py --steps 10 --warmup 2 --dtype f32 --batch 65536 --no-cpu-baseline --no-extra > $O/prof_c3.json 2>> $O/bench.err; fatal $? profc3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2col -o run -- python3 $ROOT/bench.py --collision --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/prof_c2col.json 2>> $O/bench.err; fatal $? profcol
for cfg in "4096 f64" "65536 f32"; do set -- $cfg
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch_b$1_$2 -o run -- $P $1 $2 32 3 > $O/pmc_fetch_$1_$2.log 2>&1; fatal $? pmcf
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc/write_b$1_$2 -o run -- $P $1 $2 32 3 > $O/pmc_write_$1_$2.log 2>&1; fatal $? pmcw
done
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch_b4096_f64_col -o run -- $P 4096 f64 32 3 --collision > $O/pmc_fetch_col.log 2>&1; fatal $? fcol
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc/write_b4096_f64_col -o run -- $P 4096 f64 32 3 --collision > $O/pmc_write_col.log 2>&1; fatal $? wcol
mkdir -p $O/flops/f64_b4096 $O/flops/f32_b65536
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $O/flops/f64_b4096/ops -o run -- $P 4096 f64 32 3 --save-iters $O/flops/f64_b4096/iters.npy > $O/flops_f64.log 2>&1; fatal $? flops64
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/flops/f32_b65536/ops -o run -- $P 65536 f32 32 3 --save-iters $O/flops/f32_b65536/iters.npy > $O/flops_f32.log 2>&1; fatal $? flops32
echo ALLDONE | tee -a $O/summary.txt
