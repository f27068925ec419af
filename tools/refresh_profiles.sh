#!/bin/bash
# Round-end evidence in one GPU session: parity tests, smoke, bench lines,
# rocprofv3 kernel-trace summary, PMC FETCH/WRITE passes, collision and
# config-matrix benches.  Writes gpurun_out/refresh/; tools/collect_profiles.py
# copies the judged files into profiles/<round>/.
ROOT=$(pwd); O=$ROOT/gpurun_out/refresh; mkdir -p $O; export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 0;; *) echo "FATAL $2 rc=$1" | tee -a $O/summary.txt; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; fatal $? pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; fatal $? smoke
timeout -k 10 300 python bench.py > $O/bench_b4096_f64.json 2> $O/bench.err; fatal $? bench
timeout -k 10 300 python bench.py --dtype f32 --batch 65536 --no-cpu-baseline > $O/bench_b65536_f32.json 2>> $O/bench.err; fatal $? bench32
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f64 -o run -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_f64.json 2>> $O/bench.err; fatal $? prof64
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_f32 -o run -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --dtype f32 --batch 65536 --no-cpu-baseline > $O/prof_f32.json 2>> $O/bench.err; fatal $? prof32
P="python3 $ROOT/tools/pmc_probe.py"
for cfg in "4096 f64" "65536 f32"; do set -- $cfg
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch_b$1_$2 -o run -- $P $1 $2 32 3 > $O/pmc_fetch_$1_$2.log 2>&1; fatal $? pmcf
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc/write_b$1_$2 -o run -- $P $1 $2 32 3 > $O/pmc_write_$1_$2.log 2>&1; fatal $? pmcw
done
cd $ROOT
mkdir -p $O/collision $O/matrix
run() { d=$1; n=$2; shift 2; timeout -k 10 240 python bench.py "$@" > $O/$d/$n.json 2>> $O/bench.err; fatal $? $n; }
run collision c2_f64 --collision --no-cpu-baseline
run collision c3_f32 --collision --dtype f32 --batch 65536 --no-cpu-baseline
run collision c5_f32 --collision --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline
run collision c5_f64 --collision --dtype f64 --batch 512 --multistart 256 --no-cpu-baseline
run collision c4share_f64 --collision --dtype f64 --batch 131072 --no-cpu-baseline
run collision c4share_f32 --collision --dtype f32 --batch 131072 --no-cpu-baseline
IKG_CONT_TRAJ=0 timeout -k 10 240 python bench.py --collision --no-cpu-baseline > $O/collision/c2_f64_interleaved.json 2>> $O/bench.err; fatal $? c2i
IKG_CONT_TRAJ=0 timeout -k 10 240 python bench.py --collision --dtype f32 --batch 65536 --no-cpu-baseline > $O/collision/c3_f32_interleaved.json 2>> $O/bench.err; fatal $? c3i
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_col_c2 -o run -- \
  python3 $ROOT/bench.py --collision --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_col_c2.json 2>> $O/bench.err; fatal $? profcol
cd $ROOT
run matrix c2_yaw_b4096_f64 --yaw 0.785398 --no-cpu-baseline
run matrix c3_b65536_f64 --dtype f64 --batch 65536 --no-cpu-baseline
run matrix c4share_b131072_f64 --dtype f64 --batch 131072 --no-cpu-baseline
run matrix c4share_b131072_f32 --dtype f32 --batch 131072 --no-cpu-baseline
run matrix c5share_ms256x512_f32 --dtype f32 --batch 512 --multistart 256 --no-cpu-baseline
run matrix c5share_ms256x512_f64 --dtype f64 --batch 512 --multistart 256 --no-cpu-baseline
timeout -k 10 240 python tools/collision_bench.py > $O/collision/cq_uniform.json 2>> $O/bench.err; fatal $? cq1
timeout -k 10 240 python tools/collision_bench.py --batch 4096 --converged > $O/collision/cq_solutions.json 2>> $O/bench.err; fatal $? cq2
echo done | tee -a $O/summary.txt
