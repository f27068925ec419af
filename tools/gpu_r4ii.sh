# Counter traffic of C3 fp32 with the collision term (the
# line reports counter / algorithmic traffic), then its bench line
ROOT=$(pwd); O=$ROOT/gpurun_out/r4ii; mkdir -p $O; export TMPDIR=/tmp
P="python3 $ROOT/tools/pmc_probe.py"
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch_b65536_f32_col -o run -- $P 65536 f32 32 3 --collision > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc/write_b65536_f32_col -o run -- $P 65536 f32 32 3 --collision > $O/pmc_write.log 2>&1 || exit 1
cd $ROOT
python3 tools/pmc_summary.py $O/pmc f32 65536 r04 --collision 3 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra --collision --dtype f32 --batch 65536 > $O/bench_c3col_f32.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_c3col_f32.json')); print(d['roofline']['kernel']); print(d['roofline_hbm'])"
