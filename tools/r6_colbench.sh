#!/bin/bash
# The collision bench lines (C2, C3 fp32, C5 fp32 + collision) and the default
# line, re-run after tools/pmc_summary.py regenerated profiles/pmc_*_col.json
# (the lines read their `traffic` from those): gpurun -- bash tools/r6_colbench.sh
set -o pipefail
O=gpurun_out/${TAG:-r6col}; mkdir -p $O
b() { n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra "$@" > $O/bench_$n.json 2>> $O/bench.err || exit 1; }
b c2col --collision --steps 20
b c3col_f32 --collision --dtype f32 --batch 65536
b c5col_f32 --collision --multistart 256 --batch 512 --dtype f32 --steps 5
timeout -k 10 400 python bench.py > $O/bench_c2.json 2>> $O/bench.err || exit 1
echo ALLDONE
