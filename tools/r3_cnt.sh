#!/bin/bash
# Guard trip counts (lib_cnt: -DIKG_SING_COUNT) for random-seed and C2 workloads.
export IKG_CNT_LIB=$(pwd)/ab_cnt/lib_cnt.so
for a in "131072 f64 randq0 1e-3" "131072 f32 randq0 1e-3" "8192 f64 randq0 1e-3" "4096 f64 zero 1e-3" "131072 f32 zero 1e-3"; do
  timeout -k 10 120 python tools/sing_count.py $a 2>&1 | grep -v amdgpu.ids || exit 1
done
