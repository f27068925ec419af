#!/bin/bash
# FP instruction counters of the pair batch kernel for tools/pmc_flops.py.
# usage (GPU box, repo root): bash tools/pmc_flops.sh B dtype
B=${1:-4096}; DT=${2:-f64}; SFX=$([ "$DT" = f64 ] && echo F64 || echo F32)
ROOT=$(pwd); OUT=$ROOT/gpurun_out/flops/${DT}_b$B; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_$SFX SQ_INSTS_VALU_MUL_$SFX SQ_INSTS_VALU_ADD_$SFX \
  SQ_INSTS_VALU_TRANS_$SFX --output-format csv -d $OUT/ops -o run -- python3 $ROOT/tools/pmc_probe.py $B $DT 32 3 \
  --save-iters $OUT/iters.npy > $OUT/ops.log 2>&1
