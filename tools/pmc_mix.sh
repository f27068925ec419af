#!/bin/bash
# Instruction-mix PMC passes for one IK configuration (counters only with --kernel-trace).
# usage: bash tools/pmc_mix.sh TAG B dtype ppw reps   (PMC_PASSES="p1 p3" selects passes;
# IKGRASP_LIB selects the library)
TAG=$1; shift
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
P="python3 $ROOT/tools/pmc_probe.py"
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
pass() { name=$1; shift; cnt=$1; shift;
  case " ${PMC_PASSES:-p1 p2 p3 p4 p5} " in *" $name "*) ;; *) return 0;; esac
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d $OUT/$name -o run -- $P "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
pass p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" "$@"
pass p2 "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64" "$@"
pass p3 "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES" "$@"
pass p4 "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32" "$@"
pass p5 "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INST_CYCLES_SALU" "$@"
echo done
