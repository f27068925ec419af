#!/bin/bash
# PMC passes (counters only with --kernel-trace; see MI355X_MICROARCH.md rocprofv3 section)
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
P="python3 $ROOT/tools/pmc_probe.py"
pass() { name=$1; shift; cnt=$1; shift;
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $cnt --output-format csv -d $OUT/$name -o run -- $P "$@" > $OUT/$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass fetch_b4096_f64 "FETCH_SIZE" 4096 f64 32 3
pass write_b4096_f64 "WRITE_SIZE" 4096 f64 32 3
pass sq_b4096_f64_ppw32 "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" 4096 f64 32 3
pass sq_b4096_f64_ppw16 "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" 4096 f64 16 3
pass sq_b4096_f64_ppw4 "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" 4096 f64 4 3
pass fetch_b65536_f32 "FETCH_SIZE" 65536 f32 32 3
pass write_b65536_f32 "WRITE_SIZE" 65536 f32 32 3
echo done
