#!/bin/bash
# Batch-size sweep of the headline path through bench.py (HIP events, device-resident
# targets): how converged solves/s grows as the batch fills the 1,024 SIMDs.
# Writes gpurun_out/sweep/*.json; copy into profiles/<round>/sweep/.
O=gpurun_out/sweep; mkdir -p $O
for dt in f64 f32; do
  for B in 1024 4096 16384 65536 262144 1048576; do
    timeout -k 10 240 python bench.py --dtype $dt --batch $B --steps 5 --warmup 1 --no-cpu-baseline --no-extra \
      > $O/b${B}_$dt.json 2>> $O/sweep.err
    rc=$?; if [ $rc -ne 0 ]; then echo "FATAL B=$B $dt rc=$rc" | tee -a $O/summary.txt; exit $rc; fi
    echo "B=$B $dt done" | tee -a $O/summary.txt
  done
done
