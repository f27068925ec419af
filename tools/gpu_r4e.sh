mkdir -p gpurun_out/r4e
timeout -k 10 60 tools/ubench/bin_barrier > gpurun_out/r4e/barrier.txt 2>&1; echo "rc=$?"; cat gpurun_out/r4e/barrier.txt
