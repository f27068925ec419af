# Does C3 fp32 with the collision term take the packed kernel's records under
# the default record budget?  Device memory as seen here, the workspace trace
mkdir -p gpurun_out/r4x
python -c "import torch; p=torch.cuda.get_device_properties(0); print('total_memory', p.total_memory, p.name)" > gpurun_out/r4x/dev.txt 2>&1
IKG_WS_TRACE=1 timeout -k 10 120 python tools/pmc_probe.py 65536 f32 0 1 --collision > gpurun_out/r4x/trace.txt 2>&1 || exit 1
grep -c "alloc rec" gpurun_out/r4x/trace.txt; grep "alloc rec" gpurun_out/r4x/trace.txt | head -3; cat gpurun_out/r4x/dev.txt
