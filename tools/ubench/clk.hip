// Shader clock probe (diagnostic tool): one wave spins ~N us and reports
// s_memtime (shader clock) ticks per s_memrealtime (100 MHz) tick.  Built as a
// shared library so tools/dvfs_probe.py can launch it between kernels.
#include <hip/hip_runtime.h>

__global__ void clk_kernel(unsigned long long* out, long long spin) {
  if (threadIdx.x) return;
  const unsigned long long r0 = wall_clock64(), c0 = clock64();
  unsigned long long r = r0;
  while ((long long)(r - r0) < spin) r = wall_clock64();
  const unsigned long long c1 = clock64();
  out[0] = c1 - c0;
  out[1] = r - r0;
}

extern "C" int clk_probe(void* out, long long spin_ticks, void* stream) {
  hipLaunchKernelGGL(clk_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)out, spin_ticks);
  return (int)hipGetLastError();
}
