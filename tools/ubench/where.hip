// Placement probe (diagnostic tool): one 64-lane workgroup per entry records
// its HW_ID (SIMD, CU, SE) and XCC_ID while spinning ~`spin` 100 MHz ticks, so
// tools/placement_probe.py can count waves per SIMD after a given kernel.
#include <hip/hip_runtime.h>

__global__ void where_kernel(unsigned* ids, long long spin) {
  if (threadIdx.x != 0) return;
  ids[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);       // HW_REG_HW_ID
  ids[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  const unsigned long long r0 = wall_clock64();
  while ((long long)(wall_clock64() - r0) < spin) {
  }
}

extern "C" int where_probe(void* ids, int grid, long long spin, void* stream) {
  hipLaunchKernelGGL(where_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, (unsigned*)ids, spin);
  return (int)hipGetLastError();
}
