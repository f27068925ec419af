// Microbenchmark (diagnostic tool): single-wave issue cost of the 32-bit VALU
// instructions the quad layout leans on (v_mov_b32_dpp quad_perm broadcasts,
// v_cndmask_b32, v_mov_b32) next to fp64 FMAs, one wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ __launch_bounds__(64) void k(float* out, long long* cyc, int iters) {
  int a[8];
  double f[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 3 + i;
#pragma unroll
  for (int i = 0; i < 4; ++i) f[i] = threadIdx.x * 1e-3 + i;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (KIND == 0) a[i] = __builtin_amdgcn_mov_dpp(a[i], 0x55, 0xF, 0xF, false);
        if constexpr (KIND == 1) a[i] = (a[(i + 1) & 7] & 1) ? a[i] : a[(i + 3) & 7];
        if constexpr (KIND == 2) a[i] = a[i] + a[(i + 5) & 7];
        if constexpr (KIND == 3) { if (i < 4) f[i] = fma(f[i], 1.0000001, 1e-9); }
        if constexpr (KIND == 4) {  // fp64 fma + dpp mixed 1:2
          if (i < 4) f[i] = fma(f[i], 1.0000001, 1e-9);
          a[i] = __builtin_amdgcn_mov_dpp(a[i], 0xAA, 0xF, 0xF, false);
        }
      }
    }
  }
  const long long t1 = clock64();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s += (float)f[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, double ops_per_iter) {
  const int grid = 128, iters = 20000;
  float* out;
  long long* cyc;
  hipMalloc(&out, sizeof(float) * grid * 64);
  hipMalloc(&cyc, sizeof(long long) * grid);
  hipLaunchKernelGGL((k<KIND>), dim3(grid), dim3(64), 0, 0, out, cyc, iters);
  hipLaunchKernelGGL((k<KIND>), dim3(grid), dim3(64), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  long long c;
  hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-28s cycles per instruction %.2f\n", name, (double)c / iters / ops_per_iter);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0>("v_mov_b32_dpp quad_perm", 32);
  run<1>("v_cndmask_b32 (+and/cmp)", 32);
  run<2>("v_add_u32", 32);
  run<3>("v_fma_f64 (ILP 4)", 16);
  run<4>("fma_f64 + 2 dpp (per fma)", 16);
  return 0;
}
