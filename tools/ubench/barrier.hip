// Cost of a two-wave LDS handoff per iteration (the duo layout's exchange):
// a workgroup of W waves runs `iters` iterations of a dependent fp64 FMA chain
// of length L; with SYNC the waves swap 8 doubles through LDS around one
// s_barrier per iteration.  Prints shader cycles per iteration.
//   hipcc --offload-arch=gfx950 -O3 barrier.hip -o barrier && ./barrier
#include <hip/hip_runtime.h>
#include <cstdio>

template <int L, bool SYNC, int W>
__global__ __launch_bounds__(64 * W) void chain(double* out, int iters, long long* cyc) {
  __shared__ double x[2][8][64 * W];
  const int lane = threadIdx.x;
  double a = 1.0 + lane * 1e-9, b = 0.999999;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < L; ++k) a = fma(a, b, 1e-9);
    if constexpr (SYNC) {
      const int par = it & 1;
#pragma unroll
      for (int k = 0; k < 8; ++k) x[par][k][lane] = a + k;
      __syncthreads();
      const int other = (lane + 64) % (64 * W);
      double s = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += x[par][k][other];
      a = a + s * 1e-30;
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 * W + lane] = a;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int L, bool SYNC, int W>
void run(const char* name) {
  const int blocks = 128, iters = 2000;
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(double) * blocks * 64 * W);
  (void)hipMalloc(&cyc, sizeof(long long) * blocks);
  hipLaunchKernelGGL((chain<L, SYNC, W>), dim3(blocks), dim3(64 * W), 0, 0, out, iters, cyc);  // warm-up
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL((chain<L, SYNC, W>), dim3(blocks), dim3(64 * W), 0, 0, out, iters, cyc);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  long long c[blocks];
  (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < blocks; ++i) mean += c[i];
  mean /= blocks;
  printf("%-28s L=%3d waves=%d: %8.1f shader-clock cycles/iter, %.3f us/iter wall\n", name, L, W, mean / iters,
         ms * 1e3 / iters);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<100, false, 1>("chain only");
  run<100, true, 2>("chain + LDS swap + barrier");
  run<100, false, 2>("chain, 2 waves, no sync");
  run<20, false, 1>("chain only");
  run<20, true, 2>("chain + LDS swap + barrier");
  run<0, true, 2>("LDS swap + barrier only");
  return 0;
}
