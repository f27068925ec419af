// Microbenchmark (diagnostic tool): fp64/fp32 FMA dependent latency and issue
// rate at 1 wave per SIMD, and the cost of cross-lane moves (DPP, ds_swizzle,
// LDS round trip).  Prints shader-clock cycles per loop iteration.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ILP, typename T>
__global__ __launch_bounds__(64) void chain(T* out, long long* cyc, int iters) {
  T a[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) a[i] = threadIdx.x * T(1e-3) + i;
  const T b = T(1.0000001) + threadIdx.x * T(1e-12);
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int i = 0; i < ILP; ++i) a[i] = fma(a[i], b, T(1e-9));
  }
  const long long t1 = clock64();
  T s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += a[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent chain through a DPP row_shr:1 move (fp64 = 2 movs) + add
__global__ __launch_bounds__(64) void dppchain(double* out, long long* cyc, int iters) {
  double a = threadIdx.x * 1e-3;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int lo = __double2loint(a), hi = __double2hiint(a);
      lo = __builtin_amdgcn_update_dpp(lo, lo, 0x111, 0xF, 0xF, false);
      hi = __builtin_amdgcn_update_dpp(hi, hi, 0x111, 0xF, 0xF, false);
      a = fma(__hiloint2double(hi, lo), 0.999, 1e-9);
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent chain through ds_swizzle (broadcast lane 0 of each 8-group) + fma
__global__ __launch_bounds__(64) void swzchain(double* out, long long* cyc, int iters) {
  double a = threadIdx.x * 1e-3;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int lo = __double2loint(a), hi = __double2hiint(a);
      // bitmode: and_mask=0x18, or_mask=0, xor_mask=0 -> offset = and | (or<<5) | (xor<<10)
      lo = __builtin_amdgcn_ds_swizzle(lo, 0x18);
      hi = __builtin_amdgcn_ds_swizzle(hi, 0x18);
      a = fma(__hiloint2double(hi, lo), 0.999, 1e-9);
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent chain through an LDS write + read of a neighbour's value
__global__ __launch_bounds__(64) void ldschain(double* out, long long* cyc, int iters) {
  __shared__ double s[64];
  double a = threadIdx.x * 1e-3;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[threadIdx.x] = a;
      __builtin_amdgcn_wave_barrier();
      a = fma(s[threadIdx.x ^ 1], 0.999, 1e-9);
      __builtin_amdgcn_wave_barrier();
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent sqrt / rcp chain (fp64)
__global__ __launch_bounds__(64) void sqrtchain(double* out, long long* cyc, int iters) {
  double a = 2.0 + threadIdx.x * 1e-3;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a = sqrt(a) + 1.0;
  }
  const long long t1 = clock64();
  out[blockIdx.x * 64 + threadIdx.x] = a;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
static void run(const char* name, K kern, int grid, int iters, int per_iter_ops) {
  double* o;
  long long* c;
  hipMalloc(&o, sizeof(double) * grid * 64);
  hipMalloc(&c, sizeof(long long) * grid);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, o, c, 10);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, o, c, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[4096];
  hipMemcpy(h, c, sizeof(long long) * grid, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < grid; ++i) avg += h[i];
  avg /= grid;
  printf("%-14s grid %5d: %8.3f ms  clock64 cycles per op %.2f  wall ns per op %.3f\n", name, grid, ms,
         avg / ((double)iters * per_iter_ops), ms * 1e6 / ((double)iters * per_iter_ops));
  hipFree(o);
  hipFree(c);
}

int main() {
  const int it = 20000;
  for (int g : {128, 1024, 2048}) {
    run("f64 ilp1", chain<1, double>, g, it, 8);
    run("f64 ilp2", chain<2, double>, g, it, 16);
    run("f64 ilp4", chain<4, double>, g, it, 32);
    run("f64 ilp8", chain<8, double>, g, it, 64);
    run("f64 ilp16", chain<16, double>, g, it, 128);

  }
  for (int g : {128, 1024}) {
    run("dpp f64 chain", dppchain, g, it, 8);
    run("swz f64 chain", swzchain, g, it, 8);
    run("lds f64 chain", ldschain, g, it, 8);
    run("sqrt f64 chain", sqrtchain, g, it, 8);
  }
  return 0;
}
