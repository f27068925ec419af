// Microbenchmark (diagnostic tool): v_fma_f32 vs v_pk_fma_f32 issue rate and latency at 1 wave/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
template <int ILP>
__global__ __launch_bounds__(64) void f32chain(float* out, long long* cyc, int iters) {
  float a[ILP];
  for (int i = 0; i < ILP; ++i) a[i] = threadIdx.x * 1e-3f + i;
  const float b = 1.0000001f + threadIdx.x * 1e-9f;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int i = 0; i < ILP; ++i) a[i] = fmaf(a[i], b, 1e-9f);
  }
  const long long t1 = clock64();
  float s = 0; for (int i = 0; i < ILP; ++i) s += a[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int ILP>
__global__ __launch_bounds__(64) void pkchain(float* out, long long* cyc, int iters) {
  v2f a[ILP];
  for (int i = 0; i < ILP; ++i) a[i] = v2f{threadIdx.x * 1e-3f + i, threadIdx.x * 2e-3f + i};
  const v2f b = v2f{1.0000001f + threadIdx.x * 1e-9f, 1.0000002f};
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int i = 0; i < ILP; ++i) a[i] = a[i] * b + 1e-9f;
  }
  const long long t1 = clock64();
  float s = 0; for (int i = 0; i < ILP; ++i) s += a[i].x + a[i].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <typename K>
static void run(const char* name, K kern, int grid, int iters, int ops) {
  float* o; long long* c;
  hipMalloc(&o, sizeof(float) * grid * 64); hipMalloc(&c, sizeof(long long) * grid);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, o, c, 10); hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(grid), dim3(64), 0, 0, o, c, iters); hipDeviceSynchronize();
  long long h[4096]; hipMemcpy(h, c, sizeof(long long) * grid, hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < grid; ++i) avg += h[i]; avg /= grid;
  printf("%-12s grid %5d: cycles per instr %.2f\n", name, grid, avg / ((double)iters * ops));
  hipFree(o); hipFree(c);
}
int main() {
  for (int g : {1024, 2048}) {
    run("f32 ilp1", f32chain<1>, g, 20000, 8); run("f32 ilp4", f32chain<4>, g, 20000, 32); run("f32 ilp16", f32chain<16>, g, 20000, 128);
    run("pk ilp1", pkchain<1>, g, 20000, 8); run("pk ilp4", pkchain<4>, g, 20000, 32); run("pk ilp16", pkchain<16>, g, 20000, 128);
  }
}
