// Microbenchmark (diagnostic tool): does a wave's issue rate depend on how
// many of its lanes are live, and where do single-wave workgroups land?
//   * fp64 FMA chains (ILP 8) with k live lanes (the rest leave at entry);
//   * the same with a DPP exchange and a select per step (the IK loop's mix);
//   * HW_ID / XCC_ID of every wave of a 1024-workgroup grid -> SIMD occupancy.
// Build: hipcc -O3 --offload-arch=gfx950 live.hip -o live
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

template <int ILP, bool MIX>
__global__ __launch_bounds__(64) void chain(double* out, long long* cyc, int iters, int live) {
  if ((int)threadIdx.x >= live) return;
  double a[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) a[i] = threadIdx.x * 1e-3 + i;
  const double b = 1.0000001 + threadIdx.x * 1e-12;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int i = 0; i < ILP; ++i) a[i] = fma(a[i], b, 1e-9);
      if constexpr (MIX) {
        int lo = __double2loint(a[0]), hi = __double2hiint(a[0]);
        lo = __builtin_amdgcn_update_dpp(lo, lo, 0xB1, 0xF, 0xF, false);
        hi = __builtin_amdgcn_update_dpp(hi, hi, 0xB1, 0xF, 0xF, false);
        const double o = __hiloint2double(hi, lo);
        a[1] = a[1] > o ? a[1] : o;
      }
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += a[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(64) void where(unsigned* ids) {
  if (threadIdx.x != 0) return;
  // s_getreg HW_REG_HW_ID (id 4) and HW_REG_XCC_ID (id 20), 32 bits from bit 0
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  ids[2 * blockIdx.x] = hw;
  ids[2 * blockIdx.x + 1] = xcc;
  // keep the wave resident a while so later workgroups see it occupied
  const long long t0 = clock64();
  while (clock64() - t0 < 200000) {
  }
}

template <int ILP, bool MIX>
static void run(int grid, int live, int iters) {
  double* out;
  long long* cyc;
  hipMalloc(&out, sizeof(double) * grid * 64);
  hipMalloc(&cyc, sizeof(long long) * grid);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((chain<ILP, MIX>), dim3(grid), dim3(64), 0, 0, out, cyc, iters, live);
  hipEventRecord(a);
  hipLaunchKernelGGL((chain<ILP, MIX>), dim3(grid), dim3(64), 0, 0, out, cyc, iters, live);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  std::vector<long long> c(grid);
  hipMemcpy(c.data(), cyc, sizeof(long long) * grid, hipMemcpyDeviceToHost);
  double mean = 0;
  for (long long x : c) mean += (double)x;
  mean /= grid;
  const double ops = (double)iters * 8 * (ILP + (MIX ? 3 : 0));
  printf("%s ilp%d grid %5d live %2d: %8.3f ms  cycles/op %.2f\n", MIX ? "mix " : "fma ", ILP, grid, live, ms,
         mean / ops);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  const int iters = 20000;
  for (int grid : {128, 1024, 2048})
    for (int live : {64, 32, 8, 2, 1}) run<8, false>(grid, live, iters);
  for (int grid : {128, 1024})
    for (int live : {64, 8, 2}) run<4, true>(grid, live, iters);
  // placement of 1024 single-wave workgroups
  const int G = 1024;
  unsigned* ids;
  hipMalloc(&ids, sizeof(unsigned) * 2 * G);
  hipLaunchKernelGGL(where, dim3(G), dim3(64), 0, 0, ids);
  std::vector<unsigned> h(2 * G);
  hipMemcpy(h.data(), ids, sizeof(unsigned) * 2 * G, hipMemcpyDeviceToHost);
  std::map<unsigned long long, int> per_simd, per_cu;
  for (int i = 0; i < G; ++i) {
    const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
    const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    const unsigned long long cukey = ((unsigned long long)xcc << 16) | (se << 8) | (sh << 4) | cu;
    per_cu[cukey]++;
    per_simd[(cukey << 2) | simd]++;
  }
  std::map<int, int> hist_simd, hist_cu;
  for (auto& kv : per_simd) hist_simd[kv.second]++;
  for (auto& kv : per_cu) hist_cu[kv.second]++;
  printf("grid %d: %zu distinct SIMDs, %zu distinct CUs\n", G, per_simd.size(), per_cu.size());
  for (auto& kv : hist_simd) printf("  SIMDs holding %d waves: %d\n", kv.first, kv.second);
  for (auto& kv : hist_cu) printf("  CUs holding %d waves: %d\n", kv.first, kv.second);
  return 0;
}
