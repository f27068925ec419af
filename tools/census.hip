// Wave-placement census (diagnostic tool, not part of the library).
// Each single-wave workgroup runs a fixed fp64 FMA workload (ILP 4, like the
// IK loop's issue pattern) and records HW_ID / XCC_ID and its start/end
// s_memrealtime (100 MHz).  Build: hipcc --offload-arch=gfx950 -O3 census.hip -o census
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

struct Rec {
  unsigned hwid, xcc;
  unsigned long long t0, t1;
  double sink;
};

__global__ __launch_bounds__(64) void census(Rec* out, int iters, int active_lanes) {
  unsigned hwid, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double a = threadIdx.x * 1e-3, b = 1.0000001, c = 0.5, d = 0.25, e = 0.125;
  if ((int)threadIdx.x < active_lanes) {
    for (int i = 0; i < iters; ++i) {
      a = fma(a, b, 1e-9);
      c = fma(c, b, 1e-9);
      d = fma(d, b, 1e-9);
      e = fma(e, b, 1e-9);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    Rec r{hwid, xcc, t0, t1, a + c + d + e};
    out[blockIdx.x] = r;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs reported: %d\n", cus);
  const int grids[] = {128, 256, 512, 1024, 2048};
  for (int lanes : {64, 8}) {
    for (int g : grids) {
      Rec* d;
      hipMalloc(&d, sizeof(Rec) * g);
      hipLaunchKernelGGL(census, dim3(g), dim3(64), 0, 0, d, 1000, lanes);  // warm
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(census, dim3(g), dim3(64), 0, 0, d, iters, lanes);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<Rec> h(g);
      hipMemcpy(h.data(), d, sizeof(Rec) * g, hipMemcpyDeviceToHost);
      hipFree(d);
      std::map<unsigned long long, int> per_cu, per_simd;
      std::set<unsigned> xccs;
      unsigned long long tmin = ~0ull, tmax = 0, smax = 0;
      double dmin = 1e30, dmax = 0, dsum = 0;
      for (auto& r : h) {
        const unsigned simd = (r.hwid >> 4) & 3, cu = (r.hwid >> 8) & 15, sh = (r.hwid >> 12) & 1,
                       se = (r.hwid >> 13) & 7;
        const unsigned long long cukey = ((unsigned long long)r.xcc << 32) | (se << 8) | (sh << 4) | cu;
        per_cu[cukey]++;
        per_simd[(cukey << 2) | simd]++;
        xccs.insert(r.xcc);
        tmin = std::min(tmin, r.t0);
        tmax = std::max(tmax, r.t1);
        smax = std::max(smax, r.t0);
        const double dur = (r.t1 - r.t0) / 100.0;  // us
        dmin = std::min(dmin, dur);
        dmax = std::max(dmax, dur);
        dsum += dur;
      }
      int cu_max = 0, simd_max = 0;
      for (auto& kv : per_cu) cu_max = std::max(cu_max, kv.second);
      for (auto& kv : per_simd) simd_max = std::max(simd_max, kv.second);
      printf("lanes=%2d grid=%5d: kernel %.3f ms | xcc %zu cu %zu (max %d waves/cu) simd %zu (max %d/simd) | "
             "wave us min %.1f avg %.1f max %.1f | start spread %.1f us\n",
             lanes, g, ms, xccs.size(), per_cu.size(), cu_max, per_simd.size(), simd_max, dmin, dsum / g, dmax,
             (smax - tmin) / 100.0);
    }
  }
  return 0;
}
