// The fp32 pair kernel for launches of at most one wave per SIMD (C2: 128
// waves on 1,024 SIMDs), in its own translation unit so it can be built with
// the max-ILP machine scheduler (Makefile).  Such a launch lasts as long as one
// wave takes to issue its updates in order; the in-order issue model of the
// default schedule (tools/isa_critpath.py) matches the fp64 C2 loop to 0.1%
// and predicts 14% less for the max-ILP order of the same instructions, but
// measured, the max-ILP build gains 3% on fp32 C2, nothing on fp64 C2 and
// loses 4% with collision records (profiles/r05/ilp/): only the fp32
// record-free launch takes it.  Larger launches (several waves per SIMD hide
// each other's waits) keep the default-scheduled kernel: the max-ILP build
// measured 17% slower at 131,072 problems in round 2.  Same
// source, same arithmetic, same results bit for bit: only the order differs.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ikg_device.hpp"
#include "ikg_launch.hpp"
#include "ikg_solve.hpp"
#include "ikgrasp.h"

namespace ikg {

template <bool MED>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4)))
void ikg_pair_ilp_kernel(const KModel<float>* __restrict__ gm, KParams<float> prm, const float* __restrict__ targets,
                         const float* __restrict__ q0, int64_t q0_stride, int64_t B, int64_t S, int ppw,
                         float* __restrict__ q_out, uint8_t* __restrict__ conv_out, int32_t* __restrict__ iters_out,
                         float* __restrict__ err_out) {
  pair_batch_body<float, false, SpecNextage, MED, false>(gm, prm, targets, q0, q0_stride, B, S, ppw, q_out, conv_out,
                                                         iters_out, err_out);
}

hipError_t launch_pair_ilp(const KModel<float>* dmodel, const KParams<float>& prm, const BatchArgs& a, bool med,
                           size_t lds, hipStream_t s) {
  const dim3 grid((unsigned)((a.B + a.ppw - 1) / a.ppw));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(64), lds, s, dmodel, prm, (const float*)a.targets, (const float*)a.q0,
                       a.q0_stride, a.B, a.S, a.ppw, (float*)a.q_out, a.converged, a.iters, (float*)a.err_out);
  };
  if (med)
    go(ikg_pair_ilp_kernel<true>);
  else
    go(ikg_pair_ilp_kernel<false>);
  return hipGetLastError();
}

}  // namespace ikg
