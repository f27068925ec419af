// Packed fp32 IK kernel, in its own translation unit: it is built
// with the max-ILP machine scheduler (one lane = both arms, 2-vector packed math;
// latency-bound, so ILP beats the default occupancy-first schedule: 1.66 -> 1.49 us
// per update at B = 65,536, while the same flag slows the fp64 pair kernel 17%
// at B = 131,072, tools/ablate.py).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "ikg_device.hpp"
#include "ikg_launch.hpp"
#include "ikg_solve.hpp"
#include "ikgrasp.h"

namespace ikg {

// Packed fp32 layout: one lane per problem, both arms in 2-vectors, so every
// v_pk_{fma,mul,add}_f32 advances both arms and a wave holds 64 problems
// (DESIGN.md §3).  Same loop, same arithmetic as the pair kernel's fp32 path.
//
// WPS (waves per SIMD cap, 0 = none): the kernel claims AGPRs it never uses (an
// empty asm clobber) so that the hardware fits at most WPS of its waves on a
// SIMD -- all 256 AGPRs for WPS = 1; VGPR 171 for WPS = 2 (> 512 / 3).  A
// launch of at most WPS waves per SIMD then cannot be dispatched with more
// waves sharing a SIMD while another idles, which the dispatcher does after
// some kernels (after the collision continuation, 19-46 of 1,024 SIMDs held two
// waves of the next 1,024-wave launch and the kernel took 2.2 ms instead of 1.4;
// tools/placement_probe.py).  The launcher checks the resulting occupancy.
// (amdgpu_waves_per_eu bounds the allocation at the occupancy the cap allows;
// the guarded step's LQ branch is an out-of-line call, and its spills and
// stack frame are touched only when it is taken -- DESIGN.md §3a.5)
// REC = 1: the collision continuation's window checkpoints (ikg_solve.hpp
// kWinOf), written from the first passing iterate on, both arms' by the
// problem's lane; the outputs at that iterate come from window 0's checkpoint
// (solve_pair).  REC = 2, the resume launch: one lane per (listed problem,
// window) task, grid-stride, restarting at the window's checkpoint and
// recording it (the same loop as its own instantiation, solve_pair).
template <class SP, int WPS, bool MED, int REC = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPS == 0 ? 3 : WPS)))
void ikg_packed_batch_kernel(const KModel<float>* __restrict__ m,
                                                              KParams<float> prm, const float* __restrict__ targets,
                                                              const float* __restrict__ q0, int64_t q0_stride,
                                                              int64_t B, int64_t S, float* __restrict__ q_out,
                                                              uint8_t* __restrict__ conv_out,
                                                              int32_t* __restrict__ iters_out,
                                                              float* __restrict__ err_out,
                                                              RecArgs<float> ra = RecArgs<float>{}) {
  if constexpr (WPS == 1) asm volatile("" ::: "a255");
  // v171: at least 172 VGPRs, so 2 waves fit and 3 do not; an AGPR claim
  // instead makes the allocator split the 2-wave budget 128 VGPR / 128 AGPR
  // and spill the loop (with the guarded step's cold branch in the kernel)
  if constexpr (WPS == 2) asm volatile("" ::: "v171");
  if constexpr (REC == 2) {
    constexpr int K = kWinOf<float>;
    const int nw = rec_windows<float>(prm.max_iters);
    // this launch's list entries: [ra.rbase, ra.rbase + n), records in slots 0 .. n - 1
    const int64_t n = max((int64_t)0, min((int64_t)*ra.count - ra.rbase, ra.rcap));
    const int64_t ntask = n * nw;
    const int rl = rec_len(m->n_passive);
    for (int64_t t = (int64_t)blockIdx.x * 64 + threadIdx.x; t < ntask; t += (int64_t)gridDim.x * 64) {
      const int64_t i = t / nw;
      const int w = (int)(t - i * nw);
      const int64_t p = ra.list[ra.rbase + i];
      const int k0 = iters_out[p];
      if (w < k0 / K || !win_flagged(ra.wmask + p * mask_words<float>(prm.max_iters), w)) continue;
      const int64_t tgt = S > 1 ? p / S : p;
      const int64_t row = S > 1 ? p - tgt * S : p;
      v2f RT[9], tT[3];
      hook_target_packed(m, targets + tgt * 12, RT, tT);
      float* ckw = ra.ck + p * ck_per_problem<float>(prm.max_iters) + (int64_t)w * kCkSlot;
      v2f qc = v2f{ckw[kCkQ], ckw[kCkArm + kCkQ]}, qa[kArmDof];
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qa[k] = v2f{ckw[kCkQ + 1 + k], ckw[kCkArm + kCkQ + 1 + k]};
      RecOut<float> ro{ra.rec + i * (int64_t)(prm.max_iters + 1) * rl, ra.nrec + p, q0 + row * q0_stride,
                       q_out + p * m->nq, conv_out + p, iters_out + p, err_out + p * 2, rl, ckw};
      ro.rmask = ra.rmask + p * nw + w;
      ro.k0 = k0;
      ro.it_start = max(k0, w * K);
      ro.it_stop = min((w + 1) * K, prm.max_iters + 1);
      int it;
      bool conv;
      v2f nrm, other;
      solve_pair<v2f, false, SP, MED, 2>(m, prm, 0, RT, tT, qc, qa, it, conv, nrm, other, &ro);
    }
    return;
  }
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= B) return;
  const int64_t tgt = S > 1 ? p / S : p;
  const int64_t row = S > 1 ? p - tgt * S : p;
  v2f RT[9], tT[3];
  hook_target_packed(m, targets + tgt * 12, RT, tT);
  const float* qrow = q0 + row * q0_stride;
  v2f qc = v2f(qrow[m->root_q]), qa[kArmDof];
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) qa[k] = v2f{qrow[m->arm_q[0][k]], qrow[m->arm_q[1][k]]};
  int it;
  bool conv;
  v2f nrm, other;
  if constexpr (REC == 1) {
    const int rl = rec_len(m->n_passive);
    RecOut<float> ro{ra.rec + p * (int64_t)(prm.max_iters + 1) * rl, ra.nrec + p, qrow,
                     q_out + p * m->nq, conv_out + p, iters_out + p, err_out + p * 2, rl,
                     ra.ck + p * ck_per_problem<float>(prm.max_iters)};
    ra.nrec[p] = 0;
    if (solve_pair<v2f, false, SP, MED, 1>(m, prm, 0, RT, tT, qc, qa, it, conv, nrm, other, &ro)) return;
  } else {
    solve_pair<v2f, false, SP, MED>(m, prm, 0, RT, tT, qc, qa, it, conv, nrm, other);
  }
  float* qo = q_out + p * m->nq;
  qo[m->root_q] = qc.x;
  for (int i = 0; i < m->n_passive; ++i) {  // moved only by the first update's clamp (tools.py:21-22)
    const int j = m->passive_q[i];
    const float v = qrow[j];
    qo[j] = it > 0 ? clampq(v, m->lo[j], m->hi[j]) : v;
  }
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) {
    qo[m->arm_q[0][k]] = qa[k].x;
    qo[m->arm_q[1][k]] = qa[k].y;
  }
  if (conv_out) conv_out[p] = conv ? 1 : 0;
  if (iters_out) iters_out[p] = it;
  if (err_out) {
    err_out[p * 2] = nrm.x;
    err_out[p * 2 + 1] = nrm.y;
  }
}

// Experiment knob (tools/dvfs_probe.py): dynamic LDS reserved per single-wave
// workgroup, which caps how many workgroups the dispatcher may put on one CU.
static size_t packed_lds_pad() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("IKG_PACKED_LDS_PAD");
    v = e ? atol(e) : 0;
  }
  return (size_t)v;
}

// SIMDs of the current device (4 per CU), cached per device
static unsigned simd_count() {
  constexpr int kDevs = 64;
  static std::atomic<unsigned> cache[kDevs];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDevs) return 1024;
  unsigned v = cache[dev].load(std::memory_order_relaxed);
  if (v) return v;
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  v = 4u * (unsigned)cus;
  cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// The cap instantiation really fits WPS waves per SIMD (4 WPS single-wave
// workgroups per CU) on this device; otherwise the uncapped kernel runs.
template <int WPS, int REC = 0>
static bool capped_ok() {
  constexpr int kDevs = 64;
  static std::atomic<int> cache[kDevs];  // 0 unknown, 1 ok, 2 not
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDevs) return false;
  int v = cache[dev].load(std::memory_order_relaxed);
  if (!v) {
    int blocks = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &blocks, reinterpret_cast<const void*>(ikg_packed_batch_kernel<SpecNextage, WPS, true, REC>), 64, packed_lds_pad());
    v = (e == hipSuccess && blocks == 4 * WPS) ? 1 : 2;
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

hipError_t launch_packed_batch(const KModel<float>* dmodel, const KParams<float>& prm, const BatchArgs& a,
                               hipStream_t s) {
  const dim3 grid((unsigned)((a.B + 63) / 64));
  const unsigned simds = simd_count();
  const unsigned need = (grid.x + simds - 1) / simds;  // waves per SIMD the launch needs
  RecArgs<float> ra;
  ra.rec = (float*)a.rec;
  ra.nrec = a.rec_n;
  ra.ck = (float*)a.ck;
  ra.list = a.rec_list;
  ra.count = a.rec_count;
  ra.wmask = a.rec_wmask;
  ra.rmask = a.rec_rmask;
  ra.rbase = a.rec_rbase;
  ra.rcap = a.rec_rcap;
  // resume (a.rec_list): the instantiation the batch launch took (need from a.B), grid-stride over tasks
  const dim3 g = a.rec_list ? dim3(resume_waves(std::min<int64_t>(a.B, a.rec_rcap), rec_windows<float>(prm.max_iters), 64)) : grid;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, g, dim3(64), packed_lds_pad(), s, dmodel, prm, (const float*)a.targets,
                       (const float*)a.q0, a.q0_stride, a.B, a.S, (float*)a.q_out, a.converged, a.iters,
                       (float*)a.err_out, ra);
  };
#ifndef IKG_PACKED_REC
#define IKG_PACKED_REC 1
#endif
  if (IKG_PACKED_REC && a.rec) {  // collision continuation checkpoints (0: A/B knob, the trajectory kernel instead)
    // the resume launch (a.rec_list, REC = 2) takes the cap the batch launch took (need from a.B)
    if (need == 1 && capped_ok<1, 1>())
      a.rec_list ? go(ikg_packed_batch_kernel<SpecNextage, 1, true, 2>) : go(ikg_packed_batch_kernel<SpecNextage, 1, true, 1>);
    else if (need == 2 && capped_ok<2, 1>())
      a.rec_list ? go(ikg_packed_batch_kernel<SpecNextage, 2, true, 2>) : go(ikg_packed_batch_kernel<SpecNextage, 2, true, 1>);
    else
      a.rec_list ? go(ikg_packed_batch_kernel<SpecNextage, 0, true, 2>) : go(ikg_packed_batch_kernel<SpecNextage, 0, true, 1>);
    if (a.rec_used) *a.rec_used = true;
    return hipGetLastError();
  }
  // the medium-range trig rule inline for every launch (and every q0 layout,
  // as the fp32 pair kernel): it agrees with the short-series-or-exact rule
  // to rounding, not bit for bit, on steps of 0.025..0.25 rad, and is 2%
  // faster at C3 under this kernel's max-ILP schedule (1.281 against 1.309 ms,
  // profiles/r04/trig/)
  if (need == 1 && capped_ok<1>())
    go(ikg_packed_batch_kernel<SpecNextage, 1, true>);
  else if (need == 2 && capped_ok<2>())
    go(ikg_packed_batch_kernel<SpecNextage, 2, true>);
  else
    go(ikg_packed_batch_kernel<SpecNextage, 0, true>);
  return hipGetLastError();
}

}  // namespace ikg
