// Batched dual-arm grasp-pose IK kernels for MI355X (gfx950).
//
// Hot path replaced: the iteration loop of computeqgrasppose
// (/root/reference/inverse_geometry.py:56-94):
//   FK (:58) -> 2x log6 error (:66-67) -> stop test (:70) -> 2x LOCAL frame
//   Jacobian (:75-76) -> pinv(J) e (:83) -> integrate (:86) -> clamp (:89).
//
// Layout ("pair" variant): two lanes per IK problem, one per arm.  Lane 2p
// owns the left arm of problem p, lane 2p+1 the right arm; both carry the
// shared chest joint.  The 12x13 minimum-norm solve
//     dq = J^T (J J^T)^-1 e
// is split by the block structure J = [c | blockdiag(J_L, J_R)] (c = chest
// column): each lane solves its square 6x6 arm system for two right-hand
// sides (u = J_a^-1 e_a, v = J_a^-1 c_a) and the lanes exchange two scalars
// through DPP to form the Sherman–Morrison chest step
//     s = (u_L.v_L + u_R.v_R) / (1 + |v_L|^2 + |v_R|^2),  dq_c = s,
//     dq_a = u_a - s v_a,
// which equals pinv(J) e whenever J has full row rank.
// No LDS, no barriers; the model tables are read with uniform scalar loads.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "ikg_device.hpp"
#include "ikgrasp.h"
#include "ikg_solve.hpp"
#include "ikg_jit.hpp"
#include "ikg_launch.hpp"

namespace ikg {


// One 64-lane wave per workgroup holding `ppw` problems on lanes [0, 2 ppw).
// A wave's issue cost does not depend on how many lanes are active, so small
// batches are spread with ppw < 32 to occupy every SIMD.
#ifndef IKG_WPE
#define IKG_WPE 0
#endif
// Waves per SIMD the register allocation must leave room for: the guarded
// step's LQ branch (pinv_step_f1) is cold, so spilling around it keeps the
// loop at the occupancy it had without it (fp64 226 VGPRs: 2 waves; fp32
// 103: 4); without the bound its registers took fp64 to 1 wave per SIMD.
// IKG_PAIR_MINW64: the fp64 bound as a build knob (a
// 3-wave build, at most 168 VGPRs, A/B'd in the throughput regime)
#ifndef IKG_PAIR_MINW64
#define IKG_PAIR_MINW64 2
#endif
template <typename T, bool DAMPED, class SP>
constexpr int kPairMinWaves = (kFrame1<SP> && !DAMPED) ? (sizeof(T) == 8 ? IKG_PAIR_MINW64 : 4) : 1;

template <typename T, bool DAMPED, class SP, bool MED = false, int REC = 0>
__global__ __launch_bounds__(64)
#if IKG_WPE
__attribute__((amdgpu_waves_per_eu(1, IKG_WPE)))
#else
// the resume kernel (REC = 2): few waves at most launches, so the registers of
// one wave per SIMD (no spills)
__attribute__((amdgpu_waves_per_eu(REC == 2 ? 1 : kPairMinWaves<T, DAMPED, SP>)))
#endif
void ikg_pair_batch_kernel(const KModel<T>* __restrict__ gm, KParams<T> prm,
                                                            const T* __restrict__ targets,
                                                            const T* __restrict__ q0, int64_t q0_stride, int64_t B,
                                                            int64_t S, int ppw, T* __restrict__ q_out,
                                                            uint8_t* __restrict__ conv_out,
                                                            int32_t* __restrict__ iters_out,
                                                            T* __restrict__ err_out, RecArgs<T> ra = RecArgs<T>{}) {
  // model tables stay in global memory: the compiler hoists them into
  // registers (staging them in LDS and re-reading per iteration measured 8%
  // slower)
  pair_batch_body<T, DAMPED, SP, MED, REC>(gm, prm, targets, q0, q0_stride, B, S, ppw, q_out, conv_out, iters_out,
                                           err_out, ra);
}


#ifdef IKG_STAGE_CLOCK
// the stage stamps of the pair kernel's loop (ikg_solve.hpp g_stage, this
// translation unit's copy); tools/stage_clock.py
extern "C" int ikg_debug_stage(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stage), sizeof(g_stage)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stage), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef IKG_SING_COUNT
extern "C" int ikg_debug_sing(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sing), sizeof(g_sing)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[4] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sing), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// Multi-start best-seed reduction: one wave per target reduces the S seed
// results the pair kernel wrote for it (key = worse hand error, converged
// seeds first, ties to the lower seed index) with DPP/permute wave reductions,
// then copies the winner's outputs.
template <typename T>
__global__ __launch_bounds__(256) void ikg_best_seed_kernel(int64_t T_, int64_t S, int nq,
                                                            const T* __restrict__ q_all,
                                                            const uint8_t* __restrict__ conv_all,
                                                            const int32_t* __restrict__ iters_all,
                                                            const T* __restrict__ err_all, T* __restrict__ q_out,
                                                            uint8_t* __restrict__ conv_out,
                                                            int32_t* __restrict__ iters_out,
                                                            T* __restrict__ err_out, int32_t* __restrict__ best_out) {
  const int lane = threadIdx.x & 63;
  const int64_t tgt = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (tgt >= T_) return;  // whole waves leave together
  T best_key = T(3.0e38);
  int best = 0x7fffffff;
  for (int64_t sd = lane; sd < S; sd += 64) {
    const int64_t k = tgt * S + sd;
    const T worst = fmax(err_all[2 * k], err_all[2 * k + 1]);
    const T key = conv_all[k] ? worst : T(1e30) + worst;
    if (key < best_key) {  // seeds visited in increasing order per lane
      best_key = key;
      best = (int)sd;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const T ok = __shfl_xor(best_key, off);
    const int oi = __shfl_xor(best, off);
    if (ok < best_key || (ok == best_key && oi < best)) {
      best_key = ok;
      best = oi;
    }
  }
  // every key NaN (a non-finite target or seed): no seed wins the compare, so
  // fall back to seed 0 rather than index past the target's S results
  if (best >= S) best = 0;
  const int64_t k = tgt * S + best;
  for (int j = lane; j < nq; j += 64) q_out[tgt * nq + j] = q_all[k * nq + j];
  if (lane == 0) {
    if (conv_out) conv_out[tgt] = conv_all[k];
    if (iters_out) iters_out[tgt] = iters_all[k];
    if (err_out) {
      err_out[2 * tgt] = err_all[2 * k];
      err_out[2 * tgt + 1] = err_all[2 * k + 1];
    }
    if (best_out) best_out[tgt] = best;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ikg_fk_kernel(const KModel<T>* __restrict__ m, const T* __restrict__ q,
                                                     int64_t B, T* __restrict__ hands) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B) return;
  const T* qrow = q + p * m->nq;
#pragma unroll 1
  for (int arm = 0; arm < 2; ++arm) {
    T qc, qa[kArmDof], Rh[9], th[3], sn[7], cs[7];
    load_q(m, arm, qrow, qc, qa);
    trig_exact(qc, qa, sn, cs);
    fk_arm_world<T, SpecGeneric>(m, arm, sn, cs, Rh, th);
    T* out = hands + p * 24 + arm * 12;
#pragma unroll
    for (int i = 0; i < 9; ++i) out[i] = Rh[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) out[9 + i] = th[i];
  }
}

// Diagnostic: each lane of the pair layout dumps its iteration-0 state
// [RT(9) tT(3) Rh(9) th(3) e(6) |e|] = 31 values (tests/test_gpu_parity.py).
template <typename T>
__global__ __launch_bounds__(64) void ikg_pair_state_kernel(const KModel<T>* __restrict__ m,
                                                            const T* __restrict__ targets,
                                                            const T* __restrict__ q0, int64_t q0_stride, int64_t B,
                                                            T* __restrict__ out) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = gid >> 1;
  const int arm = (int)(gid & 1);
  if (p >= B) return;
  T RT[9], tT[3];
  hook_target(m, arm, targets + p * 12, RT, tT);
  T qc, qa[kArmDof], sn[7], cs[7];
  load_q(m, arm, q0 + p * q0_stride, qc, qa);
  trig_exact(qc, qa, sn, cs);
  ArmState<T> st;
  const T nrm = sqrt(arm_fk_error<T, SpecGeneric, false, true>(m, arm, sn, cs, RT, tT, st));
  T el[6];  // world-aligned -> the reference's LOCAL error
  matvec3_t(st.Rh, st.e, el);
  matvec3_t(st.Rh, st.e + 3, el + 3);
  T* o = out + gid * 31;
  for (int i = 0; i < 9; ++i) o[i] = RT[i];
  for (int i = 0; i < 3; ++i) o[9 + i] = tT[i];
  for (int i = 0; i < 9; ++i) o[12 + i] = st.Rh[i];
  for (int i = 0; i < 3; ++i) o[21 + i] = st.th[i];
  for (int i = 0; i < 6; ++i) o[24 + i] = el[i];
  o[30] = nrm;
}

// pin.log6 over a batch of placements (B x 12 -> B x 6).
template <typename T>
__global__ __launch_bounds__(256) void ikg_log6_kernel(const T* __restrict__ M, int64_t B, T* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B) return;
  T R[9], t[3], e[6];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = M[p * 12 + i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = M[p * 12 + 9 + i];
  log6(R, t, e);
#pragma unroll
  for (int i = 0; i < 6; ++i) out[p * 6 + i] = e[i];
}

// ------------------------------------------------------------------ launchers
// Experiment knob (tools/spread_sweep.py): dynamic LDS reserved per
// single-wave workgroup, which caps how many workgroups the dispatcher packs
// onto one CU.
static size_t lds_pad_bytes() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("IKG_LDS_PAD");
    v = e ? atol(e) : 0;
  }
  return (size_t)v;
}

static int64_t packed_min_batch();

// IKG_PAIR_ILP=0: the default-scheduled pair kernel for every launch (A/B knob)
static bool pair_ilp_on() {
  static const bool v = !(getenv("IKG_PAIR_ILP") && atoi(getenv("IKG_PAIR_ILP")) == 0);
  return v;
}

template <typename T, bool DAMPED, class SP>
static void launch_pair_batch_t(const KModel<T>* dmodel, const KParams<T>& prm, const BatchArgs& a, hipStream_t s) {
  const int ppw = a.ppw;
  const dim3 grid((unsigned)((a.B + ppw - 1) / ppw));
  // IKG_FORCE_MED=1: measurement knob, the inline medium-range rule for every launch
  static const bool force_med = getenv("IKG_FORCE_MED") && atoi(getenv("IKG_FORCE_MED")) != 0;
  // per-problem seeds (multi-start, or a q0 row per target): large first steps
  // are common, so the frame-1 loop takes the medium-range trig rule inline.
  // fp64 with a broadcast q0 keeps the short-series rule (exact sincos beyond
  // its range: 4% faster at C2, the same values to rounding); fp32 takes the
  // medium-range rule for every q0 layout, as the packed kernel does, so an
  // fp32 answer does not depend on how q0 was passed
  if constexpr (kFrame1<SP> && !DAMPED) {
    const bool med = a.S > 1 || a.q0_stride != 0 || force_med || std::is_same<T, float>::value;
    // fp32, no records, at most one wave per SIMD: the max-ILP build of the
    // same kernel (ikg_pair_ilp.hip)
    if constexpr (std::is_same<SP, SpecNextage>::value && std::is_same<T, float>::value)
      if (!a.rec && pair_ilp_on() && (int64_t)grid.x * 32 < packed_min_batch()) {
        (void)launch_pair_ilp(dmodel, prm, a, med, lds_pad_bytes(), s);
        return;
      }
    if (a.rec) {  // collision continuation checkpoints (ikg_collision.hip), one fixed slot per problem
      RecArgs<T> ra;
      ra.rec = (T*)a.rec;
      ra.nrec = a.rec_n;
      ra.ck = (T*)a.ck;
      ra.list = a.rec_list;
      ra.count = a.rec_count;
      ra.wmask = a.rec_wmask;
      ra.rmask = a.rec_rmask;
      ra.rbase = a.rec_rbase;
      ra.rcap = a.rec_rcap;
      // resume (a.rec_list): the same kernel over (listed problem, window) tasks, grid-stride
      // resume: at most (windows x whole waves of the list) + one wave per first window, grid-stride
      const int64_t nl = std::min<int64_t>(a.B, a.rec_rcap);
      const int64_t rw = (int64_t)rec_windows<T>(prm.max_iters) * ((nl + ppw - 1) / ppw) + nl;
      const dim3 g = a.rec_list ? dim3((unsigned)std::min<int64_t>(rw, 4096)) : grid;
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, g, dim3(64), lds_pad_bytes(), s, dmodel, prm, (const T*)a.targets,
                           (const T*)a.q0, a.q0_stride, a.B, a.S, ppw, (T*)a.q_out, a.converged, a.iters,
                           (T*)a.err_out, ra);
      };
      if (a.rec_list) {  // the resume kernel (REC = 2)
        if (med)
          go(ikg_pair_batch_kernel<T, DAMPED, SP, true, 2>);
        else
          go(ikg_pair_batch_kernel<T, DAMPED, SP, false, 2>);
      } else if (med) {
        go(ikg_pair_batch_kernel<T, DAMPED, SP, true, 1>);
      } else {
        go(ikg_pair_batch_kernel<T, DAMPED, SP, false, 1>);
      }
      if (a.rec_used) *a.rec_used = true;
      return;
    }
    if (med) {
      hipLaunchKernelGGL((ikg_pair_batch_kernel<T, DAMPED, SP, true>), grid, dim3(64), lds_pad_bytes(), s, dmodel,
                         prm, (const T*)a.targets, (const T*)a.q0, a.q0_stride, a.B, a.S, ppw, (T*)a.q_out,
                         a.converged, a.iters, (T*)a.err_out);
      return;
    }
  }
  hipLaunchKernelGGL((ikg_pair_batch_kernel<T, DAMPED, SP>), grid, dim3(64), lds_pad_bytes(), s, dmodel, prm,
                     (const T*)a.targets, (const T*)a.q0, a.q0_stride, a.B, a.S, ppw, (T*)a.q_out, a.converged,
                     a.iters, (T*)a.err_out);
}

// The packed layout applies to fp32, the compiled Nextage specialisation and
// lambda = 0.  It halves the instructions per problem but v_pk_fma_f32 issues
// at ~4.4 cycles against ~2.7 for v_fma_f32 (tools/ubench/pkl.hip), and it
// halves the waves: measured faster only once the pair layout would need a
// second wave on some SIMD (B > 32768 on 256 CUs).  With the max-ILP build of
// ikg_packed.hip: B = 32768 pair 1.22 ms / packed 1.47, B = 49152 1.78 / 1.46,
// B = 65536 1.81 / 1.53 (bench.py, gpurun_out/thr).  AUTO takes it from there on.
template <typename T>
bool packed_applies(const KParams<T>& prm, int spec) {
  return std::is_same<T, float>::value && spec == kSpecNextage && !(prm.lambda > T(0));
}

// Per device (the launch's current device): CU counts may differ between
// devices; the cache is filled racily but every writer stores the same value.
static int64_t packed_min_batch() {
  constexpr int kDevs = 64;
  static std::atomic<int64_t> cache[kDevs];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  if (dev >= 0 && dev < kDevs) {
    const int64_t v = cache[dev].load(std::memory_order_relaxed);
    if (v > 0) return v;
  }
  int cus = 256;
  if (dev < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  const int64_t v = (int64_t)cus * 4 /* SIMDs */ * 32 /* problems per pair wave */ + 1;
  if (dev >= 0 && dev < kDevs) cache[dev].store(v, std::memory_order_relaxed);
  return v;
}

// The quad layout (ikg_quad.hip, 8 lanes and ~2/3 of the pair layout's
// instructions per problem-update, 1/4 of the problems per wave) wins while the
// batch leaves SIMDs idle; AUTO takes it up to quad_max_batch().
template <typename T>
bool quad_applies(const KParams<T>& prm, int spec) {
  return spec == kSpecNextage && !(prm.lambda > T(0));
}

static int64_t quad_max_batch() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("IKG_QUAD_MAX_BATCH");
    v = e ? atol(e) : 0;  // measured no faster than PAIR: explicit variant only
  }
  return (int64_t)v;
}

// The layout a launch of B problems runs (AUTO resolved; PAIR also stands for
// the generic, damped and model-specialised pair kernels).  The C-ABI fixes it
// from the whole batch before splitting a collision solve into record chunks
// (ikg_capi.hip), so every chunk runs the layout the batch would.
template <typename T>
int resolve_variant(const KParams<T>& prm, int spec, int variant, int64_t B, bool rec) {
  if (variant == IKG_VARIANT_QUAD || (variant == IKG_VARIANT_AUTO && B <= quad_max_batch()))
    if (quad_applies(prm, spec)) return IKG_VARIANT_QUAD;
  if constexpr (std::is_same<T, float>::value) {
    static const bool rec_pair = getenv("IKG_REC_PREFER_PAIR") && atoi(getenv("IKG_REC_PREFER_PAIR")) != 0;
    const bool want = variant == IKG_VARIANT_PACKED ||
                      (variant == IKG_VARIANT_AUTO && B >= packed_min_batch() && !(rec_pair && rec));
    if (want && packed_applies(prm, spec)) return IKG_VARIANT_PACKED;
  }
  return IKG_VARIANT_PAIR;
}

template <typename T>
hipError_t launch_pair_batch(const KModel<T>* dmodel, const KParams<T>& prm, const BatchArgs& a, int spec,
                             hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  const int v = resolve_variant(prm, spec, a.variant, a.B, a.rec != nullptr);
  if (v == IKG_VARIANT_QUAD) return launch_quad_batch<T>(dmodel, prm, a, s);
  if (a.variant == IKG_VARIANT_QUAD) return hipErrorInvalidValue;  // checked by the C-ABI first
  if constexpr (std::is_same<T, float>::value)
    if (v == IKG_VARIANT_PACKED) return launch_packed_batch(dmodel, prm, a, s);
  if (a.variant == IKG_VARIANT_PACKED) return hipErrorInvalidValue;  // checked by the C-ABI first
  const bool damped = prm.lambda > T(0);
  if (a.jit) {  // the pair loop compiled against this model's constant tables (ikg_jit.hip)
    const bool med = a.S > 1 || a.q0_stride != 0 || std::is_same<T, float>::value;
    hipFunction_t f = damped ? a.jit->damped : (med && a.jit->pair_med ? a.jit->pair_med : a.jit->pair);
    const T* targets = (const T*)a.targets;
    const T* q0 = (const T*)a.q0;
    T* q_out = (T*)a.q_out;
    T* err_out = (T*)a.err_out;
    KParams<T> p = prm;
    int64_t stride = a.q0_stride, B = a.B, S = a.S;
    int ppw = a.ppw;
    uint8_t* conv = a.converged;
    int32_t* iters = a.iters;
    void* args[] = {(void*)&dmodel, &p, &targets, &q0, &stride, &B, &S, &ppw, &q_out, &conv, &iters, &err_out};
    const unsigned grid = (unsigned)((a.B + ppw - 1) / ppw);
    return hipModuleLaunchKernel(f, grid, 1, 1, 64, 1, 1, (unsigned)lds_pad_bytes(), s, args, nullptr);
  }
  if (spec == kSpecNextage) {
    if (damped)
      launch_pair_batch_t<T, true, SpecNextage>(dmodel, prm, a, s);
    else
      launch_pair_batch_t<T, false, SpecNextage>(dmodel, prm, a, s);
  } else if (damped) {  // the damped solve does not use the wrist structure
    launch_pair_batch_t<T, true, SpecGeneric>(dmodel, prm, a, s);
  } else if (spec == kSpecGenericWrist) {
    launch_pair_batch_t<T, false, SpecGenericWrist>(dmodel, prm, a, s);
  } else {
    launch_pair_batch_t<T, false, SpecGeneric>(dmodel, prm, a, s);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_multistart(const KModel<T>* dmodel, const KParams<T>& prm, const MultiArgs& a, int spec,
                             hipStream_t s) {
  if (a.T <= 0) return hipSuccess;
  // 1) every (target, seed) problem through the pair kernel into the workspace
  // S == 1: the one seed row serves every target (broadcast), since the batch
  // kernel indexes q0 rows by problem when S == 1
  BatchArgs b{a.targets, a.seeds, a.S == 1 ? 0 : a.nq, a.T * a.S, a.ws_q, a.ws_conv, a.ws_iters, a.ws_err, 32, a.S};
  b.ws_owner = a.ws_owner;
  b.jit = a.jit;
  b.rec = a.rec;
  b.rec_n = a.rec_n;
  b.ck = a.ck;
  b.rec_slots = a.rec_slots;
  b.rec_used = a.rec_used;
  // AUTO keeps the pair layout here: seeds spread the update counts, and a
  // wave lasts as long as its slowest problem -- 64 per packed wave against 32
  // per pair wave measured 4.17 ms against 3.66 ms (256 seeds x 512 targets,
  // fp32, tools/probe/bisect_c5_trace.sh)
  b.variant = a.variant == IKG_VARIANT_AUTO ? IKG_VARIANT_PAIR : a.variant;
  // with collision records: rec_chunk targets (and their S seeds) per launch,
  // so the records' fixed slots fit the budget (ikg_capi.hip rec_chunk)
  const int64_t tc = a.rec && a.rec_chunk > 0 ? a.rec_chunk : a.T;
  for (int64_t t0 = 0; t0 < a.T; t0 += tc) {
    BatchArgs c = b;
    const int64_t nt = std::min(tc, a.T - t0);
    c.B = nt * a.S;
    c.targets = (const T*)a.targets + t0 * 12;
    c.q_out = (T*)a.ws_q + t0 * a.S * a.nq;
    c.converged = a.ws_conv + t0 * a.S;
    c.iters = a.ws_iters + t0 * a.S;
    c.err_out = (T*)a.ws_err + t0 * a.S * 2;
    hipError_t e = launch_pair_batch<T>(dmodel, prm, c, spec, s);
    if (e != hipSuccess) return e;
    if (a.collision) {  // converged-but-colliding seeds keep iterating (inverse_geometry.py:70)
      e = launch_collide_continue<T>(dmodel, (const KCollision<T>*)a.collision, prm, c, spec, a.nq, a.n_geoms, s);
      if (e != hipSuccess) return e;
    }
  }
  // 2) one wave per target picks the best seed
  const int block = 256;
  const dim3 grid((unsigned)((a.T * 64 + block - 1) / block));
  hipLaunchKernelGGL((ikg_best_seed_kernel<T>), grid, dim3(block), 0, s, a.T, a.S, a.nq, (const T*)a.ws_q,
                     (const uint8_t*)a.ws_conv, (const int32_t*)a.ws_iters, (const T*)a.ws_err, (T*)a.q_out,
                     a.converged, a.iters, (T*)a.err_out, a.best_seed);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_fk(const KModel<T>* dmodel, const void* q, int64_t B, void* hands, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  constexpr int block = 256;
  const dim3 grid((unsigned)((B + block - 1) / block));
  hipLaunchKernelGGL((ikg_fk_kernel<T>), grid, dim3(block), 0, s, dmodel, (const T*)q, B, (T*)hands);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_log6(const void* M, int64_t B, void* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  constexpr int block = 256;
  const dim3 grid((unsigned)((B + block - 1) / block));
  hipLaunchKernelGGL((ikg_log6_kernel<T>), grid, dim3(block), 0, s, (const T*)M, B, (T*)out);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pair_state(const KModel<T>* dm, const void* targets, const void* q0, int64_t stride, int64_t B,
                             void* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const dim3 grid((unsigned)((2 * B + 63) / 64));
  hipLaunchKernelGGL((ikg_pair_state_kernel<T>), grid, dim3(64), 0, s, dm, (const T*)targets, (const T*)q0, stride, B,
                     (T*)out);
  return hipGetLastError();
}
template hipError_t launch_pair_state<double>(const KModel<double>*, const void*, const void*, int64_t, int64_t,
                                              void*, hipStream_t);
template hipError_t launch_pair_state<float>(const KModel<float>*, const void*, const void*, int64_t, int64_t,
                                             void*, hipStream_t);
template hipError_t launch_log6<double>(const void*, int64_t, void*, hipStream_t);
template hipError_t launch_log6<float>(const void*, int64_t, void*, hipStream_t);
template hipError_t launch_pair_batch<double>(const KModel<double>*, const KParams<double>&, const BatchArgs&, int,
                                              hipStream_t);
template hipError_t launch_pair_batch<float>(const KModel<float>*, const KParams<float>&, const BatchArgs&, int,
                                             hipStream_t);
template int resolve_variant<double>(const KParams<double>&, int, int, int64_t, bool);
template int resolve_variant<float>(const KParams<float>&, int, int, int64_t, bool);
template hipError_t launch_multistart<double>(const KModel<double>*, const KParams<double>&, const MultiArgs&, int,
                                              hipStream_t);
template hipError_t launch_multistart<float>(const KModel<float>*, const KParams<float>&, const MultiArgs&, int,
                                             hipStream_t);
template hipError_t launch_fk<double>(const KModel<double>*, const void*, int64_t, void*, hipStream_t);
template hipError_t launch_fk<float>(const KModel<float>*, const void*, int64_t, void*, hipStream_t);

}  // namespace ikg
