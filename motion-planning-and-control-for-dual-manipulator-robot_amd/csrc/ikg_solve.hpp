// The reference loop for one IK problem (inverse_geometry.py:56-94), shared by the
// pair-layout kernels (ikg_kernels.hip) and the packed fp32 kernel (ikg_packed.hip,
// its own translation unit so it can be compiled with a different scheduler).
#pragma once
#include "ikg_device.hpp"

namespace ikg {

// q row -> this arm's (root, arm joints) and back (pair and quad layouts)
template <typename T>
__device__ inline void load_q(const KModel<T>* __restrict__ m, int arm, const T* __restrict__ qrow, T& qc, T* qa) {
  qc = qrow[m->root_q];
  const bool right = arm != 0;
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) qa[k] = qrow[right ? m->arm_q[1][k] : m->arm_q[0][k]];
}

template <typename T>
__device__ inline void store_q(const KModel<T>* __restrict__ m, int arm, const T* __restrict__ qrow, int it, T qc,
                               const T* qa, T* __restrict__ qo) {
  const bool right = arm != 0;
  if (!right) {
    qo[m->root_q] = qc;
    // passive joints (HEAD_JOINT0/1): zero Jacobian columns, so only the clamp
    // of the first update moves them (tools.py:21-22)
    for (int i = 0; i < m->n_passive; ++i) {
      const int j = m->passive_q[i];
      const T v = qrow[j];
      qo[j] = it > 0 ? clampq(v, m->lo[j], m->hi[j]) : v;
    }
  }
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) qo[right ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
}


// ---- trajectory records (collision continuation, ikg_collision.hip §3b)
// One 8-value block per arm lane, written by 16-byte stores:
//   [0, 8):  root, left arm joints 0..5, |e_L|^2
//   [8, 16): stop test passes (1/0), right arm joints 0..5, |e_R|^2
//   [16, ...): passive joints (passive_q order), padded to a multiple of 4
constexpr int kRecRoot = 0, kRecArm0 = 1, kRecErr0 = 7, kRecPass = 8, kRecArm1 = 9, kRecErr1 = 15, kRecPassive = 16;
constexpr int32_t kTrajEnded = 1 << 30;  // record count flag: the last is the iterate after max_iters
IKG_HD inline int rec_len(int n_passive) { return kRecPassive + ((n_passive + 3) & ~3); }

template <typename T>
__device__ __forceinline__ void store_block8(T* dst, const T (&v)[8]) {
#if defined(IKG_REC_NOSTORE)  // timing ablation only: records not written (answers wrong)
  (void)dst, (void)v;
#else
  struct alignas(16) V16 {
    T x[16 / sizeof(T)];
  };
  constexpr int per = 16 / (int)sizeof(T);
#pragma unroll
  for (int k = 0; k < 8 / per; ++k) {
    V16 b;
#pragma unroll
    for (int e = 0; e < per; ++e) b.x[e] = v[k * per + e];
    reinterpret_cast<V16*>(dst)[k] = b;
  }
#endif
}

template <typename T>
__device__ __forceinline__ void load_block8(const T* src, T (&v)[8]) {
  struct alignas(16) V16 {
    T x[16 / sizeof(T)];
  };
  constexpr int per = 16 / (int)sizeof(T);
#pragma unroll
  for (int k = 0; k < 8 / per; ++k) {
    const V16 b = reinterpret_cast<const V16*>(src)[k];
#pragma unroll
    for (int e = 0; e < per; ++e) v[k * per + e] = b.x[e];
  }
}

// Record-in-batch outputs of one problem (ikg_pair_batch_kernel with REC):
// the loop goes on past the first iterate whose errors pass, recording every
// iterate for the collision scan; that iterate's outputs are stored when reached.
template <typename T>
struct RecOut {
  T* rec;               // this problem's records, (max_iters + 1) x rec_len
  int32_t* nrec;        // this problem's record count (| kTrajEnded)
  const T* qrow;        // its q0 row (passive joints)
  T* qo;                // its q_out row
  uint8_t* conv;        // its outputs at the first passing iterate
  int32_t* iters;
  T* err;
  int rl;               // rec_len
};

// Diagnostic build only (-DIKG_STAGE_CLOCK, tools/stage_clock.py; no stamp
// exists in the product kernels): shader-clock stamps (s_memtime) between the
// stages of every update of the frame-1 loop, and s_memrealtime (100 MHz) around
// the loop, per wave, summed into g_stage by lane 0 of every wave:
//   [0] waves  [1] updates  [2] loop memtime  [3] loop memrealtime
//   [4] FK + log6 (arm_fk_error_f1)  [5] solve (pinv_step_f1)
//   [6] exchange + stop test  [7] integrate + clamp (arm_update)
//   [8] trig advance (trig_advance_f1)
// Each stamp is one asm statement with its lgkmcnt wait, fenced by scheduling
// barriers so no stage's instructions move across it (MI355X_MICROARCH.md
// DVFS item 6, cdna_hip_programming.md "In-kernel stamps").
#ifdef IKG_STAGE_CLOCK
static __device__ unsigned long long g_stage[16];
#define IKG_STAMP(t)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");                 \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#define IKG_RSTAMP(t)                                                                         \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");             \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#endif

// Stop test of inverse_geometry.py:70 on squared norms (KParams::eps2):
// pair layout = this lane's hand and the partner's; packed = both halves.
template <typename T, typename E>
__device__ inline bool both_below(T x, T xo, E eps2) {
  if constexpr (is_packed<T>)
    return all_of(x < T(eps2));
  else
    return x < eps2 && xo < eps2;
}

// One problem: run the reference loop to its stop condition.  T = double /
// float: this lane owns one arm (pair layout, partner = lane ^ 1); T = v2f:
// this lane owns both arms (packed layout).  Returns (through refs) the final
// q of this lane, the update count and the hand error norms at the returned q.
// REC: every iterate from the first passing one on is recorded into this
// problem's fixed slot (ikg_capi.hip sizes the launches so the slots fit the
// record budget: no shared state, so a problem's records and answer do not
// depend on which other problems share the launch or in what order they run)
template <typename T, bool DAMPED, class SP, bool MED = false, bool REC = false>
__device__ inline bool solve_pair(const KModel<typename LaneT<T>::E>* __restrict__ m,
                                  const KParams<typename LaneT<T>::E>& prm, int arm, const T* RT, const T* tT, T& qc,
                                  T* qa, int& it_out, bool& conv_out, T& nrm_out, T& other_out,
                                  const RecOut<typename LaneT<T>::E>* ro = nullptr) {
  int k0 = -1;  // REC: the first iterate whose errors pass
  using E = typename LaneT<T>::E;
  E* recp = REC ? ro->rec : nullptr;  // this problem's records
  static_assert(!(DAMPED && is_packed<T>), "the packed layout implements lambda = 0 only");
  constexpr bool F1 = kFrame1<SP> && !DAMPED;  // frame-1 path, its own trig slots
  T sn[7], cs[7];
  if constexpr (F1)
    trig_exact_f1(m, arm, qc, qa, sn, cs);
  else
    trig_exact(qc, qa, sn, cs);
  int it = 0;
  bool conv = false;
  T x, xo;  // squared error norms of this lane's hand and the partner's
  ThetaTrack<T> tk{};
#if IKG_LANE_LIMITS
  ArmLimits<T> lim;
  if constexpr (!is_packed<T>) load_limits(m, arm, lim);
  const ArmLimits<T>* limp = is_packed<T> ? nullptr : &lim;
#else
  const ArmLimits<T>* limp = nullptr;
#endif
#ifdef IKG_PAD_OPS
  // timing experiment: IKG_PAD_OPS independent fp64 FMAs per iteration (ILP 8)
  T pad[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) pad[i] = qc + T(i);
#endif
#ifdef IKG_STAGE_CLOCK
  unsigned long long sc_acc[5] = {0, 0, 0, 0, 0}, sc_t0 = 0, sc_t1 = 0, sc_r0, sc_r1, sc_l0, sc_l1;
  IKG_RSTAMP(sc_r0);
  IKG_STAMP(sc_l0);
#endif
  for (;;) {
#ifdef IKG_PAD_OPS
#pragma unroll
    for (int k = 0; k < IKG_PAD_OPS / 8; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) pad[i] = pad[i] * T(0.999999) + T(1e-7);
#endif
#if IKG_UNIFORM
    // every live lane of the wave has run the same number of updates, so the
    // count (and the resync / max_iters tests on it) is wave-uniform: scalar
    if constexpr (!is_packed<T>) it = __builtin_amdgcn_readfirstlane(it);
#endif
    // fp32: atan2f is as cheap as the tracked angle (measured)
    ThetaTrack<T>* tkp = (IKG_THETA_TRACK && is_f64<T>) ? &tk : nullptr;
    const bool resync = (it % Trig<T>::kResync) == 0;
    // the step is formed before the stop test (discarded when the loop ends)
    // so the test's exchange/compare overlaps the solve instead of heading it
    T dq[6], alpha, beta, s;
    if constexpr (F1) {
      ArmStateF1<T> st;
#ifdef IKG_STAGE_CLOCK
      IKG_STAMP(sc_t0);
      x = arm_fk_error_f1<T, SP>(m, arm, sn, cs, RT, tT, st, tkp, resync);
      IKG_STAMP(sc_t1);
      sc_acc[0] += sc_t1 - sc_t0;
      pinv_step_f1<T, SP, PairX, !REC>(m, arm, st, sn, cs, dq, s);
      IKG_STAMP(sc_t0);
      sc_acc[1] += sc_t0 - sc_t1;
#else
      x = arm_fk_error_f1<T, SP>(m, arm, sn, cs, RT, tT, st, tkp, resync);
      pinv_step_f1<T, SP, PairX, !REC>(m, arm, st, sn, cs, dq, s);
#endif
    } else {
    ArmState<T> st;
    x = arm_fk_error<T, SP>(m, arm, sn, cs, RT, tT, st, nullptr, tkp, resync);
    if constexpr (!DAMPED) {
      pinv_step_cf<T, SP>(st, arm, T(m->sing_tau), T(m->sing_beta), dq, s);
    } else {
      T A[6][8], ze[6], zc[6];
      arm_system(st, A);
      arm_solve_damped(A, prm.lambda, ze, zc, alpha, beta);
      s = chest_step(alpha + pair_swap(alpha), beta + pair_swap(beta));
      arm_dq_damped(A, ze, zc, s, dq);
    }
    }
    xo = pair_swap(x);
    if constexpr (REC) {
      const bool ended = it >= prm.max_iters;  // never tested (:56 loop exhausted)
      const bool pass = !ended && both_below(x, xo, prm.eps2);
      if (pass && k0 < 0) {  // the answer unless it collides: record 0, written out after the loop
        k0 = it;
        conv = true;
      }
      if (k0 >= 0) {
        if constexpr (is_packed<T>) {  // both arms' blocks from the one lane
          float b0[8], b1[8];
          b0[0] = qc.x;
          b1[0] = pass ? 1.f : 0.f;
#pragma unroll
          for (int k = 0; k < kArmDof; ++k) {
            b0[1 + k] = qa[k].x;
            b1[1 + k] = qa[k].y;
          }
          b0[7] = x.x;
          b1[7] = x.y;
          float* dst = recp + (int64_t)(it - k0) * ro->rl;
          store_block8(dst + kRecRoot, b0);
          store_block8(dst + kRecPass, b1);
        } else {
          T blk[8];
          blk[0] = arm ? (pass ? T(1) : T(0)) : qc;
#pragma unroll
          for (int k = 0; k < kArmDof; ++k) blk[1 + k] = qa[k];
          blk[7] = x;
          store_block8(recp + (int64_t)(it - k0) * ro->rl + (arm ? kRecPass : kRecRoot), blk);
        }
      }
      if (ended) break;
    } else {
      if (it >= prm.max_iters) break;  // loop exhausted: the reference never tests this iterate
      if (both_below(x, xo, prm.eps2)) {  // |e_L| < eps and |e_R| < eps (:70)
        conv = true;
        break;
      }
    }
    T q_old[7];
    q_old[0] = qc;
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) q_old[k + 1] = qa[k];
#ifdef IKG_STAGE_CLOCK
    IKG_STAMP(sc_t1);
    sc_acc[2] += sc_t1 - sc_t0;
#endif
    arm_update(m, arm, T(prm.dt), s, dq, qc, qa, limp);
    ++it;
#ifdef IKG_STAGE_CLOCK
    IKG_STAMP(sc_t0);
    sc_acc[3] += sc_t0 - sc_t1;
#endif
    if constexpr (F1) {
      trig_advance_f1<T, MED>(m, arm, qc, qa, q_old, (it % Trig<T>::kResync) == 0, sn, cs);
#ifdef IKG_STAGE_CLOCK
      IKG_STAMP(sc_t1);
      sc_acc[4] += sc_t1 - sc_t0;
#endif
    } else
      trig_advance<T, MED ? 1 : IKG_GENERIC_MED>(qc, qa, q_old, (it % Trig<T>::kResync) == 0, sn, cs);
  }
#ifdef IKG_STAGE_CLOCK
  IKG_STAMP(sc_l1);
  IKG_RSTAMP(sc_r1);
  if (threadIdx.x == 0) {  // lane 0 of the wave: its problem's loop ran longest only in forced runs (every lane to max_iters)
    atomicAdd(&g_stage[0], 1ull);
    atomicAdd(&g_stage[1], (unsigned long long)it);
    atomicAdd(&g_stage[2], sc_l1 - sc_l0);
    atomicAdd(&g_stage[3], sc_r1 - sc_r0);
#pragma unroll
    for (int k = 0; k < 5; ++k) atomicAdd(&g_stage[4 + k], sc_acc[k]);
  }
#endif
#ifdef IKG_PAD_OPS
  T ps = T(0);
#pragma unroll
  for (int i = 0; i < 8; ++i) ps += pad[i];
  if (any_of(ps == T(-12345.678))) it = -1;  // never true; keeps the padding live
#endif
  if constexpr (REC) {
    if (k0 >= 0) {
      // the outputs at the first passing iterate, from its record (this lane's
      // own block of record 0): writing them inside the loop put a divergent
      // branch into every update (records-in-batch kernel 4% slower)
      if constexpr (is_packed<T>) {
        float b[2][8], qa0[kArmDof];
        load_block8(recp + kRecRoot, b[0]);
        load_block8(recp + kRecPass, b[1]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int k = 0; k < kArmDof; ++k) qa0[k] = b[h][1 + k];
          store_q(m, h, ro->qrow, k0, b[0][0], qa0, ro->qo);
          ro->err[h] = sqrtf(b[h][7]);
        }
        *ro->conv = 1;
        *ro->iters = k0;
        *ro->nrec = (it - k0 + 1) | kTrajEnded;
      } else {
      T blk[8];
      load_block8(recp + (arm ? kRecPass : kRecRoot), blk);
      T qa0[kArmDof];
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qa0[k] = blk[1 + k];
      store_q(m, arm, ro->qrow, k0, blk[0], qa0, ro->qo);
      ro->err[arm] = sqrt(blk[7]);
      if (arm == 0) {
        *ro->conv = 1;
        *ro->iters = k0;
        *ro->nrec = (it - k0 + 1) | kTrajEnded;
      }
      }
    }
  }
  it_out = it;
  nrm_out = sqrt(x);
  other_out = sqrt(xo);
  conv_out = conv;
  return REC && k0 >= 0;  // the outputs came from the records
}

// Pair-layout batch kernel body (ikg_kernels.hip ikg_pair_batch_kernel, and the
// model-specialised kernels ikg_jit.cpp compiles at run time with `m` pointing
// at a constant copy of the model tables): one 64-lane wave per workgroup
// holding `ppw` problems on lanes [0, 2 ppw).
template <typename T, bool DAMPED, class SP, bool MED, bool REC = false>
__device__ inline void pair_batch_body(const KModel<T>* __restrict__ m, const KParams<T>& prm,
                                       const T* __restrict__ targets, const T* __restrict__ q0, int64_t q0_stride,
                                       int64_t B, int64_t S, int ppw, T* __restrict__ q_out,
                                       uint8_t* __restrict__ conv_out, int32_t* __restrict__ iters_out,
                                       T* __restrict__ err_out, T* __restrict__ rec = nullptr,
                                       int32_t* __restrict__ nrec = nullptr) {
  const int lane = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * ppw + (lane >> 1);
  const int arm = lane & 1;
  if (lane >= 2 * ppw || p >= B) return;  // both lanes of a pair leave together
  // multi-start (S > 1): problem p = (target p / S, seed p % S)
  const int64_t tgt = S > 1 ? p / S : p;
  const int64_t row = S > 1 ? p - tgt * S : p;
  T RT[9], tT[3];
  hook_target(m, arm, targets + tgt * 12, RT, tT);
  const T* qrow = q0 + row * q0_stride;
  T qc, qa[kArmDof];
  load_q(m, arm, qrow, qc, qa);
  int it;
  bool conv;
  T nrm, other;
  if constexpr (REC) {  // the continuation's records (ikg_collision.hip): outputs at the first passing iterate
    const int rl = rec_len(m->n_passive);
    RecOut<T> ro{rec + p * (int64_t)(prm.max_iters + 1) * rl, nrec + p, qrow, q_out + p * m->nq,
                 conv_out + p, iters_out + p, err_out + p * 2, rl};
    if (arm == 0) nrec[p] = 0;
    if (solve_pair<T, DAMPED, SP, MED, true>(m, prm, arm, RT, tT, qc, qa, it, conv, nrm, other, &ro)) return;
  } else {
    solve_pair<T, DAMPED, SP, MED>(m, prm, arm, RT, tT, qc, qa, it, conv, nrm, other);
  }
  store_q(m, arm, qrow, it, qc, qa, q_out + p * m->nq);
  if (arm == 0) {
    if (conv_out) conv_out[p] = conv ? 1 : 0;
    if (iters_out) iters_out[p] = it;
  }
  if (err_out) err_out[p * 2 + arm] = nrm;
}

}  // namespace ikg
