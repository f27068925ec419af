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

template <typename T>
__device__ __forceinline__ void store_block4(T* dst, const T (&v)[4]) {
#if defined(IKG_REC_NOSTORE)  // timing ablation only
  (void)dst, (void)v;
#else
  struct alignas(16) V16 {
    T x[16 / sizeof(T)];
  };
  constexpr int per = 16 / (int)sizeof(T);
#pragma unroll
  for (int k = 0; k < 4 / per; ++k) {
    V16 b;
#pragma unroll
    for (int e = 0; e < per; ++e) b.x[e] = v[k * per + e];
    reinterpret_cast<V16*>(dst)[k] = b;
  }
#endif
}

// ---- window checkpoints (round 6: the records' window form)
// The batch kernel no longer writes every iterate past the first passing one
// (k0).  Windows are aligned to absolute update counts (window w: iterates
// [w K, (w + 1) K), K = 32); from k0 on it writes a checkpoint at k0 (the
// loop's whole state: q, the carried trig, the rotation-angle track) and at
// each later window's first iterate (q and the previous window's path length
// L: the sum over its updates of the largest joint step), and at the end the
// record of the iterate after max_iters.  In the record-writing kernels the
// carried trig and angle are recomputed exactly every kRsRec updates, so at a
// window start they are a function of q (fp32 resyncs every 16 anyway; fp64
// every 32 there instead of 128: ~2% more work in that kernel).  Every iterate
// of window w lies within L_w of the window's first one in every joint, so the
// scan proves a whole window colliding with one certificate test on that box
// (ikg_collision.hip round -2); a window the box test does not prove is
// regenerated from its checkpoint (the resume kernel, RecArgs::list) into the
// records the scan reads.
// Slot layout per problem: rec_windows + 2 slots of kCkSlot values; window w in
// slot w (absolute); the final record (record layout, passive joints not
// filled) in the last.  Within a slot, per arm (pair layout: the arm's lane;
// packed: the arm's half) at arm * kCkArm:
//   k0's window:   [0, 8) root, the arm's joints, |e|^2 (the record block
//                  layout); [8, 15) sn; [16, 23) cs; [24, 27) angle track
//   later windows: [0, 8) root, the arm's joints, L of window w - 1
// (the last window's length goes to the next slot, before the final record's)
constexpr int kWin = 32;  // iterates per window (a power of 2, at most 64: one 64-bit record mask per window)
constexpr int kCkArm = 32, kCkSlot = 64;
constexpr int kCkQ = 0, kCkSn = 8, kCkCs = 16, kCkTk = 24, kCkL = 7;
template <typename E>
constexpr int kWinOf = kWin;
template <typename T>
#ifdef IKG_REC_RS_ABL  // timing ablation only: the batch loop's own resync period (resumed windows wrong)
constexpr int kRsRec = Trig<T>::kResync;
#else
constexpr int kRsRec = Trig<T>::kResync < kWin ? Trig<T>::kResync : kWin;  // divides kWin
#endif
template <typename E>
IKG_HD inline int rec_windows(int max_iters) { return max_iters / kWinOf<E> + 1; }
template <typename E>
IKG_HD inline int64_t ck_per_problem(int max_iters) { return (int64_t)(rec_windows<E>(max_iters) + 2) * kCkSlot; }
template <typename E>
IKG_HD inline int64_t ck_final(int max_iters) { return (int64_t)(rec_windows<E>(max_iters) + 1) * kCkSlot; }
// the windows the scan could not prove colliding (regenerated and scanned):
// one bit per window, mask_words 32-bit words per problem
template <typename E>
IKG_HD inline int mask_words(int max_iters) { return (rec_windows<E>(max_iters) + 31) / 32; }
IKG_HD inline bool win_flagged(const uint32_t* wm, int w) { return (wm[w >> 5] >> (w & 31)) & 1u; }

// Kernel argument of the record-writing (REC) batch kernels.
template <typename T>
struct RecArgs {
  T* rec = nullptr;                 // regenerated records: (max_iters + 1) x rec_len per problem
  int32_t* nrec = nullptr;          // per problem: records from k0 (| kTrajEnded)
  T* ck = nullptr;                  // window checkpoints: ck_per_problem per problem
  const int32_t* list = nullptr;    // resume launch: the problems whose windows are regenerated (null: the batch solve)
  const int32_t* count = nullptr;   // resume: list length (device)
  const uint32_t* wmask = nullptr;  // resume: per problem, the windows to regenerate (mask_words each)
  uint64_t* rmask = nullptr;        // resume: per problem and window, the iterates recorded (rec_windows each)
  int64_t rbase = 0, rcap = 0;      // resume: list entries [rbase, rbase + rcap), records in slots i - rbase
};

// Record-in-batch outputs of one problem (the REC batch kernels): the loop goes
// on past the first iterate whose errors pass (k0), writing window checkpoints
// for the collision scan; k0's outputs are stored from window 0's checkpoint.
// resume: the loop restarts at window w's checkpoint and records its iterates.
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
  T* ck;                // its checkpoint slots (resume: the window's)
  int it_start = 0, k0 = -1, it_stop = 0;  // resume: first iterate, the problem's k0, one past the last iterate
  uint64_t* rmask = nullptr;  // resume: this window's recorded iterates (bit j - first)
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
// The per-arm values of a checkpoint: pair layout, this lane's arm at
// arm * kCkArm; packed, arm 0 from .x and arm 1 from .y
template <typename T>
__device__ __forceinline__ T ck_get(const typename LaneT<T>::E* c, int arm, int off) {
  if constexpr (is_packed<T>)
    return T{c[off], c[kCkArm + off]};
  else
    return c[arm * kCkArm + off];
}
// writes v[0..N) at off of each arm (N = 4 or 8, 16-byte stores)
template <typename T, int N>
__device__ __forceinline__ void ck_put(typename LaneT<T>::E* c, int arm, int off, const T (&v)[N]) {
  using E = typename LaneT<T>::E;
  if constexpr (is_packed<T>) {
    E a[N], b[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      a[k] = v[k].x;
      b[k] = v[k].y;
    }
    if constexpr (N == 8) {
      store_block8(c + off, a);
      store_block8(c + kCkArm + off, b);
    } else {
      store_block4(c + off, a);
      store_block4(c + kCkArm + off, b);
    }
  } else {
    if constexpr (N == 8)
      store_block8(c + arm * kCkArm + off, v);
    else
      store_block4(c + arm * kCkArm + off, v);
  }
}

// REC = 1: from the first passing iterate on, the window checkpoints go into
// this problem's fixed slots (ikg_capi.hip sizes the launches so the slots fit
// the record budget: no shared state, so a problem's checkpoints and answer do
// not depend on which other problems share the launch or in what order they
// run).  REC = 2 (resume): the loop restarts at a checkpoint and records the
// window's iterates (the pair layout's waves hold tasks that start at the same
// iterate, so the count stays wave-uniform).  The two are separate instantiations of the
// same source; the compiler contracts a few products into FMAs differently in
// them, so a regenerated iterate agrees with the batch loop's to the last bits
// of q (fp64 ~1e-16), not bit for bit.  One instantiation serving both was
// bit-exact but made the batch kernel 33% slower (1,036 -> 1,382 us at C2:
// register allocation around the resume branch), profiles/r06/records/.
template <typename T, bool DAMPED, class SP, bool MED = false, int REC = 0>
__device__ inline bool solve_pair(const KModel<typename LaneT<T>::E>* __restrict__ m,
                                  const KParams<typename LaneT<T>::E>& prm, int arm, const T* RT, const T* tT, T& qc,
                                  T* qa, int& it_out, bool& conv_out, T& nrm_out, T& other_out,
                                  const RecOut<typename LaneT<T>::E>* ro = nullptr) {
  int k0 = -1;  // REC: the first iterate whose errors pass
  using E = typename LaneT<T>::E;
  E* recp = REC ? ro->rec : nullptr;  // this problem's records
  static_assert(!(DAMPED && is_packed<T>), "the packed layout implements lambda = 0 only");
  constexpr bool F1 = kFrame1<SP> && !DAMPED;  // frame-1 path, its own trig slots
  static_assert(!REC || F1, "records: the frame-1 loop only");
  T sn[7], cs[7];
  int it = 0;
  ThetaTrack<T> tk{};
  T L = T(0);  // REC: this window's path length (largest joint step per update, summed)
  uint64_t rbits = 0;  // REC = 2: the window's recorded iterates
  if constexpr (REC == 2) {  // the loop state at the checkpoint (qc, qa: the caller, from the same slot)
    it = ro->it_start;
    k0 = ro->k0;
    if (it == k0) {
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        sn[j] = ck_get<T>(ro->ck, arm, kCkSn + j);
        cs[j] = ck_get<T>(ro->ck, arm, kCkCs + j);
      }
      if constexpr (!is_packed<T>) {
        tk.th = ck_get<T>(ro->ck, arm, kCkTk);
        tk.st = ck_get<T>(ro->ck, arm, kCkTk + 1);
        tk.ct = ck_get<T>(ro->ck, arm, kCkTk + 2);
      }
    } else {  // a window start after k0: the trig resynced exactly there (kRsRec), the angle track is recomputed
      trig_exact_f1(m, arm, qc, qa, sn, cs);
    }
  } else if constexpr (F1) {
    trig_exact_f1(m, arm, qc, qa, sn, cs);
  } else {
    trig_exact(qc, qa, sn, cs);
  }
  bool conv = false;
  T x, xo;  // squared error norms of this lane's hand and the partner's
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
    // (the pair layout's resume kernel too: a wave's tasks share their window)
    if constexpr (!is_packed<T>) it = __builtin_amdgcn_readfirstlane(it);
#endif
    // fp32: atan2f is as cheap as the tracked angle (measured)
    ThetaTrack<T>* tkp = (IKG_THETA_TRACK && is_f64<T>) ? &tk : nullptr;
    // the record-writing kernels resync at every window start (kRsRec)
    constexpr int kRs = REC ? kRsRec<T> : Trig<T>::kResync;
    const bool resync = (it % kRs) == 0;
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
      // the record of iterate `it`: this lane's block(s) in the record layout
      auto put_record = [&](E* dst) {
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
          store_block8(dst + kRecRoot, b0);
          store_block8(dst + kRecPass, b1);
        } else {
          T blk[8];
          blk[0] = arm ? (pass ? T(1) : T(0)) : qc;
#pragma unroll
          for (int k = 0; k < kArmDof; ++k) blk[1 + k] = qa[k];
          blk[7] = x;
          store_block8(dst + (arm ? kRecPass : kRecRoot), blk);
        }
      };
      if (k0 >= 0) {
        constexpr int K = kWinOf<E>;
        const int j = it - k0;
        if constexpr (REC == 2) {  // a regenerated window: its passing iterates (the scan tests only those)
          if (pass) {
            put_record(recp + (int64_t)j * ro->rl);
            rbits |= 1ull << (it & (K - 1));
          }
          if (it + 1 >= ro->it_stop) break;
        } else {
          // a window starts (absolute iterate counts: wave-uniform), or this
          // problem's first passing iterate: its state, and the previous
          // window's length (slot w holds L_{w-1}, written with the state so
          // each slot goes out as whole lines)
          const bool wstart = (it & (K - 1)) == 0;
          if (wstart || j == 0) {
            E* cw = ro->ck + (int64_t)(it / K) * kCkSlot;
            const T z = T(0);
            T qb[8];
            qb[0] = qc;
#pragma unroll
            for (int k = 0; k < kArmDof; ++k) qb[1 + k] = qa[k];
            qb[7] = j == 0 ? x : L;  // k0's window: its error (the outputs); later: the last window's length
            ck_put<T, 8>(cw, arm, kCkQ, qb);
            if (j == 0) {  // k0's state (later window starts: a function of q, kRsRec)
              const T sb[8] = {sn[0], sn[1], sn[2], sn[3], sn[4], sn[5], sn[6], z};
              const T cb[8] = {cs[0], cs[1], cs[2], cs[3], cs[4], cs[5], cs[6], z};
              ck_put<T, 8>(cw, arm, kCkSn, sb);
              ck_put<T, 8>(cw, arm, kCkCs, cb);
              if constexpr (!is_packed<T>) {
                const T tb[4] = {tk.th, tk.st, tk.ct, z};
                ck_put<T, 4>(cw, arm, kCkTk, tb);
              }
            }
            L = z;
          }
          if (ended) {  // the last window's length (in the next slot), and the iterate after max_iters as a record
            E* cw = ro->ck + (int64_t)(it / K + 1) * kCkSlot;
            if constexpr (is_packed<T>) {
              cw[kCkL] = L.x;
              cw[kCkArm + kCkL] = L.y;
            } else {
              cw[arm * kCkArm + kCkL] = L;
            }
            put_record(ro->ck + ck_final<E>(prm.max_iters));
          }
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
#ifndef IKG_REC_NOL_ABL  // timing ablation only: no path length (window boxes wrong)
    if constexpr (REC == 1) {  // the window's path length: this update's largest joint step
      T mv = fabs(qc - q_old[0]);
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) mv = fmax(mv, fabs(qa[k] - q_old[k + 1]));
      L = L + mv;
    }
#endif
    ++it;
#ifdef IKG_STAGE_CLOCK
    IKG_STAMP(sc_t0);
    sc_acc[3] += sc_t0 - sc_t1;
#endif
    if constexpr (F1) {
      trig_advance_f1<T, MED>(m, arm, qc, qa, q_old, (it % (REC ? kRsRec<T> : Trig<T>::kResync)) == 0, sn, cs);
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
    if constexpr (REC == 2) {  // records only: the scan writes the outputs
      if (is_packed<T> || arm == 0) *ro->rmask = rbits;
      return true;
    }
    if (k0 >= 0) {
      // the outputs at the first passing iterate, from window 0's checkpoint
      // (this lane's own q block): writing them inside the loop put a
      // divergent branch into every update (records-in-batch kernel 4% slower)
      const E* c0 = ro->ck + (int64_t)(k0 / kWinOf<E>) * kCkSlot;  // the slot of k0's window
      if constexpr (is_packed<T>) {
        float b[2][8], qa0[kArmDof];
        load_block8(c0 + kCkQ, b[0]);
        load_block8(c0 + kCkArm + kCkQ, b[1]);
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
      load_block8(c0 + arm * kCkArm + kCkQ, blk);
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
// REC = 1: the same, writing window checkpoints.  REC = 2, the resume launch:
// tasks (listed problem i, window w), ppw per wave, grid-stride, each lane
// pair restarting problem ra.list[i] at window w's checkpoint and recording
// the windows ra.wmask flags.
template <typename T, bool DAMPED, class SP, bool MED, int REC = 0>
__device__ inline void pair_batch_body(const KModel<T>* __restrict__ m, const KParams<T>& prm,
                                       const T* __restrict__ targets, const T* __restrict__ q0, int64_t q0_stride,
                                       int64_t B, int64_t S, int ppw, T* __restrict__ q_out,
                                       uint8_t* __restrict__ conv_out, int32_t* __restrict__ iters_out,
                                       T* __restrict__ err_out, const RecArgs<T>& ra = RecArgs<T>{}) {
  const int lane = threadIdx.x;
  const int arm = lane & 1;
  if constexpr (REC == 2) {
    // the update count stays wave-uniform (as in the batch loop): waves of
    // range A hold one absolute window's tasks -- every listed problem's
    // window w after its first passing iterate, all starting at w K -- ppw
    // problems per wave (the list padded to whole waves per window); range B
    // runs each problem's first window (from k0) in a wave of its own
    constexpr int K = kWinOf<T>;
    const int nw = rec_windows<T>(prm.max_iters);
    // this launch's list entries: [ra.rbase, ra.rbase + n), records in slots 0 .. n - 1
    const int64_t n = max((int64_t)0, min((int64_t)*ra.count - ra.rbase, ra.rcap)), npad = (n + ppw - 1) / ppw * ppw;
    const int64_t wavesA = (int64_t)nw * (npad / ppw), waves = wavesA + n;
    const int rl = rec_len(m->n_passive);
    const int64_t ckpp = ck_per_problem<T>(prm.max_iters);
    for (int64_t wv = blockIdx.x; wv < waves; wv += gridDim.x) {
      int64_t i;
      int w = -1;
      if (wv < wavesA) {
        w = (int)(wv / (npad / ppw));
        i = (wv - (int64_t)w * (npad / ppw)) * ppw + (lane >> 1);
        if (lane >= 2 * ppw || i >= n) continue;  // both lanes of a pair together
      } else {
        i = wv - wavesA;
        if (lane >= 2) continue;
      }
      const int64_t p = ra.list[ra.rbase + i];
      const int k0 = iters_out[p];
      if (w < 0) w = k0 / K;  // range B: the first window
      else if (w <= k0 / K) continue;
      if (!win_flagged(ra.wmask + p * mask_words<T>(prm.max_iters), w)) continue;
      const int64_t tgt = S > 1 ? p / S : p;
      const int64_t row = S > 1 ? p - tgt * S : p;
      T RT[9], tT[3];
      hook_target(m, arm, targets + tgt * 12, RT, tT);
      T* ckw = ra.ck + p * ckpp + (int64_t)w * kCkSlot;
      const T* cq = ckw + arm * kCkArm + kCkQ;
      T qc = cq[0], qa[kArmDof];
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qa[k] = cq[1 + k];
      RecOut<T> ro{ra.rec + i * (int64_t)(prm.max_iters + 1) * rl, ra.nrec + p, q0 + row * q0_stride,
                   q_out + p * m->nq, conv_out + p, iters_out + p, err_out + p * 2, rl, ckw};
      ro.rmask = ra.rmask + p * nw + w;
      ro.k0 = k0;
      ro.it_start = max(k0, w * K);
      ro.it_stop = min((w + 1) * K, prm.max_iters + 1);
      int it;
      bool conv;
      T nrm, other;
      solve_pair<T, DAMPED, SP, MED, 2>(m, prm, arm, RT, tT, qc, qa, it, conv, nrm, other, &ro);
    }
    return;
  }
  const int64_t p = (int64_t)blockIdx.x * ppw + (lane >> 1);
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
  if constexpr (REC == 1) {  // the continuation's checkpoints (ikg_collision.hip): outputs at the first passing iterate
    const int rl = rec_len(m->n_passive);
    RecOut<T> ro{ra.rec + p * (int64_t)(prm.max_iters + 1) * rl, ra.nrec + p, qrow, q_out + p * m->nq,
                 conv_out + p, iters_out + p, err_out + p * 2, rl, ra.ck + p * ck_per_problem<T>(prm.max_iters)};
    if (arm == 0) ra.nrec[p] = 0;
    if (solve_pair<T, DAMPED, SP, MED, 1>(m, prm, arm, RT, tT, qc, qa, it, conv, nrm, other, &ro)) return;
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
