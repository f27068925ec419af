// Host emulator of the pair kernel (debug/test tool, NOT a product path and
// never called by libikgrasp.so): runs the exact stage functions of
// ikg_device.hpp for both arm lanes of a problem on the CPU, in the order the
// kernel's lanes execute them, so kernel numerics can be inspected without a
// GPU.  Built as libikgrasp_emu.so; used by tests/test_host_emu.py.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "ikg_collision.hpp"
#include "ikg_device.hpp"
#include "ikg_model_build.hpp"
#include "ikgrasp.h"

namespace {

// updates that took the LQ form (pinv_step_*), since the last ikg_emu_lq_count(1)
thread_local long long lq_count = 0;
thread_local long long big_count = 0;  // lane-updates whose step leaves the short trig series (chest-frame path)
thread_local long long jacobi_count = 0;  // arm solves of the LQ form that fell back to the Jacobi sweeps
thread_local long long svd_count = 0;  // of those, with an arm that pins the chest (bb = 0: rank-deficient M_a)
// updates whose two arm lanes computed different chest steps (must stay 0:
// each lane carries the shared chest joint); ikg_emu_solve returns -3 then
thread_local long long chest_mismatch = 0;

// collide_wave's stages run serially (same functions, same order per lane).
template <typename T>
bool emu_collide(const ikg::KModel<T>& m, const ikg::KCollision<T>& c, const T* q, const T* tgt) {
  using namespace ikg;
  T L[kMaxNq][12], F[kMaxNq][12], P[kMaxGeoms][12];
  for (int j = 0; j < m.nq; ++j) {
    T s, co;
    Prec<T>::sincos_(q[j], &s, &co);
    joint_local(&m, j, s, co, L[j]);
  }
  for (int j = 0; j < m.nq; ++j) joint_world(m.jparent, j, L, F[j]);
  for (int g = 0; g < c.n_geoms; ++g) geom_world(&c, g, F, tgt, P[g]);
  for (int k = 0; k < c.n_pairs; ++k)
    if (pair_hit(&c, k, P)) return true;
  return false;
}

template <typename T, class SP>
void emu_one(const ikg::KModel<T>& m, const ikg::KParams<T>& prm, bool damped, const T* tg, const T* qrow,
             T* qo, uint8_t* conv_out, int32_t* iters_out, T* err_out, T* trace, int trace_len,
             const ikg::KCollision<T>* col, bool med = false) {
  using namespace ikg;
  T RT[2][9], tT[2][3], qc[2], qa[2][kArmDof], sn[2][7], cs[2][7];
  for (int arm = 0; arm < 2; ++arm) {
    const bool right = arm != 0;
    T HR[9], Ht[3], d[3];
    for (int i = 0; i < 9; ++i) HR[i] = right ? m.hook_R[1][i] : m.hook_R[0][i];
    for (int i = 0; i < 3; ++i) Ht[i] = right ? m.hook_t[1][i] : m.hook_t[0][i];
    matmul3(tg, HR, RT[arm]);
    matvec3(tg, Ht, d);
    for (int i = 0; i < 3; ++i) tT[arm][i] = tg[9 + i] + d[i];
    qc[arm] = qrow[m.root_q];
    for (int k = 0; k < kArmDof; ++k) qa[arm][k] = qrow[m.arm_q[arm][k]];
  }
  int it = 0;
  bool conv = false;
  T nrm[2];
  ThetaTrack<T> tk[2] = {};
  // the kernel's frame-1 path (kFrame1 models, lambda = 0) or the chest-frame one
  const bool f1 = kFrame1<SP> && !damped;
  for (int arm = 0; arm < 2; ++arm) {
    if (f1)
      trig_exact_f1(&m, arm, qc[arm], qa[arm], sn[arm], cs[arm]);
    else
      trig_exact(qc[arm], qa[arm], sn[arm], cs[arm]);
  }
  for (;;) {
    ArmState<T> st[2];
    ArmStateF1<T> s1[2];
    const bool resync = (it % Trig<T>::kResync) == 0;
    ThetaTrack<T>* tkp[2] = {is_f64<T> ? &tk[0] : nullptr, is_f64<T> ? &tk[1] : nullptr};
    for (int arm = 0; arm < 2; ++arm) {
      if constexpr (kFrame1<SP>) {
        if (f1) {
          nrm[arm] = arm_fk_error_f1<T, SP>(&m, arm, sn[arm], cs[arm], RT[arm], tT[arm], s1[arm], tkp[arm], resync);
          continue;
        }
      }
      nrm[arm] = arm_fk_error<T, SP>(&m, arm, sn[arm], cs[arm], RT[arm], tT[arm], st[arm], nullptr, tkp[arm], resync);
    }
    if (trace && it < trace_len) {
      trace[2 * it] = std::sqrt(nrm[0]);
      trace[2 * it + 1] = std::sqrt(nrm[1]);
    }
    if (it >= prm.max_iters) break;
    if (nrm[0] < prm.eps2 && nrm[1] < prm.eps2) {
      if (!col) {
        conv = true;
        break;
      }
      T qn[kMaxNq];  // the current iterate in q order (passive joints clamped after update 1)
      for (int j = 0; j < m.nq; ++j) qn[j] = qrow[j];
      for (int i = 0; i < m.n_passive; ++i) {
        const int j = m.passive_q[i];
        qn[j] = it > 0 ? clampq(qrow[j], m.lo[j], m.hi[j]) : qrow[j];
      }
      qn[m.root_q] = qc[0];
      for (int arm = 0; arm < 2; ++arm)
        for (int k = 0; k < kArmDof; ++k) qn[m.arm_q[arm][k]] = qa[arm][k];
      if (!emu_collide(m, *col, qn, tg)) {
        conv = true;
        break;
      }
    }
    T A[2][6][8], u[2][6], v[2][6], al[2], be[2], dqa[2][6], sa[2], q_old[2][7];
    bool bad[2] = {false, false};
    for (int arm = 0; arm < 2; ++arm) {
      q_old[arm][0] = qc[arm];
      for (int k = 0; k < kArmDof; ++k) q_old[arm][k + 1] = qa[arm][k];
      if constexpr (kFrame1<SP>) {
        if (f1) {
          arm_solve_f1<T, SP>(&m, arm, s1[arm], sn[arm], cs[arm], u[arm], v[arm], al[arm], be[arm]);
          bad[arm] = beyond(be[arm], m.sing_beta);
          continue;
        }
      }
      if (damped) {
        arm_system(st[arm], A[arm]);
        arm_solve_damped(A[arm], prm.lambda, u[arm], v[arm], al[arm], be[arm]);
      } else {
        arm_solve<T, SP>(st[arm], u[arm], v[arm], al[arm], be[arm], &bad[arm], m.sing_tau);
        bad[arm] = bad[arm] || beyond(be[arm], m.sing_beta);
      }
    }
    for (int arm = 0; arm < 2; ++arm) {
      sa[arm] = chest_step(al[arm] + al[1 - arm], be[arm] + be[1 - arm]);
      if (damped)
        arm_dq_damped(A[arm], u[arm], v[arm], sa[arm], dqa[arm]);
      else
        arm_dq(u[arm], v[arm], sa[arm], dqa[arm]);
    }
    if (!damped && (bad[0] || bad[1])) {  // pinv_step_f1 / pinv_step_cf: the per-arm pinv form
      T z[2][7], pv[2][7];
      for (int arm = 0; arm < 2; ++arm) {
        if (f1) {
          if constexpr (kFrame1<SP>) arm_system_f1<T, SP>(&m, arm, s1[arm], sn[arm], cs[arm], A[arm]);
        } else {
          arm_system(st[arm], A[arm]);
        }
        if (!arm_minnorm(A[arm], z[arm], pv[arm])) ++jacobi_count;
      }
      for (int arm = 0; arm < 2; ++arm) {
        T f;
        minnorm_combine(z[arm][0], pv[arm][0], z[1 - arm][0], pv[1 - arm][0], sa[arm], f);
        for (int k = 0; k < 6; ++k) dqa[arm][k] = z[arm][1 + k] + f * pv[arm][1 + k];
      }
      if (sa[0] != sa[1]) ++chest_mismatch;  // both lanes must carry the same chest step
      ++lq_count;
      if (pv[0][0] < T(Prec<T>::kRcond) || pv[1][0] < T(Prec<T>::kRcond)) ++svd_count;  // an arm pins s
    }
    ++it;
    for (int arm = 0; arm < 2; ++arm) {
      const T s = sa[arm];
      const T* dq = dqa[arm];
      ArmLimits<T> lim;
      load_limits(&m, arm, lim);
      arm_update(&m, arm, prm.dt, s, dq, qc[arm], qa[arm], IKG_LANE_LIMITS ? &lim : nullptr);
      if (f1)
        (med ? trig_advance_f1<T, true> : trig_advance_f1<T, false>)(&m, arm, qc[arm], qa[arm], q_old[arm],
                                                                     (it % Trig<T>::kResync) == 0, sn[arm], cs[arm]);
      else {
        bool big = false;  // the exact sincos outside resyncs (diagnostic count)
        big |= fabs(qc[arm] - q_old[arm][0]) > T(Trig<T>::kIncMax);
        for (int k = 0; k < kArmDof; ++k) big |= fabs(qa[arm][k] - q_old[arm][k + 1]) > T(Trig<T>::kIncMax);
        if (big) ++big_count;
        trig_advance<T, IKG_GENERIC_MED>(qc[arm], qa[arm], q_old[arm], (it % Trig<T>::kResync) == 0, sn[arm], cs[arm]);
      }
    }
  }
  for (int j = 0; j < m.nq; ++j) qo[j] = qrow[j];
  for (int i = 0; i < m.n_passive; ++i) {
    const int j = m.passive_q[i];
    qo[j] = it > 0 ? clampq(qrow[j], m.lo[j], m.hi[j]) : qrow[j];
  }
  qo[m.root_q] = qc[0];
  for (int arm = 0; arm < 2; ++arm)
    for (int k = 0; k < kArmDof; ++k) qo[m.arm_q[arm][k]] = qa[arm][k];
  *conv_out = conv;
  *iters_out = it;
  err_out[0] = std::sqrt(nrm[0]);
  err_out[1] = std::sqrt(nrm[1]);
}

template <typename T>
void emu(const ikg_model_desc* d, const void* targets, const void* q0, int64_t stride, int64_t B,
         const ikg_params* p, void* q_out, uint8_t* conv, int32_t* iters, void* err, void* trace, int trace_len,
         const ikg_collision_desc* cd) {
  ikg::KModel<T> m;
  ikg::build_kmodel<T>(*d, m);
  static thread_local ikg::KCollision<T> kc;
  const ikg::KCollision<T>* col = nullptr;
  if (cd && p->check_collision) {
    ikg::build_kcollision<T>(*cd, kc);
    col = &kc;
  }
  const ikg::KParams<T> prm = ikg::make_kparams<T>(p);
  const int spec = p->variant == 99 ? 0 : ikg::choose_spec(m);  // variant 99: force generic
  for (int64_t i = 0; i < B; ++i) {
    const T* tg = (const T*)targets + 12 * i;
    const T* qr = (const T*)q0 + stride * i;
    T* tr = trace ? (T*)trace + (int64_t)2 * trace_len * i : nullptr;
    if (spec == 1)
      // the kernels' medium-range trig series for per-problem seeds, and for
      // every fp32 solve (ikg_kernels.hip launch_pair_batch_t)
      emu_one<T, ikg::SpecNextage>(m, prm, p->lambda > 0, tg, qr, (T*)q_out + d->nq * i, conv + i, iters + i,
                                   (T*)err + 2 * i, tr, trace_len, col, stride != 0 || sizeof(T) == 4);
    else if (spec == 2 && !(p->lambda > 0))
      emu_one<T, ikg::SpecGenericWrist>(m, prm, false, tg, qr, (T*)q_out + d->nq * i, conv + i, iters + i,
                                        (T*)err + 2 * i, tr, trace_len, col);
    else
      emu_one<T, ikg::SpecGeneric>(m, prm, p->lambda > 0, tg, qr, (T*)q_out + d->nq * i, conv + i, iters + i,
                                   (T*)err + 2 * i, tr, trace_len, col);
  }
}

}  // namespace

extern "C" long long ikg_emu_big_count(int reset) {
  const long long v = big_count;
  if (reset) big_count = 0;
  return v;
}
extern "C" long long ikg_emu_lq_count(int reset) {
  const long long v = lq_count;
  if (reset) lq_count = 0;
  return v;
}
extern "C" long long ikg_emu_jacobi_count(int reset) {
  const long long v = jacobi_count;
  if (reset) jacobi_count = 0;
  return v;
}
extern "C" long long ikg_emu_svd_count(int reset) {
  const long long v = svd_count;
  if (reset) svd_count = 0;
  return v;
}

// cd may be NULL; it is used when p->check_collision is set.
// Returns 0, or -3 when the two lanes of a problem ever carried different
// chest steps (a kernel invariant; the outputs are then not the kernel's).
extern "C" int ikg_emu_solve(const ikg_model_desc* d, int dtype, const void* targets, const void* q0,
                             int64_t q0_stride, int64_t B, const ikg_params* p, void* q_out, uint8_t* conv,
                             int32_t* iters, void* err, void* trace, int trace_len, const ikg_collision_desc* cd) {
  chest_mismatch = 0;
  if (dtype == IKG_F64)
    emu<double>(d, targets, q0, q0_stride, B, p, q_out, conv, iters, err, trace, trace_len, cd);
  else
    emu<float>(d, targets, q0, q0_stride, B, p, q_out, conv, iters, err, trace, trace_len, cd);
  return chest_mismatch ? -3 : 0;
}

template <typename T>
void emu_col(const ikg_model_desc* d, const ikg_collision_desc* cd, const void* q, const void* targets, int64_t B,
             uint8_t* out) {
  ikg::KModel<T> m;
  ikg::build_kmodel<T>(*d, m);
  static thread_local ikg::KCollision<T> kc;
  ikg::build_kcollision<T>(*cd, kc);
  for (int64_t i = 0; i < B; ++i)
    out[i] = emu_collide(m, kc, (const T*)q + d->nq * i, (const T*)targets + 12 * i) ? 1 : 0;
}

// Collision query through the device stage functions (ikg_collision_batch on the CPU).
extern "C" int ikg_emu_collision(const ikg_model_desc* d, const ikg_collision_desc* cd, int dtype, const void* q,
                                 const void* targets, int64_t B, uint8_t* out) {
  if (dtype == IKG_F64)
    emu_col<double>(d, cd, q, targets, B, out);
  else
    emu_col<float>(d, cd, q, targets, B, out);
  return 0;
}

// Inscribed-ball certificate of scene pair `pair` at configuration qc (joint
// order = q order) with the cube at `target` (ball_cert, the records scan's
// certificate), then whether it proves the pair intersecting at each of the B
// configurations q (ball_covers).  tests/test_collision.py.
template <typename T>
void emu_ball(const ikg_model_desc* d, const ikg_collision_desc* cd, int pair, const void* qc, const void* target,
              const void* q, int64_t B, double* r_out, uint8_t* covered) {
  ikg::KModel<T> m;
  ikg::build_kmodel<T>(*d, m);
  static thread_local ikg::KCollision<T> kc;
  ikg::build_kcollision<T>(*cd, kc);
  int32_t sl[ikg::kMaxNq];
  for (int k = 0; k < ikg::kMaxNq; ++k) sl[k] = k;
  static thread_local ikg::BallCert<T> bc;
  ikg::ball_cert(&m, &kc, pair, (const T*)qc, sl, (const T*)target, bc);
  *r_out = (double)bc.r;
  for (int64_t i = 0; i < B; ++i) covered[i] = ikg::ball_covers(bc, (const T*)q + d->nq * i) ? 1 : 0;
}

extern "C" int ikg_emu_ball_cert(const ikg_model_desc* d, const ikg_collision_desc* cd, int dtype, int pair,
                                 const void* qc, const void* target, const void* q, int64_t B, double* r_out,
                                 uint8_t* covered) {
  if (pair < 0 || pair >= cd->n_pairs) return -1;
  if (dtype == IKG_F64)
    emu_ball<double>(d, cd, pair, qc, target, q, B, r_out, covered);
  else
    emu_ball<float>(d, cd, pair, qc, target, q, B, r_out, covered);
  return 0;
}

// EPA depth certificate of one shape pair (tests/test_collision_epa.py):
// kinds/placements/dims per ikg_collision_desc conventions; returns
// pair_collides' verdict in *r and the certified depth bound in *depth (0 when
// no certificate).
extern "C" int ikg_emu_epa(int kindA, const double* RA, const double* tA, const double* dA, int kindB,
                           const double* RB, const double* tB, const double* dB, int* r, double* depth) {
  using namespace ikg;
  const Shape<double> A{RA, tA, dA, kindA}, B{RB, tB, dB, kindB};
  double cert[12];
  *r = pair_collides(A, B, cert);
  *depth = 0.0;
  if (*r != 2) return 0;
  double pts[4][3];
  for (int k = 0; k < 4; ++k) mink_support(A, B, cert + 3 * k, pts[k]);
  if (!tetra_encloses_origin(pts[0], pts[1], pts[2], pts[3])) return 0;
  EpaScratch s;
  *depth = epa_depth_lb(A, B, pts, s);
  return 0;
}

// The loop's math helpers over arrays (tests/test_host_emu.py accuracy checks):
// fn 0: cw_sincos (fp64), 1: cw_sincos (fp32), 2: the packed pair's sincos
// (both halves), 3: atan2_upper (fp32), 4: atan2_upper (packed pair).
// out holds 2 values per input (sin, cos) for fn 0-2, 1 for fn 3-4.
extern "C" int ikg_emu_math(int fn, int64_t n, const double* x, const double* y, double* out) {
  using namespace ikg;
  for (int64_t i = 0; i < n; ++i) {
    switch (fn) {
      case 0: cw_sincos(x[i], &out[2 * i], &out[2 * i + 1]); break;
      case 1: {
        float s, c;
        cw_sincos((float)x[i], &s, &c);
        out[2 * i] = s;
        out[2 * i + 1] = c;
        break;
      }
      case 2: {
        v2f s, c;
        Prec<v2f>::sincos_(v2f{(float)x[i], (float)-x[i]}, &s, &c);
        out[2 * i] = s.x;
        out[2 * i + 1] = c.x;
        if (s.y != -s.x || c.y != c.x) return -2;  // the halves are independent and symmetric
        break;
      }
      case 3: out[i] = atan2_upper((float)y[i], (float)x[i]); break;
      case 4: {
        const v2f r = atan2_upper(v2f{(float)y[i], (float)y[i]}, v2f{(float)x[i], (float)x[i]});
        if (r.x != r.y) return -2;
        out[i] = r.x;
        break;
      }
      default: return -1;
    }
  }
  return 0;
}
