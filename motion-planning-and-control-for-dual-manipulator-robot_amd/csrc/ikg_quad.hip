// "Quad" layout of the IK loop (inverse_geometry.py:56-94) for batches too small
// to fill the chip (BASELINE configs[1]: 4,096 targets = 128 pair waves on 1,024
// SIMDs).  One wave issues one instruction at a time, so at that size the
// update's cost is the length of one wave's instruction stream; this layout
// shortens it by giving each arm four lanes instead of one (8 lanes per
// problem, 8 problems per 64-lane wave):
//   * joint trigonometry: lane r advances trig slots r and r + 4 (of the seven
//     frame-1 slots, trig_exact_f1) and DPP quad broadcasts share them;
//   * forward kinematics: rows of the rotation chain evolve independently
//     under right-multiplication by joint rotations, so lane r (< 3) carries
//     row r from the wrist on, and the column r of the error rotation
//     Rw = RT1 Rh^T, the hand point and the position error; three broadcasts
//     of each column assemble Rw;
//   * log6, the closed-form arm solve and the update run replicated in the four
//     lanes (bit-identical inputs -> bit-identical results), so no lane ever
//     waits on another except at the broadcasts and the arm exchange.
// Per lane and update that is ~290 fp64 operations and ~70 32-bit DPP moves
// against ~405 fp64 operations for the pair layout's one lane per arm
// (DESIGN.md §3a.2).  Same device functions as the frame-1 pair path
// (ikg_device.hpp: log6_iter, arm_solve_f1, arm_update, Trig<T>::step), so the
// iterates agree with it to rounding.
#include <hip/hip_runtime.h>

#include "ikg_device.hpp"
#include "ikg_launch.hpp"
#include "ikg_solve.hpp"
#include "ikgrasp.h"

namespace ikg {

// ---------------------------------------------------------------- cross-lane (aligned quads / 8-lane groups)
// broadcast lane K of every aligned 4-lane quad: DPP quad_perm [K,K,K,K]
// (every lane is written, so no "old" operand and no copy into the destination)
template <int K>
__device__ inline int qb_i32(int x) {
  return __builtin_amdgcn_mov_dpp(x, K * 0x55, 0xF, 0xF, false);
}
template <int K>
__device__ inline double qb(double x) {
  const int lo = qb_i32<K>(__double2loint(x)), hi = qb_i32<K>(__double2hiint(x));
  return __hiloint2double(hi, lo);
}
template <int K>
__device__ inline float qb(float x) {
  return __int_as_float(qb_i32<K>(__float_as_int(x)));
}
// exchange with lane ^ 4 (the other arm's lane of the same row): row_shl:4 into
// banks 0/2 (lanes 0-3, 8-11 of each row), row_shr:4 into banks 1/3
__device__ inline int x4_i32(int x) {
  const int v = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0x5, false);
  return __builtin_amdgcn_update_dpp(v, x, 0x114, 0xF, 0xA, false);
}
__device__ inline double x4(double x) {
  const int lo = x4_i32(__double2loint(x)), hi = x4_i32(__double2hiint(x));
  return __hiloint2double(hi, lo);
}
__device__ inline float x4(float x) { return __int_as_float(x4_i32(__float_as_int(x))); }

struct QuadX {  // the other arm's lane group (pinv_step_f1)
  template <typename T>
  __device__ T operator()(T x) const { return x4(x); }
};

template <typename T>
__device__ inline T pick4(int r, T a, T b, T c, T d) {
  return r < 2 ? (r == 0 ? a : b) : (r == 2 ? c : d);
}

// ---------------------------------------------------------------- this lane's two trig slots
// slot A = r: 0 q_root+q0, 1 q0, 2 q1, 3 q1+q2; slot B = r + 4: 4 q3, 5 q4, 6 q5+hand
// (lane 3's B duplicates slot 6)
template <typename T>
__device__ inline void own_trig_exact(const KModel<T>* __restrict__ m, int arm, int r, T qc, const T* qa, T& sA,
                                      T& cA, T& sB, T& cB) {
  const T xA = pick4(r, qc, qa[0], qa[1], qa[1]);
  const T yA = pick4(r, qa[0], T(0), T(0), qa[2]);
  const T xB = pick4(r, qa[3], qa[4], qa[5], qa[5]);
  T s1, c1, s2, c2, s3, c3;
  Prec<T>::sincos_(xA, &s1, &c1);
  Prec<T>::sincos_(yA, &s2, &c2);  // (0, 1) exactly for the single-angle slots
  Prec<T>::sincos_(xB, &s3, &c3);
  add_angles(s1, c1, s2, c2, sA, cA);
  const bool right = arm != 0;
  const T hs = r >= 2 ? (right ? m->hand_sc[1][0] : m->hand_sc[0][0]) : T(0);
  const T hc = r >= 2 ? (right ? m->hand_sc[1][1] : m->hand_sc[0][1]) : T(1);
  add_angles(s3, c3, hs, hc, sB, cB);
}

// FK + pose error in frame 1, rows split over the quad (see the file comment);
// the state needed by arm_solve_f1 comes back replicated in every lane.
template <typename T, class SP>
__device__ inline T quad_fk_error(const KModel<T>* __restrict__ m, int arm, int j, const T* sn, const T* cs,
                                  const T* RT, const T* tT, ArmStateF1<T>& st, ThetaTrack<T>* tk, bool resync) {
  const bool right = arm != 0;
  // target into frame 1 (replicated; as arm_fk_error_f1)
  const T sf = sn[0], cf = cs[0];
  T p0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) p0[i] = SP::zero_t(0, i) ? T(0) : armc<T>(right, m->arm_t[0][0][i], m->arm_t[1][0][i]);
  st.k[0] = cs[1] * p0[0] + sn[1] * p0[1];
  st.k[1] = cs[1] * p0[1] - sn[1] * p0[0];
  T RT1[9], tT1[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    RT1[c] = cf * RT[c] + sf * RT[3 + c];
    RT1[3 + c] = cf * RT[3 + c] - sf * RT[c];
    RT1[6 + c] = RT[6 + c];
  }
  const T d0 = tT[0] - m->root_t[0], d1 = tT[1] - m->root_t[1];
  tT1[0] = cf * d0 + sf * d1 - st.k[0];
  tT1[1] = cf * d1 - sf * d0 - st.k[1];
  tT1[2] = tT[2] - m->root_t[2] - p0[2];
  // replicated chain up to the wrist centre: o2, Ry(q1 + q2), o3, w
  auto off = [&](int k, int i) -> T {
    return SP::zero_t(k, i) ? T(0) : armc<T>(right, m->arm_t[0][k][i], m->arm_t[1][k][i]);
  };
  const T s1 = sn[2], c1 = cs[2];
  // o2 = p1 + Ry(q1) p2
  st.o2[0] = off(1, 0) + (c1 * off(2, 0) + s1 * off(2, 2));
  st.o2[1] = off(1, 1) + off(2, 1);
  st.o2[2] = off(1, 2) + (c1 * off(2, 2) - s1 * off(2, 0));
  st.c12 = cs[3];
  st.s12 = sn[3];
  const T c12 = st.c12, s12 = st.s12;
  // o3 = o2 + Ry(q12) p3; the rotation after joint 3 (X) keeps Ry(q12)'s first column
  T o3[3];
  o3[0] = st.o2[0] + (c12 * off(3, 0) + s12 * off(3, 2));
  o3[1] = st.o2[1] + off(3, 1);
  o3[2] = st.o2[2] + (c12 * off(3, 2) - s12 * off(3, 0));
  const T s3 = sn[4], c3 = cs[4];
  // w = o3 + R3 p4, R3 = Ry(q12) Rx(q3)
  {
    const T R3[9] = {c12, s12 * s3, s12 * c3, T(0), c3, -s3, -s12, c12 * s3, c12 * c3};
    T pt[3] = {off(4, 0), off(4, 1), off(4, 2)}, dv[3];
    matvec3(R3, pt, dv);
#pragma unroll
    for (int i = 0; i < 3; ++i) st.w[i] = o3[i] + dv[i];
  }
  // row j of the chain from here: row_j(Ry(q12)) -> x Rx(q3) -> x Ry(q4) -> x Rz(q5 + hand)
  const T l0 = j == 0 ? T(1) : T(0), l1 = j == 1 ? T(1) : T(0), l2 = j == 2 ? T(1) : T(0);
  T a = l0 * c12 - l2 * s12, b = l1, g = l0 * s12 + l2 * c12;
  T y = c3 * b + s3 * g, z = c3 * g - s3 * b;  // row_j(R3) = (a, y, z)
  const T s4 = sn[5], c4 = cs[5];
  T xr = c4 * a - s4 * z;  // row_j(R4) = (xr, y, zr)
  const T zr = c4 * z + s4 * a;
  const T wj = pick4(j, st.w[0], st.w[1], st.w[2], st.w[0]);
  T o5 = wj + (xr * off(5, 0) + y * off(5, 1) + zr * off(5, 2));  // origin of joint 5, row j
  const T s5 = sn[6], c5 = cs[6];
  const T x5 = c5 * xr + s5 * y, y5 = c5 * y - s5 * xr;  // row_j(Rh) = (x5, y5, zr)
  const T hj = o5 + (x5 * armc<T>(right, m->hand_tH[0][0], m->hand_tH[1][0]) +
                     y5 * armc<T>(right, m->hand_tH[0][1], m->hand_tH[1][1]) +
                     zr * armc<T>(right, m->hand_tH[0][2], m->hand_tH[1][2]));
  // column j of Rw = RT1 Rh^T and the position error
  T col[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) col[i] = RT1[3 * i] * x5 + RT1[3 * i + 1] * y5 + RT1[3 * i + 2] * zr;
  const T dj = pick4(j, tT1[0], tT1[1], tT1[2], tT1[0]) - hj;
  T Rw[9], d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    Rw[3 * i + 0] = qb<0>(col[i]);
    Rw[3 * i + 1] = qb<1>(col[i]);
    Rw[3 * i + 2] = qb<2>(col[i]);
  }
  d[0] = qb<0>(dj);
  d[1] = qb<1>(dj);
  d[2] = qb<2>(dj);
  st.h[0] = qb<0>(hj);
  st.h[1] = qb<1>(hj);
  st.h[2] = qb<2>(hj);
  log6_iter(Rw, d, st.e, tk, resync);
  const T* e = st.e;
  return e[0] * e[0] + e[1] * e[1] + e[2] * e[2] + e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
}

template <typename T, class SP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 8 ? 2 : 4)))
void ikg_quad_batch_kernel(const KModel<T>* __restrict__ m, KParams<T> prm,
                                                            const T* __restrict__ targets,
                                                            const T* __restrict__ q0, int64_t q0_stride, int64_t B,
                                                            int64_t S, T* __restrict__ q_out,
                                                            uint8_t* __restrict__ conv_out,
                                                            int32_t* __restrict__ iters_out,
                                                            T* __restrict__ err_out) {
  static_assert(kFrame1<SP>, "the quad layout runs the frame-1 loop");
  const int lane = threadIdx.x;
  const int64_t p = (int64_t)blockIdx.x * 8 + (lane >> 3);
  if (p >= B) return;  // the 8 lanes of a problem leave together
  const int arm = (lane >> 2) & 1;
  const int r = lane & 3;
  const int j = r < 3 ? r : 0;  // lane 3 repeats row 0 (never a broadcast source)
  const int64_t tgt = S > 1 ? p / S : p;
  const int64_t row = S > 1 ? p - tgt * S : p;
  T RT[9], tT[3];
  hook_target(m, arm, targets + tgt * 12, RT, tT);
  const T* qrow = q0 + row * q0_stride;
  T qc, qa[kArmDof];
  load_q(m, arm, qrow, qc, qa);
  T sA, cA, sB, cB;
  own_trig_exact(m, arm, r, qc, qa, sA, cA, sB, cB);
  ArmLimits<T> lim;
  load_limits(m, arm, lim);
  int it = 0;
  bool conv = false;
  T x, xo;
  ThetaTrack<T> tk{};
  for (;;) {
    T sn[7], cs[7];
    sn[0] = qb<0>(sA), cs[0] = qb<0>(cA);
    sn[1] = qb<1>(sA), cs[1] = qb<1>(cA);
    sn[2] = qb<2>(sA), cs[2] = qb<2>(cA);
    sn[3] = qb<3>(sA), cs[3] = qb<3>(cA);
    sn[4] = qb<0>(sB), cs[4] = qb<0>(cB);
    sn[5] = qb<1>(sB), cs[5] = qb<1>(cB);
    sn[6] = qb<2>(sB), cs[6] = qb<2>(cB);
    ThetaTrack<T>* tkp = (IKG_THETA_TRACK && is_f64<T>) ? &tk : nullptr;
    ArmStateF1<T> st;
    x = quad_fk_error<T, SP>(m, arm, j, sn, cs, RT, tT, st, tkp, (it % Trig<T>::kResync) == 0);
    T dq[6], s;
    pinv_step_f1<T, SP, QuadX>(m, arm, st, sn, cs, dq, s);
    xo = x4(x);
    if (it >= prm.max_iters) break;
    if (x < prm.eps2 && xo < prm.eps2) {  // |e_L| < eps and |e_R| < eps (:70)
      conv = true;
      break;
    }
    T q_old[7];
    q_old[0] = qc;
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) q_old[k + 1] = qa[k];
    arm_update(m, arm, T(prm.dt), s, dq, qc, qa, &lim);
    ++it;
    // this lane's slots: increments of their angles (trig_advance_f1)
    T dj[7];
    dj[0] = qc - q_old[0];
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) dj[k + 1] = qa[k] - q_old[k + 1];
    const T dA = pick4(r, dj[0] + dj[1], dj[1], dj[2], dj[2] + dj[3]);
    const T dB = pick4(r, dj[4], dj[5], dj[6], dj[6]);
    const bool big = (it % Trig<T>::kResync) == 0 || fabs(dA) > T(Trig<T>::kIncMax) ||
                     fabs(dB) > T(Trig<T>::kIncMax);
    if (big) {
      own_trig_exact(m, arm, r, qc, qa, sA, cA, sB, cB);
    } else {
      Trig<T>::step(dA, sA, cA);
      Trig<T>::step(dB, sB, cB);
    }
  }
  if (r == 0) {
    store_q(m, arm, qrow, it, qc, qa, q_out + p * m->nq);
    if (arm == 0) {
      if (conv_out) conv_out[p] = conv ? 1 : 0;
      if (iters_out) iters_out[p] = it;
    }
    if (err_out) err_out[p * 2 + arm] = sqrt(x);
  }
}

template <typename T>
hipError_t launch_quad_batch(const KModel<T>* dmodel, const KParams<T>& prm, const BatchArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)((a.B + 7) / 8));
  hipLaunchKernelGGL((ikg_quad_batch_kernel<T, SpecNextage>), grid, dim3(64), 0, s, dmodel, prm,
                     (const T*)a.targets, (const T*)a.q0, a.q0_stride, a.B, a.S, (T*)a.q_out, a.converged, a.iters,
                     (T*)a.err_out);
  return hipGetLastError();
}

template hipError_t launch_quad_batch<double>(const KModel<double>*, const KParams<double>&, const BatchArgs&,
                                              hipStream_t);
template hipError_t launch_quad_batch<float>(const KModel<float>*, const KParams<float>&, const BatchArgs&,
                                             hipStream_t);

}  // namespace ikg
