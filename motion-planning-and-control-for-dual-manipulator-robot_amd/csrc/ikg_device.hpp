// Device-side math for the batched grasp-pose IK (gfx950 / CDNA4).
//
// Every function here restates one piece of the reference loop
// (/root/reference/inverse_geometry.py:56-94) or of the Pinocchio calls it
// makes; the oracle (oracle/ik_oracle.py) is the independent CPU statement of
// the same algorithm and is never linked into this library.
#pragma once

// (hipRTC, ikg_jit.hip: the runtime compiler provides the HIP declarations)
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

#include <type_traits>

// Math helpers are __host__ __device__ so tools/host_emu.cpp can run the
// exact kernel arithmetic on the CPU for debugging (never a product path).
#define IKG_HD __host__ __device__

// Timing-only ablation switches (tools/ablate.py builds; never the shipped
// library): bit 0 = cheap joint sincos, bit 1 = trivial log6,
// bit 2 = skip the 6x6 solve.
#ifndef IKG_ABL
#define IKG_ABL 0
#endif
// rotation angle in the loop's log6 (fp64): 0 = acos((tr R - 1)/2) as pin.log3,
// 1 = atan2(|skew|/2, (tr R - 1)/2)
#ifndef IKG_THETA
#define IKG_THETA 0
#endif
// log6's small-angle series by multiplications instead of divisions
#ifndef IKG_TAYLOR_MUL
#define IKG_TAYLOR_MUL 1
#endif
// fp64 log6 in the loop: Pinocchio's small-angle series for alpha, beta below
// precision<3>() (1) or the closed forms throughout (0)
#ifndef IKG_LOG6_SERIES
#define IKG_LOG6_SERIES 1
#endif
// pair kernel: per-lane joint limits held in registers (12 fp64) instead of
// clamping against both arms' scalar limits and selecting
#ifndef IKG_LANE_LIMITS
#define IKG_LANE_LIMITS 1
#endif
// Nextage-pattern models: iterate in the frame of the first arm joint with the
// closed-form arm solve (arm_fk_error_f1 / arm_solve_f1) instead of the chest
// frame and the two 3x3 Cramer solves
#ifndef IKG_FRAME1
#define IKG_FRAME1 1
#endif
// carry the rotation angle across iterations (ThetaTrack)
#ifndef IKG_THETA_TRACK
#define IKG_THETA_TRACK 1
#endif
// angle increment by a division-free asin series (1) or atan(y/x) (0)
#ifndef IKG_THETA_ASIN
#define IKG_THETA_ASIN 1
#endif

// The singularity guard of the closed-form step (pinv_step_*).  The closed
// form dq_a = u_a - s v_a (v_a = J_a^-1 c_a, s ~ |u| / |v|) rounds to
// ~eps |v_a| relative to the step: the cancellation grows with |v|, i.e.
// where the chest column has a component along the direction the arm block
// loses.  That is the wrist (c4 -> 0) and the shoulder (w_x -> 0), where J
// itself stays well conditioned (cond ~ 1e2) and pinv does not blow up: the
// pair then takes the per-arm pinv form.  At a straight elbow the chest cannot restore
// the lost direction, |v| stays moderate and J itself is ill conditioned, so
// the closed form is as accurate as any pinv (both ~eps cond(J)) until J is
// rank deficient to rounding, where v (and the guard) blows up and the
// branch's per-arm pinv truncates as np.linalg.pinv does (arm_pinv7).  The guard is one
// integer compare of |v|^2 (bits, so an inf/NaN from an exactly singular
// block's reciprocal also trips it) against sing_beta: fp64 1e14 (the step's
// relative rounding stays below ~1e-9 per update and the KAT-style final q
// within ~1e-11 of pinv, tools/singular_probe.py), fp32 1e12.  Tighter
// bounds trip on unconverged problems that wander near the wrist for
// hundreds of updates (C5-style random seeds: 630 of 505,859 fp64 updates at
// 1e10, 17 at 1e14), stalling their waves.
// Timing knob: IKG_SING_GUARD=0 builds the unguarded closed form.
#ifndef IKG_SING_GUARD
#define IKG_SING_GUARD 1
#endif
#ifndef IKG_SING_BETA64
#define IKG_SING_BETA64 1e14
#endif
#ifndef IKG_SING_BETA32
#define IKG_SING_BETA32 1e12f
#endif
// generic-path (chest frame, Householder / 3 x 3 adjugate) relative pivot bound
#ifndef IKG_SING_TAU64
#define IKG_SING_TAU64 1e-7
#endif
#ifndef IKG_SING_TAU32
#define IKG_SING_TAU32 1e-4
#endif

namespace ikg {

constexpr int kArmDof = 6;
constexpr int kMaxNq = 32;

// Kernel-side model tables (built once per model/dtype in ikg_capi.hip and
// uploaded to device global memory; read through uniform scalar loads).
template <typename T>
struct KModel {
  T root_R[9];
  T root_t[3];
  T root_lo, root_hi;
  T arm_R[2][kArmDof][9];
  T arm_t[2][kArmDof][3];
  T arm_lo[2][kArmDof];
  T arm_hi[2][kArmDof];
  T hand_R[2][9];
  T hand_t[2][3];
  T hook_R[2][9];
  T hook_t[2][3];
  T lo[kMaxNq];
  T hi[kMaxNq];
  int32_t arm_q[2][kArmDof];
  int32_t passive_q[kMaxNq];
  int32_t n_passive;
  int32_t root_q;
  int32_t root_axis;
  int32_t arm_axis[kArmDof];
  int32_t nq;
  int32_t rot_mask;  // bit k (k<6): arm joint k placement rotation != I; bit 6: root
  int32_t hand_axis;  // 0/1/2: hand placement rotation is R_axis(angle) (hand_sc); 3: general
  T hand_sc[2][2];    // (sin, cos) of that angle per hand
  int32_t wrist;      // 1: axes of arm joints 3,4,5 meet at the origin of arm joint 4
  int32_t pattern;    // compile-time specialisation code (ikg_model_build.hpp)
  int32_t zmask;      // bit 3k+i: arm_t[*][k][i] == 0 for both arms (k < 6)
  T hand_tH[2][3];    // hand_R^T hand_t: hand offset seen from the hand frame
  // full kinematic tree (every joint, q order) for the collision check
  T jR[kMaxNq][9];
  T jt[kMaxNq][3];
  int32_t jaxis[kMaxNq];
  int32_t jparent[kMaxNq];
  // singularity guard (pinv_step_*, build_kmodel): the bound on |v_a|^2 of
  // the closed form, and the generic path's relative pivot bound
  T sing_beta;
  T sing_tau;
};

// ---------------------------------------------------------------- kernel specialisation
// Joint-axis pattern packed 2 bits per slot: slot 0 = root, 1..6 = arm joints,
// 7 = hand frame rotation; value 3 = "read from the model at run time".
constexpr int kAxRuntime = 3;
constexpr int kPatternGeneric = 0xFFFF;

template <int PAT, bool PROT, bool WRIST, int ZMASK = 0>
struct Spec {
  static constexpr int axis(int slot) { return (PAT >> (2 * slot)) & 3; }
  static constexpr bool prot = PROT;    // arm joint placements carry rotations
  static constexpr bool wrist = WRIST;  // decoupled spherical-wrist solve
  // arm joint k's placement offset component i is exactly 0 (both arms)
  static constexpr bool zero_t(int k, int i) { return (ZMASK >> (3 * k + i)) & 1; }
  static constexpr int zmask = ZMASK;
  // the hand frame rotation turns about the last arm joint's axis: fold it
  // into that joint's angle (Rh = R5 Rot(q5 + hand angle))
  static constexpr bool fold_hand = axis(7) != kAxRuntime && axis(7) == axis(6);
};
using SpecGeneric = Spec<kPatternGeneric, true, false>;
// any model whose arm joints 3, 4, 5 meet in a point (ikg_model_build.hpp):
// generic tables, the decoupled wrist solve instead of the 6x6 QR
using SpecGenericWrist = Spec<kPatternGeneric, true, true>;
// Nextage (NextageaOpen.urdf:580-730): root Z; arm Z,Y,Y,X,Y,Z; hand Rz(1.5708);
// identity joint placements; spherical wrist at LARM/RARM_JOINT4.
constexpr int kPatternNextage = 2 | (2 << 2) | (1 << 4) | (1 << 6) | (0 << 8) | (1 << 10) | (2 << 12) | (2 << 14);
// zero offset components of the arm joint placements (URDF :580-730, both arms):
// J1 (0,0,z)  J2 (0,y,z)  J3 (x,0,z)  J4 (x,0,0)  J5 (0,0,z)
constexpr int kZeroNextage = (3 << 3) | (1 << 6) | (2 << 9) | (6 << 12) | (3 << 15);
using SpecNextage = Spec<kPatternNextage, false, true, kZeroNextage>;

template <typename T>
struct KParams {
  T eps;
  T dt;
  T lambda;
  int32_t max_iters;
  // stop threshold on the squared error norm: x < eps2 <=> sqrt(x) < eps for
  // the correctly rounded sqrt (make_kparams), so the loop's stop test
  // (inverse_geometry.py:70) needs no square root
  T eps2;
};

// ---------------------------------------------------------------- lane value types
// Scalar kernels (pair layout: one arm per lane) use T = double / float.  The
// packed fp32 kernel keeps BOTH arms of a problem in one lane as a 2-vector
// (x = left, y = right) so each v_pk_{fma,mul,add}_f32 advances both arms; the
// shared root joint is carried in both halves.  The helpers below give the
// iteration code one spelling for both (masks, selects, per-arm constants).
typedef float v2f __attribute__((ext_vector_type(2)));
typedef int v2i __attribute__((ext_vector_type(2)));

template <typename T>
struct LaneT {
  using E = T;     // element type
  using M = bool;  // comparison mask
  static constexpr bool packed = false;
};
template <>
struct LaneT<v2f> {
  using E = float;
  using M = v2i;
  static constexpr bool packed = true;
};
template <typename T>
constexpr bool is_f64 = std::is_same<typename LaneT<T>::E, double>::value;
template <typename T>
constexpr bool is_packed = LaneT<T>::packed;

IKG_HD inline bool any_of(bool m) { return m; }
IKG_HD inline bool any_of(v2i m) { return m.x != 0 || m.y != 0; }
IKG_HD inline bool all_of(bool m) { return m; }
IKG_HD inline bool all_of(v2i m) { return m.x != 0 && m.y != 0; }
// Wave-uniform branch conditions (IKG_UNIFORM): a rare per-lane path (exact
// trig / acos, the near-pi axis) is run by the whole wave when any lane needs
// it and its result selected per lane, so the branch is a scalar one -- no
// EXEC save/restore or phi copies on the common path, and every lane's value
// is the one it computed before (the selects keep the other lanes' results).
#ifndef IKG_UNIFORM
#define IKG_UNIFORM 1
#endif
// Not for the packed fp32 layout: there the scalar branches cost 2-3% at C3
// under its max-ILP schedule (round 3 A/B), so T = v2f keeps per-lane ones.
template <typename T>
IKG_HD inline bool wave_any(bool b) {
#if defined(__HIP_DEVICE_COMPILE__) && IKG_UNIFORM
  if constexpr (!LaneT<T>::packed) return __builtin_amdgcn_ballot_w64(b) != 0;
#endif
  return b;
}
IKG_HD inline bool mnot(bool m) { return !m; }
IKG_HD inline v2i mnot(v2i m) { return m == 0; }
IKG_HD inline bool mor(bool a, bool b) { return a || b; }
IKG_HD inline v2i mor(v2i a, v2i b) { return a | b; }
template <typename T, typename M>
IKG_HD inline T vsel(M m, T a, T b) {
  if constexpr (LaneT<T>::packed)
    return T{m.x ? a.x : b.x, m.y ? a.y : b.y};
  else
    return m ? a : b;
}

// per-arm model constant: the lane's arm (pair layout) or both (packed)
template <typename T, typename E>
IKG_HD inline T armc(bool right, E left_v, E right_v) {
  if constexpr (is_packed<T>)
    return T{left_v, right_v};
  else
    return right ? right_v : left_v;
}

// elementwise math on the packed type (the global overloads stay visible)
using ::atan2;
using ::atan2f;
using ::fabs;
using ::fmax;
using ::fmin;
using ::sqrt;
IKG_HD inline v2f fmax(v2f a, v2f b) { return v2f{::fmaxf(a.x, b.x), ::fmaxf(a.y, b.y)}; }
IKG_HD inline v2f fmin(v2f a, v2f b) { return v2f{::fminf(a.x, b.x), ::fminf(a.y, b.y)}; }
IKG_HD inline v2f fabs(v2f a) { return v2f{::fabsf(a.x), ::fabsf(a.y)}; }
IKG_HD inline v2f sqrt(v2f a) { return v2f{::sqrtf(a.x), ::sqrtf(a.y)}; }
IKG_HD inline v2f atan2(v2f y, v2f x) { return v2f{::atan2f(y.x, x.x), ::atan2f(y.y, x.y)}; }
IKG_HD inline v2f atan2f(v2f y, v2f x) { return atan2(y, x); }

// ---------------------------------------------------------------- precision traits
// sin/cos of a joint angle: Cody-Waite reduction by pi/2 in three FMA parts
// and Taylor polynomials on |r| <= pi/4 (truncation < 5e-17 fp64, < 2e-9
// fp32; ~1 ulp overall).  The reduction stays within ~1e-16 absolute for
// |x| < 2^40 (fp64; fp32: |x| < 2^16), far beyond any joint angle.  It replaces
// OCML's sincos, whose Payne-Hanek path for huge arguments is dead weight in
// the loop's exact trig (every 16th fp32 update: IKG_CW_SINCOS=0 restores it).
#ifndef IKG_CW_SINCOS
#define IKG_CW_SINCOS 1
#endif
// The packed pair keeps OCML's sincosf (0).  The polynomial in packed math (1)
// or per half (2) measured 4% slower at C3 (fp32, q = 0; its exact trig runs
// at resyncs only), and (1) 3% faster with random seeds (large steps)
// (profiles/r02/fp32_math_ab.txt, interleaved A/B of same-flag builds).
#ifndef IKG_CW_SINCOS_PACKED
#define IKG_CW_SINCOS_PACKED 0
#endif
template <typename T>
IKG_HD inline void cw_poly(T r, T& sr, T& cr) {
  const T r2 = r * r;
  T sp, cp;
  if constexpr (std::is_same<T, double>::value) {  // sin: r (1 - r^2/3! + ... - r^14/15!), cos: to r^16/16!
    sp = T(-1.0 / 1307674368000.0);
    sp = fma(sp, r2, T(1.0 / 6227020800.0));
    sp = fma(sp, r2, T(-1.0 / 39916800.0));
    sp = fma(sp, r2, T(1.0 / 362880.0));
    sp = fma(sp, r2, T(-1.0 / 5040.0));
    sp = fma(sp, r2, T(1.0 / 120.0));
    sp = fma(sp, r2, T(-1.0 / 6.0));
    cp = T(1.0 / 20922789888000.0);
    cp = fma(cp, r2, T(-1.0 / 87178291200.0));
    cp = fma(cp, r2, T(1.0 / 479001600.0));
    cp = fma(cp, r2, T(-1.0 / 3628800.0));
    cp = fma(cp, r2, T(1.0 / 40320.0));
    cp = fma(cp, r2, T(-1.0 / 720.0));
    cp = fma(cp, r2, T(1.0 / 24.0));
    sr = fma(r * r2, sp, r);
    cr = fma(r2 * r2, cp, fma(r2, T(-0.5), T(1)));
  } else {  // float or the packed pair (contracted to v_pk_fma_f32)
    sp = T(1.0f / 362880.0f);
    sp = sp * r2 + T(-1.0f / 5040.0f);
    sp = sp * r2 + T(1.0f / 120.0f);
    sp = sp * r2 + T(-1.0f / 6.0f);
    cp = T(-1.0f / 3628800.0f);
    cp = cp * r2 + T(1.0f / 40320.0f);
    cp = cp * r2 + T(-1.0f / 720.0f);
    cp = cp * r2 + T(1.0f / 24.0f);
    sr = (r * r2) * sp + r;
    cr = (r2 * r2) * cp + (r2 * T(-0.5f) + T(1.0f));
  }
}

// quadrant n (mod 4) of the reduction: (sin, cos)(r + n pi/2)
template <typename T>
IKG_HD inline void cw_quadrant(int n, T sr, T cr, T* s, T* c) {
  const int qd = n & 3;
  const T ss = (qd & 1) ? cr : sr;
  const T cc = (qd & 1) ? sr : cr;
  *s = (qd & 2) ? -ss : ss;
  *c = ((qd + 1) & 2) ? -cc : cc;
}

IKG_HD inline void cw_sincos(double x, double* s, double* c) {
  const double n = rint(x * 0.63661977236758134308);  // 2/pi
  double r = fma(-n, 1.5707963267948966, x);
  r = fma(-n, 6.123233995736766e-17, r);
  r = fma(-n, -1.4973849048591698e-33, r);
  double sr, cr;
  cw_poly(r, sr, cr);
  cw_quadrant((int)n, sr, cr, s, c);
}

IKG_HD inline void cw_sincos(float x, float* s, float* c) {
  const float n = rintf(x * 0.636619772f);
  float r = fmaf(-n, 1.57079637f, x);
  r = fmaf(-n, -4.37113883e-08f, r);
  r = fmaf(-n, -1.71512489e-15f, r);
  float sr, cr;
  cw_poly(r, sr, cr);
  cw_quadrant((int)n, sr, cr, s, c);
}

template <typename T>
struct Prec;

template <>
struct Prec<double> {
  // TaylorSeriesExpansion<double>::precision<3>() = eps^(1/4) (Pinocchio log3/log6)
  static constexpr double kPrec3 = 1.220703125e-04;
  static constexpr double kPi = 3.14159265358979323846;
  // relative cut-off for the triangular solve (np.linalg.pinv rcond = 1e-15)
  static constexpr double kRcond = 1e-15;
  IKG_HD static inline void sincos_(double x, double* s, double* c) {
#if IKG_CW_SINCOS
    cw_sincos(x, s, c);
#else
    ::sincos(x, s, c);
#endif
  }
};

template <>
struct Prec<float> {
  // fp32 kernel: series branches widened so the float path tracks the fp64
  // reference ("fp32 numerics"); 0.1 keeps the truncated series
  // below 1e-13 relative.
  static constexpr float kPrec3 = 0.1f;
  static constexpr float kPi = 3.14159265358979323846f;
  static constexpr float kRcond = 1e-7f;
  IKG_HD static inline void sincos_(float x, float* s, float* c) {
#if IKG_CW_SINCOS
    cw_sincos(x, s, c);
#else
    ::sincosf(x, s, c);
#endif
  }
};

template <>
struct Prec<v2f> {
  static constexpr float kPrec3 = Prec<float>::kPrec3;
  static constexpr float kPi = Prec<float>::kPi;
  static constexpr float kRcond = Prec<float>::kRcond;
  IKG_HD static inline void sincos_(v2f x, v2f* s, v2f* c) {
#if IKG_CW_SINCOS && IKG_CW_SINCOS_PACKED == 1
    // both halves' reductions and polynomials in packed math, quadrants per half
    const v2f n = v2f{rintf(x.x * 0.636619772f), rintf(x.y * 0.636619772f)};
    v2f r = x - n * 1.57079637f;  // contracted: fma(-n, C, x)
    r = r - n * -4.37113883e-08f;
    r = r - n * -1.71512489e-15f;
    v2f sr, cr;
    cw_poly(r, sr, cr);
    float s0, c0, s1, c1;
    cw_quadrant((int)n.x, sr.x, cr.x, &s0, &c0);
    cw_quadrant((int)n.y, sr.y, cr.y, &s1, &c1);
    *s = v2f{s0, s1};
    *c = v2f{c0, c1};
#elif IKG_CW_SINCOS && IKG_CW_SINCOS_PACKED == 2
    float s0, c0, s1, c1;  // the scalar polynomial per half
    cw_sincos(x.x, &s0, &c0);
    cw_sincos(x.y, &s1, &c1);
    *s = v2f{s0, s1};
    *c = v2f{c0, c1};
#else
    float s0, c0, s1, c1;
    ::sincosf(x.x, &s0, &c0);
    ::sincosf(x.y, &s1, &c1);
    *s = v2f{s0, s1};
    *c = v2f{c0, c1};
#endif
  }
};

template <typename T>
IKG_HD inline T sel(bool b, T x, T y) { return b ? x : y; }

// a / b through the hardware reciprocal refined by Newton steps (fp64: 2 steps
// + one residual correction, within ~1 ulp of the IEEE quotient) instead of the
// 11-instruction div_scale/div_fmas/div_fixup sequence; none of the quotients
// on the IK path needs correct rounding.
template <typename T>
IKG_HD inline T fdiv(T a, T b) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (is_f64<T>) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(r, fma(-b, r, 1.0), r);
    r = fma(r, fma(-b, r, 1.0), r);
    const double q = a * r;
    return fma(fma(-b, q, a), r, q);
  } else if constexpr (is_packed<T>) {
    v2f r = v2f{__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    r = r * (-b * r + 1.0f) + r;
    const v2f q = a * r;
    return (-b * q + a) * r + q;
  } else {
    float r = __builtin_amdgcn_rcpf(b);
    r = fmaf(r, fmaf(-b, r, 1.0f), r);
    const float q = a * r;
    return fmaf(fmaf(-b, q, a), r, q);
  }
#else
  return a / b;
#endif
}

// 1 / b: v_rcp_f64 is good to ~2^-24 relative; one Newton step leaves <= 11
// ulp and two give the correctly rounded reciprocal on every one of 2^20
// log-uniform inputs (tools/ubench/rcp.hip, profiles/r02/ubench_rcp.txt)
template <typename T>
IKG_HD inline T frcp(T b) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (is_f64<T>) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(r, fma(-b, r, 1.0), r);
    return fma(r, fma(-b, r, 1.0), r);
  } else if constexpr (is_packed<T>) {
    const v2f r = v2f{__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
    return r * (-b * r + 1.0f) + r;
  } else {
    float r = __builtin_amdgcn_rcpf(b);
    return fmaf(r, fmaf(-b, r, 1.0f), r);
  }
#else
  return T(1) / b;
#endif
}

// sqrt(x) for 0 <= x <= 4 (|skew| of a rotation): OCML's refinement without
// its denormal scaling and special-value selects (x = 0 gives 0); fp32: the
// hardware v_sqrt_f32 (IKG_RAW_SQRTF=0: OCML's sqrtf)
#ifndef IKG_RAW_SQRTF
#define IKG_RAW_SQRTF 1
#endif
template <typename T>
IKG_HD inline T fsqrt_unit(T x) {
#ifdef __HIP_DEVICE_COMPILE__
  if constexpr (is_f64<T>) {
    const double y = __builtin_amdgcn_rsq(fmax(x, 1e-300));
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    h = fma(h, r, h);
    // one correction already rounds correctly (tools/ubench/rcp.hip)
    const double d = fma(-g, g, x);
    return fma(d, h, g);
  } else if constexpr (!IKG_RAW_SQRTF) {
    return sqrt(x);
  } else if constexpr (is_packed<T>) {
    // v_sqrt_f32 (1 ulp) without OCML's denormal scaling and class checks
    return T{__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
  } else {
    return __builtin_amdgcn_sqrtf(x);
  }
#else
  if constexpr (is_packed<T>)
    return sqrt(x);
  else
    return std::sqrt(x);
#endif
}

// ---------------------------------------------------------------- cross-lane
// Exchange a value with the partner lane (lane ^ 1) through a DPP quad_perm
// [1,0,3,2]: no LDS traffic, one VALU op per dword.
__device__ inline int pair_swap_i32(int x) {
  // every lane is written: mov_dpp needs no "old" operand (and no copy of x)
  return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false);
}
__device__ inline float pair_swap(float x) {
  return __int_as_float(pair_swap_i32(__float_as_int(x)));
}
__device__ inline double pair_swap(double x) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  lo = pair_swap_i32(lo);
  hi = pair_swap_i32(hi);
  return __hiloint2double(hi, lo);
}
// packed: the partner arm is the other half of the same lane
IKG_HD inline v2f pair_swap(v2f x) { return x.yx; }

// ---------------------------------------------------------------- SE(3) pieces
// R is row-major: R[3*r + c].
template <typename T>
IKG_HD inline void matmul3(const T* A, const T* B, T* C) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[3 * r + 0] * B[0 + c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}

// C = A^T B
template <typename T>
IKG_HD inline void matmul3_tn(const T* A, const T* B, T* C) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[0 + r] * B[0 + c] + A[3 + r] * B[3 + c] + A[6 + r] * B[6 + c];
}

// C = A B^T
template <typename T>
IKG_HD inline void matmul3_nt(const T* A, const T* B, T* C) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      C[3 * r + c] = A[3 * r + 0] * B[3 * c + 0] + A[3 * r + 1] * B[3 * c + 1] + A[3 * r + 2] * B[3 * c + 2];
}

template <typename T>
IKG_HD inline void matvec3(const T* A, const T* x, T* y) {
#pragma unroll
  for (int r = 0; r < 3; ++r) y[r] = A[3 * r] * x[0] + A[3 * r + 1] * x[1] + A[3 * r + 2] * x[2];
}

template <typename T>
IKG_HD inline void matvec3_t(const T* A, const T* x, T* y) {
#pragma unroll
  for (int r = 0; r < 3; ++r) y[r] = A[r] * x[0] + A[3 + r] * x[1] + A[6 + r] * x[2];
}

// R <- R * Rot_axis(q) given (s, c) = sincos(q): JointModelR{X,Y,Z}::calc
// composed onto the parent rotation (only two columns change).
template <typename T>
IKG_HD inline void rotate_axis(T* R, int axis, T s, T c) {
  if (axis == 0) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      T c1 = R[3 * r + 1], c2 = R[3 * r + 2];
      R[3 * r + 1] = c * c1 + s * c2;
      R[3 * r + 2] = c * c2 - s * c1;
    }
  } else if (axis == 1) {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      T c0 = R[3 * r + 0], c2 = R[3 * r + 2];
      R[3 * r + 0] = c * c0 - s * c2;
      R[3 * r + 2] = c * c2 + s * c0;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      T c0 = R[3 * r + 0], c1 = R[3 * r + 1];
      R[3 * r + 0] = c * c0 + s * c1;
      R[3 * r + 1] = c * c1 - s * c0;
    }
  }
}

template <typename T>
IKG_HD inline void column(const T* R, int axis, T* a) {
  a[0] = axis == 0 ? R[0] : (axis == 1 ? R[1] : R[2]);
  a[1] = axis == 0 ? R[3] : (axis == 1 ? R[4] : R[5]);
  a[2] = axis == 0 ? R[6] : (axis == 1 ? R[7] : R[8]);
}

// ---------------------------------------------------------------- log3 / log6
// pin.log3 / pin.log6 -> [v; w] (inverse_geometry.py:66-67), with Pinocchio's
// branch structure: near-pi diagonal formula for
// theta >= pi - 1e-2, Taylor series below precision<3>().  The nominal branch
// is evaluated from sin(theta) = |skew(R)|/2 and cos(theta) = (tr R - 1)/2,
// which removes three transcendental calls and three divisions from the
// reference formulas (alpha = theta sin/(2(1-cos)) = theta (1+cos)/(2 sin),
// beta = 1/theta^2 - sin/(2 theta (1-cos)) = (1-alpha)/theta^2).
template <typename T>
IKG_HD inline void log6(const T* R, const T* p, T* e) {
  const T pi = Prec<T>::kPi;
  const T tr = R[0] + R[4] + R[8];
  const T sx = R[7] - R[5], sy = R[2] - R[6], sz = R[3] - R[1];
  const T ct = (tr - T(1)) * T(0.5);
  const T st = sqrt(sx * sx + sy * sy + sz * sz) * T(0.5);
  T theta;
  if constexpr (sizeof(T) == 8) {
    theta = tr > T(3) ? T(0) : (tr < T(-1) ? pi : acos(ct));  // as pin.log3
  } else {
    theta = atan2f(st, ct);  // fp32: accurate near 0 where acos is not
  }
  T w[3], alpha;
  const T t2 = theta * theta;
  if (theta >= pi - T(1e-2)) {
    T s_, cphi;
    Prec<T>::sincos_(theta - pi, &s_, &cphi);
    const T beta = t2 / (T(1) + cphi);
    const T t0 = (R[0] + cphi) * beta, t1 = (R[4] + cphi) * beta, tt = (R[8] + cphi) * beta;
    w[0] = (R[7] > R[5] ? T(1) : T(-1)) * (t0 > T(0) ? sqrt(t0) : T(0));
    w[1] = (R[2] > R[6] ? T(1) : T(-1)) * (t1 > T(0) ? sqrt(t1) : T(0));
    w[2] = (R[3] > R[1] ? T(1) : T(-1)) * (tt > T(0) ? sqrt(tt) : T(0));
    // here sin(theta) from |skew| is inaccurate; 1 - cos(theta) ~ 2 is benign
    alpha = fdiv(theta * (-s_), T(2) * (T(1) - ct));  // sin(theta) = -sin(theta - pi)
  } else {
    T f;
    if (theta > Prec<T>::kPrec3) {
      f = fdiv(theta, st);
    } else if constexpr (sizeof(T) == 8) {
      f = T(1);  // Pinocchio: theta/sin(theta) -> 1 below precision<3>()
    } else {
      f = T(1) + t2 * (T(1) / T(6) + t2 * (T(7) / T(360)));
    }
    const T hf = f * T(0.5);
    w[0] = hf * sx;
    w[1] = hf * sy;
    w[2] = hf * sz;
    // theta (1+cos)/(2 sin) for cos >= 0, theta sin/(2(1-cos)) otherwise: no cancellation
    if (ct >= T(0))
      alpha = hf * (T(1) + ct);
    else
      alpha = fdiv(theta * st, T(2) * (T(1) - ct));
  }
  T beta;
  if (theta < Prec<T>::kPrec3) {
    if constexpr (sizeof(T) == 8) {
      alpha = T(1) - t2 / T(12) - t2 * t2 / T(720);
      beta = T(1) / T(12) + t2 / T(720);
    } else {
      alpha = T(1) - t2 * (T(1) / T(12) + t2 * (T(1) / T(720) + t2 * (T(1) / T(30240))));
      beta = T(1) / T(12) + t2 * (T(1) / T(720) + t2 * (T(1) / T(30240) + t2 * (T(1) / T(1209600))));
    }
  } else {
    beta = fdiv(T(1) - alpha, t2);
  }
  const T wp = w[0] * p[0] + w[1] * p[1] + w[2] * p[2];
  const T bwp = beta * wp;
  // v = alpha p - 0.5 w x p + (beta w.p) w
  e[0] = alpha * p[0] - T(0.5) * (w[1] * p[2] - w[2] * p[1]) + bwp * w[0];
  e[1] = alpha * p[1] - T(0.5) * (w[2] * p[0] - w[0] * p[2]) + bwp * w[1];
  e[2] = alpha * p[2] - T(0.5) * (w[0] * p[1] - w[1] * p[0]) + bwp * w[2];
  e[3] = w[0];
  e[4] = w[1];
  e[5] = w[2];
}

// log6 for the IK loop: the same function as log6() above (Pinocchio's
// branches and formulas), arranged for latency.  In the loop one
// wave per SIMD runs a single dependent chain FK -> log6 -> solve, so log6's
// branches (which split the schedule) and its serial sqrt/acos/division chain
// dominated the iteration (tools/ablate.py IKG_ABL=2: 29% of it).  Here:
//  * every branch except the rare near-pi axis is a select, so the scheduler can
//    overlap log6 with the error-independent Jacobian work;
//  * the near-pi branch needs no sincos: cos(theta - pi) = -cos(theta) and
//    sin(theta) = |skew|/2 (accurate near pi in absolute terms);
//  * guarded denominators keep the unselected lanes finite.
// Rotation angle carried across iterations (log6_iter): the hand moves a little
// per update, so theta = theta_prev + atan2(sin(theta - theta_prev), cos(...))
// with the difference angle from (sin, cos) of both (angle subtraction) and a
// short odd series for its atan; exact acos/atan2 at it % kResync == 0 and
// whenever |theta - theta_prev| > kInc.
template <typename T>
struct ThetaTrack {
  T th, st, ct;
};
template <typename T>
struct ThetaInc;
template <>
struct ThetaInc<double> {
  static constexpr double kInc = 0.05;  // r^13/13 < 1e-17 r
  IKG_HD static inline double atan_small(double r) {
    const double r2 = r * r;
    return r + r * r2 * (-1.0 / 3 + r2 * (1.0 / 5 + r2 * (-1.0 / 7 + r2 * (1.0 / 9 + r2 * (-1.0 / 11)))));
  }
  // |y| <= 0.035 (the angle moves ~1% of itself per update): the first dropped
  // term 63/2816 y^11 < 3e-18
  static constexpr double kIncAsin = 0.035;
  IKG_HD static inline double asin_small(double y) {
    const double y2 = y * y;
    return y + y * y2 * (1.0 / 6 + y2 * (3.0 / 40 + y2 * (5.0 / 112 + y2 * (35.0 / 1152))));
  }
};
template <>
struct ThetaInc<float> {
  static constexpr float kInc = 0.05f;
  IKG_HD static inline float atan_small(float r) {
    const float r2 = r * r;
    return r + r * r2 * (-1.0f / 3 + r2 * (1.0f / 5 + r2 * (-1.0f / 7)));
  }
  static constexpr float kIncAsin = 0.035f;
  IKG_HD static inline float asin_small(float y) {
    const float y2 = y * y;
    return y + y * y2 * (1.0f / 6 + y2 * (3.0f / 40));
  }
};

// atan2(y, x) for y >= 0 (the rotation angle from sin >= 0 and cos) in fp32 /
// the packed pair: octant reduction a = min/max in [0, 1], an odd polynomial
// for atan(a) (fit here, max error 5.3e-8 abs evaluated in fp32, ~0.9 ulp at
// pi/4), then pi/2 - . and pi - . by selects -- all packed math for v2f,
// where OCML's atan2f ran once per half with its special-case handling.
#ifndef IKG_FAST_ATAN2
#define IKG_FAST_ATAN2 1
#endif
template <typename T>
IKG_HD inline T atan2_upper(T y, T x) {
  const T ax = fabs(x);
  const T mn = fmin(ax, y), mx = fmax(ax, y);
  const T a = fdiv<T>(mn, fmax(mx, T(1e-30f)));
  const T t = a * a;
  T u = T(0.0026226534973829985f);
  u = u * t + T(-0.015134125016629696f);
  u = u * t + T(0.0411243662238121f);
  u = u * t + T(-0.07366912066936493f);
  u = u * t + T(0.1057402640581131f);
  u = u * t + T(-0.1418599784374237f);
  u = u * t + T(0.19990399479866028f);
  u = u * t + T(-0.3333298861980438f);
  T r = a + (a * t) * u;
  r = vsel<T>(y > ax, T(1.57079637f) - r, r);
  return vsel<T>(x < T(0), T(3.14159274f) - r, r);
}

template <typename T>
IKG_HD inline void log6_iter(const T* R, const T* p, T* e, ThetaTrack<T>* tk = nullptr, bool resync = true) {
  using M = typename LaneT<T>::M;
  const T pi = T(Prec<T>::kPi);
  const T tr = R[0] + R[4] + R[8];
  const T sx = R[7] - R[5], sy = R[2] - R[6], sz = R[3] - R[1];
  const T ct = (tr - T(1)) * T(0.5);
  const T st = fsqrt_unit(sx * sx + sy * sy + sz * sz) * T(0.5);
  T theta = T(0);
  if constexpr (is_f64<T>) {
    bool exact = true;
    if (tk && !resync) {
      const T y = st * tk->ct - ct * tk->st;  // rho sin(theta - theta_prev)
      const T x = ct * tk->ct + st * tk->st;  // rho cos(theta - theta_prev)
#if IKG_THETA_ASIN
      // rho = |(st, ct)| |(st', ct')| = 1 up to the rotations' rounding (~1e-15),
      // so delta = asin(y) to that relative accuracy: a division-free series
      exact = !(fabs(y) <= ThetaInc<T>::kIncAsin && x > T(0));
      theta = tk->th + ThetaInc<T>::asin_small(y);
#else
      exact = !(fabs(y) <= ThetaInc<T>::kInc * x);
      theta = tk->th + ThetaInc<T>::atan_small(fdiv<T>(y, fmax(x, T(1e-30))));
#endif
    }
    if (wave_any<T>(exact)) {
#if IKG_THETA == 1
      const T th_x = atan2(st, ct);
#else
      const T th_x = acos(fmin(fmax(ct, T(-1)), T(1)));  // pin.log3: tr > 3 -> 0, tr < -1 -> pi
#endif
      theta = exact ? th_x : theta;
    }
    if (tk) {
      tk->th = theta;
      tk->st = st;
      tk->ct = ct;
    }
  } else {
#if IKG_FAST_ATAN2
    theta = atan2_upper(st, ct);  // fp32: accurate near 0 where acos is not
#else
    theta = atan2f(st, ct);
#endif
  }
  const T t2 = theta * theta;
  const T tiny = is_f64<T> ? T(1e-300) : T(1e-30f);
  const M above = theta > T(Prec<T>::kPrec3);
  const M below = theta < T(Prec<T>::kPrec3);
  // one reciprocal serves theta/sin(theta) and 1/theta^2: q = 1/(theta^2 sin)
  const T q = frcp<T>(fmax(t2 * st, tiny));
  const T inv_t2 = st * q;
  T f;
  if constexpr (is_f64<T>)
    f = vsel<T>(above, theta * t2 * q, T(1));  // Pinocchio: theta/sin(theta) -> 1 below precision<3>()
  else
    f = vsel<T>(above, theta * t2 * q, T(1) + t2 * (T(1.f / 6) + t2 * T(7.f / 360)));
  const T hf = f * T(0.5);
  T w[3] = {hf * sx, hf * sy, hf * sz};
  // alpha = theta sin/(2(1-cos)) = theta (1+cos)/(2 sin): the second form has no
  // cancellation below the near-pi band (there |1+cos| >= 5e-5: < 2e-14 abs.)
  T alpha = hf * (T(1) + ct);
  const M near_pi = theta >= pi - T(1e-2);
  if (wave_any<T>(any_of(near_pi))) {  // near pi (rare): the axis from the diagonal
    const T beta = fdiv<T>(t2, T(1) - ct);
    const T t0 = (R[0] - ct) * beta, t1 = (R[4] - ct) * beta, tt = (R[8] - ct) * beta;
    const T wp0 = vsel<T>(R[7] > R[5], T(1), T(-1)) * vsel<T>(t0 > T(0), sqrt(t0), T(0));
    const T wp1 = vsel<T>(R[2] > R[6], T(1), T(-1)) * vsel<T>(t1 > T(0), sqrt(t1), T(0));
    const T wp2 = vsel<T>(R[3] > R[1], T(1), T(-1)) * vsel<T>(tt > T(0), sqrt(tt), T(0));
    w[0] = vsel<T>(near_pi, wp0, w[0]);
    w[1] = vsel<T>(near_pi, wp1, w[1]);
    w[2] = vsel<T>(near_pi, wp2, w[2]);
    alpha = vsel<T>(near_pi, fdiv<T>(theta * st, T(2) * (T(1) - ct)), alpha);
  }
  T beta;
  if constexpr (is_f64<T>) {
#if IKG_LOG6_SERIES
#if IKG_TAYLOR_MUL
    // Pinocchio's series terms t2/12, t2^2/720 as products with the rounded
    // reciprocals (<= 1 ulp of each term; the branch serves theta < 1.2e-4):
    // three IEEE divisions (~11 instructions each) leave the loop
    const T as = T(1) - t2 * T(1.0 / 12) - (t2 * t2) * T(1.0 / 720);
    const T bs = T(1.0 / 12) + t2 * T(1.0 / 720);
#else
    const T as = T(1) - t2 / T(12) - t2 * t2 / T(720);
    const T bs = T(1) / T(12) + t2 / T(720);
#endif
    beta = vsel<T>(below, bs, (T(1) - alpha) * inv_t2);
    alpha = vsel<T>(below, as, alpha);
#else
    // no series branch: theta (1 + cos)/(2 sin) has no cancellation at small
    // theta, and (1 - alpha)/theta^2's cancellation error (eps/theta^2) reaches
    // v only through beta (w.p) w with |w|^2 = theta^2: ~eps |p| absolute
    (void)below;
    beta = (T(1) - alpha) * inv_t2;
#endif
  } else {
    const T as = T(1) - t2 * (T(1.f / 12) + t2 * (T(1.f / 720) + t2 * T(1.f / 30240)));
    const T bs = T(1.f / 12) + t2 * (T(1.f / 720) + t2 * (T(1.f / 30240) + t2 * T(1.f / 1209600)));
    beta = vsel<T>(below, bs, (T(1) - alpha) * inv_t2);
    alpha = vsel<T>(below, as, alpha);
  }
  const T wp = w[0] * p[0] + w[1] * p[1] + w[2] * p[2];
  const T bwp = beta * wp;
  e[0] = alpha * p[0] - T(0.5) * (w[1] * p[2] - w[2] * p[1]) + bwp * w[0];
  e[1] = alpha * p[1] - T(0.5) * (w[2] * p[0] - w[0] * p[2]) + bwp * w[1];
  e[2] = alpha * p[2] - T(0.5) * (w[0] * p[1] - w[1] * p[0]) + bwp * w[2];
  e[3] = w[0];
  e[4] = w[1];
  e[5] = w[2];
}

// ---------------------------------------------------------------- joint trigonometry
// sin/cos of every supporting joint are carried across iterations: after an
// update q -> q + d the pair is advanced by the angle-addition formula with
// Taylor series of sin d / cos d (|d| <= kIncMax keeps the truncation below
// 1e-18 in fp64), and recomputed exactly every kResync iterations, after a
// large step, or after a clamp.  This replaces 7 sincos calls per lane and
// iteration of pin.framesForwardKinematics (inverse_geometry.py:58).
template <typename T>
struct Trig;
#ifndef IKG_RESYNC64
#define IKG_RESYNC64 128
#endif
// the chest-frame path's trig rule (generic models, the damped solve, the
// collision continuation's chest-frame loop): 2 = the longer series for every
// step up to kIncMed (the tilted robot's trajectories take steps beyond the
// short series' range on ~70% of updates, and a divergent exact / series split
// cost 1.8-2.0 ms against 1.74 at B = 4,096, profiles/r05/generic/); 1 = the
// frame-1 path's medium-range rule; 0 = the short series or the exact sincos
#ifndef IKG_GENERIC_MED
#define IKG_GENERIC_MED 2
#endif
template <>
struct Trig<double> {
  // |d| <= 0.025: the dropped terms d^9/9! and d^8/8! are < 1e-18 relative.
  // Measured steps (uniform sampler, oracle): max 0.0212, 99.99% < 0.02.
  static constexpr double kIncMax = 0.025;
  // |d| <= 0.25 for step_med: the first dropped terms d^15/15!, d^16/16! < 1e-21
  static constexpr double kIncMed = 0.25;
  static constexpr int kResync = IKG_RESYNC64;
  IKG_HD static inline void step_med(double d, double& s, double& c) {
    const double d2 = d * d;
    const double sd =
        d + d * d2 *
                (-1.0 / 6 +
                 d2 * (1.0 / 120 +
                       d2 * (-1.0 / 5040 + d2 * (1.0 / 362880 + d2 * (-1.0 / 39916800 + d2 * (1.0 / 6227020800.0))))));
    const double cd =
        1.0 + d2 * (-0.5 + d2 * (1.0 / 24 +
                                 d2 * (-1.0 / 720 +
                                       d2 * (1.0 / 40320 + d2 * (-1.0 / 3628800 +
                                                                 d2 * (1.0 / 479001600 + d2 * (-1.0 / 87178291200.0)))))));
    const double sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
  IKG_HD static inline void step(double d, double& s, double& c) {
    const double d2 = d * d;
    const double sd = d + d * d2 * (-1.0 / 6 + d2 * (1.0 / 120 + d2 * (-1.0 / 5040)));
    const double cd = 1.0 + d2 * (-0.5 + d2 * (1.0 / 24 + d2 * (-1.0 / 720)));
    const double sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
};
template <>
struct Trig<float> {
  static constexpr float kIncMax = 0.1f;
  static constexpr float kIncMed = 0.5f;  // d^11/11!, d^12/12! < 2e-11 for step_med
  static constexpr int kResync = 16;
  IKG_HD static inline void step_med(float d, float& s, float& c) {
    const float d2 = d * d;
    const float sd = d + d * d2 * (-1.0f / 6 + d2 * (1.0f / 120 + d2 * (-1.0f / 5040 + d2 * (1.0f / 362880))));
    const float cd = 1.0f + d2 * (-0.5f + d2 * (1.0f / 24 + d2 * (-1.0f / 720 + d2 * (1.0f / 40320 + d2 * (-1.0f / 3628800)))));
    const float sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
  IKG_HD static inline void step(float d, float& s, float& c) {
    const float d2 = d * d;
    const float sd = d + d * d2 * (-1.0f / 6 + d2 * (1.0f / 120 + d2 * (-1.0f / 5040)));
    const float cd = 1.0f + d2 * (-0.5f + d2 * (1.0f / 24 + d2 * (-1.0f / 720)));
    const float sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
};
template <>
struct Trig<v2f> {
  static constexpr float kIncMax = Trig<float>::kIncMax;
  static constexpr float kIncMed = Trig<float>::kIncMed;
  static constexpr int kResync = Trig<float>::kResync;
  IKG_HD static inline void step_med(v2f d, v2f& s, v2f& c) {
    const v2f d2 = d * d;
    const v2f sd = d + d * d2 * (-1.0f / 6 + d2 * (1.0f / 120 + d2 * (-1.0f / 5040 + d2 * (1.0f / 362880))));
    const v2f cd = 1.0f + d2 * (-0.5f + d2 * (1.0f / 24 + d2 * (-1.0f / 720 + d2 * (1.0f / 40320 + d2 * (-1.0f / 3628800)))));
    const v2f sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
  IKG_HD static inline void step(v2f d, v2f& s, v2f& c) {
    const v2f d2 = d * d;
    const v2f sd = d + d * d2 * (-1.0f / 6 + d2 * (1.0f / 120 + d2 * (-1.0f / 5040)));
    const v2f cd = 1.0f + d2 * (-0.5f + d2 * (1.0f / 24 + d2 * (-1.0f / 720)));
    const v2f sn = s * cd + c * sd;
    c = c * cd - s * sd;
    s = sn;
  }
};

// ---------------------------------------------------------------- one arm's kinematics
template <int AX, typename T>
IKG_HD inline void rotate_ax(T* R, int runtime_axis, T s, T c) {
  if constexpr (AX == kAxRuntime)
    rotate_axis(R, runtime_axis, s, c);
  else
    rotate_axis(R, AX, s, c);
}

template <int AX, typename T>
IKG_HD inline void column_ax(const T* R, int runtime_axis, T* a) {
  if constexpr (AX == kAxRuntime)
    column(R, runtime_axis, a);
  else
    column(R, AX, a);
}

// Frame of the shared root joint after its rotation: Rc = root_R Rot(q_root),
// tc = root_t (the "chest frame"; setup_pinocchio.py:32 folds ROBOT_PLACEMENT
// into root_t).
template <typename T, class SP>
IKG_HD inline void root_frame(const KModel<typename LaneT<T>::E>* __restrict__ m, T s0, T c0, T* Rc, T* tc) {
  if constexpr (SP::prot) {
#pragma unroll
    for (int i = 0; i < 9; ++i) Rc[i] = m->root_R[i];
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) Rc[i] = (i % 4 == 0) ? T(1) : T(0);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) tc[i] = m->root_t[i];
  rotate_ax<SP::axis(0)>(Rc, m->root_axis, s0, c0);
}

// Forward kinematics of one arm (pin.forwardKinematics restricted to the
// hand's support, inverse_geometry.py:58) from the root frame (R0, t0) given
// the arm joints' (sin, cos) (slots 1..6; slot 0 = root, already in R0),
// producing
//   Rh, th  : effector frame placement (data.oMf[LARM/RARM_EFF], :62-63)
//   ax, org : axis / origin of the 7 supporting joints (root first)
//   frames  : (WANT_FRAMES) frame [R|t] of every supporting joint, stored at
//             its q index (the root only by the left lane); collision check
// in the coordinates of (R0, t0).  With (R0, t0) = (I, 0) everything is in the
// chest frame: the root rotation and the arm's zero placement components fold
// away at compile time (Spec).
template <typename T, class SP, bool WANT_AXES, bool WANT_FRAMES = false>
IKG_HD inline void fk_arm(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* R0, const T* t0, const T* sn,
                          const T* cs, T* Rh, T* th, T (*ax)[3], T (*org)[3], T (*frames)[12] = nullptr) {
  T R[9], t[3];
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = R0[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = t0[i];
  if constexpr (WANT_AXES) {
    column_ax<SP::axis(0)>(R, m->root_axis, ax[0]);
#pragma unroll
    for (int i = 0; i < 3; ++i) org[0][i] = t[i];
  }
  const bool right = arm != 0;
  if constexpr (WANT_FRAMES) {
    if (!right) {
      T* F = frames[m->root_q];
#pragma unroll
      for (int i = 0; i < 9; ++i) F[i] = R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) F[9 + i] = t[i];
    }
  }
  // hand rotation folded into the last joint's angle (not when the joint's own
  // frame is wanted)
  constexpr bool FOLD = SP::fold_hand && !WANT_FRAMES;
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) {
    T pt[3], dt_[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) pt[i] = SP::zero_t(k, i) ? T(0) : armc<T>(right, m->arm_t[0][k][i], m->arm_t[1][k][i]);
    matvec3(R, pt, dt_);
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] += dt_[i];
    if constexpr (SP::prot) {
      if (m->rot_mask & (1 << k)) {
        T P[9], Rn[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) P[i] = armc<T>(right, m->arm_R[0][k][i], m->arm_R[1][k][i]);
        matmul3(R, P, Rn);
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = Rn[i];
      }
    }
    switch (k) {  // unrolled: k is a compile-time constant after #pragma unroll
      case 0: rotate_ax<SP::axis(1)>(R, m->arm_axis[0], sn[1], cs[1]); break;
      case 1: rotate_ax<SP::axis(2)>(R, m->arm_axis[1], sn[2], cs[2]); break;
      case 2: rotate_ax<SP::axis(3)>(R, m->arm_axis[2], sn[3], cs[3]); break;
      case 3: rotate_ax<SP::axis(4)>(R, m->arm_axis[3], sn[4], cs[4]); break;
      case 4: rotate_ax<SP::axis(5)>(R, m->arm_axis[4], sn[5], cs[5]); break;
      default:
        if constexpr (FOLD) {
          // Rot(q5) Rot(h) = Rot(q5 + h): (sin, cos) by angle addition
          const T hs = armc<T>(right, m->hand_sc[0][0], m->hand_sc[1][0]);
          const T hc = armc<T>(right, m->hand_sc[0][1], m->hand_sc[1][1]);
          rotate_axis(R, SP::axis(6), sn[6] * hc + cs[6] * hs, cs[6] * hc - sn[6] * hs);
        } else {
          rotate_ax<SP::axis(6)>(R, m->arm_axis[5], sn[6], cs[6]);
        }
        break;
    }
    if constexpr (WANT_AXES) {  // a rotation about an axis leaves that column unchanged (FOLD)
      switch (k) {
        case 0: column_ax<SP::axis(1)>(R, m->arm_axis[0], ax[1]); break;
        case 1: column_ax<SP::axis(2)>(R, m->arm_axis[1], ax[2]); break;
        case 2: column_ax<SP::axis(3)>(R, m->arm_axis[2], ax[3]); break;
        case 3: column_ax<SP::axis(4)>(R, m->arm_axis[3], ax[4]); break;
        case 4: column_ax<SP::axis(5)>(R, m->arm_axis[4], ax[5]); break;
        default: column_ax<SP::axis(6)>(R, m->arm_axis[5], ax[6]); break;
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) org[k + 1][i] = t[i];
    }
    if constexpr (WANT_FRAMES) {
      T* F = frames[right ? m->arm_q[1][k] : m->arm_q[0][k]];
#pragma unroll
      for (int i = 0; i < 9; ++i) F[i] = R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) F[9 + i] = t[i];
    }
  }
  T ht[3], d[3];
  if constexpr (FOLD) {
    // R is already the hand rotation: th = t + R6 ht = t + Rh (hand_R^T ht)
#pragma unroll
    for (int i = 0; i < 3; ++i) ht[i] = armc<T>(right, m->hand_tH[0][i], m->hand_tH[1][i]);
    matvec3(R, ht, d);
#pragma unroll
    for (int i = 0; i < 3; ++i) th[i] = t[i] + d[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) Rh[i] = R[i];
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) ht[i] = armc<T>(right, m->hand_t[0][i], m->hand_t[1][i]);
    matvec3(R, ht, d);
#pragma unroll
    for (int i = 0; i < 3; ++i) th[i] = t[i] + d[i];
    constexpr int HA = SP::axis(7);
    if constexpr (HA != kAxRuntime) {
      // hand placement rotation = R_axis(angle): two columns change
#pragma unroll
      for (int i = 0; i < 9; ++i) Rh[i] = R[i];
      rotate_axis(Rh, HA, armc<T>(right, m->hand_sc[0][0], m->hand_sc[1][0]),
                  armc<T>(right, m->hand_sc[0][1], m->hand_sc[1][1]));
    } else {
      T hR[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) hR[i] = armc<T>(right, m->hand_R[0][i], m->hand_R[1][i]);
      matmul3(R, hR, Rh);
    }
  }
}

// World-frame FK of one arm (batch FK kernel, diagnostics).
template <typename T, class SP>
IKG_HD inline void fk_arm_world(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* sn, const T* cs, T* Rh, T* th) {
  T Rc[9], tc[3];
  root_frame<T, SP>(m, sn[0], cs[0], Rc, tc);
  fk_arm<T, SP, false>(m, arm, Rc, tc, sn, cs, Rh, th, nullptr, nullptr);
}

// log6(oMhand^-1 * oMtarget) (inverse_geometry.py:66-67)
template <typename T>
IKG_HD inline void pose_error(const T* Rh, const T* th, const T* RT, const T* tT, T* e) {
  T Rm[9], d[3], pm[3];
  matmul3_tn(Rh, RT, Rm);
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = tT[i] - th[i];
  matvec3_t(Rh, d, pm);
  if constexpr (IKG_ABL & 2) {
    e[0] = pm[0]; e[1] = pm[1]; e[2] = pm[2];
    e[3] = T(0.5) * (Rm[7] - Rm[5]); e[4] = T(0.5) * (Rm[2] - Rm[6]); e[5] = T(0.5) * (Rm[3] - Rm[1]);
  } else {
    log6(Rm, pm, e);
  }
}

// The same error expressed in the axes of the frame (Rh, th) is given in:
// with Rw = RT Rh^T = Rh Rm Rh^T and d = tT - th = Rh pm, log3(Rw) = Rh log3(Rm)
// and V(w)^-1 commutes with the rotation, so log6(Rw, d) = blockdiag(Rh, Rh)
// log6(Rm, pm): the reference's LOCAL error rotated into the frame's axes (same
// norm, same minimum-norm step).
template <typename T>
IKG_HD inline void pose_error_aligned(const T* Rh, const T* th, const T* RT, const T* tT, T* e,
                                      ThetaTrack<T>* tk = nullptr, bool resync = true) {
  T Rw[9], d[3];
  matmul3_nt(RT, Rh, Rw);
#pragma unroll
  for (int i = 0; i < 3; ++i) d[i] = tT[i] - th[i];
  if constexpr (IKG_ABL & 2) {
    e[0] = d[0]; e[1] = d[1]; e[2] = d[2];
    e[3] = T(0.5) * (Rw[7] - Rw[5]); e[4] = T(0.5) * (Rw[2] - Rw[6]); e[5] = T(0.5) * (Rw[3] - Rw[1]);
  } else {
    log6_iter(Rw, d, e, tk, resync);
  }
}

// ---------------------------------------------------------------- 6x6 solve, 2 RHS
// Householder QR of the square arm Jacobian A[:, 0:6] applied to the two
// right-hand sides A[:, 6] (error) and A[:, 7] (root column); returns
// x = A^-1 b for both.  Diagonal entries below rcond * max|R_kk| are
// truncated to a zero inverse (the analogue of pinv's rcond).
template <typename T>
IKG_HD inline void qr_solve6(T (&A)[6][8], T* x0, T* x1, bool* near_singular = nullptr, T tau = T(0)) {
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    T n2 = T(0);
#pragma unroll
    for (int i = k; i < 6; ++i) n2 += A[i][k] * A[i][k];
    const T nrm = sqrt(n2);
    const T akk = A[k][k];
    const T alpha = akk >= T(0) ? -nrm : nrm;
    const T vk = akk - alpha;
    const T vtv = T(2) * nrm * (nrm + fabs(akk));
    const T scale = vtv > T(0) ? T(2) / vtv : T(0);
#pragma unroll
    for (int j = k + 1; j < 8; ++j) {
      T tau = vk * A[k][j];
#pragma unroll
      for (int i = k + 1; i < 6; ++i) tau += A[i][k] * A[i][j];
      const T f = tau * scale;
      A[k][j] -= f * vk;
#pragma unroll
      for (int i = k + 1; i < 6; ++i) A[i][j] -= f * A[i][k];
    }
    A[k][k] = alpha;
  }
  T dmax = T(0);
#pragma unroll
  for (int k = 0; k < 6; ++k) dmax = fmax(dmax, fabs(A[k][k]));
  const T cut = dmax * Prec<T>::kRcond;
  if (near_singular) {
    T dmin = fabs(A[0][0]);
#pragma unroll
    for (int k = 1; k < 6; ++k) dmin = fmin(dmin, fabs(A[k][k]));
    *near_singular = dmin < tau * dmax;
  }
  T rd[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) rd[k] = fabs(A[k][k]) > cut ? T(1) / A[k][k] : T(0);
#pragma unroll
  for (int r = 5; r >= 0; --r) {
    T s0 = A[r][6], s1 = A[r][7];
#pragma unroll
    for (int j = r + 1; j < 6; ++j) {
      s0 -= A[r][j] * x0[j];
      s1 -= A[r][j] * x1[j];
    }
    x0[r] = s0 * rd[r];
    x1[r] = s1 * rd[r];
  }
}

// Cholesky solve of the damped arm block (J_a J_a^T + lambda I) for 2 RHS.
template <typename T>
IKG_HD inline void chol_solve6(T (&M)[6][6], T* b0, T* b1) {
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    T d = M[k][k];
#pragma unroll
    for (int j = 0; j < k; ++j) d -= M[k][j] * M[k][j];
    const T r = d > T(0) ? T(1) / sqrt(d) : T(0);
    M[k][k] = r;  // store the reciprocal of L_kk
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      T v = M[i][k];
#pragma unroll
      for (int j = 0; j < k; ++j) v -= M[i][j] * M[k][j];
      M[i][k] = v * r;
    }
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      b0[i] -= M[i][j] * b0[j];
      b1[i] -= M[i][j] * b1[j];
    }
    b0[i] *= M[i][i];
    b1[i] *= M[i][i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
#pragma unroll
    for (int j = i + 1; j < 6; ++j) {
      b0[i] -= M[j][i] * b0[j];
      b1[i] -= M[j][i] * b1[j];
    }
    b0[i] *= M[i][i];
    b1[i] *= M[i][i];
  }
}

template <typename T>
IKG_HD inline T clampq(T q, T lo, T hi) {
  // np.minimum(np.maximum(lower, q), upper)  (tools.py:21-22)
  return fmin(fmax(lo, q), hi);
}

// ---------------------------------------------------------------- per-lane iteration stages
// One arm-lane's share of an iteration of inverse_geometry.py:56-89.  The
// kernel composes these with DPP exchanges (ikg_kernels.hip solve_pair);
// tools/host_emu (ikg_host_emu.hip) composes the same functions for both arms
// on the CPU.
template <typename T>
struct ArmState {
  T Rh[9], th[3];         // effector placement, in the iteration's frame (below)
  T ax[7][3], org[7][3];  // axis / origin of root + arm joints, same frame
  T e[6];                 // log6(oMf^-1 oMtarget) rotated into that frame's axes
};

// exact (sin, cos) of the root and arm joints (slot 0 = root)
template <typename T>
IKG_HD inline void trig_exact(T qc, const T* qa, T* sn, T* cs) {
  Prec<T>::sincos_(qc, &sn[0], &cs[0]);
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) Prec<T>::sincos_(qa[k], &sn[k + 1], &cs[k + 1]);
}

// advance (sin, cos) after the update q_old -> (qc, qa); exact when `resync`
// or when any step exceeds the incremental range.  MED: the medium-range rule
// of the frame-1 path (trig_med_f1) -- the longer series for steps up to
// kIncMed, exact beyond and at resyncs.
template <typename T, int MED = 0>
IKG_HD inline void trig_advance(T qc, const T* qa, const T* q_old, bool resync, T* sn, T* cs) {
  T d[7];
  d[0] = qc - q_old[0];
  bool big = resync;
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) d[k + 1] = qa[k] - q_old[k + 1];
  if constexpr (MED == 2) {  // the longer series for every step up to kIncMed: no divergent short/long split
    T dmax = fabs(d[0]);
#pragma unroll
    for (int j = 1; j < 7; ++j) dmax = fmax(dmax, fabs(d[j]));
#pragma unroll
    for (int j = 0; j < 7; ++j) Trig<T>::step_med(d[j], sn[j], cs[j]);
    if (resync || any_of(dmax > T(Trig<T>::kIncMed))) trig_exact(qc, qa, sn, cs);
    return;
  }
  if constexpr (MED == 1) {
    T dmax = fabs(d[0]);
#pragma unroll
    for (int j = 1; j < 7; ++j) dmax = fmax(dmax, fabs(d[j]));
    if (resync || any_of(dmax > T(Trig<T>::kIncMax))) {
      if (!resync && all_of(mnot(dmax > T(Trig<T>::kIncMed)))) {
#pragma unroll
        for (int j = 0; j < 7; ++j) Trig<T>::step_med(d[j], sn[j], cs[j]);
      } else {
        trig_exact(qc, qa, sn, cs);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 7; ++j) Trig<T>::step(d[j], sn[j], cs[j]);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 7; ++j) big |= any_of(fabs(d[j]) > T(Trig<T>::kIncMax));
  if constexpr (IKG_ABL & 1) {  // timing ablation: no incremental trig
#pragma unroll
    for (int j = 0; j < 7; ++j) sn[j] += d[j];
    return;
  }
  if (big) {
    trig_exact(qc, qa, sn, cs);
  } else {
#pragma unroll
    for (int j = 0; j < 7; ++j) Trig<T>::step(d[j], sn[j], cs[j]);
  }
}

// Frame-1 trig slots (kFrame1 models): the sums the frame-1 FK consumes are
// carried directly, so no angle additions run per update:
//   0: q_root + q_0   1: q_0   2: q_1   3: q_1 + q_2   4: q_3   5: q_4
//   6: q_5 + hand angle (the hand rotation about the same axis, fold_hand)
template <typename T>
IKG_HD inline void add_angles(T s1, T c1, T s2, T c2, T& s, T& c) {
  s = s1 * c2 + c1 * s2;
  c = c1 * c2 - s1 * s2;
}

template <typename T>
IKG_HD inline void trig_exact_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, T qc, const T* qa, T* sn,
                                 T* cs) {
  T s[7], c[7];
  trig_exact(qc, qa, s, c);
  const bool right = arm != 0;
  const T hs = armc<T>(right, m->hand_sc[0][0], m->hand_sc[1][0]);
  const T hc = armc<T>(right, m->hand_sc[0][1], m->hand_sc[1][1]);
  add_angles(s[0], c[0], s[1], c[1], sn[0], cs[0]);
  sn[1] = s[1], cs[1] = c[1];
  sn[2] = s[2], cs[2] = c[2];
  add_angles(s[2], c[2], s[3], c[3], sn[3], cs[3]);
  sn[4] = s[4], cs[4] = c[4];
  sn[5] = s[5], cs[5] = c[5];
  add_angles(s[6], c[6], hs, hc, sn[6], cs[6]);
}

// One trig advance with the medium-range rule, per lane: the short series for
// steps within kIncMax, the longer series (kIncMed) for steps up to kIncMed,
// the exact sincos beyond that and at resyncs.
template <typename T>
IKG_HD inline void trig_med_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, T qc, const T* qa,
                               const T* d, bool resync, T* sn, T* cs) {
  T dmax = fabs(d[0]);
#pragma unroll
  for (int j = 1; j < 7; ++j) dmax = fmax(dmax, fabs(d[j]));
  if (resync || any_of(dmax > T(Trig<T>::kIncMax))) {
    // steps beyond the short series' range: first steps from random seeds
    // (multi-start took this path on 14% of its fp64 updates); a longer series
    // covers them up to kIncMed, the exact sincos beyond and at resyncs
    if (!resync && all_of(mnot(dmax > T(Trig<T>::kIncMed)))) {
#pragma unroll
      for (int j = 0; j < 7; ++j) Trig<T>::step_med(d[j], sn[j], cs[j]);
    } else {
      trig_exact_f1(m, arm, qc, qa, sn, cs);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 7; ++j) Trig<T>::step(d[j], sn[j], cs[j]);
  }
}

// MED = true: the medium-range rule (per-problem seeds: large first steps are
// common; random-seed batches 6.46 -> 5.06 ms fp64, 3.08 -> 2.73 ms fp32 at
// 131,072 against the exact fallback).  MED = false (a broadcast q0): the short
// series runs in place and a lane whose step leaves its range (or a resync)
// takes the exact sincos of every slot, in a wave-uniform branch.  The two
// rules differ only on steps of 0.025..0.25 rad, by rounding (C2 from q = 0 has
// none); the medium-range rule inline costs the broadcast kernel 4% fp64 /
// 3.5% fp32 at C2, and the out-of-line form with it 21 register copies per
// update (profiles/r04/trig/).
template <typename T, bool MED = false>
IKG_HD inline void trig_advance_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, T qc, const T* qa,
                                   const T* q_old, bool resync, T* sn, T* cs) {
  T dj[7], d[7];
  dj[0] = qc - q_old[0];
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) dj[k + 1] = qa[k] - q_old[k + 1];
  d[0] = dj[0] + dj[1];
  d[1] = dj[1];
  d[2] = dj[2];
  d[3] = dj[2] + dj[3];
  d[4] = dj[4];
  d[5] = dj[5];
  d[6] = dj[6];
  if constexpr (!MED) {
    bool big = resync;
#pragma unroll
    for (int j = 0; j < 7; ++j) big |= any_of(fabs(d[j]) > T(Trig<T>::kIncMax));
    // the step always runs in place and the exact path overwrites it: the
    // common path then needs no register copies to merge the two
#pragma unroll
    for (int j = 0; j < 7; ++j) Trig<T>::step(d[j], sn[j], cs[j]);
    if (wave_any<T>(big)) {
      T se[7], ce[7];
      trig_exact_f1(m, arm, qc, qa, se, ce);
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        sn[j] = big ? se[j] : sn[j];
        cs[j] = big ? ce[j] : cs[j];
      }
    }
    return;
  }
  trig_med_f1(m, arm, qc, qa, d, resync, sn, cs);
}

// FK + pose error; returns |e|^2 (inverse_geometry.py:58-67; the stop test
// compares it with KParams::eps2).  WORLD = false
// (the IK loop): everything in the chest frame (root_frame) -- the target is
// moved into it (Rc^T RT, Rc^T (tT - tc)) instead of the arm's 7 frames out of
// it.  WORLD = true: world frame (collision continuation, which needs world
// joint frames).  The minimum-norm step is the same in any frame (§3).
template <typename T, class SP, bool WANT_FRAMES = false, bool WORLD = WANT_FRAMES>
IKG_HD inline T arm_fk_error(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* sn, const T* cs, const T* RT,
                             const T* tT, ArmState<T>& st, T (*frames)[12] = nullptr,
                             ThetaTrack<T>* tk = nullptr, bool resync = true) {
  T Rc[9], tc[3];
  root_frame<T, SP>(m, sn[0], cs[0], Rc, tc);
  if constexpr (WORLD) {
    fk_arm<T, SP, true, WANT_FRAMES>(m, arm, Rc, tc, sn, cs, st.Rh, st.th, st.ax, st.org, frames);
    pose_error_aligned(st.Rh, st.th, RT, tT, st.e, tk, resync);
  } else {
    static_assert(!WANT_FRAMES, "joint frames are produced in the world frame");
    const T I3[9] = {T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1)};
    const T Z3[3] = {T(0), T(0), T(0)};
    fk_arm<T, SP, true>(m, arm, I3, Z3, sn, cs, st.Rh, st.th, st.ax, st.org);
    T RTc[9], dT[3], tTc[3];
    matmul3_tn(Rc, RT, RTc);
#pragma unroll
    for (int i = 0; i < 3; ++i) dT[i] = tT[i] - tc[i];
    matvec3_t(Rc, dT, tTc);
    pose_error_aligned(st.Rh, st.th, RTc, tTc, st.e, tk, resync);
  }
  const T* e = st.e;
  return e[0] * e[0] + e[1] * e[1] + e[2] * e[2] + e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
}

// Frame-aligned Jacobian at the hand point, col_j = [a_j x (p_h - o_j); a_j]
// (columns 0..5 = arm joints, 7 = root) and the aligned error (column 6).
// LOCAL = blockdiag(Rh^T, Rh^T) * aligned (:75-76), and the rotation is
// orthogonal, so the minimum-norm step is unchanged.
template <typename T>
IKG_HD inline void arm_system(const ArmState<T>& st, T (&A)[6][8]) {
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int col = j == 0 ? 7 : j - 1;
    const T dx = st.th[0] - st.org[j][0], dy = st.th[1] - st.org[j][1], dz = st.th[2] - st.org[j][2];
    A[0][col] = st.ax[j][1] * dz - st.ax[j][2] * dy;
    A[1][col] = st.ax[j][2] * dx - st.ax[j][0] * dz;
    A[2][col] = st.ax[j][0] * dy - st.ax[j][1] * dx;
    A[3][col] = st.ax[j][0];
    A[4][col] = st.ax[j][1];
    A[5][col] = st.ax[j][2];
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) A[r][6] = st.e[r];
}

template <typename T>
IKG_HD inline void cross3(const T* a, const T* b, T* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

template <typename T>
IKG_HD inline T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// [g1 g2 g3]^-1 applied to b0 and b1 by the adjugate (Cramer); an exactly
// singular block gives a zero inverse (pinv truncates only below 1e-15 sigma_max).
template <typename T>
IKG_HD inline void inv3_apply2(const T* g1, const T* g2, const T* g3, const T* b0, const T* b1, T* x0, T* x1,
                               T* det_out = nullptr) {
  T r1[3], r2[3], r3[3];
  cross3(g2, g3, r1);
  cross3(g3, g1, r2);
  cross3(g1, g2, r3);
  const T det = dot3(g1, r1);
  if (det_out) *det_out = det;
  const T rdet = vsel<T>(det != T(0), frcp(det), T(0));
  x0[0] = dot3(r1, b0) * rdet;
  x0[1] = dot3(r2, b0) * rdet;
  x0[2] = dot3(r3, b0) * rdet;
  x1[0] = dot3(r1, b1) * rdet;
  x1[1] = dot3(r2, b1) * rdet;
  x1[2] = dot3(r3, b1) * rdet;
}

// Spherical wrist (axes of arm joints 3,4,5 through w = origin of arm joint 4):
// written at w the square arm Jacobian is block lower-triangular,
//   [ G  0 ] with G = [a_j x (w - o_j)]_{j=0..2},  H = [a_j]_{j=3..5},
//   [ F  H ]      F = [a_j]_{j=0..2},
// so J_a^-1 [e c] needs two 3x3 solves.  Rows are moved from the hand point h
// to w by v_w = v_h + w_ang x (w - h) (an invertible row operation: same u, v).
template <typename T>
IKG_HD inline void arm_solve_wrist(const ArmState<T>& st, T* u, T* v, typename LaneT<T>::M* near_singular = nullptr,
                                   T tau = T(0)) {
  const T* w = st.org[5];
  const T* ev = st.e;
  const T* ew = st.e + 3;
  T bl[3], wh[3], tmp[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) wh[i] = w[i] - st.th[i];
  cross3(ew, wh, tmp);
#pragma unroll
  for (int i = 0; i < 3; ++i) bl[i] = ev[i] + tmp[i];
  T g[3][3], cl[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    T ow[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) ow[i] = w[i] - st.org[j + 1][i];
    cross3(st.ax[j + 1], ow, g[j]);
  }
  {
    T ow[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) ow[i] = w[i] - st.org[0][i];
    cross3(st.ax[0], ow, cl);
  }
  T dG, dH;
  inv3_apply2(g[0], g[1], g[2], bl, cl, u, v, &dG);
  T re[3], rcv[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    re[i] = ew[i] - (u[0] * st.ax[1][i] + u[1] * st.ax[2][i] + u[2] * st.ax[3][i]);
    rcv[i] = st.ax[0][i] - (v[0] * st.ax[1][i] + v[1] * st.ax[2][i] + v[2] * st.ax[3][i]);
  }
  inv3_apply2(st.ax[4], st.ax[5], st.ax[6], re, rcv, u + 3, v + 3, &dH);
  if (near_singular) {  // |det| against the product of the row norms (H: unit axes)
    const T ng = dot3(g[0], g[0]) * dot3(g[1], g[1]) * dot3(g[2], g[2]);
    *near_singular = mor(dG * dG < tau * tau * ng, fabs(dH) < tau);
  }
}

// lambda = 0: u = J_a^-1 e_a, v = J_a^-1 c_a; alpha = u.v, beta = v.v.
template <typename T, class SP>
IKG_HD inline void arm_solve(const ArmState<T>& st, T* u, T* v, T& alpha, T& beta,
                             typename LaneT<T>::M* near_singular = nullptr, T tau = T(0)) {
  if constexpr (IKG_ABL & 4) {
    for (int k = 0; k < 6; ++k) { u[k] = st.e[k] + st.org[k][0]; v[k] = st.ax[k][1]; }
  } else if constexpr (SP::wrist) {
    arm_solve_wrist(st, u, v, near_singular, tau);
  } else {
    static_assert(!is_packed<T>, "the generic QR solve runs in the pair layout");
    T A[6][8];
    arm_system(st, A);
    qr_solve6(A, u, v, near_singular, tau);
  }
  alpha = T(0);
  beta = T(0);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    alpha += u[k] * v[k];
    beta += v[k] * v[k];
  }
}

// ---------------------------------------------------------------- frame-1 closed form
// For the Nextage joint pattern (root Z; arm Z | Y Y | X Y Z; no placement
// rotations; hand rotation about the last axis; spherical wrist at the origin
// w of arm joint 4, ikg_model_build.hpp) the iteration runs in "frame 1": the
// frame of arm joint 0 after its rotation.  There the arm's axes are constant
// or nearly so,
//   a_0 = e_z, a_1 = a_2 = e_y (o_0 = 0, o_1 = p_1),
//   [a_3 a_4 a_5] = Ry(q1 + q2) [e_x, Rx(q3) e_y, Rx(q3) Ry(q4) e_z],
// so the wrist-decoupled solve of arm_solve_wrist,
//   G x_top = b_lin(w),  H x_bot = b_ang - F x_top,
//   G = [a_j x (w - o_j)]_{j<3}, F = [a_j]_{j<3}, H = [a_j]_{j>=3},
// has closed forms: G = [(-w_y, w_x, 0), (P1z, 0, -P1x), (P2z, 0, -P2x)] with
// P_j = w - o_j (one scalar row, then a 2x2), and H = Ry(q12) H'' with
// H'' = [[1, 0, s4], [0, c3, -s3 c4], [0, s3, c3 c4]] (a rotation, then 1/c4).
// The arm joint 0 and root rotations are both about z, so the target is moved
// into frame 1 by Rz(q_root + q_0)^T.  Same minimum-norm step as the chest-frame
// path (pinv(J) e is invariant to the frame J and e are written in, and the
// joint-space u, v are the same): ~100 fewer fp64 operations per update.
template <class SP>
constexpr bool kFrame1 = IKG_FRAME1 && SP::axis(0) == 2 && SP::axis(1) == 2 && SP::axis(2) == 1 &&
                         SP::axis(3) == 1 && SP::axis(4) == 0 && SP::axis(5) == 1 && SP::axis(6) == 2 &&
                         !SP::prot && SP::wrist && SP::fold_hand;

template <typename T>
struct ArmStateF1 {
  T w[3];      // wrist centre = origin of arm joint 4
  T o2[3];     // origin of arm joint 2
  T c12, s12;  // rotation after arm joint 2: Ry(q1 + q2)
  T k[2];      // (x, y) of Rz(q0)^T p_0: the root joint sits at -(k, p_0z)
  T h[3];      // hand point
  T e[6];      // pose error in frame-1 axes
};

// FK in frame 1 (the configuration-only half of arm_fk_error_f1): st.k,
// st.o2, st.c12/s12, st.w, st.h and the hand rotation Rh.
// sn/cs slots: 0 root, 1..6 arm joints 0..5.
template <typename T, class SP>
IKG_HD inline void fk_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* sn, const T* cs,
                         ArmStateF1<T>& st, T* R) {
  static_assert(kFrame1<SP>, "frame-1 path needs the Nextage joint pattern");
  const bool right = arm != 0;
  T p0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) p0[i] = SP::zero_t(0, i) ? T(0) : armc<T>(right, m->arm_t[0][0][i], m->arm_t[1][0][i]);
  st.k[0] = cs[1] * p0[0] + sn[1] * p0[1];
  st.k[1] = cs[1] * p0[1] - sn[1] * p0[0];
  // FK from arm joint 1 (R = I, origin of joint 0 at 0)
#pragma unroll
  for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? T(1) : T(0);
  T t[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = SP::zero_t(1, i) ? T(0) : armc<T>(right, m->arm_t[0][1][i], m->arm_t[1][1][i]);
  auto offset = [&](int k) {
    T pt[3], d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) pt[i] = SP::zero_t(k, i) ? T(0) : armc<T>(right, m->arm_t[0][k][i], m->arm_t[1][k][i]);
    matvec3(R, pt, d);
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] += d[i];
  };
  rotate_axis(R, 1, sn[2], cs[2]);  // arm joint 1 (Y)
  offset(2);
#pragma unroll
  for (int i = 0; i < 3; ++i) st.o2[i] = t[i];
  // arm joint 2 (Y): R = Ry(q1 + q2) from its carried (sin, cos)
  st.c12 = cs[3];
  st.s12 = sn[3];
  R[0] = st.c12, R[2] = st.s12, R[6] = -st.s12, R[8] = st.c12;
  offset(3);
  rotate_axis(R, 0, sn[4], cs[4]);  // arm joint 3 (X)
  offset(4);
#pragma unroll
  for (int i = 0; i < 3; ++i) st.w[i] = t[i];
  rotate_axis(R, 1, sn[5], cs[5]);  // arm joint 4 (Y)
  offset(5);
  rotate_axis(R, 2, sn[6], cs[6]);  // arm joint 5 (Z) + the hand rotation (slot 6)
  T ht[3], d[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) ht[i] = armc<T>(right, m->hand_tH[0][i], m->hand_tH[1][i]);
  matvec3(R, ht, d);
#pragma unroll
  for (int i = 0; i < 3; ++i) st.h[i] = t[i] + d[i];
}

// The pose error of frame-1 FK (the target-dependent half): the target moved
// into frame 1 = chest Rz(q_root) at root_t, then arm joint 0 at p_0 with
// Rz(q_0) (trig slots as trig_exact_f1), then log6 in the frame's axes;
// st.e and the return value |e|^2.
template <typename T, class SP>
IKG_HD inline T pose_error_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* sn, const T* cs,
                              const T* RT, const T* tT, ArmStateF1<T>& st, const T* R, ThetaTrack<T>* tk,
                              bool resync) {
  const bool right = arm != 0;
  const T sf = sn[0], cf = cs[0];
  const T p0z = SP::zero_t(0, 2) ? T(0) : armc<T>(right, m->arm_t[0][0][2], m->arm_t[1][0][2]);
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
  tT1[2] = tT[2] - m->root_t[2] - p0z;
  pose_error_aligned(R, st.h, RT1, tT1, st.e, tk, resync);
  const T* e = st.e;
  return e[0] * e[0] + e[1] * e[1] + e[2] * e[2] + e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
}

// FK + pose error in frame 1 (inverse_geometry.py:58-67); returns |e|^2.
template <typename T, class SP>
IKG_HD inline T arm_fk_error_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const T* sn, const T* cs,
                                const T* RT, const T* tT, ArmStateF1<T>& st, ThetaTrack<T>* tk, bool resync) {
  T R[9];
  fk_f1<T, SP>(m, arm, sn, cs, st, R);
  return pose_error_f1<T, SP>(m, arm, sn, cs, RT, tT, st, R, tk, resync);
}

// u = J_a^-1 e_a, v = J_a^-1 c_a in closed form (see above); alpha = u.v,
// beta = v.v.  An exactly singular block gives a zero inverse, as in
// inv3_apply2.  Split in the configuration-only half (arm_solve_f1_v: the
// inverses' scalars, v and beta) and the error half (arm_solve_f1_u: u and
// alpha); the halves were split for a two-wave layout, measured slower.
template <typename T>
struct SolveF1V {
  T iP0, iD, rH, c4r;  // 1/P0-type scalars of G^-1 and 1/c4 of H''^-1
  T v[6];              // J_a^-1 c_a
  T beta;              // |v|^2
};

template <typename T, class SP>
IKG_HD inline void arm_solve_f1_v(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm,
                                  const ArmStateF1<T>& st, const T* sn, const T* cs, SolveF1V<T>& sv) {
  const bool right = arm != 0;
  const T* w = st.w;
  // G: P0 = w, P1 = w - p_1, P2 = w - o_2
  T P1[3], P2[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    P1[i] = SP::zero_t(1, i) ? w[i] : w[i] - armc<T>(right, m->arm_t[0][1][i], m->arm_t[1][1][i]);
    P2[i] = w[i] - st.o2[i];
  }
  const T det2 = P1[0] * P2[2] - P1[2] * P2[0];
  const T dG = w[0] * det2;
  // an exactly singular block gives inf / NaN here; the guard (pinv_step_f1,
  // on the bits of |v|^2) sends it to the per-arm pinv form
  const T rG = frcp(dG);
  sv.iP0 = det2 * rG;
  sv.iD = w[0] * rG;
  T* v = sv.v;
  {  // root column at w: e_z x (w + (k, .)) = (-(w_y + k_y), w_x + k_x, 0)
    v[0] = (w[0] + st.k[0]) * sv.iP0;
    const T r0 = w[1] * v[0] - (w[1] + st.k[1]);
    v[1] = -P2[0] * r0 * sv.iD;
    v[2] = P1[0] * r0 * sv.iD;
  }
  // H = Ry(q12) H''; slots 4, 5 = arm joints 3, 4
  const T s3 = sn[4], c3 = cs[4], s4 = sn[5], c4 = cs[5];
  sv.rH = frcp(c4);
  sv.c4r = c4 * sv.rH;
  const T c12 = st.c12, s12 = st.s12;
  {  // root column: z = Ry(q12)^T (e_z - (0, v1 + v2, v0))
    const T z1 = -(v[1] + v[2]), z2 = T(1) - v[0];
    const T y0 = -s12 * z2, y2 = c12 * z2;
    v[5] = (c3 * y2 - s3 * z1) * sv.rH;
    v[4] = (c3 * z1 + s3 * y2) * sv.c4r;
    v[3] = y0 - s4 * v[5];
  }
  sv.beta = T(0);
#pragma unroll
  for (int k = 0; k < 6; ++k) sv.beta += v[k] * v[k];
}

template <typename T, class SP>
IKG_HD inline void arm_solve_f1_u(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm,
                                  const ArmStateF1<T>& st, const T* sn, const T* cs, const SolveF1V<T>& sv, T* u,
                                  T& alpha) {
  const bool right = arm != 0;
  const T* w = st.w;
  const T* ev = st.e;
  const T* ew = st.e + 3;
  // linear rows moved from the hand point to w
  T wh[3], cr[3], bl[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) wh[i] = w[i] - st.h[i];
  cross3(ew, wh, cr);
#pragma unroll
  for (int i = 0; i < 3; ++i) bl[i] = ev[i] + cr[i];
  T P1[3], P2[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    P1[i] = SP::zero_t(1, i) ? w[i] : w[i] - armc<T>(right, m->arm_t[0][1][i], m->arm_t[1][1][i]);
    P2[i] = w[i] - st.o2[i];
  }
  {
    u[0] = bl[1] * sv.iP0;
    const T r0 = bl[0] + w[1] * u[0];
    u[1] = -(P2[0] * r0 + P2[2] * bl[2]) * sv.iD;
    u[2] = (P1[2] * bl[2] + P1[0] * r0) * sv.iD;
  }
  const T s3 = sn[4], c3 = cs[4], s4 = sn[5];
  const T c12 = st.c12, s12 = st.s12;
  {  // e: z = Ry(q12)^T (e_w - (0, x1 + x2, x0))
    const T z0 = ew[0], z1 = ew[1] - (u[1] + u[2]), z2 = ew[2] - u[0];
    const T y0 = c12 * z0 - s12 * z2, y2 = s12 * z0 + c12 * z2;
    u[5] = (c3 * y2 - s3 * z1) * sv.rH;
    u[4] = (c3 * z1 + s3 * y2) * sv.c4r;
    u[3] = y0 - s4 * u[5];
  }
  alpha = T(0);
#pragma unroll
  for (int k = 0; k < 6; ++k) alpha += u[k] * sv.v[k];
}

template <typename T, class SP>
IKG_HD inline void arm_solve_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const ArmStateF1<T>& st,
                                const T* sn, const T* cs, T* u, T* v, T& alpha, T& beta) {
  SolveF1V<T> sv;
  arm_solve_f1_v<T, SP>(m, arm, st, sn, cs, sv);
  arm_solve_f1_u<T, SP>(m, arm, st, sn, cs, sv, u, alpha);
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] = sv.v[k];
  beta = sv.beta;
}

// The guard's test: x beyond the bound, or inf / NaN (compared as unsigned
// bits, which -ffinite-math-only cannot fold away; x >= 0 or NaN here).
IKG_HD inline bool beyond(double x, double b) {
  return __builtin_bit_cast(uint64_t, x) > __builtin_bit_cast(uint64_t, b);
}
IKG_HD inline bool beyond(float x, float b) {
  return __builtin_bit_cast(uint32_t, x) > __builtin_bit_cast(uint32_t, b);
}
IKG_HD inline v2i beyond(v2f x, float b) { return v2i{beyond(x.x, b) ? -1 : 0, beyond(x.y, b) ? -1 : 0}; }
// The guard over this lane's and the partner arm's |v|^2.  A packed lane
// holds both arms, so the partner's is its own other half: one unsigned max and
// one compare instead of two masked 2-vectors (round 4: 10 fewer VALU per update).
IKG_HD inline bool guard_test(double x, double xo, double b) { return beyond(x, b) || beyond(xo, b); }
IKG_HD inline bool guard_test(float x, float xo, float b) { return beyond(x, b) || beyond(xo, b); }
IKG_HD inline bool guard_test(v2f x, v2f, float b) {
  const uint32_t hx = __builtin_bit_cast(uint32_t, x.x), hy = __builtin_bit_cast(uint32_t, x.y);
  return (hx > hy ? hx : hy) > __builtin_bit_cast(uint32_t, b);
}

// ---------------------------------------------------------------- singular arm blocks
// pinv(J) e for J = [c | blockdiag(J_L, J_R)] without inverting the arm
// blocks, for the iterates where one of them is (nearly) singular.  Per arm,
// M_a = [c_a | J_a] (6 x 7).  With z_a = M_a^+ e_a (minimum-norm least
// squares) and p_a = P_null(M_a) e_0 = e_0 - M_a^+ c_a (the chest axis e_0
// projected on M_a's null space, bb_a = p_a[0] = |p_a|^2), the least-squares
// solutions of the arm's rows with chest value s are z_a + p_a t_a + (null
// directions without a chest component), s = a_a + bb_a t_a (a = z_a[0]),
// and pinv's minimum of s^2 + |x_L|^2 + |x_R|^2 = |z_L|^2 + |z_R|^2 - s^2 + ...
// over them is attained at
//   s = (a_L bb_R + a_R bb_L) / D,  D = bb_L + bb_R - bb_L bb_R,
//   z_L + p_L (a_R - a_L (1 - bb_R)) / D   (the right arm likewise).
// With invertible blocks this is the Sherman-Morrison step (bb = 1/(1+|v|^2),
// a = alpha bb).  A block that loses rank even with the chest column (a
// straight elbow) has bb = 0 and pins s; its least-squares z_a is pinv's.
// D = 0 only if both arms pin s (J loses rank through the coupling): s is then
// the mean of the two values (not pinv's least-squares compromise).
//
// M_a^+ by one-sided (Hestenes) Jacobi on M_a's 6 rows: rotations G make the
// rows w_i orthogonal, M^+ b = sum_i w_i (G b)_i / |w_i|^2 over the rows with
// |w_i| > 1e-15 max |w|, np.linalg.pinv's cut (Jacobi's small singular values
// are accurate, so the rank decision is pinv's).  Both right-hand sides (e, c)
// are rotated along.
// sqrt in the lane type's own precision (the global ::sqrt would take a float
// through double)
template <typename T>
IKG_HD inline T tsqrt(T x) {
  if constexpr (is_packed<T> || is_f64<T>)
    return sqrt(x);
  else
    return sqrtf(x);
}

template <typename T>
IKG_HD inline T tabs(T x) {
  if constexpr (is_packed<T> || is_f64<T>)
    return fabs(x);
  else
    return fabsf(x);
}
template <typename T>
IKG_HD inline T tmax(T x, T y) {
  if constexpr (is_packed<T> || is_f64<T>)
    return fmax(x, y);
  else
    return fmaxf(x, y);
}

#ifdef IKG_SING_COUNT
// diagnostic build: [0] lanes that took the branch, [1] Jacobi sweeps (per TU)
static __device__ unsigned long long g_sing[4];
#define IKG_SING_TALLY(k, n) atomicAdd(&g_sing[k], (unsigned long long)(n))
#else
#define IKG_SING_TALLY(k, n) ((void)0)
#endif

template <typename T>
IKG_HD inline void arm_pinv7(const T (&A)[6][8], T* z, T* p) {
  using E = typename LaneT<T>::E;
  // column order: 0 = chest (A[.][7]), 1..6 = arm joints (A[.][0..5])
  T W[6][7], e[6], c[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    W[r][0] = A[r][7];
#pragma unroll
    for (int k = 0; k < 6; ++k) W[r][1 + k] = A[r][k];
    e[r] = A[r][6];
    c[r] = A[r][7];
  }
  const T tol = T(E(Prec<E>::kRcond));
#pragma nounroll
  for (int sweep = 0; sweep < 12; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = i + 1; j < 6; ++j) {
        T a = T(0), b = T(0), d = T(0);
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          a += W[i][k] * W[i][k];
          b += W[j][k] * W[j][k];
          d += W[i][k] * W[j][k];
        }
        const auto rot = tabs(d) > tol * tsqrt(a * b);
        rotated |= any_of(rot);
        const T dd = vsel(rot, d, T(1));
        const T zeta = fdiv(b - a, T(2) * dd);
        const T t = fdiv(vsel(zeta >= T(0), T(1), T(-1)), tabs(zeta) + tsqrt(T(1) + zeta * zeta));
        const T cs = vsel(rot, fdiv(T(1), tsqrt(T(1) + t * t)), T(1));
        const T sn = vsel(rot, cs * t, T(0));
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          const T wi = W[i][k], wj = W[j][k];
          W[i][k] = cs * wi - sn * wj;
          W[j][k] = sn * wi + cs * wj;
        }
        const T ei = e[i], ej = e[j], ci = c[i], cj = c[j];
        e[i] = cs * ei - sn * ej;
        e[j] = sn * ei + cs * ej;
        c[i] = cs * ci - sn * cj;
        c[j] = sn * ci + cs * cj;
      }
#if defined(IKG_SING_COUNT) && defined(__HIP_DEVICE_COMPILE__)
    IKG_SING_TALLY(1, 1);
#endif
    if (!rotated) break;
  }
  T s2[6], smax = T(0);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    T a = T(0);
#pragma unroll
    for (int k = 0; k < 7; ++k) a += W[i][k] * W[i][k];
    s2[i] = a;
    smax = tmax(smax, a);
  }
  const T cut2 = smax * tol * tol;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    z[k] = T(0);
    p[k] = k == 0 ? T(1) : T(0);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const auto keep = s2[i] > cut2;
    const T r = vsel(keep, fdiv(T(1), vsel(keep, s2[i], T(1))), T(0));
    const T fe = e[i] * r, fc = c[i] * r;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      z[k] += W[i][k] * fe;
      p[k] -= W[i][k] * fc;
    }
  }
}

// The same z_a, p_a from M_a's normal equations, for the guard's usual case:
// an arm block J_a near singular at the wrist or shoulder, where the chest
// column keeps M_a = [c_a | J_a] well conditioned (cond ~ 1e2).  G = M_a M_a^T
// (6 x 6) by Cholesky, y = G^-1 e, w = G^-1 c_a; z = M_a^T y, p = e_0 - M_a^T w,
// in the lane type (packed: both arms at once).  The error is ~eps
// cond(M_a)^2 of the step; it is taken where every Cholesky pivot is >= kNeTol
// of G's largest diagonal entry (cond(M_a) <~ 1e3: fp64 <= ~2e-10 of the step,
// fp32 below the closed form's own error at its guard bound); elsewhere (a
// straight elbow, rank deficiency) the Jacobi form decides the rank as pinv
// does.  ~350 operations against ~10^4 for the Jacobi sweeps, which made a
// wave holding a problem that lingers near the wrist several times slower
// (random seeds, multi-start: round 3).
constexpr double kNeTol = 1e-6;

template <typename T>
IKG_HD inline typename LaneT<T>::M minnorm_ne(const T (&A)[6][8], T* z, T* p) {
  using E = typename LaneT<T>::E;
  // rows of M_a = [c | J_a]: column 0 = chest (A[.][7]), 1..6 = A[.][0..5]
  auto M = [&](int r, int k) -> T { return k == 0 ? A[r][7] : A[r][k - 1]; };
  T G[6][6];
  T gmax = T(0);
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c <= r; ++c) {
      T acc = T(0);
#pragma unroll
      for (int k = 0; k < 7; ++k) acc += M(r, k) * M(c, k);
      G[r][c] = acc;
      if (r == c) gmax = tmax(gmax, acc);
    }
  auto ok = gmax > T(0);
  T rinv[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    T d = G[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= G[j][k] * G[j][k];
    ok = ok & (d >= T(E(kNeTol)) * gmax);
    rinv[j] = fdiv(T(1), tsqrt(tmax(d, T(E(Prec<E>::kRcond)) * gmax + T(E(1e-30)))));
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      T a = G[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) a -= G[i][k] * G[j][k];
      G[i][j] = a * rinv[j];
    }
  }
  // forward (L) then backward (L^T) substitution for e and c = M[.][0]
  T y[6], w[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    T a = A[i][6], b = A[i][7];
#pragma unroll
    for (int k = 0; k < i; ++k) {
      a -= G[i][k] * y[k];
      b -= G[i][k] * w[k];
    }
    y[i] = a * rinv[i];
    w[i] = b * rinv[i];
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    T a = y[i], b = w[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) {
      a -= G[k][i] * y[k];
      b -= G[k][i] * w[k];
    }
    y[i] = a * rinv[i];
    w[i] = b * rinv[i];
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    T a = T(0), b = T(0);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      a += M(r, k) * y[r];
      b += M(r, k) * w[r];
    }
    z[k] = a;
    p[k] = (k == 0 ? T(1) : T(0)) - b;
  }
  return ok;
}

// z_a, p_a for one lane (both halves of a packed lane): the normal equations
// where they are accurate, the Jacobi form elsewhere.  Returns whether every
// half took the normal equations (diagnostics).
template <typename T>
IKG_HD inline bool arm_minnorm(const T (&A)[6][8], T* z, T* p) {
  const auto ok = minnorm_ne(A, z, p);
  const auto need_j = mnot(ok);
  if (any_of(need_j)) {
    T zj[7], pj[7];
    arm_pinv7(A, zj, pj);
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      z[k] = vsel(need_j, zj[k], z[k]);
      p[k] = vsel(need_j, pj[k], p[k]);
    }
  }
  return !any_of(need_j);
}

// The chest value s and this arm's coefficient f (z_a + p_a f) from the two
// arms' (a, bb) (partner: ao, bbo).  Both lanes of a pair must get the same s
// bit for bit (each carries the chest joint), so every product is rounded on
// its own (no contraction) and the sums are commutative.
template <typename T>
IKG_HD inline void minnorm_combine(T a, T bb, T ao, T bbo, T& s, T& f) {
#pragma clang fp contract(off)
  const T pr = a * bbo, po = ao * bb;
  const T num = pr + po;
  const T D = (bb + bbo) - bb * bbo;
  const auto ok = D > T(Prec<T>::kRcond);
  const T Ds = vsel(ok, D, T(1));
  s = vsel(ok, fdiv(num, Ds), (a + ao) * T(0.5));
  f = vsel(ok, fdiv(ao - a * (T(1) - bbo), Ds), T(0));
}

// The 6 x 8 arm system in frame-1 axes at the hand point (the layout of
// arm_system: columns 0..5 arm joints, 6 the error, 7 the chest), from the
// frame-1 state (arm_fk_error_f1): axes a0 = e_z, a1 = a2 = e_y,
// [a3 a4 a5] = Ry(q12) [e_x, Rx(q3) e_y, Rx(q3) Ry(q4) e_z]; the wrist axes
// pass through w, the chest axis (e_z) through -(k, p0z).
template <typename T, class SP>
IKG_HD inline void arm_system_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const ArmStateF1<T>& st,
                                 const T* sn, const T* cs, T (&A)[6][8]) {
  const bool right = arm != 0;
  const T* h = st.h;
  T ax[7][3], org[7][3];
  const T s3 = sn[4], c3 = cs[4], s4 = sn[5], c4 = cs[5], c12 = st.c12, s12 = st.s12;
  // local wrist axes before Ry(q12): e_x, Rx(q3) e_y = (0, c3, s3), Rx(q3) Ry(q4) e_z = (s4, -s3 c4, c3 c4)
  const T loc[3][3] = {{T(1), T(0), T(0)}, {T(0), c3, s3}, {s4, -s3 * c4, c3 * c4}};
  const T ez[3] = {T(0), T(0), T(1)}, ey[3] = {T(0), T(1), T(0)};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    ax[0][i] = ez[i];  // chest
    ax[1][i] = ez[i];
    ax[2][i] = ey[i];
    ax[3][i] = ey[i];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {  // Ry(q12) loc[k]
    ax[4 + k][0] = c12 * loc[k][0] + s12 * loc[k][2];
    ax[4 + k][1] = loc[k][1];
    ax[4 + k][2] = c12 * loc[k][2] - s12 * loc[k][0];
  }
  const T p0z = SP::zero_t(0, 2) ? T(0) : armc<T>(right, m->arm_t[0][0][2], m->arm_t[1][0][2]);
  org[0][0] = -st.k[0];
  org[0][1] = -st.k[1];
  org[0][2] = -p0z;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    org[1][i] = T(0);
    org[2][i] = SP::zero_t(1, i) ? T(0) : armc<T>(right, m->arm_t[0][1][i], m->arm_t[1][1][i]);
    org[3][i] = st.o2[i];
    org[4][i] = st.w[i];
    org[5][i] = st.w[i];
    org[6][i] = st.w[i];
  }
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int col = j == 0 ? 7 : j - 1;
    const T dx = h[0] - org[j][0], dy = h[1] - org[j][1], dz = h[2] - org[j][2];
    A[0][col] = ax[j][1] * dz - ax[j][2] * dy;
    A[1][col] = ax[j][2] * dx - ax[j][0] * dz;
    A[2][col] = ax[j][0] * dy - ax[j][1] * dx;
    A[3][col] = ax[j][0];
    A[4][col] = ax[j][1];
    A[5][col] = ax[j][2];
  }
#pragma unroll
  for (int r = 0; r < 6; ++r) A[r][6] = st.e[r];
}


// lambda > 0: z_e, z_c = (J_a J_a^T + lambda I)^-1 [e_a, c_a]; alpha = c.z_e, beta = c.z_c.
template <typename T>
IKG_HD inline void arm_solve_damped(const T (&A)[6][8], T lambda, T* ze, T* zc, T& alpha, T& beta) {
  T M[6][6];
#pragma unroll
  for (int r = 0; r < 6; ++r)
#pragma unroll
    for (int c = 0; c <= r; ++c) {
      T acc = r == c ? lambda : T(0);
#pragma unroll
      for (int k = 0; k < 6; ++k) acc += A[r][k] * A[c][k];
      M[r][c] = acc;
    }
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    ze[r] = A[r][6];
    zc[r] = A[r][7];
  }
  chol_solve6(M, ze, zc);
  alpha = T(0);
  beta = T(0);
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    alpha += A[r][7] * ze[r];
    beta += A[r][7] * zc[r];
  }
}

// Sherman–Morrison chest step from the pair-summed scalars.
template <typename T>
IKG_HD inline T chest_step(T alpha_sum, T beta_sum) {
  return fdiv(alpha_sum, T(1) + beta_sum);
}

template <typename T>
IKG_HD inline void arm_dq(const T* u, const T* v, T s, T* dq) {
#pragma unroll
  for (int k = 0; k < 6; ++k) dq[k] = u[k] - s * v[k];
}

template <typename T>
IKG_HD inline void arm_dq_damped(const T (&A)[6][8], const T* ze, const T* zc, T s, T* dq) {
  T y[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) y[r] = ze[r] - s * zc[r];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    T acc = T(0);
#pragma unroll
    for (int r = 0; r < 6; ++r) acc += A[r][k] * y[r];
    dq[k] = acc;
  }
}

// pinv(J) e for the pair (inverse_geometry.py:83): the closed-form
// Sherman-Morrison step, and the per-arm pinv form (arm_pinv7) for both lanes of a
// pair when either arm block is near singular.  The guard travels in the sign
// of the exchanged |v|^2 (never negative otherwise), so it costs no extra
// exchange; both lanes of a pair take the branch together.
struct PairX {  // the partner arm: lane ^ 1 (pair layout) or the other half (packed)
  template <typename T>
  __device__ T operator()(T x) const { return pair_swap(x); }
};

template <typename T, class X = PairX>
__device__ inline void pinv_step_tail(const T* u, const T* v, T alpha, T beta, typename LaneT<T>::E bound, T* dq,
                                      T& s, bool& need) {
  const X xc;
  const T bo = xc(beta);
  s = chest_step(alpha + xc(alpha), beta + bo);
  arm_dq(u, v, s, dq);
  need = guard_test(beta, bo, bound);
}

template <typename T, class X = PairX>
__device__ inline void pinv_step_lq(const T (&A)[6][8], int, T* dq, T& s) {
  const X xc;
  T z[7], p[7], f;
#ifdef IKG_SING_COUNT
  IKG_SING_TALLY(0, 1);
#endif
  arm_minnorm(A, z, p);
  minnorm_combine(z[0], p[0], xc(z[0]), xc(p[0]), s, f);
#pragma unroll
  for (int k = 0; k < 6; ++k) dq[k] = z[1 + k] + f * p[1 + k];
}

// The guard's branch as an out-of-line call (IKG_COLD_CALL): the loop is then
// register-allocated as if the branch did not exist, and only a taken branch
// pays for saving the loop's state around the call (round 3: the inlined
// branch cost the never-taken loop 3-4% at C2 / C3).
#ifndef IKG_COLD_CALL
#define IKG_COLD_CALL 1
#endif
template <typename T>
struct ColdIO {  // the branch's inputs and outputs, copied only when it is taken
  ArmStateF1<T> st;
  T sn[7], cs[7], dq[6], s;
};
template <typename T, class SP, class X>
__device__ __attribute__((noinline)) void pinv_step_f1_cold(const KModel<typename LaneT<T>::E>* __restrict__ m,
                                                            int arm, ColdIO<T>* io) {
  T A[6][8];
  arm_system_f1<T, SP>(m, arm, io->st, io->sn, io->cs, A);
  pinv_step_lq<T, X>(A, arm, io->dq, io->s);
}

// COLD: the out-of-line branch, for fp64 and the packed fp32 layout; the pair
// fp32 kernel keeps it inline (the call measured +0.4% at C2 fp32, DESIGN
// §3a.5), and so does the records-in-batch loop (REC: 3% slower with it at C2
// with the collision term)
template <typename T, class SP, class X = PairX, bool COLD = true>
__device__ inline void pinv_step_f1(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, const ArmStateF1<T>& st,
                                    const T* sn, const T* cs, T* dq, T& s) {
  T u[6], v[6], alpha, beta;
  arm_solve_f1<T, SP>(m, arm, st, sn, cs, u, v, alpha, beta);
  bool need;
  pinv_step_tail<T, X>(u, v, alpha, beta, m->sing_beta, dq, s, need);
  if (__builtin_expect(IKG_SING_GUARD && need, 0)) {
#if IKG_COLD_CALL
    if constexpr ((is_f64<T> || is_packed<T>) && COLD) {
      ColdIO<T> io;
      io.st = st;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        io.sn[j] = sn[j];
        io.cs[j] = cs[j];
      }
      pinv_step_f1_cold<T, SP, X>(m, arm, &io);
#pragma unroll
      for (int k = 0; k < 6; ++k) dq[k] = io.dq[k];
      s = io.s;
      return;
    }
#endif
    T A[6][8];
    arm_system_f1<T, SP>(m, arm, st, sn, cs, A);
    pinv_step_lq<T, X>(A, arm, dq, s);
  }
}

template <typename T, class SP>
__device__ inline void pinv_step_cf(const ArmState<T>& st, int arm, T tau, T bound, T* dq, T& s) {
  T u[6], v[6], alpha, beta;
  typename LaneT<T>::M bad;
  arm_solve<T, SP>(st, u, v, alpha, beta, &bad, tau);
  bool need;
  // a small relative pivot (truncated by the QR, or a small 3 x 3
  // determinant) travels as an out-of-bound |v|^2
  pinv_step_tail(u, v, alpha, vsel(bad, T(3e38), beta), bound, dq, s, need);
  if (__builtin_expect(IKG_SING_GUARD && need, 0)) {
    T A[6][8];
    arm_system(st, A);
    pinv_step_lq(A, arm, dq, s);
  }
}

// This lane's arm limits (pair layout), loaded once per solve when the
// registers are available (IKG_LANE_LIMITS).
template <typename T>
struct ArmLimits {
  T lo[kArmDof], hi[kArmDof];
};
template <typename T>
IKG_HD inline void load_limits(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, ArmLimits<T>& L) {
  const bool right = arm != 0;
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) {
    L.lo[k] = armc<T>(right, m->arm_lo[0][k], m->arm_lo[1][k]);
    L.hi[k] = armc<T>(right, m->arm_hi[0][k], m->arm_hi[1][k]);
  }
}

// pin.integrate (q + dq * DT, :86) then projecttojointlimits (:89).
template <typename T>
IKG_HD inline void arm_update(const KModel<typename LaneT<T>::E>* __restrict__ m, int arm, T dt, T s, const T* dq, T& qc, T* qa,
                              const ArmLimits<T>* lim = nullptr) {
  const bool right = arm != 0;
  qc = clampq(qc + s * dt, T(m->root_lo), T(m->root_hi));
  if (lim) {
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) qa[k] = clampq(qa[k] + dq[k] * dt, lim->lo[k], lim->hi[k]);
    return;
  }
  if constexpr (is_packed<T>) {  // both arms in the lane: packed limits
#pragma unroll
    for (int k = 0; k < kArmDof; ++k)
      qa[k] = clampq(qa[k] + dq[k] * dt, T{m->arm_lo[0][k], m->arm_lo[1][k]}, T{m->arm_hi[0][k], m->arm_hi[1][k]});
  } else {
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) {
      // clamp against both arms' (scalar) limits and select the result: 2 VALU
      // ops per bound with scalar operands instead of materialising per-lane
      // limits (the pair kernel has no registers to keep them)
      const T v = qa[k] + dq[k] * dt;
      const T qL = clampq(v, m->arm_lo[0][k], m->arm_hi[0][k]);
      const T qR = clampq(v, m->arm_lo[1][k], m->arm_hi[1][k]);
      qa[k] = sel(right, qR, qL);
    }
  }
}

// tools.getcubeplacement: oMcube * hook (tools.py:54-59), for this lane's arm.
template <typename T>
IKG_HD inline void hook_target(const KModel<T>* __restrict__ m, int arm, const T* __restrict__ tg, T* RT,
                                   T* tT) {
  const bool right = arm != 0;
  T CR[9], Ct[3], HR[9], Ht[3], d[3];
#pragma unroll
  for (int i = 0; i < 9; ++i) CR[i] = tg[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) Ct[i] = tg[9 + i];
#pragma unroll
  for (int i = 0; i < 9; ++i) HR[i] = sel(right, m->hook_R[1][i], m->hook_R[0][i]);
#pragma unroll
  for (int i = 0; i < 3; ++i) Ht[i] = sel(right, m->hook_t[1][i], m->hook_t[0][i]);
  matmul3(CR, HR, RT);
  matvec3(CR, Ht, d);
#pragma unroll
  for (int i = 0; i < 3; ++i) tT[i] = Ct[i] + d[i];
}

// Both arms' hook targets in one packed lane (x = left, y = right).
IKG_HD inline void hook_target_packed(const KModel<float>* __restrict__ m, const float* __restrict__ tg, v2f* RT,
                                      v2f* tT) {
  float RL[9], tL[3], RR[9], tR[3];
  hook_target(m, 0, tg, RL, tL);
  hook_target(m, 1, tg, RR, tR);
#pragma unroll
  for (int i = 0; i < 9; ++i) RT[i] = v2f{RL[i], RR[i]};
#pragma unroll
  for (int i = 0; i < 3; ++i) tT[i] = v2f{tL[i], tR[i]};
}

}  // namespace ikg
