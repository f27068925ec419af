// Host-side construction of the kernel model tables from ikg_model_desc
// (shared by the C-ABI and the host emulator).
#pragma once

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "ikg_collision.hpp"
#include "ikg_device.hpp"
#include "ikgrasp.h"

namespace ikg {

// |t x a| <= 1e-14 |t| |a|: the line through the origin along a contains t
inline bool parallel_or_zero(const double* t, const double* a) {
  const double c[3] = {t[1] * a[2] - t[2] * a[1], t[2] * a[0] - t[0] * a[2], t[0] * a[1] - t[1] * a[0]};
  const double nc = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
  const double nt = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
  const double na = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  return nc <= 1e-14 * nt * na;
}

inline bool is_identity(const double* R) {
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      if (R[3 * r + c] != (r == c ? 1.0 : 0.0)) return false;
  return true;
}

// A numeric test knob from the environment: parsed whole by strtod, finite and
// >= 0, else ignored with a message; an accepted override is announced on
// stderr (once per table build), so a stray value never changes results silently.
template <typename T>
inline void env_knob(const char* name, T& v) {
  const char* e = std::getenv(name);
  if (!e) return;
  char* end = nullptr;
  const double x = std::strtod(e, &end);
  if (end == e || *end != '\0' || !std::isfinite(x) || x < 0) {
    std::fprintf(stderr, "[ikgrasp] ignoring %s=\"%s\": not a finite number >= 0\n", name, e);
    return;
  }
  std::fprintf(stderr, "[ikgrasp] test override %s=%g active\n", name, x);
  v = (T)x;
}

template <typename T>
inline void build_kmodel(const ikg_model_desc& d, KModel<T>& k) {
  std::memset(&k, 0, sizeof(k));
  const int r = d.root_q;
  for (int i = 0; i < 9; ++i) k.root_R[i] = (T)d.placement[r][i];
  for (int i = 0; i < 3; ++i) k.root_t[i] = (T)d.placement[r][9 + i];
  k.root_lo = (T)d.lower[r];
  k.root_hi = (T)d.upper[r];
  k.root_q = r;
  k.root_axis = d.axis[r];
  k.rot_mask = 0;
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < IKG_ARM_DOF; ++j) {
      const int q = d.arm_q[a][j];
      for (int i = 0; i < 9; ++i) k.arm_R[a][j][i] = (T)d.placement[q][i];
      for (int i = 0; i < 3; ++i) k.arm_t[a][j][i] = (T)d.placement[q][9 + i];
      k.arm_lo[a][j] = (T)d.lower[q];
      k.arm_hi[a][j] = (T)d.upper[q];
      k.arm_q[a][j] = q;
      k.arm_axis[j] = d.axis[q];
      if (!is_identity(d.placement[q])) k.rot_mask |= 1 << j;
    }
  for (int a = 0; a < 2; ++a) {
    for (int i = 0; i < 9; ++i) k.hand_R[a][i] = (T)d.hand[a][i];
    for (int i = 0; i < 3; ++i) k.hand_t[a][i] = (T)d.hand[a][9 + i];
    for (int i = 0; i < 9; ++i) k.hook_R[a][i] = (T)d.hook[a][i];
    for (int i = 0; i < 3; ++i) k.hook_t[a][i] = (T)d.hook[a][9 + i];
  }
  for (int q = 0; q < d.nq; ++q) {
    k.lo[q] = (T)d.lower[q];
    k.hi[q] = (T)d.upper[q];
    for (int i = 0; i < 9; ++i) k.jR[q][i] = (T)d.placement[q][i];
    for (int i = 0; i < 3; ++i) k.jt[q][i] = (T)d.placement[q][9 + i];
    k.jaxis[q] = d.axis[q];
    k.jparent[q] = d.parent[q];
  }
  k.nq = d.nq;
  // singularity guard (ikg_device.hpp pinv_step): below these the closed-form
  // arm solve's cancellation (u - s v with |u|, |v| ~ 1/tau) would cost more
  // than ~1e-12 (fp64) / 1e-5 (fp32) of the step, so the pair takes the
  // 6 x 7 LQ form instead
  k.sing_beta = (T)(sizeof(T) == 8 ? IKG_SING_BETA64 : IKG_SING_BETA32);
  k.sing_tau = (T)(sizeof(T) == 8 ? IKG_SING_TAU64 : IKG_SING_TAU32);
  // test knobs, read when the tables are built: IKG_SING_BETA=0 (with
  // IKG_SING_TAU=1e30 for the generic path) sends every update through the
  // LQ form.  A value must parse whole as a finite number >= 0; anything else
  // is ignored with a message, and an accepted override is announced.
  env_knob("IKG_SING_BETA", k.sing_beta);
  env_knob("IKG_SING_TAU", k.sing_tau);
  bool used[IKG_MAX_NQ] = {};
  used[r] = true;
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < IKG_ARM_DOF; ++j) used[d.arm_q[a][j]] = true;
  k.n_passive = 0;
  for (int q = 0; q < d.nq; ++q)
    if (!used[q]) k.passive_q[k.n_passive++] = q;
  if (!is_identity(d.placement[r])) k.rot_mask |= 1 << 6;

  // hand frame rotation: a principal-axis rotation R_a(angle) shared by both hands?
  k.hand_axis = 3;
  for (int ax = 0; ax < 3 && k.hand_axis == 3; ++ax) {
    const int b = (ax + 1) % 3, c = (ax + 2) % 3;
    bool ok = true;
    for (int h = 0; h < 2; ++h) {
      const double* R = d.hand[h];
      auto at = [&](int i, int j) { return R[3 * i + j]; };
      ok = ok && at(ax, ax) == 1.0 && at(ax, b) == 0.0 && at(ax, c) == 0.0 && at(b, ax) == 0.0 &&
           at(c, ax) == 0.0 && at(b, b) == at(c, c) && at(b, c) == -at(c, b);
    }
    if (ok) {
      k.hand_axis = ax;
      for (int h = 0; h < 2; ++h) {
        k.hand_sc[h][0] = (T)d.hand[h][3 * c + b];  // sin
        k.hand_sc[h][1] = (T)d.hand[h][3 * b + b];  // cos
      }
    }
  }
  // spherical wrist: the axes of arm joints 3, 4, 5 meet at joint 4's origin,
  // i.e. joint 4's origin lies on joint 3's axis (t4 || e3 in joint 3's frame)
  // and joint 5's axis passes through it (t5 || R5 e5 in joint 4's frame).
  // Any placement rotations; parallel up to 1e-14 relative (a tilted URDF's
  // rpy round trip leaves ~1e-17 m).
  k.wrist = 1;
  for (int a = 0; a < 2; ++a) {
    const int q3 = d.arm_q[a][3], q4 = d.arm_q[a][4], q5 = d.arm_q[a][5];
    const double* P4 = d.placement[q4];
    const double* P5 = d.placement[q5];
    double e3[3] = {0.0, 0.0, 0.0}, a5[3];
    e3[d.axis[q3]] = 1.0;
    for (int i = 0; i < 3; ++i) a5[i] = P5[3 * i + d.axis[q5]];  // R5 e5 (row-major)
    if (!parallel_or_zero(P4 + 9, e3) || !parallel_or_zero(P5 + 9, a5)) k.wrist = 0;
  }
  // zero placement offsets shared by both arms (Spec zero mask)
  k.zmask = 0;
  for (int j = 0; j < IKG_ARM_DOF; ++j)
    for (int i = 0; i < 3; ++i)
      if (d.placement[d.arm_q[0][j]][9 + i] == 0.0 && d.placement[d.arm_q[1][j]][9 + i] == 0.0)
        k.zmask |= 1 << (3 * j + i);
  for (int a = 0; a < 2; ++a)
    for (int i = 0; i < 3; ++i) {
      const double* H = d.hand[a];
      k.hand_tH[a][i] = (T)(H[i] * H[9] + H[3 + i] * H[10] + H[6 + i] * H[11]);
    }
  int pat = d.axis[r];
  for (int j = 0; j < IKG_ARM_DOF; ++j) pat |= d.axis[d.arm_q[0][j]] << (2 * (j + 1));
  pat |= k.hand_axis << 14;
  k.pattern = pat;
}

// Smallest x with sqrt(x) >= eps (both in T, IEEE): the loop tests x < eps2,
// which is exactly sqrt(x) < eps for a correctly rounded sqrt.
template <typename T>
inline T stop_threshold(T eps) {
  if (!(eps > T(0))) return T(0);
  T m = eps * eps;
  while (m > T(0) && std::sqrt(m) >= eps) m = std::nextafter(m, T(0));
  while (std::sqrt(m) < eps) m = std::nextafter(m, std::numeric_limits<T>::max());
  return m;
}

template <typename T>
inline KParams<T> make_kparams(const ikg_params* p) {
  KParams<T> k;
  k.eps = (T)p->eps;
  k.dt = (T)p->dt;
  k.lambda = (T)p->lambda;
  k.max_iters = p->max_iters;
  k.eps2 = stop_threshold<T>((T)p->eps);
  return k;
}

// The compiled specialisation this model can use (ikg_launch.hpp kSpec*).
template <typename T>
inline int choose_spec(const KModel<T>& k) {
  if (k.pattern == kPatternNextage && k.rot_mask == 0 && k.wrist && (k.zmask & kZeroNextage) == kZeroNextage)
    return 1;  // kSpecNextage
  if (k.wrist) return 2;  // kSpecGenericWrist
  return 0;  // kSpecGeneric
}


// Collision scene tables (bounding radii padded so rounding never rejects a
// touching pair).
template <typename T>
inline void build_kcollision(const ikg_collision_desc& d, KCollision<T>& c) {
  std::memset(&c, 0, sizeof(c));
  c.n_geoms = d.n_geoms;
  c.n_pairs = d.n_pairs;
  c.target_geom = d.target_geom;
  for (int g = 0; g < d.n_geoms; ++g) {
    for (int i = 0; i < 9; ++i) c.R[g][i] = (T)d.placement[g][i];
    for (int i = 0; i < 3; ++i) c.t[g][i] = (T)d.placement[g][9 + i];
    for (int i = 0; i < 3; ++i) c.dims[g][i] = (T)d.dims[g][i];
    c.kind[g] = d.kind[g];
    c.joint[g] = d.joint[g];
    const double* h = d.dims[g];
    double r;  // bounding sphere about the placement origin, padded for rounding
    if (d.kind[g] == IKG_GEOM_SPHERE)
      r = h[0];
    else if (d.kind[g] == IKG_GEOM_CYLINDER)
      r = std::sqrt(h[0] * h[0] + h[1] * h[1]);
    else
      r = std::sqrt(h[0] * h[0] + h[1] * h[1] + h[2] * h[2]);
    c.brad[g] = (T)(r * (1.0 + 1e-6) + 1e-9);
  }
  for (int k = 0; k < d.n_pairs; ++k) {
    c.pairs[k][0] = (int16_t)d.pairs[k][0];
    c.pairs[k][1] = (int16_t)d.pairs[k][1];
    const T r = c.brad[d.pairs[k][0]] + c.brad[d.pairs[k][1]];  // as the device would form it
    c.pr2[k] = r * r;
  }
}

}  // namespace ikg
