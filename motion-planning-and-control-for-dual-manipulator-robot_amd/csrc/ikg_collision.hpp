// Collision term of the reference's `success`:
// tools.collision(robot, q) = pin.updateGeometryPlacements + pin.computeCollisions
// over the active pairs of setup_pinocchio.py:53-60 (hpp-fcl narrow phase).
// Restated for gfx950 as a wave-cooperative check: one wave per problem, the
// joint frames and geometry placements staged in LDS, the ~745 pairs split
// over the 64 lanes with a bounding-sphere broad phase, exact sphere tests and
// boolean GJK on support functions for boxes / cylinders / the cube mesh hull.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ikg_device.hpp"

namespace ikg {

constexpr int kMaxGeoms = 64;
constexpr int kMaxPairs = 1024;
constexpr int kGjkIters = 48;

enum { kSphere = 0, kBox = 1, kCylinder = 2, kMeshBox = 3 };

template <typename T>
struct KCollision {
  T R[kMaxGeoms][9];
  T t[kMaxGeoms][3];
  T dims[kMaxGeoms][3];
  T brad[kMaxGeoms];  // bounding-sphere radius about the placement origin
  int32_t kind[kMaxGeoms];
  int32_t joint[kMaxGeoms];
  int16_t pairs[kMaxPairs][2];
  int32_t n_geoms;
  int32_t n_pairs;
  int32_t target_geom;
};

// LDS scratch of one collision check (one wave).
template <typename T>
struct CollideScratch {
  T q[kMaxNq];
  T L[kMaxNq][12];   // joint-local transforms placement * R_axis(q)
  T F[kMaxNq][12];   // world joint frames
  T P[kMaxGeoms][12];  // world geometry placements
};

template <typename T>
struct Shape {
  const T* R;  // 9, row-major
  const T* t;  // 3
  const T* dims;
  int kind;
};

template <typename T>
IKG_HD inline void shape_support(const Shape<T>& s, const T* d, T* out) {
  if (s.kind == kSphere) {
    const T n2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const T f = n2 > T(0) ? s.dims[0] / sqrt(n2) : T(0);
    for (int i = 0; i < 3; ++i) out[i] = s.t[i] + f * d[i];
    return;
  }
  T dl[3], loc[3];
  matvec3_t(s.R, d, dl);  // R^T d
  if (s.kind == kCylinder) {
    const T rad2 = dl[0] * dl[0] + dl[1] * dl[1];
    const T f = rad2 > T(0) ? s.dims[0] / sqrt(rad2) : T(0);
    loc[0] = f * dl[0];
    loc[1] = f * dl[1];
    loc[2] = dl[2] >= T(0) ? s.dims[1] : -s.dims[1];
  } else {  // box / mesh hull
    for (int i = 0; i < 3; ++i) loc[i] = dl[i] >= T(0) ? s.dims[i] : -s.dims[i];
  }
  T w[3];
  matvec3(s.R, loc, w);
  for (int i = 0; i < 3; ++i) out[i] = s.t[i] + w[i];
}

template <typename T>
IKG_HD inline void triple(const T* a, const T* b, const T* c, T* out) {  // (a x b) x c
  T ab[3];
  cross3(a, b, ab);
  cross3(ab, c, out);
}

// Boolean GJK: do the convex shapes intersect (origin inside A - B)?
template <typename T>
IKG_HD inline bool gjk_intersect(const Shape<T>& A, const Shape<T>& B) {
  T sim[4][3];
  int n;
  T d[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
  if (dot3(d, d) == T(0)) d[0] = T(1);
  auto sup = [&](const T* dir, T* out) {
    T pa[3], pb[3], nd[3] = {-dir[0], -dir[1], -dir[2]};
    shape_support(A, dir, pa);
    shape_support(B, nd, pb);
    for (int i = 0; i < 3; ++i) out[i] = pa[i] - pb[i];
  };
  sup(d, sim[0]);
  n = 1;
  for (int i = 0; i < 3; ++i) d[i] = -sim[0][i];
  for (int iter = 0; iter < kGjkIters; ++iter) {
    if (dot3(d, d) < T(1e-30)) return true;
    T a[3];
    sup(d, a);
    if (dot3(a, d) < T(0)) return false;  // separating direction
    for (int i = 0; i < 3; ++i) sim[n][i] = a[i];
    ++n;
    // ---- reduce the simplex towards the origin (a = newest point)
    for (int pass = 0; pass < 3; ++pass) {
      const T* A0 = sim[n - 1];
      T ao[3] = {-A0[0], -A0[1], -A0[2]};
      if (n == 2) {
        T ab[3] = {sim[0][0] - A0[0], sim[0][1] - A0[1], sim[0][2] - A0[2]};
        if (dot3(ab, ao) > T(0)) {
          triple(ab, ao, ab, d);
          if (dot3(d, d) < T(1e-30)) return true;  // origin on the segment
        } else {
          for (int i = 0; i < 3; ++i) sim[0][i] = A0[i];
          n = 1;
          for (int i = 0; i < 3; ++i) d[i] = ao[i];
        }
        break;
      }
      if (n == 3) {
        T ab[3], ac[3], abc[3], t1[3];
        for (int i = 0; i < 3; ++i) {
          ab[i] = sim[1][i] - A0[i];
          ac[i] = sim[0][i] - A0[i];
        }
        cross3(ab, ac, abc);
        cross3(abc, ac, t1);
        if (dot3(t1, ao) > T(0)) {
          if (dot3(ac, ao) > T(0)) {  // keep [c, a]
            for (int i = 0; i < 3; ++i) sim[1][i] = A0[i];
            n = 2;
            triple(ac, ao, ac, d);
            if (dot3(d, d) < T(1e-30)) return true;
            break;
          }
          for (int i = 0; i < 3; ++i) {  // line [b, a]
            sim[0][i] = sim[1][i];
            sim[1][i] = A0[i];
          }
          n = 2;
          continue;
        }
        cross3(ab, abc, t1);
        if (dot3(t1, ao) > T(0)) {
          for (int i = 0; i < 3; ++i) {
            sim[0][i] = sim[1][i];
            sim[1][i] = A0[i];
          }
          n = 2;
          continue;
        }
        if (dot3(abc, ao) > T(0)) {
          for (int i = 0; i < 3; ++i) d[i] = abc[i];  // [c, b, a]
        } else {
          for (int i = 0; i < 3; ++i) {  // [b, c, a]
            const T tmp = sim[0][i];
            sim[0][i] = sim[1][i];
            sim[1][i] = tmp;
            d[i] = -abc[i];
          }
        }
        break;
      }
      // n == 4: sim = [d, c, b, a]
      T ab[3], ac[3], ad[3], f[3];
      for (int i = 0; i < 3; ++i) {
        ab[i] = sim[2][i] - A0[i];
        ac[i] = sim[1][i] - A0[i];
        ad[i] = sim[0][i] - A0[i];
      }
      cross3(ab, ac, f);
      if (dot3(f, ao) > T(0)) {  // triangle [c, b, a]
        for (int i = 0; i < 3; ++i) {
          sim[0][i] = sim[1][i];
          sim[1][i] = sim[2][i];
          sim[2][i] = A0[i];
        }
        n = 3;
        continue;
      }
      cross3(ac, ad, f);
      if (dot3(f, ao) > T(0)) {  // triangle [d, c, a]
        for (int i = 0; i < 3; ++i) sim[2][i] = A0[i];
        n = 3;
        continue;
      }
      cross3(ad, ab, f);
      if (dot3(f, ao) > T(0)) {  // triangle [b, d, a]
        for (int i = 0; i < 3; ++i) {
          sim[1][i] = sim[0][i];
          sim[0][i] = sim[2][i];
          sim[2][i] = A0[i];
        }
        n = 3;
        continue;
      }
      return true;  // origin enclosed
    }
  }
  return true;  // iteration cap: treat as touching
}

// Narrow phase of one pair (hpp-fcl collide(): intersection <=> collision).
template <typename T>
IKG_HD inline bool pair_collides(const Shape<T>& A, const Shape<T>& B) {
  if (A.kind == kSphere && B.kind == kSphere) {
    T d[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
    const T r = A.dims[0] + B.dims[0];
    return dot3(d, d) < r * r;
  }
  if ((A.kind == kSphere) != (B.kind == kSphere)) {
    const Shape<T>& S = A.kind == kSphere ? A : B;
    const Shape<T>& X = A.kind == kSphere ? B : A;
    if (X.kind == kBox || X.kind == kMeshBox) {  // closest point on the box
      T d[3] = {S.t[0] - X.t[0], S.t[1] - X.t[1], S.t[2] - X.t[2]}, p[3];
      matvec3_t(X.R, d, p);
      T e2 = T(0);
      for (int i = 0; i < 3; ++i) {
        const T c = fmin(fmax(p[i], -X.dims[i]), X.dims[i]);
        e2 += (p[i] - c) * (p[i] - c);
      }
      return e2 < S.dims[0] * S.dims[0];
    }
  }
  return gjk_intersect(A, B);
}

// ---------------------------------------------------------------- check stages
// The stages of one check, shared by the wave-parallel driver (collide_wave,
// ikg_collision.hip) and the host emulator.  Frames are [R(9) row-major, t(3)].

// Joint-local transform placement * R_axis(q_j) (JointModelR*::calc).
template <typename T>
IKG_HD inline void joint_local(const KModel<T>* __restrict__ m, int j, T qj, T* L) {
  T s, co, R[9];
  Prec<T>::sincos_(qj, &s, &co);
  for (int i = 0; i < 9; ++i) R[i] = m->jR[j][i];
  rotate_axis(R, m->jaxis[j], s, co);
  for (int i = 0; i < 9; ++i) L[i] = R[i];
  for (int i = 0; i < 3; ++i) L[9 + i] = m->jt[j][i];
}

// World frame of joint j (oMi): compose the local transforms up the parent chain.
template <typename T>
IKG_HD inline void joint_world(const KModel<T>* __restrict__ m, int j, const T (*L)[12], T* F) {
  T R[9], t[3];
  for (int i = 0; i < 9; ++i) R[i] = L[j][i];
  for (int i = 0; i < 3; ++i) t[i] = L[j][9 + i];
  for (int k = m->jparent[j]; k >= 0; k = m->jparent[k]) {
    T Rn[9], tn[3];
    matmul3(L[k], R, Rn);
    matvec3(L[k], t, tn);
    for (int i = 0; i < 9; ++i) R[i] = Rn[i];
    for (int i = 0; i < 3; ++i) t[i] = L[k][9 + i] + tn[i];
  }
  for (int i = 0; i < 9; ++i) F[i] = R[i];
  for (int i = 0; i < 3; ++i) F[9 + i] = t[i];
}

// World placement of geometry g (pin.updateGeometryPlacements); the target
// geometry sits at the solve's cube placement (setcubeplacement).
template <typename T>
IKG_HD inline void geom_world(const KCollision<T>* __restrict__ c, int g, const T (*F)[12], const T* tgt, T* P) {
  if (g == c->target_geom) {
    for (int i = 0; i < 12; ++i) P[i] = tgt[i];
  } else if (c->joint[g] < 0) {
    for (int i = 0; i < 9; ++i) P[i] = c->R[g][i];
    for (int i = 0; i < 3; ++i) P[9 + i] = c->t[g][i];
  } else {
    const T* Fj = F[c->joint[g]];
    T tn[3];
    matmul3(Fj, c->R[g], P);
    matvec3(Fj, c->t[g], tn);
    for (int i = 0; i < 3; ++i) P[9 + i] = Fj[9 + i] + tn[i];
  }
}

// Pair k of the active list: bounding-sphere rejection, then the narrow phase.
template <typename T>
IKG_HD inline bool pair_hit(const KCollision<T>* __restrict__ c, int k, const T (*P)[12]) {
  const int a = c->pairs[k][0], b = c->pairs[k][1];
  const T* Pa = P[a];
  const T* Pb = P[b];
  T d[3] = {Pa[9] - Pb[9], Pa[10] - Pb[10], Pa[11] - Pb[11]};
  const T r = c->brad[a] + c->brad[b];
  if (dot3(d, d) >= r * r) return false;
  const Shape<T> A{Pa, Pa + 9, c->dims[a], c->kind[a]};
  const Shape<T> B{Pb, Pb + 9, c->dims[b], c->kind[b]};
  return pair_collides(A, B);
}

}  // namespace ikg
