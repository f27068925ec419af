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
  T pr2[kMaxPairs];  // per pair: (brad[a] + brad[b])^2, the bounding-sphere test's threshold
  int32_t n_geoms;
  int32_t n_pairs;
  int32_t target_geom;
};

// LDS scratch of one collision check (one wave).
template <typename T>
struct CollideScratch {
  T q[kMaxNq];
  T sn[kMaxNq];      // sin / cos of q (filled by the caller or by collide_wave)
  T cs[kMaxNq];
  int32_t par[kMaxNq];  // jparent staged in LDS
  T L[kMaxNq][12];   // joint-local transforms placement * R_axis(q)
  T F[kMaxNq][12];   // world joint frames
  T P[kMaxGeoms][12];  // world geometry placements
  int16_t cand[kMaxPairs];  // pairs past the bounding-sphere test, in pair order (collide_wave)
};

// Expanding-polytope scratch (epa_depth_lb): at most kEpaIters expansions of
// the starting tetrahedron.
constexpr int kEpaIters = 5;
// continuation -> stretch kernel record per problem: the certified margin,
// Rmot of the root + left arm joints and of (0 +) the right arm's, then the
// certified iterate's values of the same joints per arm
constexpr int kStretchRec = 32;
constexpr int kEpaV = 4 + kEpaIters;
constexpr int kEpaF = 2 * kEpaV - 4;
struct EpaScratch {
  double V[kEpaV][3];
  double N[kEpaF][4];      // face planes: unit outward normal, offset
  int8_t F[kEpaF][3];
  int8_t H[kEpaF + 4][2];  // horizon edges of one expansion (serial form)
  int8_t Fx[kEpaF + 4][2]; // new faces of one expansion (group form)
};

// Witness of the previous check of one problem (LDS): the colliding pair and,
// when its GJK ended on an enclosing tetrahedron, the 4 search directions.
// Continuation only: a certified penetration margin of the witness pair
// (budget, from epa_depth_lb) and the lever arms Rmot of its geometries; the
// IK lanes keep the certified iterate and, while sum_j |q_j - qcert_j| Rmot[j]
// stays below budget, the pair provably still intersects, so the check's
// answer is known.
template <typename T>
struct Witness {
  int32_t pair;     // -1: none
  int32_t cert_ok;  // dir[] valid
  int32_t skip_ok;  // budget valid for this pair
  int32_t epa_wait; // checks before the next certificate attempt
  int32_t gen;      // bumped whenever skip_ok / budget / Rmot change (the IK lanes cache them)
  int32_t epa_go;   // this check's hit asks for a certificate (continuation)
  double budget;
  T Rmot[kMaxNq];   // per joint: lever-arm bound of the two geometries about it
  T gbrad[2];
  EpaScratch epa;
  T dir[12];
  T pts[4][3];
  // the pair's two geometries, cached when the witness is set (continuation)
  int32_t gjoint[2];
  int32_t gkind[2];
  int32_t gtarget[2];
  T gR[2][9];
  T gt[2][3];
  T gdims[2][3];
  T P[2][12];  // their world placements at the current iterate
};

template <typename T>
struct Shape {
  const T* R;  // 9, row-major
  const T* t;  // 3
  const T* dims;
  int kind;
};

// IKG_SUPPORT_RELOAD (default 1): the placement's rotation and translation are
// re-read from LDS at every support call.  Held in registers across the GJK
// loop (the compiler hoists the loads: 2 x 12 values) they took the fp64 check
// kernels -- pre-screen, window boxes, records scan -- past 256 registers
// (248-256 VGPRs + 18 AGPRs: one wave per SIMD); re-read they fit 2 waves
// (244-256 VGPRs, no AGPRs): C4 share + collision 6.97 -> 6.11 ms, C2 + collision
// 1.259 -> 1.248 (profiles/r06/records/reload/).  fp32 (3 waves per SIMD either
// way) keeps the hoisted loads: C3 unchanged, C5 within +-1%.  The values and
// the arithmetic are the same: answers bit for bit.
#ifndef IKG_SUPPORT_RELOAD
#define IKG_SUPPORT_RELOAD 1
#endif
template <typename T>
IKG_HD inline void shape_support(const Shape<T>& s0, const T* d, T* out) {
  Shape<T> s = s0;
#if defined(__HIP_DEVICE_COMPILE__) && IKG_SUPPORT_RELOAD
  if constexpr (sizeof(T) == 8) asm volatile("" : "+v"(s.R), "+v"(s.t));  // opaque pointers: the loads stay in the loop
#endif
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
// The simplex lives in named registers (s1..s3 = older vertices, oldest
// first; `a` = newest); every case below indexes them statically, so nothing
// spills to scratch.  Each vertex carries the search direction that produced
// it, so an enclosing tetrahedron can be handed back as a certificate: the
// four directions whose support points, re-evaluated at nearby poses, are
// checked for enclosure first (tetra_encloses_origin) before a fresh GJK.
template <typename T>
struct GVert {
  T p[3];  // support point of A - B
  T d[3];  // direction it was taken in
};

template <typename T>
IKG_HD inline void cp3(T* d, const T* s) {
  d[0] = s[0];
  d[1] = s[1];
  d[2] = s[2];
}

// [s1, a]: keep the segment or drop to {a}.  Returns true if the origin is on it.
template <typename T>
IKG_HD inline bool gjk_line(const GVert<T>& a, GVert<T>& s1, GVert<T>& s2, int& m, T* dir) {
  const T ao[3] = {-a.p[0], -a.p[1], -a.p[2]};
  const T ab[3] = {s1.p[0] - a.p[0], s1.p[1] - a.p[1], s1.p[2] - a.p[2]};
  if (dot3(ab, ao) > T(0)) {
    s2 = a;
    m = 2;
    triple(ab, ao, ab, dir);
    return dot3(dir, dir) < T(1e-30);
  }
  s1 = a;
  m = 1;
  cp3(dir, ao);
  return false;
}

// [s1 = c, s2 = b, a]
template <typename T>
IKG_HD inline bool gjk_triangle(const GVert<T>& a, GVert<T>& s1, GVert<T>& s2, GVert<T>& s3, int& m, T* dir) {
  const T ao[3] = {-a.p[0], -a.p[1], -a.p[2]};
  T ab[3], ac[3], abc[3], t1[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = s2.p[i] - a.p[i];
    ac[i] = s1.p[i] - a.p[i];
  }
  cross3(ab, ac, abc);
  cross3(abc, ac, t1);
  if (dot3(t1, ao) > T(0)) {
    if (dot3(ac, ao) > T(0)) {  // keep [c, a]
      s2 = a;
      m = 2;
      triple(ac, ao, ac, dir);
      return dot3(dir, dir) < T(1e-30);
    }
    s1 = s2;  // line [b, a]
    return gjk_line(a, s1, s2, m, dir);
  }
  cross3(ab, abc, t1);
  if (dot3(t1, ao) > T(0)) {
    s1 = s2;  // line [b, a]
    return gjk_line(a, s1, s2, m, dir);
  }
  if (dot3(abc, ao) > T(0)) {  // [c, b, a]
    cp3(dir, abc);
  } else {  // [b, c, a]
    const GVert<T> tmp = s1;
    s1 = s2;
    s2 = tmp;
    for (int i = 0; i < 3; ++i) dir[i] = -abc[i];
  }
  s3 = a;
  m = 3;
  return false;
}

// [s1 = d, s2 = c, s3 = b, a]; returns 2 when the tetrahedron encloses the origin.
template <typename T>
IKG_HD inline int gjk_tetra(const GVert<T>& a, GVert<T>& s1, GVert<T>& s2, GVert<T>& s3, int& m, T* dir) {
  const T ao[3] = {-a.p[0], -a.p[1], -a.p[2]};
  T ab[3], ac[3], ad[3], f[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = s3.p[i] - a.p[i];
    ac[i] = s2.p[i] - a.p[i];
    ad[i] = s1.p[i] - a.p[i];
  }
  cross3(ab, ac, f);
  if (dot3(f, ao) > T(0)) {  // triangle [c, b, a]
    s1 = s2;
    s2 = s3;
    return gjk_triangle(a, s1, s2, s3, m, dir) ? 1 : 0;
  }
  cross3(ac, ad, f);
  if (dot3(f, ao) > T(0)) return gjk_triangle(a, s1, s2, s3, m, dir) ? 1 : 0;  // triangle [d, c, a]
  cross3(ad, ab, f);
  if (dot3(f, ao) > T(0)) {  // triangle [b, d, a]
    s2 = s1;
    s1 = s3;
    return gjk_triangle(a, s1, s2, s3, m, dir) ? 1 : 0;
  }
  return 2;  // origin enclosed
}

template <typename T>
IKG_HD inline void mink_support(const Shape<T>& A, const Shape<T>& B, const T* dir, T* out) {
  T pa[3], pb[3], nd[3] = {-dir[0], -dir[1], -dir[2]};
  shape_support(A, dir, pa);
  shape_support(B, nd, pb);
  for (int i = 0; i < 3; ++i) out[i] = pa[i] - pb[i];
}

// 0: separated; 1: intersecting; 2: intersecting with `cert` (12 values = the
// 4 search directions of an origin-enclosing tetrahedron) filled when non-null.
template <typename T>
IKG_HD inline int gjk_intersect(const Shape<T>& A, const Shape<T>& B, T* cert = nullptr) {
  GVert<T> s1, s2, s3, a;
  T d[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
  if (dot3(d, d) == T(0)) d[0] = T(1);
  cp3(s1.d, d);
  mink_support(A, B, d, s1.p);
  int m = 1;
  for (int i = 0; i < 3; ++i) d[i] = -s1.p[i];
  for (int iter = 0; iter < kGjkIters; ++iter) {
    if (dot3(d, d) < T(1e-30)) return 1;
    cp3(a.d, d);
    mink_support(A, B, d, a.p);
    if (dot3(a.p, d) < T(0)) return 0;  // separating direction
    int in;
    if (m == 1)
      in = gjk_line(a, s1, s2, m, d) ? 1 : 0;
    else if (m == 2)
      in = gjk_triangle(a, s1, s2, s3, m, d) ? 1 : 0;
    else
      in = gjk_tetra(a, s1, s2, s3, m, d);
    if (in == 2 && cert) {
      cp3(cert, s1.d);
      cp3(cert + 3, s2.d);
      cp3(cert + 6, s3.d);
      cp3(cert + 9, a.d);
    }
    if (in) return in;
  }
  return 1;  // iteration cap: treat as touching
}

// Strict origin-in-tetrahedron test (barycentric signs): a certificate that
// the convex set holding the four points, here A - B, contains the origin.
template <typename T>
IKG_HD inline bool tetra_encloses_origin(const T* P0, const T* P1, const T* P2, const T* P3) {
  auto vol = [](const T* a, const T* b, const T* c, const T* d) {
    T u[3], v[3], w[3], x[3];
    for (int i = 0; i < 3; ++i) {
      u[i] = b[i] - a[i];
      v[i] = c[i] - a[i];
      w[i] = d[i] - a[i];
    }
    cross3(u, v, x);
    return dot3(x, w);
  };
  const T O[3] = {T(0), T(0), T(0)};
  const T V = vol(P0, P1, P2, P3);
  if (V == T(0)) return false;
  return vol(O, P1, P2, P3) * V > T(0) && vol(P0, O, P2, P3) * V > T(0) && vol(P0, P1, O, P3) * V > T(0) &&
         vol(P0, P1, P2, O) * V > T(0);
}

// Certified lower bound on the penetration depth of two intersecting convex
// shapes: the expanding polytope algorithm (EPA) started from an
// origin-enclosing tetrahedron P of support points of A - B.  Every vertex is
// a support point, so the polytope lies inside A - B; with the origin inside
// it, the ball of radius min over faces of the plane distance lies inside
// A - B too, i.e. translating either shape by less than that keeps them
// intersecting (for any rigid motion: every point moving by less than the
// bound keeps h_{A-B}(u) > 0 for all u).  A few expansions along the closest
// face's normal approach the true depth fast (round-1 probe on the
// colliding fixtures: ~90% after 4).  Returns 0 when no certificate results
// (degenerate or non-convex numerics: the final polytope is verified).
template <typename T>
IKG_HD inline double epa_depth_lb(const Shape<T>& A, const Shape<T>& B, const T (*P)[3], EpaScratch& s) {
  for (int v = 0; v < 4; ++v)
    for (int i = 0; i < 3; ++i) s.V[v][i] = (double)P[v][i];
  int nV = 4, nF = 4;
  // plane of face f into s.N[f]; false if degenerate
  auto plane = [&](int f) {
    const double *a = s.V[s.F[f][0]], *b = s.V[s.F[f][1]], *c = s.V[s.F[f][2]];
    const double u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, w[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
    double n[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
    const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    if (!(nn > 1e-300)) return false;
    const double r = 1.0 / nn;
    for (int i = 0; i < 3; ++i) s.N[f][i] = n[i] * r;
    s.N[f][3] = s.N[f][0] * a[0] + s.N[f][1] * a[1] + s.N[f][2] * a[2];
    return true;
  };
  const int8_t F0[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  double cen[3];
  for (int i = 0; i < 3; ++i) cen[i] = 0.25 * (s.V[0][i] + s.V[1][i] + s.V[2][i] + s.V[3][i]);
  for (int f = 0; f < 4; ++f) {
    for (int k = 0; k < 3; ++k) s.F[f][k] = F0[f][k];
    if (!plane(f)) return 0.0;
    if (s.N[f][0] * cen[0] + s.N[f][1] * cen[1] + s.N[f][2] * cen[2] > s.N[f][3]) {  // inward: flip
      const int8_t t = s.F[f][1];
      s.F[f][1] = s.F[f][2];
      s.F[f][2] = t;
      for (int i = 0; i < 4; ++i) s.N[f][i] = -s.N[f][i];
    }
  }
  double best = 0.0, scale = 0.0;
  for (int v = 0; v < 4; ++v)
    for (int i = 0; i < 3; ++i) scale = fmax(scale, fabs(s.V[v][i]));
  for (int it = 0;; ++it) {
    int fmin = 0;
    for (int f = 1; f < nF; ++f)
      if (s.N[f][3] < s.N[fmin][3]) fmin = f;
    const double dmin = s.N[fmin][3];
    if (!(dmin >= 0.0)) return 0.0;  // the origin is not inside
    best = dmin;
    if (it == kEpaIters || nV == kEpaV) break;
    T dir[3] = {(T)s.N[fmin][0], (T)s.N[fmin][1], (T)s.N[fmin][2]}, wt[3];
    mink_support(A, B, dir, wt);
    const double w[3] = {(double)wt[0], (double)wt[1], (double)wt[2]};
    if (w[0] * s.N[fmin][0] + w[1] * s.N[fmin][1] + w[2] * s.N[fmin][2] - dmin <= 1e-12 * scale) break;
    bool vis[kEpaF];
    int nvis = 0;
    for (int f = 0; f < nF; ++f) {
      vis[f] = s.N[f][0] * w[0] + s.N[f][1] * w[1] + s.N[f][2] * w[2] - s.N[f][3] > 1e-14 * scale;
      nvis += vis[f];
    }
    if (!vis[fmin]) break;
    int nH = 0;
    bool overflow = false;
    for (int f = 0; f < nF && !overflow; ++f) {
      if (!vis[f]) continue;
      for (int e = 0; e < 3; ++e) {
        const int8_t a = s.F[f][e], b = s.F[f][(e + 1) % 3];
        bool shared = false;
        for (int g = 0; g < nF && !shared; ++g) {
          if (g == f || !vis[g]) continue;
          for (int e2 = 0; e2 < 3; ++e2)
            if (s.F[g][e2] == b && s.F[g][(e2 + 1) % 3] == a) shared = true;
        }
        if (!shared) {
          if (nH == kEpaF + 4) {
            overflow = true;
            break;
          }
          s.H[nH][0] = a;
          s.H[nH][1] = b;
          ++nH;
        }
      }
    }
    if (overflow || nF - nvis + nH > kEpaF) break;  // the current polytope stays valid
    int k = 0;
    for (int f = 0; f < nF; ++f) {  // drop the visible faces
      if (vis[f]) continue;
      for (int e = 0; e < 3; ++e) s.F[k][e] = s.F[f][e];
      for (int i = 0; i < 4; ++i) s.N[k][i] = s.N[f][i];
      ++k;
    }
    for (int i = 0; i < 3; ++i) s.V[nV][i] = w[i];
    for (int h = 0; h < nH; ++h) {
      s.F[k][0] = s.H[h][0];
      s.F[k][1] = s.H[h][1];
      s.F[k][2] = (int8_t)nV;
      if (!plane(k)) return 0.0;
      ++k;
    }
    nF = k;
    ++nV;
    for (int i = 0; i < 3; ++i) scale = fmax(scale, fabs(w[i]));
  }
  // verify: every vertex on the inner side of every face plane (convex hull)
  for (int f = 0; f < nF; ++f)
    for (int v = 0; v < nV; ++v)
      if (s.N[f][0] * s.V[v][0] + s.N[f][1] * s.V[v][1] + s.N[f][2] * s.V[v][2] - s.N[f][3] > 1e-9 * scale)
        return 0.0;
  return best;
}

// Narrow phase of one pair (hpp-fcl collide(): intersection <=> collision).
// `cert` as for gjk_intersect (only GJK pairs produce one).
template <typename T>
IKG_HD inline int pair_collides(const Shape<T>& A, const Shape<T>& B, T* cert = nullptr) {
  if (A.kind == kSphere && B.kind == kSphere) {
    T d[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
    const T r = A.dims[0] + B.dims[0];
    return dot3(d, d) < r * r ? 1 : 0;
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
      return e2 < S.dims[0] * S.dims[0] ? 1 : 0;
    }
  }
  return gjk_intersect(A, B, cert);
}

// ---------------------------------------------------------------- distance
// hpp-fcl computeDistance().min_distance for one pair (tools.py:37-51,
// distanceToObstacle): the Euclidean distance between two separated convex
// shapes.  Spheres are handled as their centre point (radius subtracted at
// the end), a sphere against a box exactly; everything else by GJK with the
// closest point of the simplex computed by Voronoi-region tests (Ericson,
// Real-Time Collision Detection §5.1).  Returns <= 0 when the shapes
// intersect (the reference only queries collision-free configurations).
template <typename T>
struct DSimplex {
  T w[4][3];
  int n;
};

// Closest point to the origin of segment [a, b]; keeps the supporting subset.
template <typename T>
IKG_HD inline void closest_seg(DSimplex<T>& S, T* v) {
  const T* a = S.w[0];
  const T* b = S.w[1];
  T ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const T t = -dot3(a, ab);
  const T l2 = dot3(ab, ab);
  if (t <= T(0) || l2 <= T(0)) {
    S.n = 1;
    cp3(v, a);
    return;
  }
  if (t >= l2) {
    S.n = 1;
    cp3(S.w[0], b);
    cp3(v, b);
    return;
  }
  const T u = t / l2;
  for (int i = 0; i < 3; ++i) v[i] = a[i] + u * ab[i];
}

// Closest point to the origin of segment [a, b] (no simplex bookkeeping).
template <typename T>
IKG_HD inline void seg_point(const T* a, const T* b, T* v, T& t_out) {
  T ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const T l2 = dot3(ab, ab);
  T t = l2 > T(0) ? -dot3(a, ab) / l2 : T(0);
  t = fmin(fmax(t, T(0)), T(1));
  t_out = t;
  for (int i = 0; i < 3; ++i) v[i] = a[i] + t * ab[i];
}

// Closest point to the origin of triangle (a, b, c) (Ericson 5.1.5, p = 0);
// region: 0/1/2 vertex a/b/c, 3 edge ab, 4 edge ac, 5 edge bc, 6 face.  A
// degenerate (zero-area) triangle resolves to the closest of its edges.
template <typename T>
IKG_HD inline void closest_tri(const T* a, const T* b, const T* c, T* v, int& region) {
  T ab[3], ac[3], ap[3];
  for (int i = 0; i < 3; ++i) {
    ab[i] = b[i] - a[i];
    ac[i] = c[i] - a[i];
    ap[i] = -a[i];
  }
  T n[3];
  cross3(ab, ac, n);
  const T scale = dot3(ab, ab) * dot3(ac, ac);
  if (!(dot3(n, n) > T(1e-24) * scale)) {  // degenerate: best edge
    T v1[3], v2[3], v3[3], t1, t2, t3;
    seg_point(a, b, v1, t1);
    seg_point(a, c, v2, t2);
    seg_point(b, c, v3, t3);
    const T d1 = dot3(v1, v1), d2 = dot3(v2, v2), d3 = dot3(v3, v3);
    if (d1 <= d2 && d1 <= d3) {
      cp3(v, v1);
      region = t1 <= T(0) ? 0 : (t1 >= T(1) ? 1 : 3);
    } else if (d2 <= d3) {
      cp3(v, v2);
      region = t2 <= T(0) ? 0 : (t2 >= T(1) ? 2 : 4);
    } else {
      cp3(v, v3);
      region = t3 <= T(0) ? 1 : (t3 >= T(1) ? 2 : 5);
    }
    return;
  }
  const T d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= T(0) && d2 <= T(0)) {
    region = 0;
    cp3(v, a);
    return;
  }
  T bp[3] = {-b[0], -b[1], -b[2]};
  const T d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= T(0) && d4 <= d3) {
    region = 1;
    cp3(v, b);
    return;
  }
  const T vc = d1 * d4 - d3 * d2;
  if (vc <= T(0) && d1 >= T(0) && d3 <= T(0)) {
    const T u = d1 / (d1 - d3);
    region = 3;
    for (int i = 0; i < 3; ++i) v[i] = a[i] + u * ab[i];
    return;
  }
  T cpn[3] = {-c[0], -c[1], -c[2]};
  const T d5 = dot3(ab, cpn), d6 = dot3(ac, cpn);
  if (d6 >= T(0) && d5 <= d6) {
    region = 2;
    cp3(v, c);
    return;
  }
  const T vb = d5 * d2 - d1 * d6;
  if (vb <= T(0) && d2 >= T(0) && d6 <= T(0)) {
    const T w_ = d2 / (d2 - d6);
    region = 4;
    for (int i = 0; i < 3; ++i) v[i] = a[i] + w_ * ac[i];
    return;
  }
  const T va = d3 * d6 - d5 * d4;
  if (va <= T(0) && (d4 - d3) >= T(0) && (d5 - d6) >= T(0)) {
    const T w_ = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    region = 5;
    for (int i = 0; i < 3; ++i) v[i] = b[i] + w_ * (c[i] - b[i]);
    return;
  }
  const T den = T(1) / (va + vb + vc);
  const T u = vb * den, w_ = vc * den;
  region = 6;
  for (int i = 0; i < 3; ++i) v[i] = a[i] + ab[i] * u + ac[i] * w_;
}

// Reduce S (a triangle, w[0..2]) to the supporting feature of its closest point.
template <typename T>
IKG_HD inline void closest_tri_reduce(DSimplex<T>& S, T* v) {
  int region = 6;
  closest_tri(S.w[0], S.w[1], S.w[2], v, region);
  switch (region) {
    case 0: S.n = 1; break;
    case 1: S.n = 1; cp3(S.w[0], S.w[1]); break;
    case 2: S.n = 1; cp3(S.w[0], S.w[2]); break;
    case 3: S.n = 2; break;
    case 4: S.n = 2; cp3(S.w[1], S.w[2]); break;
    case 5: S.n = 2; cp3(S.w[0], S.w[2]); break;  // (c, b)
    default: S.n = 3; break;
  }
}

// Tetrahedron w[0..3]: origin inside -> intersecting (returns true);
// otherwise the closest point over its faces (all four when the tetrahedron
// is flat, e.g. a triangle extended by a coplanar box corner; else those
// facing the origin), reduced to that face's supporting feature.
template <typename T>
IKG_HD inline bool closest_tet_reduce(DSimplex<T>& S, T* v) {
  const int face[4][4] = {{0, 1, 2, 3}, {0, 2, 3, 1}, {0, 3, 1, 2}, {1, 3, 2, 0}};  // 3 verts + opposite
  T e1[3], e2[3], e3[3], cr[3];
  for (int i = 0; i < 3; ++i) {
    e1[i] = S.w[1][i] - S.w[0][i];
    e2[i] = S.w[2][i] - S.w[0][i];
    e3[i] = S.w[3][i] - S.w[0][i];
  }
  cross3(e2, e3, cr);
  const T vol = dot3(e1, cr);
  const T l = fmax(fmax(dot3(e1, e1), dot3(e2, e2)), dot3(e3, e3));
  const bool flat = !(vol * vol > T(1e-24) * l * l * l);
  bool inside = !flat;
  T best = T(0);
  int best_f = -1;
  for (int f = 0; f < 4; ++f) {
    const T* a = S.w[face[f][0]];
    const T* b = S.w[face[f][1]];
    const T* c = S.w[face[f][2]];
    const T* d = S.w[face[f][3]];
    if (!flat) {
      T ab[3], ac[3], n[3];
      for (int i = 0; i < 3; ++i) {
        ab[i] = b[i] - a[i];
        ac[i] = c[i] - a[i];
      }
      cross3(ab, ac, n);
      T ad[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
      const T sd = dot3(n, ad);  // opposite vertex side
      const T so = -dot3(n, a);  // origin side
      if (so * sd >= T(0)) continue;  // origin on the inner side of this face
      inside = false;
    }
    T fv[3];
    int region = 6;
    closest_tri(a, b, c, fv, region);
    const T d2 = dot3(fv, fv);
    if (best_f < 0 || d2 < best) {
      best = d2;
      best_f = f;
    }
  }
  if (inside) return true;
  T a[3], b[3], c[3];
  cp3(a, S.w[face[best_f][0]]);
  cp3(b, S.w[face[best_f][1]]);
  cp3(c, S.w[face[best_f][2]]);
  cp3(S.w[0], a);
  cp3(S.w[1], b);
  cp3(S.w[2], c);
  S.n = 3;
  closest_tri_reduce(S, v);
  return false;
}

template <typename T>
IKG_HD inline T gjk_distance_raw(const Shape<T>& A, const Shape<T>& B) {
  DSimplex<T> S;
  T v[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
  if (dot3(v, v) == T(0)) v[0] = T(1);
  {
    T d[3] = {-v[0], -v[1], -v[2]};
    mink_support(A, B, d, S.w[0]);
  }
  S.n = 1;
  cp3(v, S.w[0]);
  const T eps_rel = sizeof(T) == 8 ? T(1e-12) : T(1e-6);
  for (int it = 0; it < 64; ++it) {
    const T vv = dot3(v, v);
    if (vv <= (sizeof(T) == 8 ? T(1e-30) : T(1e-14))) return T(0);  // origin on the simplex: touching
    T d[3] = {-v[0], -v[1], -v[2]}, w[3];
    mink_support(A, B, d, w);
    if (vv - dot3(v, w) <= eps_rel * vv) break;  // no progress towards the origin: |v| is the distance
    // the new point is never already in the simplex once it made progress
    cp3(S.w[S.n == 1 ? 1 : (S.n == 2 ? 2 : 3)], w);
    S.n += 1;
    T vn[3];
    if (S.n == 2) {
      closest_seg(S, vn);
    } else if (S.n == 3) {
      closest_tri_reduce(S, vn);
    } else if (closest_tet_reduce(S, vn)) {
      return T(0);  // origin inside: intersecting
    }
    if (!(dot3(vn, vn) < vv)) break;  // rounding stall: keep the best point found
    cp3(v, vn);
  }
  return sqrt(dot3(v, v));
}

// distance of one pair (min_distance of hpp-fcl's DistanceResult)
template <typename T>
IKG_HD inline T pair_distance(const Shape<T>& A, const Shape<T>& B) {
  if (A.kind == kSphere && B.kind == kSphere) {
    T d[3] = {A.t[0] - B.t[0], A.t[1] - B.t[1], A.t[2] - B.t[2]};
    return sqrt(dot3(d, d)) - A.dims[0] - B.dims[0];
  }
  if ((A.kind == kSphere) != (B.kind == kSphere)) {
    const Shape<T>& Sp = A.kind == kSphere ? A : B;
    const Shape<T>& X = A.kind == kSphere ? B : A;
    if (X.kind == kBox || X.kind == kMeshBox) {  // exact: closest point on the box
      T d[3] = {Sp.t[0] - X.t[0], Sp.t[1] - X.t[1], Sp.t[2] - X.t[2]}, p[3];
      matvec3_t(X.R, d, p);
      T e2 = T(0);
      for (int i = 0; i < 3; ++i) {
        const T c = fmin(fmax(p[i], -X.dims[i]), X.dims[i]);
        e2 += (p[i] - c) * (p[i] - c);
      }
      return sqrt(e2) - Sp.dims[0];
    }
    const T zero[3] = {T(0), T(0), T(0)};
    const Shape<T> P{Sp.R, Sp.t, zero, kSphere};  // the centre: a sphere of radius 0
    return gjk_distance_raw(P, X) - Sp.dims[0];
  }
  return gjk_distance_raw(A, B);
}

// ---------------------------------------------------------------- check stages
// The stages of one check, shared by the wave-parallel driver (collide_wave,
// ikg_collision.hip) and the host emulator.  Frames are [R(9) row-major, t(3)].

// Joint-local transform placement * R_axis(q_j) (JointModelR*::calc), given
// (s, co) = sincos(q_j).
template <typename T>
IKG_HD inline void joint_local(const KModel<T>* __restrict__ m, int j, T s, T co, T* L) {
  T R[9];
  for (int i = 0; i < 9; ++i) R[i] = m->jR[j][i];
  rotate_axis(R, m->jaxis[j], s, co);
  for (int i = 0; i < 9; ++i) L[i] = R[i];
  for (int i = 0; i < 3; ++i) L[9 + i] = m->jt[j][i];
}

// World frame of joint j (oMi): compose the local transforms up the parent
// chain (`par` = jparent, staged wherever the caller keeps it).
template <typename T>
IKG_HD inline void joint_world(const int32_t* par, int j, const T (*L)[12], T* F) {
  T R[9], t[3];
  for (int i = 0; i < 9; ++i) R[i] = L[j][i];
  for (int i = 0; i < 3; ++i) t[i] = L[j][9 + i];
  for (int k = par[j]; k >= 0; k = par[k]) {
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
IKG_HD inline int pair_hit(const KCollision<T>* __restrict__ c, int k, const T (*P)[12], T* cert = nullptr) {
  const int a = c->pairs[k][0], b = c->pairs[k][1];
  const T* Pa = P[a];
  const T* Pb = P[b];
  T d[3] = {Pa[9] - Pb[9], Pa[10] - Pb[10], Pa[11] - Pb[11]};
  const T r = c->brad[a] + c->brad[b];
  if (dot3(d, d) >= r * r) return 0;
  const Shape<T> A{Pa, Pa + 9, c->dims[a], c->kind[a]};
  const Shape<T> B{Pb, Pb + 9, c->dims[b], c->kind[b]};
  return pair_collides(A, B, cert);
}

template <typename T>
IKG_HD inline Shape<T> pair_shape(const KCollision<T>* __restrict__ c, int g, const T (*P)[12]) {
  return Shape<T>{P[g], P[g] + 9, c->dims[g], c->kind[g]};
}

// ---------------------------------------------------------------- inscribed-ball certificate
// A cheap proof that a colliding pair still collides after the joints moved
// (the records scan, ikg_collision.hip traj_scan_body):
//  * at a certified iterate c, a point p inside both geometries and the radius
//    r of a ball around p inside both (shape_depth: exact for the primitives);
//  * the two geometries move relative to the joint frame of their lowest
//    common ancestor only through the joints below it.  Moving those joints
//    from q_c to q one at a time, distal first, rotates a geometry about each
//    joint's axis at its q_c position, so the point of the geometry that ends
//    at p travels a path D with D <= sum_k |dq_k| (|p - o_k| + D) (o_k: joint
//    k's origin at q_c): D <= S1 / (1 - S0), S1 = sum_k |dq_k| |p - o_k|,
//    S0 = sum_k |dq_k|.  If S1 + r S0 < r for both geometries, D < r, that
//    point was inside the ball, hence inside the geometry at q_c, and p lies in
//    both geometries at q: the pair intersects there and collision(q) is True
//    (the OR over all pairs), with no narrow phase.
// r is taken net of the placements' rounding (1e-9 fp64, 1e-5 fp32, as the
// EPA certificate); a certificate with r <= 0 proves nothing.

// Radius of the largest ball around x inside the primitive (negative outside).
template <typename T>
IKG_HD inline T shape_depth(const Shape<T>& s, const T* x) {
  const T d[3] = {x[0] - s.t[0], x[1] - s.t[1], x[2] - s.t[2]};
  if (s.kind == kSphere) return s.dims[0] - sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  T l[3];
  matvec3_t(s.R, d, l);  // R^T d
  if (s.kind == kCylinder) {
    const T rad = sqrt(l[0] * l[0] + l[1] * l[1]);
    return fmin(s.dims[0] - rad, s.dims[1] - fabs(l[2]));
  }
  return fmin(fmin(s.dims[0] - fabs(l[0]), s.dims[1] - fabs(l[1])), s.dims[2] - fabs(l[2]));
}

// The primitive's core: a segment [a, b] every point of which carries a ball
// of radius rho inside the shape (sphere: its centre; cylinder: the axis
// shortened by rho at both ends, rho = min(R, half length); box: the longest
// axis shortened likewise, rho = the smallest half extent).
template <typename T>
IKG_HD inline void shape_core(const Shape<T>& s, T* a, T* b, T& rho) {
  int k = 2;
  T half = T(0);
  rho = s.dims[0];
  if (s.kind == kCylinder) {
    rho = fmin(s.dims[0], s.dims[1]);
    half = s.dims[1] - rho;
  } else if (s.kind != kSphere) {
    k = s.dims[0] >= s.dims[1] ? (s.dims[0] >= s.dims[2] ? 0 : 2) : (s.dims[1] >= s.dims[2] ? 1 : 2);
    rho = fmin(fmin(s.dims[0], s.dims[1]), s.dims[2]);
    half = s.dims[k] - rho;
  }
  for (int i = 0; i < 3; ++i) {
    const T ax = s.kind == kSphere ? T(0) : s.R[3 * i + k];  // column k: the local axis in the world
    a[i] = s.t[i] - half * ax;
    b[i] = s.t[i] + half * ax;
  }
}

// Closest points s = a0 + u (a1 - a0), t = b0 + v (b1 - b0) of two segments.
template <typename T>
IKG_HD inline void closest_segments(const T* a0, const T* a1, const T* b0, const T* b1, T* s, T* t) {
  T d1[3], d2[3], r[3];
  for (int i = 0; i < 3; ++i) {
    d1[i] = a1[i] - a0[i];
    d2[i] = b1[i] - b0[i];
    r[i] = a0[i] - b0[i];
  }
  const T a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  const T tiny = T(1e-24);
  T u = T(0), v = T(0);
  if (a <= tiny && e <= tiny) {
  } else if (a <= tiny) {
    v = fmin(fmax(f / e, T(0)), T(1));
  } else {
    const T cc = dot3(d1, r);
    if (e <= tiny) {
      u = fmin(fmax(-cc / a, T(0)), T(1));
    } else {
      const T bb = dot3(d1, d2), den = a * e - bb * bb;
      u = den > tiny ? fmin(fmax((bb * f - cc * e) / den, T(0)), T(1)) : T(0);
      v = (bb * u + f) / e;
      if (v < T(0)) {
        v = T(0);
        u = fmin(fmax(-cc / a, T(0)), T(1));
      } else if (v > T(1)) {
        v = T(1);
        u = fmin(fmax((bb - cc) / a, T(0)), T(1));
      }
    }
  }
  for (int i = 0; i < 3; ++i) {
    s[i] = a0[i] + u * d1[i];
    t[i] = b0[i] + v * d2[i];
  }
}

// The primitive's interior as at most 6 concave constraints c_k(x) >= 0 (the
// depth is their minimum) and their gradients: box faces h_i -+ l_i, cylinder
// radius R - |l_xy| and caps h -+ l_z, sphere R - |x - c|.  Unused slots get
// a large value so they never bind.
template <typename T>
IKG_HD inline void shape_constraints(const Shape<T>& s, const T* x, T (&c)[6], T (&g)[6][3]) {
  const T d[3] = {x[0] - s.t[0], x[1] - s.t[1], x[2] - s.t[2]};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    c[k] = T(1e30);
    g[k][0] = g[k][1] = g[k][2] = T(0);
  }
  if (s.kind == kSphere) {
    const T n = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    const T f = n > T(0) ? T(-1) / n : T(0);
    c[0] = s.dims[0] - n;
#pragma unroll
    for (int i = 0; i < 3; ++i) g[0][i] = f * d[i];
    return;
  }
  T l[3];
  matvec3_t(s.R, d, l);
  if (s.kind == kCylinder) {
    const T rad = sqrt(l[0] * l[0] + l[1] * l[1]);
    const T f = rad > T(0) ? T(-1) / rad : T(0);
    c[0] = s.dims[0] - rad;
    c[1] = s.dims[1] - l[2];
    c[2] = s.dims[1] + l[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      g[0][i] = f * (s.R[3 * i] * l[0] + s.R[3 * i + 1] * l[1]);
      g[1][i] = -s.R[3 * i + 2];
      g[2][i] = s.R[3 * i + 2];
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    c[2 * a] = s.dims[a] - l[a];
    c[2 * a + 1] = s.dims[a] + l[a];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      g[2 * a][i] = -s.R[3 * i + a];
      g[2 * a + 1][i] = s.R[3 * i + a];
    }
  }
}

// Certificate point search, in fp32 whatever the solve's type (it only has to
// find a good point; its depth is then evaluated exactly): ascent on a soft
// minimum of the two shapes' constraints towards the Chebyshev centre of
// A n B (weights max(0, 1 - (c_k - min)/tau)^2 -- no transcendental -- with the
// softness and the step shrinking geometrically), from one of kCertStarts
// starting points: start 0 is the best of the two centres, their midpoint and
// the point between the closest points of the two cores where the cores' depth
// estimates meet; start s > 0 is one of those four moved by half the smaller
// core radius along an axis of either shape.  The wave runs one start per lane
// and keeps the deepest (traj_scan_body); deep_common_point runs them in turn.
constexpr int kCertStarts = 64;
constexpr int kCertIters = 8;

IKG_HD inline void deep_point_from(const Shape<float>& A, const Shape<float>& B, int start, float* p) {
  float a0[3], a1[3], b0[3], b1[3], ra, rb, s[3], t[3];
  shape_core(A, a0, a1, ra);
  shape_core(B, b0, b1, rb);
  closest_segments(a0, a1, b0, b1, s, t);
  float D = 0.f;
  for (int i = 0; i < 3; ++i) D += (t[i] - s[i]) * (t[i] - s[i]);
  D = sqrtf(D);
  const float fm = D > 0.f ? fminf(fmaxf((D + ra - rb) / (2.f * D), 0.f), 1.f) : 0.5f;
  // the candidates and the start's choice by selects, never a run-time index
  // into a private array (that put the arrays in scratch memory: ~6.6 KB of
  // scratch traffic per certificate wave)
  float best = -1e30f, base[4][3];
  int bi = 0;
#pragma unroll
  for (int cnd = 0; cnd < 4; ++cnd) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      base[cnd][i] = cnd == 0 ? s[i] + fm * (t[i] - s[i]) : cnd == 1 ? A.t[i] : cnd == 2 ? B.t[i]
                                                                       : 0.5f * (A.t[i] + B.t[i]);
    const float r = fminf(shape_depth(A, base[cnd]), shape_depth(B, base[cnd]));
    if (r > best) {
      best = r;
      bi = cnd;
    }
  }
  const int b = start == 0 ? bi : start & 3;
  float x[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) x[i] = b == 0 ? base[0][i] : b == 1 ? base[1][i] : b == 2 ? base[2][i] : base[3][i];
  if (start != 0) {
    const int j = (start >> 2) % 3, side = (start / 12) & 1, sg = (start / 24) & 1;
    const float mag = 0.5f * fmaxf(fminf(ra, rb), 1e-3f) * (1.f + (float)(start / 48));
    const int kind = side ? B.kind : A.kind;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float ra0 = A.R[3 * i], ra1 = A.R[3 * i + 1], ra2 = A.R[3 * i + 2];
      const float rb0 = B.R[3 * i], rb1 = B.R[3 * i + 1], rb2 = B.R[3 * i + 2];
      const float axis = j == 0 ? (side ? rb0 : ra0) : j == 1 ? (side ? rb1 : ra1) : (side ? rb2 : ra2);
      x[i] = x[i] + (sg ? -mag : mag) * (kind == kSphere ? (i == j ? 1.f : 0.f) : axis);
    }
  }
  float scale = 0.f;
  for (int i = 0; i < 3; ++i) scale = fmaxf(scale, fmaxf(A.dims[i], B.dims[i]));
  float tau = 0.2f * scale, eta = 0.5f * scale;
  best = -1e30f;
  for (int i = 0; i < 3; ++i) p[i] = x[i];
  for (int it = 0; it <= kCertIters; ++it) {
    float ca[6], ga[6][3], cb[6], gb[6][3];
    shape_constraints(A, x, ca, ga);
    shape_constraints(B, x, cb, gb);
    float m = ca[0];
#pragma unroll
    for (int k = 0; k < 6; ++k) m = fminf(m, fminf(ca[k], cb[k]));
    if (m > best) {
      best = m;
      for (int i = 0; i < 3; ++i) p[i] = x[i];
    }
    if (it == kCertIters) break;
    const float itau = 1.f / tau;
    float u[3] = {0.f, 0.f, 0.f}, wsum = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      float wa = fmaxf(1.f - (ca[k] - m) * itau, 0.f), wb = fmaxf(1.f - (cb[k] - m) * itau, 0.f);
      wa *= wa;
      wb *= wb;
      wsum += wa + wb;
#pragma unroll
      for (int i = 0; i < 3; ++i) u[i] += wa * ga[k][i] + wb * gb[k][i];
    }
    const float f = eta / wsum;  // wsum >= 1: the binding constraint weighs 1
    for (int i = 0; i < 3; ++i) x[i] += f * u[i];
    tau *= 0.7f;
    eta *= 0.8f;
  }
}

// fp32 copies of a shape's placement and dimensions (for the search)
template <typename T>
IKG_HD inline void shape_f32(const Shape<T>& S, float* R, float* t, float* d) {
  for (int i = 0; i < 9; ++i) R[i] = (float)S.R[i];
  for (int i = 0; i < 3; ++i) {
    t[i] = (float)S.t[i];
    d[i] = (float)S.dims[i];
  }
}

// Start `start`'s point and its exact ball radius in both shapes (in T).
template <typename T>
IKG_HD inline T deep_point_depth(const Shape<T>& A, const Shape<T>& B, int start, T* p) {
  float RA[9], tA[3], dA[3], RB[9], tB[3], dB[3], pf[3];
  shape_f32(A, RA, tA, dA);
  shape_f32(B, RB, tB, dB);
  const Shape<float> Af{RA, tA, dA, A.kind}, Bf{RB, tB, dB, B.kind};
  deep_point_from(Af, Bf, start, pf);
  for (int i = 0; i < 3; ++i) p[i] = T(pf[i]);
  return fmin(shape_depth(A, p), shape_depth(B, p));
}

// A point deep inside both shapes and the radius of the ball around it that
// lies in both (<= 0: none found): the deepest of the kCertStarts searches
// (ties: the lowest start), as the wave's reduction picks it.  The depth of
// every point is evaluated exactly, so the search only decides how large the
// certified radius is, never whether it holds (on random colliding fixture
// poses it finds a positive radius for ~97% of the colliding pairs; a full
// optimiser: all of them).
template <typename T>
IKG_HD inline T deep_common_point(const Shape<T>& A, const Shape<T>& B, T* p) {
  T best = T(-1e30);
  for (int st = 0; st < kCertStarts; ++st) {
    T x[3];
    const T r = deep_point_depth(A, B, st, x);
    if (r > best) {
      best = r;
      for (int i = 0; i < 3; ++i) p[i] = x[i];
    }
  }
  return best;
}

// Certificate of one pair at one iterate: the joints below the pair's common
// ancestor with their values at the iterate and lever arms |p - o_k|.
constexpr int kCertJoints = kMaxNq;  // the two branches below the common ancestor are disjoint
constexpr int kCoverBatch = 16;  // ball_covers' one batch of loads (two 6-7-joint chains fit)
template <typename T>
struct BallCert {
  T r;  // certified radius, net of rounding; <= 0: no certificate
  int32_t n;
  int32_t joint[kCertJoints];
  int32_t side[kCertJoints];  // which geometry the joint moves
  int32_t off[kCertJoints];   // the joint's column in q (sl[joint]); entries n .. kCoverBatch - 1: zero
  T qc[kCertJoints];
  T lev[kCertJoints];
  // working state (LDS in the scan, where dynamically indexed per-lane arrays
  // would live in scratch memory): the pair's joint chains, the joint origins
  // and the two placements (the chains' local transforms go to a workspace of
  // kMaxNq x 12 the caller passes: the scan's collision scratch)
  int32_t g[2];                 // the pair's geometries
  int32_t lca;                  // their joints' lowest common ancestor (-1: none)
  int32_t nl[3];                // chain lengths: root .. lca, lca .. geometry 0, lca .. geometry 1
  int32_t ok;                   // the chains fit the workspace (a tree of at most kMaxNq joints)
  int32_t list[3][kMaxNq];      // each chain, leaf first (joint indices)
  T org[kCertJoints][3];        // joint origins at the certified iterate
  T P[2][12];                   // the two geometries' placements
  T p[3];                       // the certified point
};

// The pair's chains (one lane): geometries, common ancestor, the joints from
// the root to it and from it to each geometry's joint (`par`: jparent, e.g.
// staged in LDS).
template <typename T>
IKG_HD inline void cert_chains(const KCollision<T>* __restrict__ c, const int32_t* par, int pair, BallCert<T>& out) {
  const int gg[2] = {c->pairs[pair][0], c->pairs[pair][1]};
  int jj[2];
  for (int h = 0; h < 2; ++h) {
    out.g[h] = gg[h];
    jj[h] = gg[h] == c->target_geom ? -1 : c->joint[gg[h]];
  }
  // every walk is bounded by kMaxNq steps whatever the tables hold; a chain
  // that does not end within it leaves the certificate empty (ok = 0)
  int lca = -1;
  bool ok = true;
  if (jj[0] >= 0 && jj[1] >= 0) {
    uint32_t anc = 0;
    int k = jj[0], steps = 0;
    for (; k >= 0 && k < kMaxNq && steps < kMaxNq; k = par[k], ++steps) anc |= 1u << k;
    ok = ok && k < 0;
    lca = jj[1];
    for (steps = 0; lca >= 0 && lca < kMaxNq && steps < kMaxNq && !((anc >> lca) & 1u); ++steps) lca = par[lca];
    ok = ok && lca < kMaxNq && steps < kMaxNq;
  }
  out.lca = lca;
  int n = 0, k = lca;
  for (; k >= 0 && k < kMaxNq && n < kMaxNq; k = par[k]) out.list[0][n++] = k;
  ok = ok && k < 0;
  out.nl[0] = n;
  for (int h = 0; h < 2; ++h) {
    n = 0;
    k = (gg[h] != c->target_geom && jj[h] >= 0) ? jj[h] : lca;
    for (; k != lca && k >= 0 && k < kMaxNq && n < kMaxNq; k = par[k]) out.list[1 + h][n++] = k;
    ok = ok && (k == lca || k < 0);
    out.nl[1 + h] = n;
  }
  out.ok = ok && out.nl[0] + out.nl[1] + out.nl[2] <= kMaxNq;
}

// Local transform of entry e (chains in order) at configuration q.
template <typename T>
IKG_HD inline void cert_local(const KModel<T>* __restrict__ m, const T* __restrict__ q, const int32_t* sl, int e,
                              BallCert<T>& out, T (*Lt)[12]) {
  const int ch = e < out.nl[0] ? 0 : e < out.nl[0] + out.nl[1] ? 1 : 2;
  const int i = e - (ch > 0 ? out.nl[0] : 0) - (ch > 1 ? out.nl[1] : 0);
  const int k = out.list[ch][i];
  T sk, ck;
  Prec<T>::sincos_(q[sl[k]], &sk, &ck);
  joint_local(m, k, sk, ck, Lt[e]);  // entries in chain order: chain 0, then 1, then 2
}

// Compose the chains (one lane): the common ancestor's frame, then each
// branch down to its geometry: joint origins, the moving joints' list, the
// two placements.
template <typename T>
IKG_HD inline void cert_compose(const KCollision<T>* __restrict__ c, const T* __restrict__ q, const int32_t* sl,
                                const T* tgt, BallCert<T>& out, const T (*Lt)[12]) {
  T Fs[12] = {T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0)};
  int n = 0;
  for (int ch = 0; ch < 3; ++ch) {
    const int h = ch - 1;
    if (ch > 0) {
      const int g = out.g[h];
      if (g == c->target_geom || c->joint[g] < 0) {
        for (int i = 0; i < 9; ++i) out.P[h][i] = g == c->target_geom ? tgt[i] : c->R[g][i];
        for (int i = 0; i < 3; ++i) out.P[h][9 + i] = g == c->target_geom ? tgt[9 + i] : c->t[g][i];
        continue;
      }
    }
    T W[12];
    for (int i = 0; i < 12; ++i) W[i] = ch == 0 ? ((i == 0 || i == 4 || i == 8) ? T(1) : T(0)) : Fs[i];
    for (int u = out.nl[ch] - 1; u >= 0; --u) {  // down the chain: W <- W L_k
      const T* L = Lt[(ch > 0 ? out.nl[0] : 0) + (ch > 1 ? out.nl[1] : 0) + u];
      T Rn[9], tn[3];
      matmul3(W, L, Rn);
      matvec3(W, L + 9, tn);
      for (int i = 0; i < 9; ++i) W[i] = Rn[i];
      for (int i = 0; i < 3; ++i) W[9 + i] += tn[i];
      if (ch > 0 && n < kCertJoints) {
        const int k = out.list[ch][u];
        out.joint[n] = k;
        out.side[n] = h;
        out.off[n] = sl[k];
        out.qc[n] = q[sl[k]];
        for (int i = 0; i < 3; ++i) out.org[n][i] = W[9 + i];
        ++n;
      }
    }
    if (ch == 0) {
      for (int i = 0; i < 12; ++i) Fs[i] = W[i];
    } else {
      const int g = out.g[h];
      T Rg[9], tg3[3];
      matmul3(W, c->R[g], Rg);
      matvec3(W, c->t[g], tg3);
      for (int i = 0; i < 9; ++i) out.P[h][i] = Rg[i];
      for (int i = 0; i < 3; ++i) out.P[h][9 + i] = W[9 + i] + tg3[i];
    }
  }
  out.n = n;
  for (int e = n; e < kCoverBatch; ++e) {  // unused batch entries weigh nothing (ball_covers)
    out.joint[e] = out.side[e] = out.off[e] = 0;
    out.qc[e] = T(0);
  }
}

// The two geometries as shapes (their placements copied out of `out`).
template <typename T>
IKG_HD inline void cert_shapes(const KCollision<T>* __restrict__ c, const BallCert<T>& out, T (&PA)[12], T (&PB)[12],
                               Shape<T>& A, Shape<T>& B) {
  for (int i = 0; i < 12; ++i) {
    PA[i] = out.P[0][i];
    PB[i] = out.P[1][i];
  }
  A = Shape<T>{PA, PA + 9, c->dims[out.g[0]], c->kind[out.g[0]]};
  B = Shape<T>{PB, PB + 9, c->dims[out.g[1]], c->kind[out.g[1]]};
}

// The radius (net of the placements' rounding: 1e-9 fp64, 1e-5 fp32, as the
// EPA certificate) and the lever arms |p - o_k| for the point found.
template <typename T>
IKG_HD inline void cert_finish(T r, const T* p, BallCert<T>& out) {
  for (int i = 0; i < 3; ++i) out.p[i] = p[i];
  for (int e = 0; e < out.n; ++e) {
    const T d[3] = {p[0] - out.org[e][0], p[1] - out.org[e][1], p[2] - out.org[e][2]};
    out.lev[e] = sqrt(dot3(d, d));
  }
  out.r = r - (sizeof(T) == 8 ? T(1e-9) : T(1e-5));
}

// Build the certificate for `pair` at configuration q (q[sl[k]] = joint k:
// a record row and its slot map), one lane doing every stage in turn (the host
// emulator; the scan runs the same stages over the wave, traj_scan_body).
template <typename T>
IKG_HD inline void ball_cert(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c, int pair,
                             const T* __restrict__ q, const int32_t* sl, const T* tgt, BallCert<T>& out) {
  cert_chains(c, m->jparent, pair, out);
  if (!out.ok) {
    out.n = 0;
    out.r = T(-1);
    return;
  }
  T Lt[kMaxNq][12];
  for (int e = 0; e < out.nl[0] + out.nl[1] + out.nl[2]; ++e) cert_local(m, q, sl, e, out, Lt);
  cert_compose(c, q, sl, tgt, out, Lt);
  T PA[12], PB[12];
  Shape<T> A{}, B{};
  cert_shapes(c, out, PA, PB, A, B);
  T p[3];
  const T r = deep_common_point(A, B, p);
  cert_finish(r, p, out);
}

// Does the certificate prove the pair intersecting at configuration q (q[off]:
// a record row, or a configuration in joint order with the slot map the
// certificate was built with)?  Up to kCoverBatch joints the loads go out as
// one batch (unused entries read q[0] and weigh nothing) instead of one
// dependent global load per joint (the scan's cover step ran ~35k cycles per
// chunk that way, profiles/r05/collision/).
template <typename T>
IKG_HD inline bool ball_covers(const BallCert<T>& bc, const T* __restrict__ q) {
  T s0[2] = {T(0), T(0)}, s1[2] = {T(0), T(0)};
  const int n = bc.n;
  if (n <= kCoverBatch) {
    T v[kCoverBatch];
#pragma unroll
    for (int e = 0; e < kCoverBatch; ++e) v[e] = q[bc.off[e]];
#pragma unroll
    for (int e = 0; e < kCoverBatch; ++e) {
      const T d = e < n ? fabs(v[e] - bc.qc[e]) : T(0);
      const T l = bc.lev[e < n ? e : 0];
      const bool h1 = bc.side[e] != 0;
      s0[0] += h1 ? T(0) : d;
      s0[1] += h1 ? d : T(0);
      s1[0] += h1 ? T(0) : d * l;
      s1[1] += h1 ? d * l : T(0);
    }
  } else {
    for (int e = 0; e < n; ++e) {
      const T d = fabs(q[bc.off[e]] - bc.qc[e]);
      const int h = bc.side[e];
      s0[h] += d;
      s1[h] += d * bc.lev[e];
    }
  }
  return bc.r > T(0) && s1[0] + bc.r * s0[0] < bc.r && s1[1] + bc.r * s0[1] < bc.r;
}

}  // namespace ikg
