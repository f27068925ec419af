// Collision kernels (gfx950): the collision term of computeqgrasppose's
// `success` (inverse_geometry.py:70, :97-98; tools.py:25-35).
//
//  * ikg_collision_kernel: tools.collision(robot, q) for a batch, one wave per
//    problem (ikg_collision_batch).
//  * ikg_collide_continue_kernel: the reference loop from the first iterate
//    whose hand errors pass (found by the pair kernel) onwards: while that
//    iterate collides the loop keeps updating (:70 is `errors and not
//    collision`), checking collision at every iterate whose errors pass,
//    until a collision-free one or max_iters.  One wave per problem: lanes 0/1
//    run the pair iteration (ikg_device.hpp stages), all 64 lanes share the
//    ~745-pair check.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdlib>

#include "ikg_collision.hpp"
#include "ikg_device.hpp"
#include "ikg_launch.hpp"
#include "ikg_solve.hpp"

namespace ikg {

// Phase timing of the continuation kernel (diagnostic build only: -DIKG_CPROF,
// tools/cprof.sh).  Lane 0 of each wave accumulates shader-clock cycles per
// phase; totals are summed into g_cprof.
#ifdef IKG_CPROF
__device__ unsigned long long g_cprof[8];
// certificate statistics: checks run, checks answered by the certificate,
// tetrahedra available on a hit, EPA attempts, EPA certificates, sum of
// certified margins (nm)
__device__ unsigned long long g_skip[8];
// trajectory scan, per problem and window: max / sum of checks, max cycles,
// sum / max of sweeps, windows scanned, certificates, sum of cycles
__device__ unsigned long long g_scan[28];
#define SKIP_STAT(i, v) atomicAdd(&g_skip[i], (unsigned long long)(v))
// single-lane witness work: cycles in GJK (pair_collides + supports), in
// certify_witness (of which EPA), calls of each
__device__ unsigned long long g_wprof[6];
#define WPROF(i, v) atomicAdd(&g_wprof[i], (unsigned long long)(v))
// `cp_lead` (in scope at every use): this lane accumulates for its problem
#define CPROF_MARK(acc, t)                   \
  do {                                       \
    const unsigned long long _n = clock64(); \
    if (cp_lead) acc += _n - t;              \
    t = _n;                                  \
  } while (0)
#define CPROF_ADD(i, v)                 \
  do {                                  \
    if (prof && cp_lead) prof[i] += v; \
  } while (0)
#else
#define SKIP_STAT(i, v) \
  do {                  \
  } while (0)
#define WPROF(i, v) \
  do {              \
  } while (0)
#define CPROF_MARK(acc, t) \
  do {                     \
  } while (0)
#define CPROF_ADD(i, v) \
  do {                  \
  } while (0)
#endif

// World joint frames -> geometry placements -> pair tests; wave-uniform result.
// Must be called by all 64 lanes of the (single-wave) workgroup, with S.q,
// S.sn/S.cs (= sincos of S.q) and S.par ready.
//
// The witness W (LDS) is the pair that collided at the previous check of this
// problem.  It is tested first: along the continuation the robot moves by
// ~1e-5 rad per update, so a colliding pair almost always still collides.
// If its last GJK ended on an origin-enclosing tetrahedron, the support points
// along the same 4 directions are re-evaluated at the new poses (lanes 0-3)
// and an enclosure is again a proof of intersection; otherwise lane 0 re-runs
// GJK (refreshing the certificate).  Failing that, the pairs are swept in
// wave-wide rounds of 64 with an early exit on the first round holding a hit,
// whose lowest pair becomes the new witness.  The result is the OR over all
// active pairs either way: only the order of the tests changes.
#ifndef IKG_SWEEP_COMPACT
#define IKG_SWEEP_COMPACT 1
#endif
template <typename T, bool WITNESS>
__device__ bool collide_wave(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                             CollideScratch<T>& S, const T* tgt, Witness<T>& W,
                             unsigned long long* prof = nullptr) {
  const int lane = threadIdx.x & 63;
  const int nq = m->nq;
#ifdef IKG_CPROF
  unsigned long long t = clock64(), a_fr = 0, a_w = 0, a_sw = 0;
  const bool cp_lead = lane == 0;
#endif
  if (lane < nq) joint_local(m, lane, S.sn[lane], S.cs[lane], S.L[lane]);
  __syncthreads();
  if (lane < nq) joint_world(S.par, lane, S.L, S.F[lane]);
  __syncthreads();
  CPROF_MARK(a_fr, t);
  CPROF_ADD(0, a_fr);
  const int w = WITNESS ? W.pair : -1;
  if (WITNESS && w >= 0) {
    const int ga = c->pairs[w][0], gb = c->pairs[w][1];
    if (lane < 2) geom_world(c, lane ? gb : ga, S.F, tgt, S.P[lane ? gb : ga]);
    __syncthreads();
    const Shape<T> A = pair_shape(c, ga, S.P), B = pair_shape(c, gb, S.P);
    if (W.cert_ok) {
      if (lane < 4) mink_support(A, B, W.dir + 3 * lane, W.pts[lane]);
      __syncthreads();
      const bool h = lane == 0 && tetra_encloses_origin(W.pts[0], W.pts[1], W.pts[2], W.pts[3]);
      if (__any(h)) {
        CPROF_MARK(a_w, t);
        CPROF_ADD(1, a_w);
        return true;
      }
    }
    int r = 0;
    if (lane == 0) {
      T cert[12];
      r = pair_collides(A, B, cert);
      W.cert_ok = r == 2;
      if (r == 2)
        for (int i = 0; i < 12; ++i) W.dir[i] = cert[i];
    }
    const bool any = __any(r != 0);
    CPROF_MARK(a_w, t);
    CPROF_ADD(1, a_w);
    if (any) return true;
  }
  CPROF_ADD(3, 1ull);  // full sweeps
  for (int g = lane; g < c->n_geoms; g += 64) geom_world(c, g, S.F, tgt, S.P[g]);
  __syncthreads();
  bool found = false;
#if IKG_SWEEP_COMPACT
  // Two passes: the bounding-sphere test of every pair, the survivors listed
  // in pair order (ballot + popcount), then the exact tests over the list in
  // rounds of 64.  A collision-free pose runs ~2 narrow-phase rounds instead of
  // a GJK-latency round in each of the 12 rounds of 64 pairs; the answer and
  // the witness (lowest colliding pair) are the single pass's.
  // Every round's pair indices and thresholds are loaded before the first
  // test (one memory round trip per check instead of two dependent ones per
  // round of 64 pairs; the thresholds are precomputed per pair, pr2)
  int ncand = 0;
  {
    constexpr int kRounds = kMaxPairs / 64;
    const int np = c->n_pairs;
    const uint32_t* __restrict__ pw = reinterpret_cast<const uint32_t*>(&c->pairs[0][0]);
    uint32_t pk[kRounds];
    T r2[kRounds];
#pragma unroll
    for (int i = 0; i < kRounds; ++i) {
      const int k = i * 64 + lane;
      const bool in = k < np;
      pk[i] = in ? pw[k] : 0u;
      r2[i] = in ? c->pr2[k] : T(0);
    }
#pragma unroll
    for (int i = 0; i < kRounds; ++i) {
      if (i * 64 >= np) break;  // wave-uniform
      const int k = i * 64 + lane;
      bool pass = false;
      if (k < np && k != w) {
        const int a = (int16_t)(pk[i] & 0xFFFFu), b = (int16_t)(pk[i] >> 16);
        const T d0 = S.P[a][9] - S.P[b][9], d1 = S.P[a][10] - S.P[b][10], d2 = S.P[a][11] - S.P[b][11];
        pass = d0 * d0 + d1 * d1 + d2 * d2 < r2[i];
      }
      const unsigned long long bal = __ballot(pass);
      if (pass) S.cand[ncand + __popcll(bal & ((1ull << lane) - 1))] = (int16_t)k;
      ncand += __popcll(bal);
    }
  }
  __syncthreads();
#ifdef IKG_CPROF
  {  // prof[4]: the bounding-sphere pass (its share of the sweep, prof[2])
    const unsigned long long _n = clock64();
    if (prof && cp_lead) prof[4] += _n - t;
  }
#endif
  for (int base = 0; base < ncand; base += 64) {
    const int i = base + lane;
    const int k = i < ncand ? S.cand[i] : 0;
    bool hit = false;
    if (i < ncand) {
      const int a = c->pairs[k][0], b = c->pairs[k][1];
      hit = pair_collides(pair_shape(c, a, S.P), pair_shape(c, b, S.P)) != 0;
    }
    const unsigned long long bal = __ballot(hit);
    if (bal) {
      if (WITNESS && lane == 0) W.pair = S.cand[base + __ffsll((long long)bal) - 1];
      found = true;
      break;
    }
  }
#else
  for (int base = 0; base < c->n_pairs; base += 64) {
    const int k = base + lane;
    const bool hit = k < c->n_pairs && k != w && pair_hit(c, k, S.P) != 0;
    const unsigned long long bal = __ballot(hit);
    if (bal) {
      if (WITNESS && lane == 0) W.pair = base + __ffsll((long long)bal) - 1;
      found = true;
      break;
    }
  }
#endif
  if (WITNESS && lane == 0) {
    if (!found) W.pair = -1;
    W.cert_ok = 0;
  }
  CPROF_MARK(a_sw, t);
  CPROF_ADD(2, a_sw);
  return found;
}

template <typename T>
__device__ inline void stage_trig_par(const KModel<T>* __restrict__ m, CollideScratch<T>& S) {
  const int lane = threadIdx.x & 63;
  if (lane < m->nq) {
    Prec<T>::sincos_(S.q[lane], &S.sn[lane], &S.cs[lane]);
    S.par[lane] = m->jparent[lane];
  }
}

template <typename T>
__global__ __launch_bounds__(64) void ikg_collision_kernel(const KModel<T>* __restrict__ m,
                                                           const KCollision<T>* __restrict__ c,
                                                           const T* __restrict__ q, const T* __restrict__ targets,
                                                           int64_t B, uint8_t* __restrict__ out) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  __shared__ Witness<T> W;
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (lane < m->nq) S.q[lane] = q[p * m->nq + lane];
  if (lane < 12) tgt[lane] = targets[p * 12 + lane];
  if (lane == 0) {
    W.pair = -1;
    W.cert_ok = 0;
  }
  __syncthreads();
  stage_trig_par(m, S);
  __syncthreads();
  const bool col = collide_wave<T, false>(m, c, S, tgt, W);
  if (lane == 0) out[p] = col ? 1 : 0;
}

// ---------------------------------------------------------------- planner queries
// distanceToObstacle (tools.py:37-51): min over the given active pairs of the
// pair distance at configuration q, one wave per configuration.
template <typename T>
__global__ __launch_bounds__(64) void ikg_distance_kernel(const KModel<T>* __restrict__ m,
                                                          const KCollision<T>* __restrict__ c,
                                                          const T* __restrict__ q, const T* __restrict__ targets,
                                                          int64_t B, const int32_t* __restrict__ pair_idx, int n_idx,
                                                          T* __restrict__ out) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (lane < m->nq) S.q[lane] = q[p * m->nq + lane];
  if (lane < 12) tgt[lane] = targets[p * 12 + lane];
  __syncthreads();
  stage_trig_par(m, S);
  __syncthreads();
  if (lane < m->nq) joint_local(m, lane, S.sn[lane], S.cs[lane], S.L[lane]);
  __syncthreads();
  if (lane < m->nq) joint_world(S.par, lane, S.L, S.F[lane]);
  __syncthreads();
  for (int g = lane; g < c->n_geoms; g += 64) geom_world(c, g, S.F, tgt, S.P[g]);
  __syncthreads();
  // GJK in fp64 whatever the I/O type: the fp32 rounding of the simplex tests
  // (flat tetrahedra against the table's faces) is not worth a separate tuning
  double d = 1e30;
  for (int k = lane; k < n_idx; k += 64) {
    const int pr = pair_idx[k];
    double P2[2][12], D2[2][3];
    int K2[2];
    for (int h = 0; h < 2; ++h) {
      const int g = c->pairs[pr][h];
      for (int i = 0; i < 12; ++i) P2[h][i] = (double)S.P[g][i];
      for (int i = 0; i < 3; ++i) D2[h][i] = (double)c->dims[g][i];
      K2[h] = c->kind[g];
    }
    const Shape<double> A{P2[0], P2[0] + 9, D2[0], K2[0]}, Bs{P2[1], P2[1] + 9, D2[1], K2[1]};
    d = fmin(d, pair_distance(A, Bs));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) d = fmin(d, __shfl_xor(d, off));
  if (lane == 0) out[p] = (T)d;
}

// The cube's own collision model (setup_pinocchio.py:62-70): the target
// geometry placed at each candidate placement against the given world-fixed
// geometries (table, obstacle), one thread per placement.
template <typename T>
__global__ __launch_bounds__(256) void ikg_target_env_kernel(const KCollision<T>* __restrict__ c,
                                                             const T* __restrict__ targets, int64_t B,
                                                             const int32_t* __restrict__ geoms, int n_geoms,
                                                             uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const T* P = targets + 12 * i;
  const int tg = c->target_geom;
  const Shape<T> A{P, P + 9, c->dims[tg], c->kind[tg]};
  int hit = 0;
  for (int k = 0; k < n_geoms; ++k) {
    const int g = geoms[k];
    const Shape<T> Bs{c->R[g], c->t[g], c->dims[g], c->kind[g]};
    hit |= pair_collides(A, Bs) != 0;
  }
  out[i] = hit ? 1 : 0;
}

template <typename T>
hipError_t launch_distance(const KModel<T>* dm, const KCollision<T>* dc, const void* q, const void* targets,
                           int64_t B, const int32_t* pair_idx, int n_idx, void* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL((ikg_distance_kernel<T>), dim3((unsigned)B), dim3(64), 0, s, dm, dc, (const T*)q,
                     (const T*)targets, B, pair_idx, n_idx, (T*)out);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_target_env(const KCollision<T>* dc, const void* targets, int64_t B, const int32_t* geoms,
                             int n_geoms, uint8_t* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL((ikg_target_env_kernel<T>), dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, dc,
                     (const T*)targets, B, geoms, n_geoms, out);
  return hipGetLastError();
}
template hipError_t launch_distance<double>(const KModel<double>*, const KCollision<double>*, const void*,
                                            const void*, int64_t, const int32_t*, int, void*, hipStream_t);
template hipError_t launch_distance<float>(const KModel<float>*, const KCollision<float>*, const void*,
                                           const void*, int64_t, const int32_t*, int, void*, hipStream_t);
template hipError_t launch_target_env<double>(const KCollision<double>*, const void*, int64_t, const int32_t*, int,
                                              uint8_t*, hipStream_t);
template hipError_t launch_target_env<float>(const KCollision<float>*, const void*, int64_t, const int32_t*, int,
                                             uint8_t*, hipStream_t);

// ---------------------------------------------------------------- continuation
// G problems per wave (LG = 64/G lanes each).  Per-problem state lives in a
// slice of dynamic LDS sized for the model (group_lds_bytes).
template <typename T>
struct GroupLds {
  T* q;
  T* sn;
  T* cs;
  T (*F)[12];   // world joint frames of the current iterate
  T (*L)[12];   // joint-local transforms of the passive joints (constant here)
  T (*P)[12];   // geometry placements
  T* tgt;
  T* flag;
  int32_t* par;
  Witness<T>* W;
};

template <typename T>
IKG_HD inline size_t group_lds_real_bytes(int nq, int ng) {
  return (sizeof(T) * (27 * (size_t)nq + 12 * (size_t)ng + 16) + 15) & ~(size_t)15;
}

template <typename T>
IKG_HD inline size_t group_lds_bytes(int nq, int ng) {
  return group_lds_real_bytes<T>(nq, ng) + ((sizeof(int32_t) * (size_t)nq + 15) & ~(size_t)15) +
         ((sizeof(Witness<T>) + 15) & ~(size_t)15);
}

template <typename T>
__device__ inline GroupLds<T> group_view(char* base, int g, int nq, int ng) {
  char* p = base + (size_t)g * group_lds_bytes<T>(nq, ng);
  GroupLds<T> v;
  T* t = (T*)p;
  v.q = t;
  t += nq;
  v.sn = t;
  t += nq;
  v.cs = t;
  t += nq;
  v.F = (T(*)[12])t;
  t += 12 * nq;
  v.L = (T(*)[12])t;
  t += 12 * nq;
  v.P = (T(*)[12])t;
  t += 12 * ng;
  v.tgt = t;
  t += 12;
  v.flag = t;
  char* c = p + group_lds_real_bytes<T>(nq, ng);
  v.par = (int32_t*)c;
  c += (sizeof(int32_t) * nq + 15) & ~(size_t)15;
  v.W = (Witness<T>*)c;
  return v;
}

// ---- group-parallel EPA (continuation): the LG lanes of one problem's group
// each own one face slot of the polytope (LG >= kEpaF); vertices and the new
// faces of an expansion pass through LDS.  Same polytope sequence as the
// serial epa_depth_lb (the reference form, host-tested): the closest face is
// the lowest slot at the minimum offset, the horizon is the set of edges of
// visible faces whose reverse edge lies on no visible face, and every face's
// plane is computed by the same expression -- only slot order differs.
template <int LG>
__device__ __forceinline__ unsigned long long group_bits(bool p, int lane0) {
  const unsigned long long b = __ballot(p);
  return LG == 64 ? b : (b >> lane0) & ((1ull << LG) - 1ull);
}

template <int LG>
__device__ __forceinline__ double group_min(double x) {
#pragma unroll
  for (int o = LG / 2; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, LG));
  return x;
}

// LDS writes of one lane visible to the other lanes of its wave (one wave
// per workgroup here; the groups of a wave run the same code in lockstep)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// plane of face (a, b, c) of V: unit normal + offset; false if degenerate
__device__ __forceinline__ bool epa_plane(const double (*V)[3], int a, int b, int c, double* n) {
  const double *pa = V[a], *pb = V[b], *pc = V[c];
  const double u[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
  const double w[3] = {pc[0] - pa[0], pc[1] - pa[1], pc[2] - pa[2]};
  const double m[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
  const double nn = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
  if (!(nn > 1e-300)) return false;
  const double r = 1.0 / nn;
  for (int i = 0; i < 3; ++i) n[i] = m[i] * r;
  n[3] = n[0] * pa[0] + n[1] * pa[1] + n[2] * pa[2];
  return true;
}

template <typename T, int LG>
__device__ double epa_depth_lb_group(const Shape<T>& A, const Shape<T>& B, const T (*P)[3], EpaScratch& s, int li,
                                     int lane0) {
  static_assert(LG >= kEpaF, "one face slot per lane");
  if (li < 4)
    for (int i = 0; i < 3; ++i) s.V[li][i] = (double)P[li][i];
  wave_lds_sync();
  constexpr int8_t F0[4][3] = {{0, 1, 2}, {0, 3, 1}, {0, 2, 3}, {1, 3, 2}};
  int fa = 0, fb = 0, fc = 0;
  double n[4] = {0.0, 0.0, 0.0, 0.0};
  bool alive = li < 4, bad = false;
  double cen[3], scale = 0.0;
  for (int i = 0; i < 3; ++i) cen[i] = 0.25 * (s.V[0][i] + s.V[1][i] + s.V[2][i] + s.V[3][i]);
  for (int v = 0; v < 4; ++v)
    for (int i = 0; i < 3; ++i) scale = fmax(scale, fabs(s.V[v][i]));
  if (alive) {
    fa = F0[li][0];
    fb = F0[li][1];
    fc = F0[li][2];
    bad = !epa_plane(s.V, fa, fb, fc, n);
    if (!bad && n[0] * cen[0] + n[1] * cen[1] + n[2] * cen[2] > n[3]) {  // inward: flip
      const int t = fb;
      fb = fc;
      fc = t;
      for (int i = 0; i < 4; ++i) n[i] = -n[i];
    }
  }
  if (group_bits<LG>(bad, lane0)) return 0.0;
  int nV = 4;
  double best = 0.0;
  const unsigned long long below = li == 0 ? 0ull : (~0ull >> (64 - li));  // lanes < li of the group
  for (int it = 0;; ++it) {
    const double dmin = group_min<LG>(alive ? n[3] : 1e300);
    if (!(dmin >= 0.0)) return 0.0;  // the origin is not inside
    best = dmin;
    if (it == kEpaIters || nV == kEpaV) break;
    const int fmin = __ffsll((long long)group_bits<LG>(alive && n[3] == dmin, lane0)) - 1;
    double nd[3];
    for (int i = 0; i < 3; ++i) nd[i] = __shfl(n[i], fmin, LG);
    T dir[3] = {(T)nd[0], (T)nd[1], (T)nd[2]}, wt[3];
    mink_support(A, B, dir, wt);
    const double w[3] = {(double)wt[0], (double)wt[1], (double)wt[2]};
    if (w[0] * nd[0] + w[1] * nd[1] + w[2] * nd[2] - dmin <= 1e-12 * scale) break;
    const bool vis = alive && n[0] * w[0] + n[1] * w[1] + n[2] * w[2] - n[3] > 1e-14 * scale;
    const unsigned long long vm = group_bits<LG>(vis, lane0);
    if (!((vm >> fmin) & 1ull)) break;
    // horizon edges of this face: reverse edge on no other visible face
    const int e0[3] = {fa, fb, fc}, e1[3] = {fb, fc, fa};
    bool hz[3] = {vis, vis, vis};
    for (unsigned long long m = vm; m; m &= m - 1) {
      const int g = __ffsll((long long)m) - 1;
      const int ga = __shfl(fa, g, LG), gb = __shfl(fb, g, LG), gc = __shfl(fc, g, LG);
      if (g != li)
        for (int e = 0; e < 3; ++e)
          if ((ga == e1[e] && gb == e0[e]) || (gb == e1[e] && gc == e0[e]) || (gc == e1[e] && ga == e0[e]))
            hz[e] = false;
    }
    const int nh = (int)hz[0] + (int)hz[1] + (int)hz[2];
    const unsigned long long h1 = group_bits<LG>(nh >= 1, lane0), h2 = group_bits<LG>(nh >= 2, lane0),
                             h3 = group_bits<LG>(nh >= 3, lane0);
    const int nH = __popcll(h1) + __popcll(h2) + __popcll(h3);
    const int nalive = __popcll(group_bits<LG>(alive, lane0));
    if (nH > kEpaF + 4 || nalive - __popcll(vm) + nH > kEpaF) break;  // the current polytope stays valid
    const int pre = __popcll(h1 & below) + __popcll(h2 & below) + __popcll(h3 & below);
    for (int e = 0, k = pre; e < 3; ++e)
      if (hz[e]) {
        s.Fx[k][0] = (int8_t)e0[e];
        s.Fx[k][1] = (int8_t)e1[e];
        ++k;
      }
    if (li == 0)
      for (int i = 0; i < 3; ++i) s.V[nV][i] = w[i];
    wave_lds_sync();
    // free slots: dead or visible; the r-th free slot takes the r-th new face
    alive = alive && !vis;
    const unsigned long long fm = group_bits<LG>(!alive, lane0);
    const int r = __popcll(fm & below);
    bad = false;
    if (!alive && r < nH) {
      fa = s.Fx[r][0];
      fb = s.Fx[r][1];
      fc = nV;
      alive = true;
      bad = !epa_plane(s.V, fa, fb, fc, n);
    }
    if (group_bits<LG>(bad, lane0)) return 0.0;
    ++nV;
    for (int i = 0; i < 3; ++i) scale = fmax(scale, fabs(w[i]));
    wave_lds_sync();  // Fx is rewritten by the next expansion
  }
  // verify: every vertex on the inner side of every face plane (convex hull)
  bool out = false;
  if (alive)
    for (int v = 0; v < nV; ++v)
      out = out || n[0] * s.V[v][0] + n[1] * s.V[v][1] + n[2] * s.V[v][2] - n[3] > 1e-9 * scale;
  return group_bits<LG>(out, lane0) ? 0.0 : best;
}

// Penetration certificate of the witness pair, by the problem's group (rare,
// so kept out of line: inlined, its temporaries raised the register pressure
// of the whole continuation loop).  EPA lower bound on the depth minus the
// placement rounding of the I/O type; per joint j, the lever-arm bound Rmot[j]
// of the two geometries about it (distance of the geometry's centre from the
// joint origin + its bounding radius + twice the margin, which bounds that
// distance over the motions the margin allows).
template <typename T, int LG>
__device__ __attribute__((always_inline)) inline void certify_witness(int nq, Shape<T> A, Shape<T> B, Witness<T>& W,
                                                          const T (*Fa)[12], const int32_t* par, int li, int lane0) {
  const double tol = sizeof(T) == 8 ? 1e-9 : 1e-5;
#ifdef IKG_CPROF
  const unsigned long long t0 = clock64();
#endif
  const double d = epa_depth_lb_group<T, LG>(A, B, W.pts, W.epa, li, lane0) - tol;
#ifdef IKG_CPROF
  if (li == 0) {
    WPROF(2, clock64() - t0);
    WPROF(5, 1);
  }
#endif
  if (li == 0) SKIP_STAT(3, 1);
  if (!(d > 0.0)) {
    if (li == 0) W.epa_wait = 32;
    return;
  }
  if (li == 0) {
    SKIP_STAT(4, 1);
    SKIP_STAT(5, d * 1e9);
  }
  for (int j = li; j < nq; j += LG) {
    T r = T(0);
    for (int g = 0; g < 2; ++g) {
      if (W.gtarget[g]) continue;
      bool anc = false;
      for (int k = W.gjoint[g]; k >= 0 && !anc; k = par[k]) anc = k == j;
      if (!anc) continue;
      const T* c = W.P[g] + 9;
      const T dx = c[0] - Fa[j][9], dy = c[1] - Fa[j][10], dz = c[2] - Fa[j][11];
      r += sqrt(dx * dx + dy * dy + dz * dz) + W.gbrad[g] + T(2.0 * d);
    }
    W.Rmot[j] = r;
  }
  if (li == 0) {
    W.budget = d;
    W.skip_ok = 1;
    ++W.gen;
  }
}

// One collision check for every group with `need` set (group-uniform); all 64
// lanes call it.  Joint frames come from the IK lanes' FK of the same iterate
// (fk_arm WANT_FRAMES), so only the passive joints are composed here; then
// witness-first / certificate / sweep exactly as collide_wave.  Returns the
// group's verdict.
template <typename T, int LG>
__device__ bool collide_group(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                              const GroupLds<T>& V, int li, int lane0, bool need, unsigned long long gmask,
                              unsigned long long* prof) {
#ifdef IKG_CPROF
  unsigned long long t = clock64(), a_fr = 0, a_w = 0, a_sw = 0;
  const bool cp_lead = li == 0 && need;
#endif
  // root / arm joint frames were written by the IK lanes' FK of this iterate;
  // the remaining (passive) joints hang off them, parents first (q order)
  if (need && li == 0)
    for (int i = 0; i < m->n_passive; ++i) {
      const int j = m->passive_q[i];
      const T* Lj = V.L[j];
      const int a = V.par[j];
      if (a < 0) {
        for (int k = 0; k < 12; ++k) V.F[j][k] = Lj[k];
      } else {
        const T* Fp = V.F[a];
        T tn[3];
        matmul3(Fp, Lj, V.F[j]);
        matvec3(Fp, Lj + 9, tn);
        for (int k = 0; k < 3; ++k) V.F[j][9 + k] = Fp[9 + k] + tn[k];
      }
    }
  __syncthreads();
  const T(*Fa)[12] = V.F;
  CPROF_MARK(a_fr, t);
  CPROF_ADD(0, a_fr);
  const int w = need ? V.W->pair : -1;
  const bool has_w = w >= 0;
  Witness<T>& W = *V.W;
  if (has_w && li < 2) {  // the witness geometries' placements, from LDS only
    T* P = W.P[li];
    if (W.gtarget[li]) {
      for (int i = 0; i < 12; ++i) P[i] = V.tgt[i];
    } else if (W.gjoint[li] < 0) {
      for (int i = 0; i < 9; ++i) P[i] = W.gR[li][i];
      for (int i = 0; i < 3; ++i) P[9 + i] = W.gt[li][i];
    } else {
      const T* Fj = Fa[W.gjoint[li]];
      T tn[3];
      matmul3(Fj, W.gR[li], P);
      matvec3(Fj, W.gt[li], tn);
      for (int i = 0; i < 3; ++i) P[9 + i] = Fj[9 + i] + tn[i];
    }
  }
  __syncthreads();
  const Shape<T> A{W.P[0], W.P[0] + 9, W.gdims[0], W.gkind[0]};
  const Shape<T> B{W.P[1], W.P[1] + 9, W.gdims[1], W.gkind[1]};
  const bool cert = has_w && W.cert_ok;
  if (cert && li < 4) mink_support(A, B, W.dir + 3 * li, W.pts[li]);
  __syncthreads();
  if (has_w && li == 0) {
    int r = 0;
    bool tetra = false;  // W.pts hold an origin-enclosing tetrahedron of this iterate
    if (cert && tetra_encloses_origin(W.pts[0], W.pts[1], W.pts[2], W.pts[3])) {
      r = 1;
      tetra = true;
    } else {
      T cd[12];
#ifdef IKG_CPROF
      const unsigned long long t0 = clock64();
#endif
      r = pair_collides(A, B, cd);
#ifdef IKG_CPROF
      WPROF(0, clock64() - t0);
      WPROF(3, 1);
#endif
      W.cert_ok = r == 2;
      if (r == 2) {
        for (int i = 0; i < 12; ++i) W.dir[i] = cd[i];
        for (int k = 0; k < 4; ++k) mink_support(A, B, W.dir + 3 * k, W.pts[k]);
        tetra = tetra_encloses_origin(W.pts[0], W.pts[1], W.pts[2], W.pts[3]);
      }
    }
    V.flag[1] = r ? T(1) : T(0);
    if (r && tetra) SKIP_STAT(2, 1);
    // penetration certificate: while the accumulated motion bound stays below
    // it, later checks of this problem are answered without running them
    W.epa_go = r && tetra && !W.skip_ok && --W.epa_wait <= 0;
  }
  __syncthreads();
  if (has_w && W.epa_go) {
#ifdef IKG_CPROF
    const unsigned long long t0 = clock64();
#endif
    certify_witness<T, LG>(m->nq, A, B, W, Fa, V.par, li, lane0);
#ifdef IKG_CPROF
    if (li == 0) {
      WPROF(1, clock64() - t0);
      WPROF(4, 1);
    }
#endif
  }
  __syncthreads();
  bool hit = has_w && V.flag[1] != T(0);
  CPROF_MARK(a_w, t);
  CPROF_ADD(1, a_w);
  const bool sweep = need && !hit;
  if (__any(sweep)) {
    CPROF_ADD(3, sweep ? 1ull : 0ull);
    if (sweep)
      for (int g = li; g < c->n_geoms; g += LG) geom_world(c, g, Fa, V.tgt, V.P[g]);
    __syncthreads();
    bool done = !sweep, found = false;
    int wnew = -1;
    for (int base = 0;; base += LG) {
      const int k = base + li;
      const bool h = !done && k < c->n_pairs && k != w && pair_hit(c, k, V.P) != 0;
      const unsigned long long bal = __ballot(h) & gmask;
      if (!done && bal) {
        found = true;
        wnew = base + (__ffsll((long long)bal) - 1 - lane0);
      }
      done = done || bal != 0 || base + LG >= c->n_pairs;
      if (!__any(!done)) break;
    }
    if (sweep && li == 0) {
      W.pair = wnew;
      W.cert_ok = 0;
      if (W.skip_ok) ++W.gen;
      W.skip_ok = 0;
      W.epa_wait = 0;
    }
    if (sweep && found && li < 2) {  // cache the new witness's geometry constants
      const int g = c->pairs[wnew][li];
      W.gjoint[li] = c->joint[g];
      W.gkind[li] = c->kind[g];
      W.gtarget[li] = g == c->target_geom;
      for (int i = 0; i < 9; ++i) W.gR[li][i] = c->R[g][i];
      for (int i = 0; i < 3; ++i) W.gt[li][i] = c->t[g][i];
      for (int i = 0; i < 3; ++i) W.gdims[li][i] = c->dims[g][i];
      W.gbrad[li] = c->brad[g];
    }
    if (sweep) hit = found;
    CPROF_MARK(a_sw, t);
    CPROF_ADD(2, a_sw);
  }
  return hit;
}

// One continuation iteration's FK + errors + step of this lane's arm
// (inverse_geometry.py:58-83; the IK lanes' frames go to F for the check).
// Returns the squared error norm of the lane's hand.
// FRAMES = false (certified stretches, no check ahead): the batch kernel's
// chest-frame FK with the tracked rotation angle, no joint frames.
template <typename T, bool DAMPED, class SP, bool FRAMES = true>
__device__ __forceinline__ T cont_step(const KModel<T>* __restrict__ m, const KParams<T>& prm, int arm, const T* sn,
                                       const T* cs, const T* RT, const T* tT, T (*F)[12], T* dq, T& s,
                                       ThetaTrack<T>* tk = nullptr, bool resync = true) {
  ArmState<T> st;
  T x;
  if constexpr (FRAMES)
    x = arm_fk_error<T, SP, true>(m, arm, sn, cs, RT, tT, st, F);
  else if constexpr (IKG_THETA_TRACK && is_f64<T>)
    x = arm_fk_error<T, SP>(m, arm, sn, cs, RT, tT, st, nullptr, tk, resync);
  else
    x = arm_fk_error<T, SP>(m, arm, sn, cs, RT, tT, st);
  T alpha, beta;
  if constexpr (!DAMPED) {
    pinv_step_cf<T, SP>(st, arm, m->sing_tau, m->sing_beta, dq, s);
  } else {
    T A[6][8], ze[6], zc[6];
    arm_system(st, A);
    arm_solve_damped(A, prm.lambda, ze, zc, alpha, beta);
    s = chest_step(alpha + pair_swap(alpha), beta + pair_swap(beta));
    arm_dq_damped(A, ze, zc, s, dq);
  }
  return x;
}

// Certificate motion bound of this lane's joints between the certified
// iterate and q: sum_j |q_j - qcert_j| Rmot_j.  Moving one joint at a time
// from qcert to q, every point of the witness geometries moves by at most
// Rmot_j |dq_j| per joint while the total stays below the margin (Rmot holds
// the 2 x margin lever-arm allowance), so the net displacement bounds any
// iterate -- tighter than summing the per-update motion when iterates drift
// back and forth near a fixed point.
template <typename T>
__device__ __forceinline__ T motion_bound(T qc, const T* qa, const T* qcert, const T* Rr) {
  T e = fabs(qc - qcert[0]) * Rr[0];
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) e += fabs(qa[k] - qcert[k + 1]) * Rr[k + 1];
  return e;
}

// q <- clip(q + dt dq) (:86-89) and the trig state.
template <typename T>
__device__ __forceinline__ void cont_update(const KModel<T>* __restrict__ m, const KParams<T>& prm, int arm, T s,
                                            const T* dq, int it, T& qc, T* qa,
                                            T* sn, T* cs) {
  T q_old[7];
  q_old[0] = qc;
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) q_old[k + 1] = qa[k];
  arm_update(m, arm, prm.dt, s, dq, qc, qa);
  trig_advance<T, IKG_GENERIC_MED>(qc, qa, q_old, ((it + 1) % Trig<T>::kResync) == 0, sn, cs);  // as solve_pair
}

// Certified-stretch updates (no collision check ahead, so no joint frames):
// the batch kernel's frame-1 loop for kFrame1 models with lambda = 0 (trig
// slots of trig_exact_f1), else the chest-frame loop of cont_step.
template <class SP, bool DAMPED>
constexpr bool kStretchF1 = kFrame1<SP> && !DAMPED;

template <typename T, bool DAMPED, class SP>
__device__ __forceinline__ T stretch_step(const KModel<T>* __restrict__ m, const KParams<T>& prm, int arm,
                                          const T* sn, const T* cs, const T* RT, const T* tT, T* dq, T& s,
                                          ThetaTrack<T>* tk, bool resync) {
  if constexpr (kStretchF1<SP, DAMPED>) {
    ArmStateF1<T> st;
    const T x = arm_fk_error_f1<T, SP>(m, arm, sn, cs, RT, tT, st, (IKG_THETA_TRACK && is_f64<T>) ? tk : nullptr,
                                       resync);
    pinv_step_f1<T, SP>(m, arm, st, sn, cs, dq, s);
    return x;
  } else {
    return cont_step<T, DAMPED, SP, false>(m, prm, arm, sn, cs, RT, tT, nullptr, dq, s, tk, resync);
  }
}

template <typename T, bool DAMPED, class SP>
__device__ __forceinline__ void stretch_update(const KModel<T>* __restrict__ m, const KParams<T>& prm, int arm, T s,
                                               const T* dq, int it, T& qc, T* qa, T* sn, T* cs,
                                               const ArmLimits<T>& lim) {
  if constexpr (kStretchF1<SP, DAMPED>) {
    T q_old[7];
    q_old[0] = qc;
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) q_old[k + 1] = qa[k];
    arm_update(m, arm, prm.dt, s, dq, qc, qa, &lim);
    trig_advance_f1(m, arm, qc, qa, q_old, ((it + 1) % Trig<T>::kResync) == 0, sn, cs);
  } else {
    cont_update(m, prm, arm, s, dq, it, qc, qa, sn, cs);
  }
}

// In-kernel certified stretch (IK lanes of the continuation).  The wave's
// problems leave together, as soon as one of them needs the main loop (a
// check, or max_iters): a problem left waiting while the others finish their
// stretches would run its own remainder after them (measured: 4x the wave's
// iterations with 4 problems per wave).  The others simply redo their current
// iterate in the main loop.  Out of line so that the loop gets a register
// allocation of its own: inlined into the continuation kernel, whose live
// state spills it to AGPRs, the same iteration issued 4.5x the VALU
// instructions of ikg_cert_stretch_kernel's (PMC).  The caller's state is
// saved once per stretch instead.
template <typename T, bool DAMPED, class SP>
__device__ __noinline__ void cert_stretch(const KModel<T>* __restrict__ m, int max_iters, T eps2, T dt, T lambda,
                                          int arm, int li, const T* RT_, const T* tT_, const T* Rr_,
                                          const T* qcert_, T cbudget, T& qc_io, T* qa_io, T* sn_io, T* cs_io,
                                          int& it_io) {
  KParams<T> prm;
  prm.max_iters = max_iters;
  prm.eps2 = eps2;
  prm.dt = dt;
  prm.lambda = lambda;
  T RT[9], tT[3], Rr[7], qcert[7], qa[kArmDof], sn[7], cs[7];
#pragma unroll
  for (int i = 0; i < 9; ++i) RT[i] = RT_[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) tT[i] = tT_[i];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    Rr[i] = Rr_[i];
    qcert[i] = qcert_[i];
    sn[i] = sn_io[i];
    cs[i] = cs_io[i];
  }
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) qa[k] = qa_io[k];
  T qc = qc_io;
  int it = it_io;
  ThetaTrack<T> tk{};
  ArmLimits<T> lim;
  load_limits(m, arm, lim);
  if constexpr (kStretchF1<SP, DAMPED>) trig_exact_f1(m, arm, qc, qa, sn, cs);  // frame-1 slots (a resync)
  for (int n = 0;; ++n) {
    if (__any(it >= max_iters)) break;
    T dq[6], s;
    const T x = stretch_step<T, DAMPED, SP>(m, prm, arm, sn, cs, RT, tT, dq, s, &tk,
                                            n == 0 || (it % Trig<T>::kResync) == 0);
    const T xo = pair_swap(x);
    const T em = motion_bound(qc, qa, qcert, Rr);
    const T et = em + pair_swap(em);
    const bool conv2 = x < eps2 && xo < eps2;
    if (__any(conv2 && !(et < cbudget))) break;
    if (conv2 && li == 0) SKIP_STAT(1, 1);
    if (li == 0) SKIP_STAT(6, 1);
    stretch_update<T, DAMPED, SP>(m, prm, arm, s, dq, it, qc, qa, sn, cs, lim);
    ++it;
  }
  // the caller's loop reads the chest-frame slots
  if constexpr (kStretchF1<SP, DAMPED>) trig_exact(qc, qa, sn, cs);
  qc_io = qc;
  it_io = it;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    sn_io[i] = sn[i];
    cs_io[i] = cs[i];
  }
#pragma unroll
  for (int k = 0; k < kArmDof; ++k) qa_io[k] = qa[k];
}

// occupancy the guarded step's cold LQ branch (pinv_step_*) must not cost:
// the register bound of the kernels before it (spills go to that branch)
template <typename T, bool DAMPED, class SP>
constexpr int kContMinWaves = (sizeof(T) == 4 && kFrame1<SP> && !DAMPED) ? 2 : 1;
template <typename T, bool DAMPED, class SP>
constexpr int kStretchMinWaves = (kFrame1<SP> && !DAMPED) ? (sizeof(T) == 8 ? 2 : 4) : 1;

template <typename T, bool DAMPED, class SP, int G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kContMinWaves<T, DAMPED, SP>)))
void ikg_collide_continue_kernel(const KModel<T>* __restrict__ m,
                                                                  const KCollision<T>* __restrict__ c,
                                                                  KParams<T> prm, const T* __restrict__ targets,
                                                                  int64_t S_per_target, int64_t B,
                                                                  T* __restrict__ q_out,
                                                                  uint8_t* __restrict__ conv,
                                                                  int32_t* __restrict__ iters,
                                                                  T* __restrict__ err,
                                                                  int32_t* __restrict__ witness, int handoff,
                                                                  int32_t* __restrict__ stretch_list,
                                                                  int32_t* __restrict__ stretch_count,
                                                                  T* __restrict__ stretch_rec,
                                                                  const int32_t* __restrict__ cont_list,
                                                                  const int32_t* __restrict__ cont_count) {
  extern __shared__ __align__(16) char lds[];
  constexpr int LG = 64 / G;
  const int lane = threadIdx.x;
  const int g = lane / LG, li = lane % LG, lane0 = g * LG;
  const unsigned long long gmask = LG == 64 ? ~0ull : (((1ull << LG) - 1ull) << lane0);
  const int nq = m->nq;
  const GroupLds<T> V = group_view<T>(lds, g, nq, c->n_geoms);
  // the pre-screen's colliding problems, compacted in problem order
  // (ikg_compact_*_kernel): G per wave instead of ~G * fraction colliding
  const int64_t slot = (int64_t)blockIdx.x * G + g;
  const int64_t p = slot < (int64_t)*cont_count ? (int64_t)cont_list[slot] : B;
  // problems whose hand errors passed in the pair kernel and whose first
  // check collided (ikg_prescreen_kernel: the others are final, success)
  const bool started = p < B && conv[p] != 0 && witness[p] >= 0;
  if (!__any(started)) return;  // whole wave
  bool active = started;
  if (active) {
    const int64_t t_idx = S_per_target > 1 ? p / S_per_target : p;
    for (int j = li; j < nq; j += LG) {
      const T qj = q_out[p * nq + j];
      V.q[j] = qj;
      Prec<T>::sincos_(qj, &V.sn[j], &V.cs[j]);
      joint_local(m, j, V.sn[j], V.cs[j], V.L[j]);  // the passive joints' entries are used
      V.par[j] = m->jparent[j];
    }
    if (li < 12) V.tgt[li] = targets[t_idx * 12 + li];
    if (li < 2) {  // the pre-screen's colliding pair is the first witness
      const int w = witness[p];
      const int gg = c->pairs[w][li];
      Witness<T>& W = *V.W;
      W.gjoint[li] = c->joint[gg];
      W.gkind[li] = c->kind[gg];
      W.gtarget[li] = gg == c->target_geom;
      for (int i = 0; i < 9; ++i) W.gR[li][i] = c->R[gg][i];
      for (int i = 0; i < 3; ++i) W.gt[li][i] = c->t[gg][i];
      for (int i = 0; i < 3; ++i) W.gdims[li][i] = c->dims[gg][i];
      W.gbrad[li] = c->brad[gg];
    }
    if (li == 0) {
      V.W->pair = witness[p];
      V.W->cert_ok = 0;
      V.W->skip_ok = 0;
      V.W->epa_wait = 0;
      V.W->gen = 0;
      V.W->budget = 0.0;
      V.flag[3] = T(0);
    }
  }
  __syncthreads();
  const int arm = li & 1;
  const bool ik = active && li < 2;
  T RT[9], tT[3], qc = T(0), qa[kArmDof] = {}, sn[7], cs[7];
  if (ik) {
    hook_target(m, arm, V.tgt, RT, tT);
    qc = V.q[m->root_q];
    for (int k = 0; k < kArmDof; ++k) qa[k] = V.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]];
    trig_exact(qc, qa, sn, cs);
  }
  int it = active ? iters[p] : 0;
  bool success = false, passive_clamped = it > 0;
  T nrm = T(0);
#ifdef IKG_CPROF
  unsigned long long prof[5] = {0, 0, 0, 0, 0}, t = clock64(), a_fk = 0, a_up = 0, a_col = 0;
  const int it0 = it;
  bool cp_lead = li == 0 && active;
#else
  unsigned long long* prof = nullptr;
#endif
  // the IK lanes' copy of the penetration certificate (Witness gen / skip_ok /
  // budget / Rmot of their chain joints) and the motion bound accumulated
  // against it, in registers: no LDS traffic per iteration but one int read
  int cgen = 0;
  bool cert_live = false, handed = false;
  T Rr[7] = {};
  T qcert[7] = {}, cbudget = T(0);
  for (;;) {
#ifdef IKG_CPROF
    cp_lead = li == 0 && active;
#endif
    // Certified stretch: while the witness pair provably intersects, the
    // reference's stop test cannot pass, so the IK lanes iterate alone (no
    // LDS flags, no barriers, no joint frames).  handoff != 0: the problem
    // leaves for ikg_cert_stretch_kernel (pair layout, the batch kernel's
    // registers and pace) with its remaining margin; otherwise the stretch
    // runs here.  Either way it ends at the first iterate whose errors pass
    // once the margin is spent (redone below with a real check) or at max_iters.
    // the group's decision (its IK lanes'), for every lane of the group
    const bool go_ik = active && li < 2 && cert_live && passive_clamped;
    const bool go = __shfl(go_ik ? 1 : 0, lane0) != 0;
    if (!handoff && go) {
      // every lane of the group runs the stretch, the others mirroring their
      // arm's IK lane bit for bit: a wave issues the same instruction stream
      // either way, but with 2 live lanes out of 64 it ran 2.5x slower
      // (tools/probe/mirror.sh); only the IK lanes keep the results
      const int src = lane0 + arm;
      qc = __shfl(qc, src);
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qa[k] = __shfl(qa[k], src);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        sn[k] = __shfl(sn[k], src);
        cs[k] = __shfl(cs[k], src);
        Rr[k] = __shfl(Rr[k], src);
        qcert[k] = __shfl(qcert[k], src);
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) RT[k] = __shfl(RT[k], src);
#pragma unroll
      for (int k = 0; k < 3; ++k) tT[k] = __shfl(tT[k], src);
      cbudget = __shfl(cbudget, src);
      cert_stretch<T, DAMPED, SP>(m, prm.max_iters, prm.eps2, prm.dt, prm.lambda, arm, li, RT, tT, Rr, qcert,
                                  cbudget, qc, qa, sn, cs, it);
      if (li < 2) {
        if (arm == 0) V.q[m->root_q] = qc;
        for (int k = 0; k < kArmDof; ++k) V.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
      }
    }
    if (handoff && go_ik) {
      if (li == 0) {
        V.flag[3] = T(1);
        stretch_rec[p * kStretchRec] = cbudget;
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        stretch_rec[p * kStretchRec + 1 + 7 * arm + k] = Rr[k];
        stretch_rec[p * kStretchRec + 15 + 7 * arm + k] = qcert[k];
      }
    }
    if (handoff) {
      __syncthreads();
      if (active && V.flag[3] != T(0)) {
        handed = true;
        active = false;
      }
    }
    __syncthreads();
    // FK + errors at the current iterate (:58-67) and, before the collision
    // check, the update it would take (:75-83): the Jacobian state dies here,
    // so only q, dq and the trig state stay live across the check
    T dq[6], s = T(0);
    if (active && li < 2) {
      nrm = cont_step<T, DAMPED, SP>(m, prm, arm, sn, cs, RT, tT, V.F, dq, s);
      const T other = pair_swap(nrm);
      if (li == 0) V.flag[0] = (nrm < prm.eps2 && other < prm.eps2) ? T(1) : T(0);
      if (V.W->gen != cgen) {  // only invalidations reach here (passive clamp): drop it
        cgen = V.W->gen;
        cert_live = false;
      }
      // collision(q) is known True while the motion bound stays below the margin
      const T em = cert_live ? motion_bound(qc, qa, qcert, Rr) : T(0);
      const T tot = em + pair_swap(em);
      if (li == 0) V.flag[2] = (cert_live && tot < cbudget) ? T(1) : T(0);
    }
    __syncthreads();
    CPROF_MARK(a_fk, t);
    if (active && it >= prm.max_iters) active = false;  // loop exhausted: success stays false
    const bool need = active && V.flag[0] != T(0);
    // the witness pair provably still intersects (certified margin not yet
    // used up by the motion bound): collision(q) is True without a check
    const bool known = need && V.flag[2] != T(0);
    if (need && !known && li == 0 && V.W->skip_ok) {  // spent: check, then certify afresh
      V.W->skip_ok = 0;
      V.W->epa_wait = 0;
      ++V.W->gen;
    }
    const bool check = need && !known;
    if (li == 0 && check) SKIP_STAT(0, 1);
    if (li == 0 && active) SKIP_STAT(7, 1);
    if (li == 0 && known) SKIP_STAT(1, 1);
    if (__any(check)) {
      const bool col = collide_group<T, LG>(m, c, V, li, lane0, check, gmask, prof);
      if (check && !col) {
        success = true;  // :70 errors pass and no collision
        active = false;
      }
    }
    CPROF_MARK(a_col, t);
    if (__any(check)) __syncthreads();  // collide_group's last witness / certificate writes
    if (active && li < 2 && V.W->gen != cgen) {
      // certificate (re)made or dropped at this iterate's check: reload it; the
      // bound counts the motion from this iterate on
      cgen = V.W->gen;
      cert_live = V.W->skip_ok != 0;
      qcert[0] = qc;
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qcert[k + 1] = qa[k];
      if (cert_live) {
        cbudget = T(V.W->budget);
        Rr[0] = arm == 0 ? V.W->Rmot[m->root_q] : T(0);  // the root is counted once (left lane)
        for (int k = 0; k < kArmDof; ++k) Rr[k + 1] = V.W->Rmot[arm ? m->arm_q[1][k] : m->arm_q[0][k]];
      }
    }
    if (active && li < 2) {  // apply the update (:86-89)
      cont_update(m, prm, arm, s, dq, it, qc, qa, sn, cs);
      if (arm == 0) V.q[m->root_q] = qc;
      for (int k = 0; k < kArmDof; ++k) V.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
    }
    if (active && !passive_clamped && li == 0 && V.W->skip_ok) {  // the passive joints may move: drop it
      V.W->skip_ok = 0;
      ++V.W->gen;
    }
    if (active && !passive_clamped) {  // projecttojointlimits on every joint after the first update
      for (int i = li; i < m->n_passive; i += LG) {
        const int j = m->passive_q[i];
        V.q[j] = clampq(V.q[j], m->lo[j], m->hi[j]);
        Prec<T>::sincos_(V.q[j], &V.sn[j], &V.cs[j]);
        joint_local(m, j, V.sn[j], V.cs[j], V.L[j]);
      }
    }
    if (active) {
      passive_clamped = true;
      ++it;
    }
    CPROF_MARK(a_up, t);
    if (!__any(active)) break;
    __syncthreads();
  }
  __syncthreads();
#ifdef IKG_CPROF
  if (li == 0 && started) {
    atomicAdd(&g_cprof[0], a_fk);
    atomicAdd(&g_cprof[1], a_col);
    atomicAdd(&g_cprof[2], a_up);
    atomicAdd(&g_cprof[3], prof[0]);
    atomicAdd(&g_cprof[4], prof[1]);
    atomicAdd(&g_cprof[5], prof[2]);
    atomicAdd(&g_cprof[6], prof[3]);
    atomicAdd(&g_cprof[7], (unsigned long long)(it - it0));
  }
#endif
  if (started) {
    for (int j = li; j < nq; j += LG) q_out[p * nq + j] = V.q[j];
    if (handed) {  // continues in ikg_cert_stretch_kernel: pending (-2 - pair), listed
      if (li == 0) {
        iters[p] = it;
        witness[p] = -2 - V.W->pair;
        stretch_list[atomicAdd(stretch_count, 1)] = (int32_t)p;
      }
    } else {
      if (li < 2) err[p * 2 + arm] = sqrt(nrm);
      if (li == 0) {
        conv[p] = success ? 1 : 0;
        iters[p] = it;
        witness[p] = -1;  // final
      }
    }
  }
}

// Certified stretches handed off by the continuation (stretch_list): pair
// layout as in ikg_pair_batch_kernel (two lanes per problem, up to 32 per
// wave, spread over the chip when few), the batch kernel's chest-frame
// iteration, with the continuation's margin test: while the motion bound
// stays below the remaining certified margin the witness pair still
// intersects, so the stop test of inverse_geometry.py:70 cannot pass.  Ends
// at max_iters (final: not converged) or at the first iterate whose errors
// pass once the margin is spent (witness[p] back to the pair: the next
// continuation launch redoes that iterate with a real check).
template <typename T, bool DAMPED, class SP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? kStretchMinWaves<T, DAMPED, SP> : 1)))
void ikg_cert_stretch_kernel(const KModel<T>* __restrict__ m, KParams<T> prm,
                                                              const T* __restrict__ targets, int64_t S_per_target,
                                                              T* __restrict__ q_out, uint8_t* __restrict__ conv,
                                                              int32_t* __restrict__ iters, T* __restrict__ err,
                                                              int32_t* __restrict__ witness,
                                                              const int32_t* __restrict__ stretch_list,
                                                              const int32_t* __restrict__ stretch_count,
                                                              const T* __restrict__ stretch_rec, int ppw_min) {
  const int n = *stretch_count;
  const int lane = threadIdx.x, arm = lane & 1;
  const int nb = (int)gridDim.x;
  // ppw_min < 0 (timing experiment): one problem per wave, every lane pair
  // of the wave computing it, lanes 0/1 storing
  const bool mirror = ppw_min < 0;
  const int ppw = mirror ? 1 : min(32, max(ppw_min, (n + nb - 1) / nb));
  const bool writer = !mirror || lane < 2;
  const int nq = m->nq;
  for (int base = (int)blockIdx.x * ppw; base < n; base += nb * ppw) {
    const int i = base + (mirror ? 0 : lane >> 1);
    if ((!mirror && lane >= 2 * ppw) || i >= n) continue;  // both lanes of a pair together
    const int64_t p = stretch_list[i];
    const int64_t tgt = S_per_target > 1 ? p / S_per_target : p;
    T RT[9], tT[3], qc, qa[kArmDof], sn[7], cs[7], Rr[7], qcert[7];
    hook_target(m, arm, targets + tgt * 12, RT, tT);
    T* qrow = q_out + p * nq;
    qc = qrow[m->root_q];
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) qa[k] = qrow[arm ? m->arm_q[1][k] : m->arm_q[0][k]];
    if constexpr (kStretchF1<SP, DAMPED>)
      trig_exact_f1(m, arm, qc, qa, sn, cs);
    else
      trig_exact(qc, qa, sn, cs);
    ArmLimits<T> lim;
    load_limits(m, arm, lim);
    const T budget = stretch_rec[p * kStretchRec];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      Rr[k] = stretch_rec[p * kStretchRec + 1 + 7 * arm + k];
      qcert[k] = stretch_rec[p * kStretchRec + 15 + 7 * arm + k];
    }
    int it = iters[p];
    T x;
    bool final = false;
    ThetaTrack<T> tk{};
    for (int r = 0;; ++r) {
      T dq[6], s;
      x = stretch_step<T, DAMPED, SP>(m, prm, arm, sn, cs, RT, tT, dq, s, &tk,
                                      r == 0 || (it % Trig<T>::kResync) == 0);
      const T xo = pair_swap(x);
      const T em = motion_bound(qc, qa, qcert, Rr);
      const T et = em + pair_swap(em);
      if (it >= prm.max_iters) {  // loop exhausted (:100): the last errors are reported
        final = true;
        break;
      }
      if (x < prm.eps2 && xo < prm.eps2) {
        if (!(et < budget)) break;
        if (arm == 0) SKIP_STAT(1, 1);
      }
      stretch_update<T, DAMPED, SP>(m, prm, arm, s, dq, it, qc, qa, sn, cs, lim);
      ++it;
    }
    if (!writer) continue;
    if (arm == 0) qrow[m->root_q] = qc;
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) qrow[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
    if (final) err[p * 2 + arm] = sqrt(x);
    if (arm == 0) {
      iters[p] = it;
      if (final) conv[p] = 0;
      witness[p] = final ? -1 : -2 - witness[p];
    }
  }
}

// Problems the pre-screen left colliding (witness >= 0), listed in problem
// order: ikg_compact_count_kernel counts each block's chunk, then
// ikg_compact_write_kernel adds the earlier chunks' counts and writes its
// chunk's problems in rounds of 256 (wave ballots + a 4-wave prefix).
// Order-preserving, so the continuation's grouping (and with it the results,
// bit for bit) does not depend on scheduling.  Coalesced: one thread per
// element per round (the single-workgroup form, one thread per contiguous
// chunk, took 100 us at 131,072 problems).
constexpr int kCompactChunk = 4096;

__global__ __launch_bounds__(256) void ikg_compact_count_kernel(const int32_t* __restrict__ witness, int64_t B,
                                                                int32_t* __restrict__ counts) {
  __shared__ int32_t part[4];
  const int t = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kCompactChunk, b1 = min(B, b0 + kCompactChunk);
  int n = 0;
  for (int64_t i = b0 + t; i < b1; i += 256) n += witness[i] >= 0;
  n = __popcll(__ballot(n & 1)) + 2 * __popcll(__ballot(n & 2)) + 4 * __popcll(__ballot(n & 4)) +
      8 * __popcll(__ballot(n & 8)) + 16 * __popcll(__ballot(n & 16));  // n <= 16 per thread
  if ((t & 63) == 0) part[t >> 6] = n;
  __syncthreads();
  if (t == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void ikg_compact_write_kernel(const int32_t* __restrict__ witness, int64_t B,
                                                                const int32_t* __restrict__ counts,
                                                                int32_t* __restrict__ list,
                                                                int32_t* __restrict__ count) {
  __shared__ int32_t part[4];
  __shared__ int32_t base;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (wv == 0) {  // offset of this chunk: the earlier chunks' counts
    int s = 0;
    for (int j = lane; j < (int)blockIdx.x; j += 64) s += counts[j];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) base = s;
  }
  __syncthreads();
  int off = base;
  const int64_t b0 = (int64_t)blockIdx.x * kCompactChunk, b1 = min(B, b0 + kCompactChunk);
  const unsigned long long below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int64_t r = b0; r < b1; r += 256) {
    const int64_t i = r + t;
    const bool f = i < b1 && witness[i] >= 0;
    const unsigned long long m = __ballot(f);
    if (lane == 0) part[wv] = __popcll(m);
    __syncthreads();
    int wo = off;
    for (int k = 0; k < wv; ++k) wo += part[k];
    if (f) list[wo + __popcll(m & below)] = (int32_t)i;
    off += part[0] + part[1] + part[2] + part[3];
    __syncthreads();
  }
  if (blockIdx.x == gridDim.x - 1 && t == 0) *count = off;
}

// First check of the collision continuation for every problem whose errors
// passed (inverse_geometry.py:70), one wave per problem (64 lanes per sweep,
// against 16 in the continuation's groups): collision-free ones are final
// (success); for colliding ones the colliding pair found seeds the
// continuation's witness.  witness[p] = that pair, -1 if none / not converged.
template <typename T>
__global__ __launch_bounds__(64) void ikg_prescreen_kernel(const KModel<T>* __restrict__ m,
                                                           const KCollision<T>* __restrict__ c,
                                                           const T* __restrict__ q, const T* __restrict__ targets,
                                                           int64_t S_per_target, int64_t B,
                                                           const uint8_t* __restrict__ conv,
                                                           int32_t* __restrict__ witness,
                                                           int32_t* __restrict__ app_list = nullptr,
                                                           int32_t* __restrict__ app_count = nullptr) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  __shared__ Witness<T> W;
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (!conv[p]) {  // wave-uniform
    if (lane == 0) witness[p] = -1;
    return;
  }
  const int64_t t_idx = S_per_target > 1 ? p / S_per_target : p;
  if (lane < m->nq) S.q[lane] = q[p * m->nq + lane];
  if (lane < 12) tgt[lane] = targets[t_idx * 12 + lane];
  if (lane == 0) {
    W.pair = -1;
    W.cert_ok = 0;
  }
  __syncthreads();
  stage_trig_par(m, S);
  __syncthreads();
#ifdef IKG_CPROF
  unsigned long long prof[5] = {0, 0, 0, 0, 0};
  const bool col = collide_wave<T, true>(m, c, S, tgt, W, prof);
  if (lane == 0) {  // pre-screen: checks, frames, sweep, of it the sphere pass (tools/scan_prof.py)
    atomicAdd(&g_scan[24], 1ull);
    atomicAdd(&g_scan[25], prof[0]);
    atomicAdd(&g_scan[26], prof[2]);
    atomicAdd(&g_scan[27], prof[4]);
  }
#else
  const bool col = collide_wave<T, true>(m, c, S, tgt, W);
#endif
  if (lane == 0) {
    witness[p] = col ? W.pair : -1;
    if (col && app_list) app_list[atomicAdd(app_count, 1)] = (int32_t)p;  // colliding: listed (no compaction)
  }
}

// ---------------------------------------------------------------- trajectory-first continuation
// The iterates of inverse_geometry.py:56-89 do not depend on the collision
// test: `and not collision(robot, q)` (:70) only decides at which iterate the
// loop stops, the update is the same either way.  So for the problems the
// pre-screen left colliding, the updates and the checks are decoupled:
//   ikg_traj_kernel       runs the IK updates at the batch kernel's pace (pair
//                         layout, the frame-1 loop, no checks, no LDS) and
//                         records every iterate's q, hand errors and stop-test
//                         verdict, in windows of Wn iterates;
//   ikg_traj_scan_kernel  one wave per problem walks the window's records in
//                         order: witness-first checks at the iterates whose
//                         errors pass, a penetration certificate after a
//                         colliding one, and the certificate's motion bound
//                         (evaluated 64 records at a time, one per lane) to
//                         skip the iterates it proves colliding; the first
//                         passing iterate without collision is the answer.
// The answer is the reference's: the first passing iterate that is
// collision-free, else the iterate after max_iters updates with
// success = False.  Replaces the interleaved continuation, whose certified
// stretches ran at ~2.9 us per update inside the check kernel against ~1 us
// here.
template <typename T>
struct TrajCert {  // a problem's witness pair between windows
  int32_t pair;
};

// Windows alternate between two record buffers (parity r & 1): window r + 1's
// updates run in the same launch as window r's scan.
template <typename T>
struct TrajWs {
  T* rec;             // [parity][slot][Wn][rec_len]: q, squared hand errors, stop test (see below)
  T* qrun;            // [slot][nq]: the iterate the next window starts from
  int32_t* itrun;     // its update count
  int32_t* it0;       // [parity][slot]: update count of the window's first record
  int32_t* nrec;      // [parity][slot]: records; bit 30: the last is the iterate after max_iters
  int32_t* done;      // answered
  TrajCert<T>* cst;
  int64_t slots;      // slots per parity
  int by_p = 0;       // records, counts and it0 indexed by problem (the pair kernel's records)
  int cert = 1;       // inscribed-ball certificates before the witness tests (IKG_SCAN_CERT=0: off)
  // round -2 (window checkpoints, ikg_solve.hpp kWinOf): problem i = index i of
  // the batch, every converged one checked first, then a colliding one's
  // windows tested against certificates; wit_out[i] = the colliding pair
  // found when some window is left to regenerate (flagged in wmask), -1 if
  // none, not converged or answered
  int32_t* wit_out = nullptr;
  const T* ck = nullptr;        // the batch kernel's window checkpoints
  uint32_t* wmask = nullptr;    // per problem, the windows left (mask_words each): written by round -2, read by round 0
  // round -2 over the whole batch: a problem with windows left is appended to
  // this list (its order is the atomic's: no answer depends on it -- a
  // problem's records, resume tasks and scan are its own), else compacted after
  int32_t* app_list = nullptr;
  int32_t* app_count = nullptr;
  const uint64_t* rmask = nullptr;  // round 0: per problem and window, the iterates the resume kernel recorded
  int box = 1;                  // round -2: window boxes tested (IKG_BOX_COVER)
  // round 0 after round -2: this launch scans list entries [rbase, rbase + rcap),
  // whose records are in slots i - rbase (ikg_capi.hip records capacity)
  int64_t rbase = 0, rcap = INT64_MAX;
  // round 0 after round -2, split scan: a listed problem's 64-record chunks
  // dealt round-robin to G waves (G from the listed count: about split_waves
  // waves in all, at most kScanSplitMax per problem); each wave's first
  // collision-free passing record goes to best[p] (atomicMin), and the last of
  // the G waves to arrive (arrive[p]) writes the answer.  best / arrive are set
  // by round -2 (fused) or by the host (split first check).  split_waves 0: off
  int32_t* best = nullptr;
  int32_t* arrive = nullptr;
  int split_waves = 0;
};
constexpr int kScanSplitMax = 8;
constexpr int32_t kScanNone = 0x7f7f7f7f;  // best[p] before any wave found an answer (a byte-fill value)

// IKG_SCAN_CERT=0: the records scan without inscribed-ball certificates (A/B
// knob, read at every launch so one process can compare both: the answers do
// not depend on it, tests/test_gpu_collision.py)
static int scan_cert() {
  const char* e = getenv("IKG_SCAN_CERT");
  return e ? atoi(e) : 1;
}
// waves of the records scan (grid-stride over the listed problems): one per
// problem up to 65,536.  The listed count is known only on the device, so the
// grid is sized by B and waves past it return at once.  A grid of 1,024 (one
// wave per SIMD, ~8.5 windows each at C3) took C3 + collision 2.21 ms against
// 1.98 (profiles/r05/collision/scan_waves/); IKG_SCAN_WAVES (read at every
// launch) sets it for A/Bs
// IKG_BOX_COVER=0 (read at every launch): round -2 proves no window by its box,
// so every problem that collides at its first passing iterate has all its
// records regenerated and scanned -- the round-5 records' work, for the tests
// that pin the window form's answers to it (and for A/Bs)
// The first check of a records solve: the lean pre-screen kernel checks every
// converged problem and lists the colliding ones itself, then
// ikg_first_check_kernel runs the window boxes over that list.  The fused form
// (IKG_PRESCAN=1, read at every launch: one wave per problem of the batch for
// both) carries the certificate code's registers into every problem's check --
// 1 wave per SIMD in fp64, 1.6 ms for C4's 131,072-problem share; with the
// kernels' own appends (no compaction launches) the split form is also the
// faster at C2 (70 against 75 us) and C3 (254 against 267 us),
// profiles/r06/records/prescan/
static bool first_fused(int64_t B) {
  (void)B;
  const char* e = getenv("IKG_PRESCAN");
  return e ? atoi(e) != 0 : false;
}
static int box_cover() {
  const char* e = getenv("IKG_BOX_COVER");
  return e ? atoi(e) != 0 : 1;
}
// IKG_SCAN_SPLIT (read at every launch): the split scan's wave target (0: one
// wave per listed problem)
static int scan_split() {
  const char* e = getenv("IKG_SCAN_SPLIT");
  return e ? std::max(0, atoi(e)) : 2048;
}
static int64_t scan_waves(int64_t B) {
  const char* e = getenv("IKG_SCAN_WAVES");
  const int64_t w = e ? std::max(1, atoi(e)) : 65536;
  return std::min<int64_t>(w, B);
}
// the record layout (kRec*, rec_len, store_block8) is in ikg_solve.hpp

template <typename T>
__device__ inline void rec_slots(const KModel<T>* __restrict__ m, int lane, int32_t* sl) {
  if (lane < kArmDof) {
    sl[m->arm_q[0][lane]] = kRecArm0 + lane;
    sl[m->arm_q[1][lane]] = kRecArm1 + lane;
  }
  if (lane < m->n_passive) sl[m->passive_q[lane]] = kRecPassive + lane;
  if (lane == 0) sl[m->root_q] = kRecRoot;
}

template <typename T, bool DAMPED, class SP>
__device__ __forceinline__ void traj_window(const KModel<T>* __restrict__ m, const KParams<T>& prm,
                                            const T* __restrict__ targets, int64_t S_per_target,
                                            const T* __restrict__ q_out, const int32_t* __restrict__ iters,
                                            const int32_t* __restrict__ clist, int n, const TrajWs<T>& w,
                                            int Wn, int round, int blk, int nb) {
  const int lane = threadIdx.x, arm = lane & 1;
  // full waves: a wave with few live lanes issues the same loop up to 2.5x
  // slower (Live lanes)
  constexpr int ppw = 32;
  const int nq = m->nq, RL = rec_len(m->n_passive);
  const int64_t par = (int64_t)(round & 1) * w.slots;
  for (int base = blk * ppw; base < n; base += nb * ppw) {
    const int i = base + (lane >> 1);
    if (lane >= 2 * ppw || i >= n) continue;  // both lanes of a pair together
    // answered, or its loop already exhausted: the window before recorded the
    // iterate after max_iters (itrun = max_iters + 1 marks that), and its scan,
    // running beside this window, answers it.  `done` may be stale here: extra
    // work only.  A skipped problem's record count is cleared, so the scan of
    // this window never reads the slot's records from two windows back.
    if (round > 0 && (w.done[i] || w.itrun[i] > prm.max_iters)) {
      if (arm == 0) w.nrec[par + i] = 0;
      continue;
    }
    const int64_t p = clist[i];
    const int64_t tgt = S_per_target > 1 ? p / S_per_target : p;
    T RT[9], tT[3], qc, qa[kArmDof], sn[7], cs[7];
    hook_target(m, arm, targets + tgt * 12, RT, tT);
    const T* src = round == 0 ? q_out + p * nq : w.qrun + (int64_t)i * nq;
    int it = round == 0 ? iters[p] : w.itrun[i];
    qc = src[m->root_q];
#pragma unroll
    for (int k = 0; k < kArmDof; ++k) qa[k] = src[arm ? m->arm_q[1][k] : m->arm_q[0][k]];
    if constexpr (kStretchF1<SP, DAMPED>)
      trig_exact_f1(m, arm, qc, qa, sn, cs);
    else
      trig_exact(qc, qa, sn, cs);
    ArmLimits<T> lim;
    load_limits(m, arm, lim);
    if (arm == 0) w.it0[par + i] = it;
    T* rec = w.rec + (par + i) * Wn * RL;
    // the passive joints, constant from the first update on (projecttojointlimits),
    // are written ahead: a vector load in the loop would wait for every record
    // store before it (one vmcnt for loads and stores)
    if (arm == 0)
      for (int k = 0; k < m->n_passive; ++k) {
        const int pj = m->passive_q[k];
        const T raw = src[pj], cl = clampq(raw, m->lo[pj], m->hi[pj]);
        const int jn = min(Wn, prm.max_iters + 1 - it);
        for (int j = 0; j < jn; ++j) rec[(int64_t)j * RL + kRecPassive + k] = it + j > 0 ? cl : raw;
      }
    ThetaTrack<T> tk{};
    int j = 0;
    bool ended = false;
    for (;;) {
      T dq[6], s;
      const T x = stretch_step<T, DAMPED, SP>(m, prm, arm, sn, cs, RT, tT, dq, s, &tk,
                                              j == 0 || (it % Trig<T>::kResync) == 0);
      const T xo = pair_swap(x);
      ended = it >= prm.max_iters;
      {
        // the iterate after max_iters is never tested (:56 loop exhausted)
        const T pass = (!ended && x < prm.eps2 && xo < prm.eps2) ? T(1) : T(0);
        T blk[8];
        blk[0] = arm ? pass : qc;
#pragma unroll
        for (int k = 0; k < kArmDof; ++k) blk[1 + k] = qa[k];
        blk[7] = x;  // squared: the scan takes the root of the answer's only
        store_block8(rec + (int64_t)j * RL + (arm ? kRecPass : kRecRoot), blk);
      }
      ++j;
      if (ended) break;
      stretch_update<T, DAMPED, SP>(m, prm, arm, s, dq, it, qc, qa, sn, cs, lim);
      ++it;
      if (j == Wn) break;
    }
    if (!ended) {  // the next window starts at this iterate
      T* qr = w.qrun + (int64_t)i * nq;
      if (arm == 0) {
        qr[m->root_q] = qc;
        for (int k = 0; k < m->n_passive; ++k) {
          const int pj = m->passive_q[k];
          qr[pj] = clampq(src[pj], m->lo[pj], m->hi[pj]);
        }
      }
#pragma unroll
      for (int k = 0; k < kArmDof; ++k) qr[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
    }
    if (arm == 0) {
      // a window that stops at it == max_iters without having recorded that
      // iterate (it0 + Wn == max_iters) is not `ended`: the next one records it
      w.itrun[i] = ended ? prm.max_iters + 1 : it;
      w.nrec[par + i] = j | (ended ? kTrajEnded : 0);
    }
  }
}

// Does pair `pair` intersect at configuration q (a record row)?  One lane's
// own test: the two geometries' placements from their joint chains, then the
// narrow phase.  The chains' common part (the lowest common ancestor joint up
// to the root) is built once: each branch is accumulated leaf to LCA
// (left-multiplying the local transforms), then left-multiplied by the shared
// product (round 3: the witness pairs are mostly on one arm, where the shared
// part was half of the per-record sincos and products).
template <typename T>
__device__ inline void chain_mul(const KModel<T>* __restrict__ m, const T* __restrict__ q, const int32_t* sl, int from,
                                 int stop, T (&F)[12]) {
  for (int k = from; k != stop; k = m->jparent[k]) {
    T L[12], Rn[9], tn[3], sk, ck;
    Prec<T>::sincos_(q[sl[k]], &sk, &ck);
    joint_local(m, k, sk, ck, L);
    matmul3(L, F, Rn);
    matvec3(L, F + 9, tn);
    for (int i = 0; i < 9; ++i) F[i] = Rn[i];
    for (int i = 0; i < 3; ++i) F[9 + i] = L[9 + i] + tn[i];
  }
}

template <typename T>
__device__ inline bool witness_hit_lane(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                                        int pair, const T* __restrict__ q, const int32_t* sl, const T* tgt,
                                        T (*P)[12]) {
  const int gg[2] = {c->pairs[pair][0], c->pairs[pair][1]};
  int jj[2];
  for (int h = 0; h < 2; ++h) jj[h] = gg[h] == c->target_geom ? -1 : c->joint[gg[h]];
  // lowest common ancestor of the two joints (-1: none)
  int lca = -1;
  if (jj[0] >= 0 && jj[1] >= 0) {
    uint32_t anc = 0;
    for (int k = jj[0]; k >= 0; k = m->jparent[k]) anc |= 1u << k;
    lca = jj[1];
    while (lca >= 0 && !((anc >> lca) & 1u)) lca = m->jparent[lca];
  }
  T Fs[12] = {T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0)};
  if (lca >= 0) chain_mul(m, q, sl, lca, -1, Fs);
  for (int h = 0; h < 2; ++h) {
    const int g = gg[h];
    if (g == c->target_geom) {
      for (int i = 0; i < 12; ++i) P[h][i] = tgt[i];
      continue;
    }
    const int j = jj[h];
    if (j < 0) {
      for (int i = 0; i < 9; ++i) P[h][i] = c->R[g][i];
      for (int i = 0; i < 3; ++i) P[h][9 + i] = c->t[g][i];
      continue;
    }
    T F[12] = {T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0), T(1), T(0), T(0), T(0)};
    chain_mul(m, q, sl, j, lca, F);  // leaf up to (not including) the LCA, or to the root
    if (lca >= 0) {
      T Rn[9], tn[3];
      matmul3(Fs, F, Rn);
      matvec3(Fs, F + 9, tn);
      for (int i = 0; i < 9; ++i) F[i] = Rn[i];
      for (int i = 0; i < 3; ++i) F[9 + i] = Fs[9 + i] + tn[i];
    }
    T tn[3];
    matmul3(F, c->R[g], P[h]);
    matvec3(F, c->t[g], tn);
    for (int i = 0; i < 3; ++i) P[h][9 + i] = F[9 + i] + tn[i];
  }
  const Shape<T> A{P[0], P[0] + 9, c->dims[gg[0]], c->kind[gg[0]]};
  const Shape<T> B{P[1], P[1] + 9, c->dims[gg[1]], c->kind[gg[1]]};
  return pair_collides(A, B) != 0;
}

// The scan of one window, one wave per problem (grid-stride).  Records are
// taken 64 at a time, one per lane: every record whose stop test passes is
// tested against the witness pair on its own lane (a hit proves collision(q),
// the OR over all pairs); at the first record the witness does not prove,
// the whole wave runs the full check (collide_wave's sweep): collision-free
// is the answer, else the pair found becomes the witness and the chunk's
// unproved records after it are tested against it.
// round = -1 (no pre-screen): the first check of every listed problem, at the
// iterate the batch kernel stopped at (q_out): collision-free problems are
// final there, the others get their first witness.
// ball_cert over the wave: lane 0 walks the chains, the lanes place a joint
// each, lane 0 composes, then every lane runs the point search from its own
// start (deep_point_from) and the deepest point (lowest start on a tie, as
// deep_common_point) is the certificate's.  Wave-uniform; ends synchronised.
// (inlined at each of its call sites: out of line, the call made the scan's
// registers the callee's and the scan kernels fell from 3 waves per SIMD to 2)
template <typename T>
__device__ __forceinline__ void scan_ball_cert(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c, int pair,
                                      const T* __restrict__ q, const int32_t* sl, const int32_t* par, const T* tgt,
                                      BallCert<T>& bc, T (*Lt)[12], unsigned long long* pc = nullptr) {
  const int lane = threadIdx.x;
#ifdef IKG_CPROF
  const unsigned long long c0 = clock64();
#endif
  if (lane == 0) cert_chains(c, par, pair, bc);
  __syncthreads();
  if (!bc.ok) {  // wave-uniform (LDS): no certificate
    __syncthreads();
    if (lane == 0) {
      bc.n = 0;
      bc.r = T(-1);
    }
    __syncthreads();
    return;
  }
  const int ne = bc.nl[0] + bc.nl[1] + bc.nl[2];
  for (int e = lane; e < ne; e += 64) cert_local(m, q, sl, e, bc, Lt);
  __syncthreads();
  if (lane == 0) cert_compose(c, q, sl, tgt, bc, Lt);
  __syncthreads();
#ifdef IKG_CPROF
  const unsigned long long c1 = clock64();
#endif
  T PA[12], PB[12], x[3];
  Shape<T> A{}, B{};
  cert_shapes(c, bc, PA, PB, A, B);
  static_assert(kCertStarts == 64, "one start per lane");
  const T r = deep_point_depth(A, B, lane, x);
  T best = r;
  int bl = lane;
  for (int o = 32; o > 0; o >>= 1) {
    const T ob = __shfl_xor(best, o);
    const int ol = __shfl_xor(bl, o);
    if (ob > best || (ob == best && ol < bl)) {
      best = ob;
      bl = ol;
    }
  }
#ifdef IKG_CPROF
  const unsigned long long c2 = clock64();
#endif
  __syncthreads();  // every lane has read the placements
  if (lane == bl) cert_finish(r, x, bc);
  __syncthreads();
#ifdef IKG_CPROF
  if (pc) {  // cycles: placements, point search, radius and levers (the caller's per-window counters)
    pc[4] += c1 - c0;
    pc[5] += c2 - c1;
    pc[6] += clock64() - c2;
  }
#endif
}

// Does the certificate prove every iterate of window w colliding?  Its
// iterates lie within L (the window's path length, per arm) of its first one
// in every arm joint (ikg_solve.hpp kWinOf), so |q_k - qc_k| <= |first_k - qc_k|
// + L for each; ball_covers' motion bound over that box (L widened by 1e-4 for
// the rounding of its sum).  Passive joints: constant after the first update.
// The certificate's columns are record slots (built on a record-layout row).
template <typename T>
__device__ inline bool box_covers(const BallCert<T>& bc, const T* __restrict__ cw, const T* PVr, const T* PVc,
                                  bool first_it) {
  const T L0 = cw[kCkSlot + kCkL], L1 = cw[kCkSlot + kCkArm + kCkL];  // L_w: in slot w + 1 (never k0's slot)
  T s0[2] = {T(0), T(0)}, s1[2] = {T(0), T(0)};
  for (int e = 0; e < bc.n; ++e) {
    const int rs = bc.off[e];
    T cv, hw;
    if (rs < kRecPass) {
      cv = cw[rs];
      hw = L0;
    } else if (rs < kRecPassive) {
      cv = cw[kCkArm + rs - kRecPass];
      hw = L1;
    } else {
      const int pi = rs - kRecPassive;
      cv = first_it ? PVr[pi] : PVc[pi];
      hw = first_it ? fabs(PVc[pi] - PVr[pi]) : T(0);
    }
    const T d = fabs(cv - bc.qc[e]) + hw * T(1.0001);
    const int h = bc.side[e];
    s0[h] += d;
    s1[h] += d * bc.lev[e];
  }
  return bc.r > T(0) && s1[0] + bc.r * s0[0] < bc.r && s1[1] + bc.r * s0[1] < bc.r;
}

// Round -2, a converged problem that collides at its first passing iterate
// (W.pair the pair found there).  A certificate for that pair at that
// iterate, every window's box tested against it (64 windows at a time); then,
// at the first window left, a certificate at its first iterate (a checkpoint:
// an iterate of the loop) and the windows left tested again -- up to
// kCoverCerts certificates.  All proved: every later passing iterate
// collides, so the answer is the iterate after max_iters with success = False
// (inverse_geometry.py:70, :97-98), from the final record.  Else the problem
// is listed (wit_out) with the windows left (wmask) for the resume launch and
// the records scan.  Wave-uniform; ends synchronised.
constexpr int kCoverCerts = 1;
constexpr int kCoverChunks = 4;  // windows tested: up to 64 x 4 (max_iters < 8,192); beyond, all left to the scan
template <typename T>
__device__ inline void window_covers(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                                     CollideScratch<T>& S, const T* tgt, const Witness<T>& W, const int32_t* SL,
                                     BallCert<T>& BC, const TrajWs<T>& w, int64_t p, T* __restrict__ q_out,
                                     uint8_t* __restrict__ conv, int32_t* __restrict__ iters, T* __restrict__ err) {
  __shared__ T PVr[kMaxNq], PVc[kMaxNq];  // passive joints: the first passing iterate's values, and every later one's
  __shared__ T RQ[kRecPassive + kMaxNq];  // the row a certificate is built at (record layout)
  const int lane = threadIdx.x, nq = m->nq, npv = m->n_passive;
  const int k0 = iters[p];
  const int nrec = w.nrec[p] & ~kTrajEnded;
  const int max_iters = k0 + nrec - 1;
  constexpr int K = kWinOf<T>;
  const int wf = k0 / K, nwp = rec_windows<T>(max_iters);  // this problem's windows: wf .. nwp - 1 (absolute)
  const T* ckp = w.ck + p * ck_per_problem<T>(max_iters);
  if (lane < npv) {
    const int pj = m->passive_q[lane];
    const T v = q_out[p * nq + pj];
    PVr[lane] = v;
    PVc[lane] = clampq(v, m->lo[pj], m->hi[pj]);
  }
  bool open[kCoverChunks];
#pragma unroll
  for (int k = 0; k < kCoverChunks; ++k) open[k] = lane + 64 * k >= wf && lane + 64 * k < nwp;
  const bool boxes = w.box && nwp <= 64 * kCoverChunks;
  for (int wt = wf, nc = 0; boxes && nc < kCoverCerts; ++nc) {  // wt: wave-uniform
    const T* ct = ckp + (int64_t)wt * kCkSlot;
    __syncthreads();  // RQ, BC, S.L free (the check, or the last round's tests, are done)
    if (lane < kRecPass)
      RQ[lane] = ct[kCkQ + lane];
    else if (lane < kRecPassive)
      RQ[lane] = ct[kCkArm + kCkQ + lane - kRecPass];
    else if (lane < kRecPassive + npv)
      RQ[lane] = max(k0, wt * K) > 0 ? PVc[lane - kRecPassive] : PVr[lane - kRecPassive];
    __syncthreads();
    scan_ball_cert(m, c, W.pair, RQ, SL, S.par, tgt, BC, S.L);
    const bool ok = BC.r > T(0);  // wave-uniform (LDS)
    int nxt = -1;
#pragma unroll
    for (int k = 0; k < kCoverChunks; ++k) {
      const int wi = lane + 64 * k;
      if (ok && open[k]) open[k] = !box_covers(BC, ckp + (int64_t)wi * kCkSlot, PVr, PVc, max(k0, wi * K) == 0);
      const unsigned long long b = __ballot(open[k] && wi > wt);
      if (nxt < 0 && b) nxt = 64 * k + __ffsll((long long)b) - 1;
    }
    if (nxt < 0) break;
    wt = nxt;
  }
  bool any = false;
  uint32_t* wm = w.wmask + p * mask_words<T>(max_iters);
  const int nmw = mask_words<T>(max_iters);
#pragma unroll
  for (int k = 0; k < kCoverChunks; ++k) {
    const unsigned long long b = __ballot(boxes ? open[k] : lane + 64 * k >= wf && lane + 64 * k < nwp);
    any = any || b != 0;
    if (lane < 2 && 2 * k + lane < nmw) wm[2 * k + lane] = (uint32_t)(b >> (32 * lane));
  }
  for (int k = 2 * kCoverChunks + lane; k < nmw; k += 64) wm[k] = ~0u;  // windows past the tested ones
  any = any || nmw > 2 * kCoverChunks;
  if (!any) {
    const T* fr = ckp + ck_final<T>(max_iters);
    if (lane < nq) {
      const int rs = SL[lane];
      q_out[p * nq + lane] = rs < kRecPassive ? fr[rs] : PVc[rs - kRecPassive];
    }
    if (lane < 2) err[p * 2 + lane] = sqrt(fr[lane ? kRecErr1 : kRecErr0]);
    if (lane == 0) {
      conv[p] = 0;
      iters[p] = max_iters;
    }
  }
  if (lane == 0) {
    w.wit_out[p] = any ? W.pair : -1;
    if (any && w.app_list) w.app_list[atomicAdd(w.app_count, 1)] = (int32_t)p;
  }
  __syncthreads();
}

// FIRST: round -2 only (ikg_first_check_kernel: the first check and the window
// boxes, none of the records scan's code, so its registers stay the check's)
template <typename T, bool FIRST = false>
__device__ __forceinline__ void traj_scan_body(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                                               const T* __restrict__ targets, int64_t S_per_target,
                                               const int32_t* __restrict__ clist, int n,
                                               const int32_t* __restrict__ witness0, const TrajWs<T>& w, int Wn,
                                               int round, T* __restrict__ q_out, uint8_t* __restrict__ conv,
                                               int32_t* __restrict__ iters, T* __restrict__ err, int blk, int nb) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  __shared__ Witness<T> W;
  // per-lane witness placements: live only inside a witness round, so they
  // share S's transform tables (S.L..S.cand), which the certificate (S.L as
  // its joint table) and the full check (collide_wave) use only between rounds;
  // 6 KB less LDS per wave in fp32 (17.9 -> 11.7 KB: 3 waves per SIMD)
  static_assert(offsetof(CollideScratch<T>, cand) + sizeof(S.cand) - offsetof(CollideScratch<T>, L) >=
                    sizeof(T) * 64 * 2 * 12, "witness placements fit S's transform tables");
  T(*const PL)[2][12] = reinterpret_cast<T(*)[2][12]>(&S.L[0][0]);
  __shared__ int32_t SL[kMaxNq];  // joint -> record slot
  __shared__ BallCert<T> BC;   // the witness pair's inscribed-ball certificate (ball_cert)
  __shared__ int32_t bc_pair;  // the pair BC certifies (-1: none yet for this problem)
  __shared__ int32_t bc_fail;  // a pair whose certificate came out empty: not tried again for this problem
  const int lane = threadIdx.x;
  const int nq = m->nq, RL = rec_len(m->n_passive);
  const int64_t par = (int64_t)(round & 1) * w.slots;
  rec_slots(m, lane, SL);
  const int i_end = (int)std::min<int64_t>(n, w.rbase + std::min<int64_t>(w.rcap, INT32_MAX));
  __shared__ int32_t sp_best;  // split scan: the answer of the last wave to arrive (-1: none), else -2
  // split scan (round 0 after round -2): G waves per listed problem, the same G in every wave
  const int n_ent = std::max(0, i_end - (int)w.rbase);
  const int G = (!FIRST && round == 0 && w.wmask && w.by_p && w.best && w.split_waves > 0 && n_ent > 0)
                    ? std::max(1, std::min(kScanSplitMax, w.split_waves / n_ent))
                    : 1;
  for (int64_t t = blk; t < (int64_t)n_ent * G; t += nb) {
    const int i = (int)w.rbase + (int)(t / G), g = (int)(t % G);
    // answered by an earlier scan: window r - 1's, or (no pre-screen: witness0
    // null) the first checks' before window 0
    if ((round > 0 || (round == 0 && !witness0)) && w.done[i]) continue;  // wave-uniform
    if constexpr (FIRST) round = -2;
    // FIRST: every problem of the batch (its first check, then the window
    // boxes), or with witness0 the pre-screen's colliding list (boxes only)
    const bool fused = FIRST && !witness0;
    const int64_t p = fused ? (int64_t)i : (int64_t)clist[i];
    if (FIRST && w.best && lane == 0) {  // the split scan's per-problem state (a listed problem passes here)
      w.best[p] = kScanNone;
      w.arrive[p] = 0;
    }
    if (fused && !conv[p]) {  // wave-uniform
      if (lane == 0) w.wit_out[p] = -1;
      continue;
    }
    const int64_t t_idx = S_per_target > 1 ? p / S_per_target : p;
    if (lane < 12) tgt[lane] = targets[t_idx * 12 + lane];
    if (lane < nq) S.par[lane] = m->jparent[lane];
    if (lane == 0) {  // the pre-screen's colliding pair, else the one the last window ended with
      const int wp0 = fused || (round < 0 && !FIRST) ? -1 : witness0 && (round == 0 || FIRST) ? witness0[p] : w.cst[i].pair;
      W.pair = wp0 >= 0 && wp0 < c->n_pairs ? wp0 : -1;  // a witness is only a hint: never trust an index
      W.cert_ok = 0;
      bc_pair = -1;
      bc_fail = -1;
    }
    if (round < 0 && lane < nq) S.q[lane] = q_out[p * nq + lane];
    __syncthreads();
    if (round < 0) {
      bool col = true;  // FIRST over the pre-screen's list: colliding (W.pair the pair it found)
      if (!FIRST || fused) {
        stage_trig_par(m, S);
        __syncthreads();
        col = collide_wave<T, true>(m, c, S, tgt, W);
      }
      if (lane == 0) {
        if (FIRST)
          w.wit_out[p] = -1;  // window_covers sets it when windows are left to regenerate
        else if (col)
          w.cst[i].pair = W.pair;
        else
          w.done[i] = 1;  // :70 errors pass and no collision: final as the batch kernel left it
      }
      __syncthreads();
      if constexpr (FIRST)
        if (col && W.pair >= 0) window_covers(m, c, S, tgt, W, SL, BC, w, p, q_out, conv, iters, err);
      continue;  // wave-uniform
    }
    const int64_t ix = w.by_p ? p : par + i;
    const int nr = w.nrec[ix];
    const int nrec = nr & ~kTrajEnded;
    const bool ended = (nr & kTrajEnded) != 0;
    const int it0 = w.it0[ix];
    T* rec = w.rec + (w.wmask ? (int64_t)i - w.rbase : ix) * Wn * RL;  // round 0 after round -2: slot by list entry
#ifdef IKG_CPROF
    // per-window counters, flushed once at the window's end (atomics inside the
    // loop would make the next load wait on them): 0 certificates, 1 positive,
    // 2 records tested against one, 3 proved, 4-6 certificate cycles, 7 cover
    // cycles, 8 cover calls, 9 chunk stage cycles, 10 witness cycles, 11 passive fill
    unsigned long long pc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long cp0 = clock64();
#else
    unsigned long long* pc = nullptr;
#endif
    // regenerated records (round 0 after round -2): only the windows the box
    // tests left (wm), the others proved colliding
    constexpr int K = kWinOf<T>;
    const uint32_t* wm = w.wmask ? w.wmask + p * mask_words<T>(it0 + nrec - 1) : nullptr;
    const uint64_t* rmw = w.rmask ? w.rmask + p * rec_windows<T>(it0 + nrec - 1) : nullptr;
    int rstart = 0;  // record j is iterate it0 + j, in absolute window (it0 + j) / K
    if (wm)
      for (int wa = it0 / K; rstart < nrec && !win_flagged(wm, wa); ++wa) rstart = (wa + 1) * K - it0;
    rstart = min(rstart, nrec);
    if (w.by_p) {  // the batch kernels record no passive joints: constant from the first update on
      // staged in LDS first: read from q_out inside the loop, they were reloaded
      // after every record store (q_out may alias the records), a memory round
      // trip per 64 records
      const int npv = m->n_passive;
      if (lane < npv) {
        const int pj = m->passive_q[lane];
        const T v = q_out[p * nq + pj];
        S.sn[lane] = v;                                // the first iterate's value (it0 + j = 0)
        S.cs[lane] = clampq(v, m->lo[pj], m->hi[pj]);  // every later one
      }
      __syncthreads();
      for (int j = rstart + 64 * g + lane; j < nrec; j += 64 * G)  // this wave's chunks
        if (!wm || (win_flagged(wm, (it0 + j) / K) && ((rmw[(it0 + j) / K] >> ((it0 + j) & (K - 1))) & 1ull)))
          for (int k = 0; k < npv; ++k) rec[(int64_t)j * RL + kRecPassive + k] = it0 + j > 0 ? S.cs[k] : S.sn[k];
      __syncthreads();
    }
    int ans = -1;
#ifdef IKG_CPROF
    unsigned long long sprof[5] = {0, 0, 0, 0, 0}, n_chk = 0, n_lane = 0;
    const unsigned long long st0 = clock64();
    unsigned long long* prof = sprof;
#else
    unsigned long long* prof = nullptr;
#endif
#ifdef IKG_CPROF
    pc[11] += clock64() - cp0;  // passive columns
#endif
    for (int start = rstart + 64 * g; start < nrec && ans < 0; start += 64 * G) {
#ifdef IKG_CPROF
      const unsigned long long cc0 = clock64();
#endif
      const int j = start + lane;
      // a record the resume kernel wrote: a window it regenerated, an iterate the certificate left
      const bool live = j < nrec && (!wm || (win_flagged(wm, (it0 + j) / K) &&
                                             ((rmw[(it0 + j) / K] >> ((it0 + j) & (K - 1))) & 1ull)));
      if (G > 1) {  // another wave already answered before this chunk: nothing here can be the first
        if (!__any(live)) continue;
        const int b = __builtin_amdgcn_readfirstlane(__hip_atomic_load(w.best + p, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT));
        if (b < start) break;
      }
      const T* r = rec + (int64_t)(live ? j : rstart) * RL;
      bool need = live && r[kRecPass] != T(0);
      // inscribed-ball certificates of the witness pair: every lane's motion
      // bound against the current certificate (ball_covers) proves its record
      // colliding with no narrow phase; a new certificate (one lane's
      // placements and point search, ball_cert) at the first record left
      // unproved, at most one per chunk; what they leave goes to the witness
      // tests.  A certificate carries over to the next chunk while its pair
      // stays the witness.  It costs about a witness round and a half, so it
      // pays only when it proves most of a chunk: a pair whose new certificate
      // comes out empty (it barely intersects) or proves fewer than
      // kCertYield of the chunk's records is left to the witness tests for the
      // rest of the window.
      constexpr int kCertYield = 32;
      int n_before = 0;
      for (int cr = 0; w.cert && W.pair >= 0 && W.pair != bc_fail; ++cr) {
        if (bc_pair == W.pair) {  // wave-uniform (LDS)
#ifdef IKG_CPROF
          const unsigned long long cv0 = clock64();
#endif
          const bool cov = need && ball_covers(BC, r);
#ifdef IKG_CPROF
          const unsigned long long nn = __popcll(__ballot(need)), nc = __popcll(__ballot(cov));
          pc[7] += clock64() - cv0;
          pc[8] += 1;
          pc[2] += nn;
          pc[3] += nc;
#endif
          need = need && !cov;
        }
        const unsigned long long bn = __ballot(need);
        if (cr == 1) {  // the new certificate's yield
          if (lane == 0 && n_before - __popcll(bn) < kCertYield) bc_fail = W.pair;
          __syncthreads();
        }
        if (!bn || cr == 1) break;
        n_before = __popcll(bn);
        const int f = start + __ffsll((long long)bn) - 1;
        __syncthreads();  // every lane has read BC
        scan_ball_cert(m, c, W.pair, rec + (int64_t)f * RL, SL, S.par, tgt, BC, S.L, pc);  // S.L: free between full checks
        if (lane == 0) {
          bc_pair = BC.r > T(0) ? W.pair : -1;
          if (bc_pair < 0) bc_fail = W.pair;
        }
#ifdef IKG_CPROF
        pc[0] += 1;
        pc[1] += BC.r > T(0) ? 1 : 0;
#endif
        __syncthreads();
        if (bc_pair < 0) break;
      }
#ifdef IKG_CPROF
      const unsigned long long cw = clock64();
      pc[9] += cw - cc0;  // record reads, covers and certificates
#endif
      while (__any(need)) {
        const int wp = W.pair;
        const bool hit = need && wp >= 0 && witness_hit_lane(m, c, wp, r, SL, tgt, PL[lane]);
#ifdef IKG_CPROF
        ++n_lane;
#endif
        const unsigned long long bal = __ballot(need && !hit);
        if (!bal) break;  // every passing record of the chunk collides
        const int f = start + __ffsll((long long)bal) - 1;
        if (lane < nq) S.q[lane] = rec[(int64_t)f * RL + SL[lane]];
        if (lane == 0) W.pair = -1;  // the witness does not hit here: sweep every pair
        __syncthreads();
        stage_trig_par(m, S);
        __syncthreads();
#ifdef IKG_CPROF
        ++n_chk;
#endif
        if (!collide_wave<T, true>(m, c, S, tgt, W, prof)) {
          ans = f;  // :70 errors pass and no collision
          break;
        }
        __syncthreads();
        need = need && !hit && j > f;  // unproved records after f: try the new witness
      }
#ifdef IKG_CPROF
      pc[10] += clock64() - cw;  // witness rounds and full checks
#endif
    }
#ifdef IKG_CPROF
    if (lane == 0) {
      const unsigned long long cyc = clock64() - st0;
      atomicMax(&g_scan[0], n_chk);
      atomicAdd(&g_scan[1], n_chk);
      atomicMax(&g_scan[2], cyc);
      atomicAdd(&g_scan[3], sprof[3]);
      atomicMax(&g_scan[4], n_lane);
      atomicAdd(&g_scan[5], 1ull);
      atomicAdd(&g_scan[6], n_lane);
      atomicAdd(&g_scan[7], cyc);
      const int map[12] = {8, 9, 10, 11, 12, 13, 14, 18, 19, 16, 15, 17};
#pragma unroll
      for (int k = 0; k < 12; ++k) atomicAdd(&g_scan[map[k]], pc[k]);
    }
#endif
    if (G > 1) {  // the last of the problem's G waves writes its answer: the first over all of them
      if (lane == 0) {
        if (ans >= 0) atomicMin(w.best + p, ans);
        __threadfence();
        const bool last = atomicAdd(w.arrive + p, 1) == G - 1;
        __threadfence();
        const int b = last ? atomicMin(w.best + p, kScanNone) : kScanNone;
        sp_best = !last ? -2 : b < nrec ? b : -1;
      }
      __syncthreads();
      ans = sp_best;
      __syncthreads();
      if (ans == -2) continue;  // wave-uniform: another of the problem's waves answers
    }
    const int a = ans >= 0 ? ans : (ended ? nrec - 1 : -1);
    if (a >= 0) {  // final: the answer, or the iterate after max_iters (success = False)
      // the latter from the batch kernel's final record when its window was not regenerated
      const bool fin = ans < 0 && wm;
      const T* r = fin ? w.ck + p * ck_per_problem<T>(it0 + nrec - 1) + ck_final<T>(it0 + nrec - 1)
                       : rec + (int64_t)a * RL;
      // a passive joint keeps its value in q_out (the batch kernels never move
      // it), clamped from the first update on: not from S.sn / S.cs, which a
      // full check (stage_trig_par) overwrites, nor from the record, whose
      // passive slots another wave of a split scan fills
      if (lane < nq) {
        T v;
        if (w.by_p && SL[lane] >= kRecPassive) {
          v = q_out[p * nq + lane];
          if (fin || it0 + a > 0) v = clampq(v, m->lo[lane], m->hi[lane]);
        } else {
          v = r[SL[lane]];
        }
        q_out[p * nq + lane] = v;
      }
      if (lane < 2) err[p * 2 + lane] = sqrt(r[lane ? kRecErr1 : kRecErr0]);
      if (lane == 0) {
        conv[p] = ans >= 0 ? 1 : 0;
        iters[p] = it0 + a;
        w.done[i] = 1;
      }
    } else if (lane == 0 && G == 1) {  // the witness carries over to the next window
      w.cst[i].pair = W.pair;
    }
    __syncthreads();
  }
}

// out of line in the fused kernel: the scan's registers stay out of the update loop's allocation
template <typename T>
__device__ __noinline__ void traj_scan(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                                       const T* __restrict__ targets, int64_t S_per_target,
                                       const int32_t* __restrict__ clist, int n,
                                       const int32_t* __restrict__ witness0, const TrajWs<T>& w, int Wn, int round,
                                       T* __restrict__ q_out, uint8_t* __restrict__ conv,
                                       int32_t* __restrict__ iters, T* __restrict__ err, int blk, int nb) {
  traj_scan_body<T>(m, c, targets, S_per_target, clist, n, witness0, w, Wn, round, q_out, conv, iters, err, blk, nb);
}

// Separate launches (IKG_TRAJ_FUSE=0): window r's updates, then its scan.
template <typename T, bool DAMPED, class SP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kStretchMinWaves<T, DAMPED, SP>)))
void ikg_traj_update_kernel(const KModel<T>* __restrict__ m, KParams<T> prm,
                                                             const T* __restrict__ targets, int64_t S_per_target,
                                                             const T* __restrict__ q_out,
                                                             const int32_t* __restrict__ iters,
                                                             const int32_t* __restrict__ clist,
                                                             const int32_t* __restrict__ count, TrajWs<T> w, int Wn,
                                                             int r) {
  traj_window<T, DAMPED, SP>(m, prm, targets, S_per_target, q_out, iters, clist, *count, w, Wn, r, (int)blockIdx.x,
                             (int)gridDim.x);
}

// Round -2 over the batch (one wave per problem, grid-stride): the first
// check at the batch kernel's iterate and the window boxes (window_covers);
// with witness0, over the pre-screen's colliding list (clist, *count): the
// window boxes only
#ifndef IKG_FC_WAVES64  // timing knob: waves per SIMD the fp64 first check and records scan are compiled for
#define IKG_FC_WAVES64 1
#endif
template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 3 : IKG_FC_WAVES64)))
void ikg_first_check_kernel(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                            const T* __restrict__ targets, int64_t S_per_target, int64_t B,
                            const int32_t* __restrict__ clist, const int32_t* __restrict__ count,
                            const int32_t* __restrict__ witness0, TrajWs<T> w, T* __restrict__ q_out,
                            uint8_t* __restrict__ conv, int32_t* __restrict__ iters, T* __restrict__ err) {
  traj_scan_body<T, true>(m, c, targets, S_per_target, clist, count ? *count : (int)B, witness0, w, 0, -2, q_out, conv,
                          iters, err, (int)blockIdx.x, (int)gridDim.x);
}

// fp32: at most 168 VGPRs, so 3 waves fit a SIMD as before the certificate
// code (which alone would take the kernel to 182 and 2 waves)
template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 4 ? 3 : IKG_FC_WAVES64)))
void ikg_traj_scan_kernel(const KModel<T>* __restrict__ m,
                                                           const KCollision<T>* __restrict__ c,
                                                           const T* __restrict__ targets, int64_t S_per_target,
                                                           const int32_t* __restrict__ clist,
                                                           const int32_t* __restrict__ count,
                                                           const int32_t* __restrict__ witness0, TrajWs<T> w, int Wn,
                                                           int r, T* __restrict__ q_out, uint8_t* __restrict__ conv,
                                                           int32_t* __restrict__ iters, T* __restrict__ err) {
  traj_scan_body<T>(m, c, targets, S_per_target, clist, count ? *count : (int)w.slots, witness0, w, Wn, r, q_out,
                    conv, iters, err, (int)blockIdx.x, (int)gridDim.x);
}

// Launch r of rounds + 1: window r's updates on the first `tblocks`
// workgroups, window r - 1's scan on the others (both read only what launch
// r - 1 wrote; the two windows use different record buffers).  first != 0
// (no pre-screen): launch 0's scan part runs the first checks (round -1).
template <typename T, bool DAMPED, class SP>
__global__ __launch_bounds__(64) void ikg_traj_kernel(const KModel<T>* __restrict__ m,
                                                      const KCollision<T>* __restrict__ c, KParams<T> prm,
                                                      const T* __restrict__ targets, int64_t S_per_target,
                                                      const int32_t* __restrict__ clist,
                                                      const int32_t* __restrict__ count,
                                                      const int32_t* __restrict__ witness0, TrajWs<T> w, int Wn,
                                                      int r, int rounds, int tblocks, int first, T* __restrict__ q_out,
                                                      uint8_t* __restrict__ conv, int32_t* __restrict__ iters,
                                                      T* __restrict__ err) {
  const int n = *count;
  const int blk = (int)blockIdx.x;
  if (blk < tblocks) {
    if (r < rounds)
      traj_window<T, DAMPED, SP>(m, prm, targets, S_per_target, q_out, iters, clist, n, w, Wn, r, blk, tblocks);
  } else if (r > 0 || first) {
    traj_scan<T>(m, c, targets, S_per_target, clist, n, witness0, w, Wn, r - 1, q_out, conv, iters, err,
                 blk - tblocks, (int)gridDim.x - tblocks);
  }
}

// ------------------------------------------------------------------ launchers
template <typename T>
hipError_t launch_collision(const KModel<T>* dm, const KCollision<T>* dc, const void* q, const void* targets,
                            int64_t B, uint8_t* out, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL((ikg_collision_kernel<T>), dim3((unsigned)B), dim3(64), 0, s, dm, dc, (const T*)q,
                     (const T*)targets, B, out);
  return hipGetLastError();
}

// problems per continuation wave (IKG_CONT_G=1 selects one per wave; timing knob)
static int cont_groups() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("IKG_CONT_G");
    v = (e && atoi(e) == 1) ? 1 : 4;
  }
  return v;
}

// stream-ordered workspace of one continuation: witness / state per problem
// (>= 0: continue with this pair, -1: final, <= -2: stretch pending), the
// stretch list and its count, the stretch records (remaining margin + Rmot)
template <typename T>
struct ContWs {
  int32_t* wit;
  int32_t* list;    // stretch hand-off list
  int32_t* count;   // its length; [1]: length of clist
  int32_t* clist;   // the continuation's problems (ikg_compact_*_kernel)
  T* rec;
};

// Continuation launches that hand certified stretches to the stretch kernel
// before the last one, which runs any remaining stretch itself.  Every round
// is a grid-wide sync, and a problem whose margin runs out mid-stretch waits
// for the round's longest stretch before its re-check.  With the
// continuation's problems compacted (4 per wave), the in-kernel stretch wins
// at every measured size, so the default is 0 rounds.  Measured
// (tools/probe/rounds.sh, kernel ms per solve, 0/1/2 rounds): C2 fp64
// B=4096: 2.39/3.35/3.19; C3 fp32 B=65536: 5.10/5.38/5.71.  Before the
// compaction (problems in place, ~0.5 per wave): C2 2.47/3.45/3.17, C3
// 6.06/5.20/5.72.  IKG_HANDOFF_ROUNDS overrides (read per launch: the tests
// run both paths).
static int handoff_rounds() {
  const char* e = getenv("IKG_HANDOFF_ROUNDS");
  return e ? std::min(64, std::max(0, atoi(e))) : 0;
}

// least problems per stretch wave (IKG_STRETCH_PPW; timing knob)
static int stretch_ppw() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("IKG_STRETCH_PPW");
    v = e ? std::min(32, std::max(-1, atoi(e))) : 32;
    if (v == 0) v = 1;
  }
  return v;
}

template <typename T, bool DAMPED, class SP, int G>
static void launch_continue_g(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                              const BatchArgs& a, int nq, int ng, const ContWs<T>& w, hipStream_t s) {
  const size_t lds = (size_t)G * group_lds_bytes<T>(nq, ng);
  const dim3 grid((unsigned)((a.B + G - 1) / G));
  // stretch kernel: enough waves to give every SIMD of the chip one, at most
  const unsigned sgrid = (unsigned)std::min<int64_t>(1024, a.B);
  const int rounds = handoff_rounds();
  for (int r = 0; r <= rounds; ++r) {
    const int handoff = r < rounds;
    if (handoff) (void)hipMemsetAsync(w.count, 0, sizeof(int32_t), s);
    hipLaunchKernelGGL((ikg_collide_continue_kernel<T, DAMPED, SP, G>), grid, dim3(64), lds, s, dm, dc, prm,
                       (const T*)a.targets, a.S, a.B, (T*)a.q_out, a.converged, a.iters, (T*)a.err_out, w.wit,
                       handoff, w.list, w.count, w.rec, (const int32_t*)w.clist, (const int32_t*)(w.count + 1));
    if (handoff)
      hipLaunchKernelGGL((ikg_cert_stretch_kernel<T, DAMPED, SP>), dim3(sgrid), dim3(64), 0, s, dm, prm,
                         (const T*)a.targets, a.S, (T*)a.q_out, a.converged, a.iters, (T*)a.err_out, w.wit,
                         (const int32_t*)w.list, (const int32_t*)w.count, (const T*)w.rec, stretch_ppw());
  }
}

template <typename T, bool DAMPED, class SP>
static void launch_continue_t(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                              const BatchArgs& a, int nq, int ng, const ContWs<T>& w, hipStream_t s) {
  if (cont_groups() == 1)
    launch_continue_g<T, DAMPED, SP, 1>(dm, dc, prm, a, nq, ng, w, s);
  else
    launch_continue_g<T, DAMPED, SP, 4>(dm, dc, prm, a, nq, ng, w, s);
}

// IKG_CONT_TRAJ=0 selects the interleaved continuation (read per launch: the
// tests run both).  Above kTrajMaxB problems per launch the record windows
// shrink below 32 iterates (kTrajBudget), so the interleaved one runs there.
constexpr int64_t kTrajMaxB = 262144;
static bool cont_traj(int64_t B) {
  const char* e = getenv("IKG_CONT_TRAJ");
  if (e) return atoi(e) != 0;
  return B <= kTrajMaxB;
}

// IKG_TRAJ_FUSE=0: the updates and the scan of a window as separate launches
// (no overlap of window r + 1's updates with window r's scan)
static bool traj_fuse() {
  const char* e = getenv("IKG_TRAJ_FUSE");
  return !(e && atoi(e) == 0);
}

// record window per problem: kTrajWindow iterates per (update, scan) round,
// fewer (at least 16) when two buffers of Wn records for every problem of the
// launch would exceed kTrajBudget.  The buffers are sized by the whole batch B
// because the number of problems that continue is only known on the device:
// 2 x 128 x rec_len x sizeof(T) = 40 KB per problem in fp64 (164 MB at C2,
// 2.7 GB at B = 65,536).  Windows are relative to each problem's first
// passing iterate; every problem needs ceil((max_iters + 1 - k0) / Wn) rounds.
constexpr size_t kTrajBudget = size_t(4) << 30;
constexpr int kTrajWindow = 128;

__global__ __launch_bounds__(256) void ikg_fill_i32_kernel(int32_t* __restrict__ x, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = v;
}

template <typename T, bool DAMPED, class SP>
static hipError_t launch_traj_t(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                                const BatchArgs& a, int nq, const ContWs<T>& cw, bool first, hipStream_t s) {
  // every joint is the root, an arm joint or passive (ikg_model_build.hpp)
  const size_t RL = (size_t)rec_len(std::max(0, nq - 1 - 2 * kArmDof)), B = (size_t)a.B;
  const size_t full = (size_t)prm.max_iters + 1;
  const size_t per = 2 * RL * sizeof(T) * B;  // one iterate of every slot, both buffers
  int Wn = (int)std::min({full, (size_t)kTrajWindow, std::max<size_t>(16, kTrajBudget / per)});
  if (const char* ev = getenv("IKG_TRAJ_WINDOW"))  // timing / test knob
    Wn = (int)std::min<size_t>(full, (size_t)std::max(16, atoi(ev)));
  const int rounds = (int)((full + Wn - 1) / Wn);
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_rec = al(per * Wn), b_q = al(sizeof(T) * nq * B), b_i = al(sizeof(int32_t) * B),
               b_c = al(sizeof(TrajCert<T>) * B);
  char* ws = nullptr;
  hipError_t e = ws_alloc(a.ws_owner, (void**)&ws, b_rec + b_q + 6 * b_i + b_c, s);
  if (e != hipSuccess) return e;
  TrajWs<T> w;
  char* c = ws;
  w.rec = (T*)c, c += b_rec;
  w.qrun = (T*)c, c += b_q;
  w.itrun = (int32_t*)c, c += b_i;
  w.it0 = (int32_t*)c, c += 2 * b_i;
  w.nrec = (int32_t*)c, c += 2 * b_i;
  w.done = (int32_t*)c, c += b_i;
  w.cst = (TrajCert<T>*)c;
  w.slots = (int64_t)B;
  w.cert = scan_cert();
  ws_trace("alloc traj", ws, b_rec + b_q + 6 * b_i + b_c, s);
  poison_float(w.rec, b_rec + b_q, s);  // records, qrun
  poison_int(w.itrun, 6 * b_i + b_c, s);  // itrun, it0, nrec, done, cst
  hipLaunchKernelGGL(ikg_fill_i32_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, w.done, a.B, 0);
  const int32_t* wit0 = first ? nullptr : (const int32_t*)cw.wit;
  const int32_t* clist = (const int32_t*)cw.clist;
  const int32_t* cnt = (const int32_t*)(cw.count + 1);
  // updates: full waves of 32 problems, at most one wave per SIMD; scan: one
  // wave per problem, grid-stride
  const int tblocks = (int)std::min<int64_t>(1024, (a.B + 31) / 32);
  const int sblocks = (int)std::min<int64_t>(1024, a.B);
  if (!traj_fuse()) {
    for (int r = first ? -1 : 0; r < rounds; ++r) {
      if (r >= 0)
        hipLaunchKernelGGL((ikg_traj_update_kernel<T, DAMPED, SP>), dim3(tblocks), dim3(64), 0, s, dm, prm,
                           (const T*)a.targets, a.S, (const T*)a.q_out, (const int32_t*)a.iters, clist, cnt, w, Wn, r);
      hipLaunchKernelGGL((ikg_traj_scan_kernel<T>), dim3(sblocks), dim3(64), 0, s, dm, dc, (const T*)a.targets,
                         a.S, clist, cnt, wit0, w, Wn, r, (T*)a.q_out, a.converged, a.iters, (T*)a.err_out);
    }
  }
  for (int r = 0; traj_fuse() && r <= rounds; ++r) {
    const int nblk = tblocks + (r > 0 || first ? sblocks : 0);
    hipLaunchKernelGGL((ikg_traj_kernel<T, DAMPED, SP>), dim3(nblk), dim3(64), 0, s, dm, dc, prm,
                       (const T*)a.targets, a.S, clist, cnt, wit0, w, Wn, r, rounds, tblocks, first ? 1 : 0,
                       (T*)a.q_out, a.converged, a.iters, (T*)a.err_out);
  }
  e = hipGetLastError();
  ws_trace("free traj", ws, 0, s);
  const hipError_t ef = ws_free(a.ws_owner, ws, s);
  return e != hipSuccess ? e : ef;
}


// listed for the trajectory continuation without a pre-screen: every problem
// whose errors passed in the batch kernel (marker >= 0 for the compaction)
__global__ __launch_bounds__(256) void ikg_mark_converged_kernel(const uint8_t* __restrict__ conv, int64_t B,
                                                                 int32_t* __restrict__ mark) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < B) mark[i] = conv[i] ? 0 : -1;
}

// Pre-screen before the trajectory continuation (default), or
// IKG_TRAJ_PRESCREEN=0: every converged problem runs the updates and the first
// checks run beside window 0's updates, in its first launch.  That form took
// C2 with the collision term from 1.64 to 1.57 ms, but one in three runs of
// tests/test_gpu_graph.py gave a replay that differed from the direct solve
// (cause not found), so it stays an opt-in experiment.
static bool traj_prescreen(int64_t) {
  const char* e = getenv("IKG_TRAJ_PRESCREEN");
  return !(e && atoi(e) == 0);
}

template <typename T, bool DAMPED, class SP>
static void launch_continue_sel(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                                const BatchArgs& a, int nq, int ng, const ContWs<T>& w, hipStream_t s,
                                hipError_t& err, bool first) {
  if (cont_traj(a.B)) {
    err = launch_traj_t<T, DAMPED, SP>(dm, dc, prm, a, nq, w, first, s);
    if (err != hipErrorOutOfMemory || first) return;
    (void)hipGetLastError();  // no room for the record buffers: the interleaved continuation needs none
    err = hipSuccess;
  }
  launch_continue_t<T, DAMPED, SP>(dm, dc, prm, a, nq, ng, w, s);
}

template <typename T>
hipError_t launch_collide_continue(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                                   const BatchArgs& a, int spec, int nq, int ng, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  if (a.B > 0x7fffffff) return hipErrorInvalidValue;
  // stream-ordered workspace: the pre-screen's witness pair per problem
  const size_t ib = ((sizeof(int32_t) * (size_t)a.B + 255) & ~(size_t)255);
  char* ws = nullptr;
  hipError_t e = ws_alloc(a.ws_owner, (void**)&ws, 3 * ib + 256 + sizeof(T) * kStretchRec * (size_t)a.B, s);
  if (e != hipSuccess) return e;
  ContWs<T> w{(int32_t*)ws, (int32_t*)(ws + ib), (int32_t*)(ws + 3 * ib), (int32_t*)(ws + 2 * ib),
              (T*)(ws + 3 * ib + 256)};
  ws_trace("alloc cont", ws, 3 * ib + 256 + sizeof(T) * kStretchRec * (size_t)a.B, s);
  poison_int(ws, 3 * ib + 256, s);  // witness, lists, counts
  poison_float(w.rec, sizeof(T) * kStretchRec * (size_t)a.B, s);
  const bool damped = prm.lambda > T(0);
  hipError_t ec = hipSuccess;
  const unsigned nb = (unsigned)((a.B + kCompactChunk - 1) / kCompactChunk);
  auto compact = [&] {  // listed: witness >= 0 (the chunk counts borrow the stretch list, written only after)
    hipLaunchKernelGGL(ikg_compact_count_kernel, dim3(nb), dim3(256), 0, s, (const int32_t*)w.wit, a.B, w.list);
    hipLaunchKernelGGL(ikg_compact_write_kernel, dim3(nb), dim3(256), 0, s, (const int32_t*)w.wit, a.B,
                       (const int32_t*)w.list, w.clist, w.count + 1);
  };
  if (a.rec_used && *a.rec_used) {
    // the batch kernel wrote window checkpoints from each problem's first
    // passing iterate (ikg_solve.hpp kWinOf): (1) one wave per problem of the
    // batch checks it there and, when it collides, tests every window's box
    // against a certificate at that iterate (round -2); (2) the problems with
    // a window left are listed; (3) the batch kernel regenerates their
    // records from that window on (resume launch); (4) the records scan
    const size_t bi = ((sizeof(int32_t) * (size_t)a.B + 255) & ~(size_t)255);
    const size_t bm = ((sizeof(uint32_t) * (size_t)mask_words<T>(prm.max_iters) * (size_t)a.B + 255) & ~(size_t)255);
    const size_t bc = ((sizeof(TrajCert<T>) * (size_t)a.B + 255) & ~(size_t)255);
    const size_t br = ((sizeof(uint64_t) * (size_t)rec_windows<T>(prm.max_iters) * (size_t)a.B + 255) & ~(size_t)255);
    char* dws = nullptr;
    e = ws_alloc(a.ws_owner, (void**)&dws, bi + bm + bc + br + 2 * bi, s);
    if (e != hipSuccess) return e;
    TrajWs<T> tw{};
    tw.rec = (T*)a.rec;
    tw.nrec = a.rec_n;
    tw.it0 = a.iters;
    tw.done = (int32_t*)dws;
    tw.wmask = (uint32_t*)(dws + bi);
    tw.cst = (TrajCert<T>*)(dws + bi + bm);
    uint64_t* rmask = (uint64_t*)(dws + bi + bm + bc);
    tw.rmask = rmask;
    tw.slots = a.B;
    tw.by_p = 1;
    tw.cert = scan_cert();
    tw.ck = (const T*)a.ck;
    tw.box = box_cover();
    tw.split_waves = scan_split();
    if (tw.split_waves > 0) {
      tw.best = (int32_t*)(dws + bi + bm + bc + br);
      tw.arrive = (int32_t*)(dws + bi + bm + bc + br + bi);
    }
    ws_trace("alloc scan", dws, bi + bm + bc + br + 2 * bi, s);
    poison_int(dws, bi + bm + bc, s);
    poison_int(rmask, br, s);
    if (tw.best) poison_int(tw.best, 2 * bi, s);  // the first check sets them for every problem it may list
    // `done` is only written (read by later rounds, of which there are none here), so it needs no fill
    tw.wit_out = w.wit;
    // the problems with windows left are appended to w.clist (count w.count[1])
    // by the kernels themselves (no compaction launches; the order is the
    // atomics', and no answer depends on it)
    TrajWs<T> tf = tw;
    tf.app_list = w.clist;
    tf.app_count = w.count + 1;
    (void)hipMemsetAsync(w.count + 1, 0, 2 * sizeof(int32_t), s);
    if (first_fused(a.B)) {  // one wave per problem of the batch: the first check and the window boxes
      hipLaunchKernelGGL((ikg_first_check_kernel<T>), dim3((unsigned)std::min<int64_t>(a.B, int64_t(1) << 20)), dim3(64),
                         0, s, dm, dc, (const T*)a.targets, a.S, a.B, (const int32_t*)nullptr,
                         (const int32_t*)nullptr, (const int32_t*)nullptr, tf, (T*)a.q_out, a.converged, a.iters,
                         (T*)a.err_out);
    } else {  // the pre-screen lists the colliding (w.list, count w.count[2]), the window boxes run over that list
      hipLaunchKernelGGL((ikg_prescreen_kernel<T>), dim3((unsigned)a.B), dim3(64), 0, s, dm, dc, (const T*)a.q_out,
                         (const T*)a.targets, a.S, a.B, (const uint8_t*)a.converged, w.wit, w.list, w.count + 2);
      hipLaunchKernelGGL((ikg_first_check_kernel<T>), dim3((unsigned)scan_waves(a.B)), dim3(64), 0, s, dm, dc,
                         (const T*)a.targets, a.S, a.B, (const int32_t*)w.list, (const int32_t*)(w.count + 2),
                         (const int32_t*)w.wit, tf, (T*)a.q_out, a.converged, a.iters, (T*)a.err_out);
    }
    // the listed problems' records hold rec_slots problems (ikg_capi.hip
    // records capacity): the resume kernel and the scan run in rounds of that
    // many list entries -- launched for every round the batch could need, a
    // round past the list's end exits at once
    const int64_t cap = a.rec_slots > 0 ? std::min<int64_t>(a.rec_slots, a.B) : a.B;
    tw.wit_out = nullptr;
    for (int64_t rb = 0; rb < a.B && ec == hipSuccess; rb += cap) {
      BatchArgs r = a;
      r.rec_list = w.clist;
      r.rec_count = w.count + 1;
      r.rec_wmask = tw.wmask;
      r.rec_rmask = rmask;
      r.rec_rbase = rb;
      r.rec_rcap = cap;
      ec = launch_pair_batch<T>(dm, prm, r, spec, s);
      if (ec != hipSuccess) break;
      tw.rbase = rb;
      tw.rcap = cap;
      hipLaunchKernelGGL((ikg_traj_scan_kernel<T>), dim3((unsigned)scan_waves(cap)), dim3(64), 0, s, dm, dc,
                         (const T*)a.targets, a.S, (const int32_t*)w.clist, (const int32_t*)(w.count + 1),
                         (const int32_t*)w.wit, tw, prm.max_iters + 1, 0, (T*)a.q_out, a.converged, a.iters,
                         (T*)a.err_out);
      ec = hipGetLastError();
    }
    ws_trace("free scan", dws, 0, s);
    const hipError_t ef2 = ws_free(a.ws_owner, dws, s);
    if (ec == hipSuccess) ec = ef2;
    e = ec != hipSuccess ? ec : hipGetLastError();
    ws_trace("free cont", ws, 0, s);
    const hipError_t ef = ws_free(a.ws_owner, ws, s);
    return e != hipSuccess ? e : ef;
  }
  // trajectory continuation without a pre-screen: the first checks run in its
  // first launch, so every converged problem is listed
  const bool first = cont_traj(a.B) && !traj_prescreen(a.B);
  if (first)
    hipLaunchKernelGGL(ikg_mark_converged_kernel, dim3((unsigned)((a.B + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t*)a.converged, a.B, w.wit);
  else
    hipLaunchKernelGGL((ikg_prescreen_kernel<T>), dim3((unsigned)a.B), dim3(64), 0, s, dm, dc, (const T*)a.q_out,
                       (const T*)a.targets, a.S, a.B, (const uint8_t*)a.converged, w.wit);
  compact();
  if (spec == kSpecNextage) {
    if (damped)
      launch_continue_sel<T, true, SpecNextage>(dm, dc, prm, a, nq, ng, w, s, ec, first);
    else
      launch_continue_sel<T, false, SpecNextage>(dm, dc, prm, a, nq, ng, w, s, ec, first);
  } else if (damped) {
    launch_continue_sel<T, true, SpecGeneric>(dm, dc, prm, a, nq, ng, w, s, ec, first);
  } else if (spec == kSpecGenericWrist) {
    launch_continue_sel<T, false, SpecGenericWrist>(dm, dc, prm, a, nq, ng, w, s, ec, first);
  } else {
    launch_continue_sel<T, false, SpecGeneric>(dm, dc, prm, a, nq, ng, w, s, ec, first);
  }
  e = ec != hipSuccess ? ec : hipGetLastError();
  ws_trace("free cont", ws, 0, s);
  const hipError_t ef = ws_free(a.ws_owner, ws, s);
  return e != hipSuccess ? e : ef;
}

#ifdef IKG_CPROF
extern "C" int ikg_debug_skip(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_skip), sizeof(g_skip)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_skip), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
extern "C" int ikg_debug_wprof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wprof), sizeof(g_wprof)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[6] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wprof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
extern "C" int ikg_debug_scan(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_scan), sizeof(g_scan)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[28] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_scan), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
extern "C" int ikg_debug_cprof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cprof), sizeof(g_cprof)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_cprof), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

template hipError_t launch_collision<double>(const KModel<double>*, const KCollision<double>*, const void*,
                                             const void*, int64_t, uint8_t*, hipStream_t);
template hipError_t launch_collision<float>(const KModel<float>*, const KCollision<float>*, const void*,
                                            const void*, int64_t, uint8_t*, hipStream_t);
template hipError_t launch_collide_continue<double>(const KModel<double>*, const KCollision<double>*,
                                                    const KParams<double>&, const BatchArgs&, int, int, int,
                                                    hipStream_t);
template hipError_t launch_collide_continue<float>(const KModel<float>*, const KCollision<float>*,
                                                   const KParams<float>&, const BatchArgs&, int, int, int,
                                                   hipStream_t);

}  // namespace ikg
