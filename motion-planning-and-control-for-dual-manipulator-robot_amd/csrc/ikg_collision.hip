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

#include "ikg_collision.hpp"
#include "ikg_device.hpp"
#include "ikg_launch.hpp"

namespace ikg {

// Phase timing of the continuation kernel (diagnostic build only: -DIKG_CPROF,
// tools/cprof.sh).  Lane 0 of each wave accumulates shader-clock cycles per
// phase; totals are summed into g_cprof.
#ifdef IKG_CPROF
__device__ unsigned long long g_cprof[8];
#define CPROF_MARK(acc, t)                      \
  do {                                          \
    const unsigned long long _n = clock64();    \
    if ((threadIdx.x & 63) == 0) acc += _n - t; \
    t = _n;                                     \
  } while (0)
#define CPROF_ADD(i, v)                             \
  do {                                              \
    if (prof && (threadIdx.x & 63) == 0) prof[i] += v; \
  } while (0)
#else
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
template <typename T, bool WITNESS>
__device__ bool collide_wave(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                             CollideScratch<T>& S, const T* tgt, Witness<T>& W,
                             unsigned long long* prof = nullptr) {
  const int lane = threadIdx.x & 63;
  const int nq = m->nq;
#ifdef IKG_CPROF
  unsigned long long t = clock64(), a_fr = 0, a_w = 0, a_sw = 0;
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

template <typename T, bool DAMPED, class SP>
__global__ __launch_bounds__(64) void ikg_collide_continue_kernel(const KModel<T>* __restrict__ m,
                                                                  const KCollision<T>* __restrict__ c,
                                                                  KParams<T> prm, const T* __restrict__ targets,
                                                                  int64_t S_per_target, T* __restrict__ q_out,
                                                                  uint8_t* __restrict__ conv,
                                                                  int32_t* __restrict__ iters,
                                                                  T* __restrict__ err) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  __shared__ T flag[4];
  __shared__ Witness<T> W;
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (!conv[p]) return;  // only problems whose hand errors passed (uniform per workgroup)
  const int nq = m->nq;
  const int64_t t_idx = S_per_target > 1 ? p / S_per_target : p;
  if (lane < nq) S.q[lane] = q_out[p * nq + lane];
  if (lane < 12) tgt[lane] = targets[t_idx * 12 + lane];
  if (lane == 0) {
    W.pair = -1;
    W.cert_ok = 0;
  }
  __syncthreads();
  stage_trig_par(m, S);  // passive joints keep these; lanes 0/1 refresh the rest
  const int arm = lane & 1;
  const bool pair_lane = lane < 2;
  T RT[9], tT[3], qc = T(0), qa[kArmDof] = {};
  if (pair_lane) {
    hook_target(m, arm, tgt, RT, tT);
    qc = S.q[m->root_q];
    for (int k = 0; k < kArmDof; ++k) qa[k] = S.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]];
  }
  int it = iters[p];
  bool success = false;
  T nrm = T(0), other = T(0);
#ifdef IKG_CPROF
  unsigned long long prof[4] = {0, 0, 0, 0}, t = clock64(), a_fk = 0, a_up = 0, a_col = 0;
  const int it0 = it;
#else
  unsigned long long* prof = nullptr;
#endif
  bool passive_clamped = it > 0;
  for (;;) {
    __syncthreads();  // stage_trig_par / the previous update wrote S
    ArmState<T> st;
    if (pair_lane) {  // hand errors at the current iterate (:58-67)
      T sn[7], cs[7];
      trig_exact(qc, qa, sn, cs);
      nrm = arm_fk_error<T, SP>(m, arm, sn, cs, RT, tT, st);
      other = pair_swap(nrm);
      if (lane == 0) {
        flag[0] = (nrm < prm.eps && other < prm.eps) ? T(1) : T(0);
        S.sn[m->root_q] = sn[0];
        S.cs[m->root_q] = cs[0];
      }
      for (int k = 0; k < kArmDof; ++k) {
        const int j = arm ? m->arm_q[1][k] : m->arm_q[0][k];
        S.sn[j] = sn[k + 1];
        S.cs[j] = cs[k + 1];
      }
    }
    __syncthreads();
    CPROF_MARK(a_fk, t);
    if (it >= prm.max_iters) break;  // loop exhausted: success stays false
    if (flag[0] != T(0) && !collide_wave<T, true>(m, c, S, tgt, W, prof)) {
      success = true;  // :70 errors pass and no collision
      break;
    }
    CPROF_MARK(a_col, t);
    if (pair_lane) {  // one update (:75-89)
      T dq[6], alpha, beta, s;
      if constexpr (!DAMPED) {
        T u[6], v[6];
        arm_solve<T, SP>(st, u, v, alpha, beta);
        s = chest_step(alpha + pair_swap(alpha), beta + pair_swap(beta));
        arm_dq(u, v, s, dq);
      } else {
        T A[6][8], ze[6], zc[6];
        arm_system(st, A);
        arm_solve_damped(A, prm.lambda, ze, zc, alpha, beta);
        s = chest_step(alpha + pair_swap(alpha), beta + pair_swap(beta));
        arm_dq_damped(A, ze, zc, s, dq);
      }
      arm_update(m, arm, prm.dt, s, dq, qc, qa);
    }
    __syncthreads();  // the collision check may still be reading S.q
    if (pair_lane) {
      if (arm == 0) S.q[m->root_q] = qc;
      for (int k = 0; k < kArmDof; ++k) S.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
    }
    if (!passive_clamped) {  // projecttojointlimits on every joint after the first update
      for (int i = lane; i < m->n_passive; i += 64) {
        const int j = m->passive_q[i];
        S.q[j] = clampq(S.q[j], m->lo[j], m->hi[j]);
        Prec<T>::sincos_(S.q[j], &S.sn[j], &S.cs[j]);
      }
      passive_clamped = true;
    }
    ++it;
    CPROF_MARK(a_up, t);
  }
  __syncthreads();
#ifdef IKG_CPROF
  if (lane == 0) {
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
  if (lane < nq) q_out[p * nq + lane] = S.q[lane];
  if (pair_lane) {
    err[p * 2 + arm] = nrm;
    if (lane == 0) {
      conv[p] = success ? 1 : 0;
      iters[p] = it;
    }
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

template <typename T, bool DAMPED, class SP>
static void launch_continue_t(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                              const BatchArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((ikg_collide_continue_kernel<T, DAMPED, SP>), dim3((unsigned)a.B), dim3(64), 0, s, dm, dc, prm,
                     (const T*)a.targets, a.S, (T*)a.q_out, a.converged, a.iters, (T*)a.err_out);
}

template <typename T>
hipError_t launch_collide_continue(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                                   const BatchArgs& a, int spec, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  const bool damped = prm.lambda > T(0);
  if (spec == kSpecNextage) {
    if (damped)
      launch_continue_t<T, true, SpecNextage>(dm, dc, prm, a, s);
    else
      launch_continue_t<T, false, SpecNextage>(dm, dc, prm, a, s);
  } else {
    if (damped)
      launch_continue_t<T, true, SpecGeneric>(dm, dc, prm, a, s);
    else
      launch_continue_t<T, false, SpecGeneric>(dm, dc, prm, a, s);
  }
  return hipGetLastError();
}

#ifdef IKG_CPROF
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
                                                    const KParams<double>&, const BatchArgs&, int, hipStream_t);
template hipError_t launch_collide_continue<float>(const KModel<float>*, const KCollision<float>*,
                                                   const KParams<float>&, const BatchArgs&, int, hipStream_t);

}  // namespace ikg
