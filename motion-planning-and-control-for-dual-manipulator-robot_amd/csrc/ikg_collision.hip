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

// World joint frames -> geometry placements -> pair tests; wave-uniform result.
// Must be called by all 64 lanes of the (single-wave) workgroup.
template <typename T>
__device__ bool collide_wave(const KModel<T>* __restrict__ m, const KCollision<T>* __restrict__ c,
                             CollideScratch<T>& S, const T* tgt) {
  const int lane = threadIdx.x & 63;
  const int nq = m->nq;
  if (lane < nq) joint_local(m, lane, S.q[lane], S.L[lane]);
  __syncthreads();
  if (lane < nq) joint_world(m, lane, S.L, S.F[lane]);
  __syncthreads();
  for (int g = lane; g < c->n_geoms; g += 64) geom_world(c, g, S.F, tgt, S.P[g]);
  __syncthreads();
  bool hit = false;
  for (int k = lane; k < c->n_pairs && !hit; k += 64) hit = pair_hit(c, k, S.P);
  return __any(hit) != 0;
}

template <typename T>
__global__ __launch_bounds__(64) void ikg_collision_kernel(const KModel<T>* __restrict__ m,
                                                           const KCollision<T>* __restrict__ c,
                                                           const T* __restrict__ q, const T* __restrict__ targets,
                                                           int64_t B, uint8_t* __restrict__ out) {
  __shared__ CollideScratch<T> S;
  __shared__ T tgt[12];
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (lane < m->nq) S.q[lane] = q[p * m->nq + lane];
  if (lane < 12) tgt[lane] = targets[p * 12 + lane];
  __syncthreads();
  const bool col = collide_wave(m, c, S, tgt);
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
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  if (!conv[p]) return;  // only problems whose hand errors passed (uniform per workgroup)
  const int nq = m->nq;
  const int64_t t_idx = S_per_target > 1 ? p / S_per_target : p;
  if (lane < nq) S.q[lane] = q_out[p * nq + lane];
  if (lane < 12) tgt[lane] = targets[t_idx * 12 + lane];
  __syncthreads();
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
  for (;;) {
    ArmState<T> st;
    if (pair_lane) {  // hand errors at the current iterate (:58-67)
      T sn[7], cs[7];
      trig_exact(qc, qa, sn, cs);
      nrm = arm_fk_error<T, SP>(m, arm, sn, cs, RT, tT, st);
      other = pair_swap(nrm);
      if (lane == 0) flag[0] = (nrm < prm.eps && other < prm.eps) ? T(1) : T(0);
    }
    __syncthreads();
    if (it >= prm.max_iters) break;  // loop exhausted: success stays false
    if (flag[0] != T(0) && !collide_wave(m, c, S, tgt)) {
      success = true;  // :70 errors pass and no collision
      break;
    }
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
      if (arm == 0) {
        S.q[m->root_q] = qc;
        for (int i = 0; i < m->n_passive; ++i) {  // projecttojointlimits on every joint
          const int j = m->passive_q[i];
          S.q[j] = clampq(S.q[j], m->lo[j], m->hi[j]);
        }
      }
      for (int k = 0; k < kArmDof; ++k) S.q[arm ? m->arm_q[1][k] : m->arm_q[0][k]] = qa[k];
    }
    ++it;
    __syncthreads();
  }
  __syncthreads();
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

template hipError_t launch_collision<double>(const KModel<double>*, const KCollision<double>*, const void*,
                                             const void*, int64_t, uint8_t*, hipStream_t);
template hipError_t launch_collision<float>(const KModel<float>*, const KCollision<float>*, const void*,
                                            const void*, int64_t, uint8_t*, hipStream_t);
template hipError_t launch_collide_continue<double>(const KModel<double>*, const KCollision<double>*,
                                                    const KParams<double>&, const BatchArgs&, int, hipStream_t);
template hipError_t launch_collide_continue<float>(const KModel<float>*, const KCollision<float>*,
                                                   const KParams<float>&, const BatchArgs&, int, hipStream_t);

}  // namespace ikg
