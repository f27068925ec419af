// Controller kinematics: the per-tick kinematic terms of
// the task-space controller, /root/reference/control.py:284-345, for a batch of
// robot states in one launch:
//
//   pin.computeAllTerms / updateFramePlacements      -> oMf[LARM_EFF], oMf[RARM_EFF]   (:284-287, :305)
//   pin.getFrameVelocity(..., rf)                      -> frame velocity                 (:310-313)
//   pin.computeFrameJacobian(..., rf)                  -> J   (6 x nq per hand)          (:341-342)
//   pin.getFrameJacobianTimeVariation(..., rf)         -> dJ  (6 x nq per hand)          (:343-344)
//   J_dot @ vq                                         -> dJ v                           (:345)
//   desired-state FK (:292-294) and the PD errors      -> e = [x_des - x; log3(R_des R^T)],
//                                                         edot = v_des - v (LOCAL_WORLD_ALIGNED, :314-333)
//
// rf is Pinocchio's ReferenceFrame: WORLD = 0, LOCAL = 1, LOCAL_WORLD_ALIGNED = 2
// (the controller uses LOCAL_WORLD_ALIGNED).  dJ is the time derivative of the
// frame Jacobian in rf along q' = v, the quantity Pinocchio's
// getFrameJacobianTimeVariation returns.
//
// Layout: one lane per (state, hand), 32 states per 64-lane workgroup.  A lane
// walks its hand's support chain (root joint + 6 arm joints) and produces the
// 7 non-zero columns of its 6 rows of J / dJ from the point-velocity form
//   J col k  (LWA) = [a_k x (p_f - o_k); a_k]
//   dJ col k (LWA) = [a'_k x (p_f - o_k) + a_k x (p'_f - o'_k); a'_k],   a'_k = w_{k-1} x a_k
// (a_k world axis, o_k world origin, o'_k its velocity, w_{k-1} the angular
// velocity of the parent body).  The dense [12, nq] matrices of the tile's 32
// states are assembled in LDS (zeros written once per workgroup; every tile
// writes the same non-zero positions) and streamed out with 16-byte coalesced
// stores: the kernel is bound by those writes.
#include <hip/hip_runtime.h>

#include "ikg_launch.hpp"

namespace ikg {

namespace {

constexpr int kStatesPerTile = 32;

template <typename T>
__device__ inline void cross3(const T* a, const T* b, T* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// One joint of the hand's support chain: parent body frame (R, o), the point
// velocity o' of the current origin and the parent body's angular velocity w
// advance across joint j (placement (jR, jt), axis, angle (s, c), rate vj).
// Out: the joint's world axis a, its derivative a' = w_parent x a.
template <typename T>
struct ChainState {
  T R[9], o[3], od[3], w[3];
};

template <typename T>
__device__ inline void chain_joint(const KModel<T>* __restrict__ m, int j, bool first, T s, T c, T vj,
                                   ChainState<T>& st, T* a, T* ad) {
  T on[3];
  if (first) {
#pragma unroll
    for (int i = 0; i < 9; ++i) st.R[i] = m->jR[j][i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      on[i] = m->jt[j][i];
      st.od[i] = T(0);
      st.w[i] = T(0);
    }
  } else {
    T d[3];
    matvec3(st.R, m->jt[j], d);
    T wd[3];
    cross3(st.w, d, wd);  // velocity of the new origin: o' + w x (o_new - o)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      on[i] = st.o[i] + d[i];
      st.od[i] += wd[i];
    }
    T Rn[9];
    matmul3(st.R, m->jR[j], Rn);
#pragma unroll
    for (int i = 0; i < 9; ++i) st.R[i] = Rn[i];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) st.o[i] = on[i];
  // Rot_axis leaves its own axis fixed; one branch per axis keeps every index
  // compile-time (a select chain over a runtime axis is lowered to scratch)
  const int ax = m->jaxis[j];
  if (ax == 0) {
    column(st.R, 0, a);
    rotate_axis(st.R, 0, s, c);
  } else if (ax == 1) {
    column(st.R, 1, a);
    rotate_axis(st.R, 1, s, c);
  } else {
    column(st.R, 2, a);
    rotate_axis(st.R, 2, s, c);
  }
  cross3(st.w, a, ad);
#pragma unroll
  for (int i = 0; i < 3; ++i) st.w[i] += a[i] * vj;
}

// q index of chain slot k (0 = root, 1..6 = arm joints)
template <typename T>
__device__ inline int chain_q(const KModel<T>* __restrict__ m, int arm, int k) {
  return k == 0 ? m->root_q : m->arm_q[arm][k - 1];
}

template <typename T>
struct FramePass {
  T R[9], p[3], pd[3], w[3];  // effector placement, origin velocity, angular velocity (world)
};

// (sin, cos, rate) of chain slot k, read from the state's q / v rows
template <typename T>
__device__ inline int load_joint(const KModel<T>* __restrict__ m, int arm, int k, const T* __restrict__ qrow,
                                 const T* __restrict__ vrow, T& s, T& c, T& vj) {
  const int j = chain_q(m, arm, k);
  Prec<T>::sincos_(qrow[j], &s, &c);
  vj = vrow ? vrow[j] : T(0);
  return j;
}

// Forward pass to the effector frame (pin.forwardKinematics first order +
// updateFramePlacements, frame = LARM_EFF / RARM_EFF on the last arm joint).
// The chain loops stay rolled (the joint tables are indexed per lane), which
// keeps the kernel far below the register file; the compute is small next to
// the output stream.
template <typename T>
__device__ inline void frame_pass(const KModel<T>* __restrict__ m, int arm, const T* __restrict__ qrow,
                                  const T* __restrict__ vrow, FramePass<T>& f) {
  ChainState<T> st;
  T a[3], ad[3];
#pragma unroll 1
  for (int k = 0; k < 7; ++k) {
    T s, c, vj;
    const int j = load_joint(m, arm, k, qrow, vrow, s, c, vj);
    chain_joint(m, j, k == 0, s, c, vj, st, a, ad);
  }
  T d[3];
  matvec3(st.R, m->hand_t[arm], d);
  T wd[3];
  cross3(st.w, d, wd);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    f.p[i] = st.o[i] + d[i];
    f.pd[i] = st.od[i] + wd[i];
    f.w[i] = st.w[i];
  }
  matmul3(st.R, m->hand_R[arm], f.R);
}

// express a LOCAL_WORLD_ALIGNED motion column in rf (WORLD: shift to the world
// origin; LOCAL: rotate into the frame)
template <typename T>
__device__ inline void to_rf(int rf, const FramePass<T>& f, const T* lin, const T* ang, T* out) {
  if (rf == 2) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      out[i] = lin[i];
      out[3 + i] = ang[i];
    }
  } else if (rf == 0) {  // v_O = v_p + w x (0 - p) = v_p + p x w
    T pw[3];
    cross3(f.p, ang, pw);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      out[i] = lin[i] + pw[i];
      out[3 + i] = ang[i];
    }
  } else {
    matvec3_t(f.R, lin, out);
    matvec3_t(f.R, ang, out + 3);
  }
}

// 16-byte coalesced copy of a finished LDS tile to global memory
template <typename T>
__device__ inline void tile_store(const T* __restrict__ tile, T* __restrict__ dst, int n) {
  const int lane = threadIdx.x;
  if ((((uintptr_t)dst) & 15) == 0 && ((n * (int)sizeof(T)) & 15) == 0) {
    const int nv = n * (int)sizeof(T) / 16;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* s = reinterpret_cast<const u32x4*>(tile);
    u32x4* d = reinterpret_cast<u32x4*>(dst);
    for (int i = lane; i < nv; i += 64) __builtin_nontemporal_store(s[i], d + i);
  } else {
    for (int i = lane; i < n; i += 64) dst[i] = tile[i];
  }
}

}  // namespace

template <typename T>
__global__ __launch_bounds__(64) void ikg_frame_kin_kernel(const KModel<T>* __restrict__ m, const T* __restrict__ q,
                                                           const T* __restrict__ v, const T* __restrict__ qd,
                                                           const T* __restrict__ vd, int64_t B, int rf,
                                                           FrameKinOut o) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* tile = reinterpret_cast<T*>(smem);
  const int nq = m->nq;
  const int per_state = 12 * nq;
  const bool mats = o.J || o.dJ;
  if (mats) {
    for (int i = threadIdx.x; i < kStatesPerTile * per_state; i += 64) tile[i] = T(0);
  }
  const int lane = threadIdx.x;
  const int arm = lane & 1;
  const int64_t ntiles = (B + kStatesPerTile - 1) / kStatesPerTile;
  for (int64_t tix = blockIdx.x; tix < ntiles; tix += gridDim.x) {
    const int64_t p0 = tix * kStatesPerTile;
    const int ns = (int)min((int64_t)kStatesPerTile, B - p0);
    const int sl = lane >> 1;
    const bool live = sl < ns;
    const int64_t p = p0 + sl;
    const T* qrow = q + p * nq;
    const T* vrow = v ? v + p * nq : nullptr;
    FramePass<T> f;
    if (live) {
      frame_pass(m, arm, qrow, vrow, f);
      if (o.placement) {
        T* out = (T*)o.placement + p * 24 + arm * 12;
#pragma unroll
        for (int i = 0; i < 9; ++i) out[i] = f.R[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) out[9 + i] = f.p[i];
      }
      if (o.velocity) {
        T vf[6];
        to_rf(rf, f, f.pd, f.w, vf);
        T* out = (T*)o.velocity + p * 12 + arm * 6;
#pragma unroll
        for (int i = 0; i < 6; ++i) out[i] = vf[i];
      }
      if (o.err || o.derr) {  // control.py:314-333 (always LOCAL_WORLD_ALIGNED)
        FramePass<T> fd;
        frame_pass(m, arm, qd + p * nq, vd ? vd + p * nq : nullptr, fd);
        if (o.err) {
          T Re[9], zero[3] = {T(0), T(0), T(0)}, lg[6];
          matmul3_nt(fd.R, f.R, Re);  // R_des R^T
          log6(Re, zero, lg);         // rotation part = pin.log3
          T* out = (T*)o.err + p * 12 + arm * 6;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            out[i] = fd.p[i] - f.p[i];
            out[3 + i] = lg[3 + i];
          }
        }
        if (o.derr) {
          T* out = (T*)o.derr + p * 12 + arm * 6;
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            out[i] = fd.pd[i] - f.pd[i];
            out[3 + i] = fd.w[i] - f.w[i];
          }
        }
      }
    }
    // J, then dJ (+ dJ v): second pass along the chain emits the columns
#pragma unroll 1
    for (int which = 0; which < 2; ++which) {
      T* dst = which == 0 ? (T*)o.J : (T*)o.dJ;
      const bool want_dJv = which == 1 && o.dJv;
      if (!dst && !want_dJv) continue;
      if (live) {
        ChainState<T> st;
        T acc[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
        T* rows = tile + sl * per_state + 6 * arm * nq;
#pragma unroll 1
        for (int k = 0; k < 7; ++k) {
          T sj, cj, vj, a[3], ad[3];
          const int j = load_joint(m, arm, k, qrow, vrow, sj, cj, vj);
          chain_joint(m, j, k == 0, sj, cj, vj, st, a, ad);
          T r[3], lin[3], col[6];
#pragma unroll
          for (int i = 0; i < 3; ++i) r[i] = f.p[i] - st.o[i];
          if (which == 0) {
            cross3(a, r, lin);
            to_rf(rf, f, lin, a, col);
          } else {
            T rd[3], t1[3], t2[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) rd[i] = f.pd[i] - st.od[i];
            cross3(ad, r, t1);
            cross3(a, rd, t2);
#pragma unroll
            for (int i = 0; i < 3; ++i) lin[i] = t1[i] + t2[i];
            if (rf == 1) {  // d/dt (R^T J_lwa) = R^T (dJ_lwa - w x J_lwa)
              T jl[3], wl[3], wa[3];
              cross3(a, r, jl);
              cross3(f.w, jl, wl);
              cross3(f.w, a, wa);
              T l2[3], a2[3];
#pragma unroll
              for (int i = 0; i < 3; ++i) {
                l2[i] = lin[i] - wl[i];
                a2[i] = ad[i] - wa[i];
              }
              to_rf(rf, f, l2, a2, col);
            } else if (rf == 0) {  // d/dt [o x a; a] = [o' x a + o x a'; a']
              T t3[3], t4[3];
              cross3(st.od, a, t3);
              cross3(st.o, ad, t4);
#pragma unroll
              for (int i = 0; i < 3; ++i) {
                col[i] = t3[i] + t4[i];
                col[3 + i] = ad[i];
              }
            } else {
              to_rf(rf, f, lin, ad, col);
            }
#pragma unroll
            for (int i = 0; i < 6; ++i) acc[i] += col[i] * vj;
          }
          if (dst) {
#pragma unroll
            for (int i = 0; i < 6; ++i) rows[i * nq + j] = col[i];
          }
        }
        if (want_dJv) {
          T* out = (T*)o.dJv + p * 12 + arm * 6;
#pragma unroll
          for (int i = 0; i < 6; ++i) out[i] = acc[i];
        }
      }
      if (dst) {
        __syncthreads();
        tile_store(tile, dst + p0 * per_state, ns * per_state);
        __syncthreads();
      }
    }
  }
}

template <typename T>
hipError_t launch_frame_kin(const KModel<T>* dm, int nq, const void* q, const void* v, const void* qd, const void* vd,
                            int64_t B, int rf, const FrameKinOut& o, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int64_t ntiles = (B + kStatesPerTile - 1) / kStatesPerTile;
  const size_t lds = (o.J || o.dJ) ? sizeof(T) * kStatesPerTile * 12 * nq : 0;
  // enough workgroups to fill the chip several times over; each zeroes its
  // LDS tile once and then strides over tiles
  const int64_t grid = ntiles < 8192 ? ntiles : 8192;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)ikg_frame_kin_kernel<T>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((ikg_frame_kin_kernel<T>), dim3((unsigned)grid), dim3(64), lds, s, dm, (const T*)q,
                     (const T*)v, (const T*)qd, (const T*)vd, B, rf, o);
  return hipGetLastError();
}

template hipError_t launch_frame_kin<double>(const KModel<double>*, int, const void*, const void*, const void*,
                                             const void*, int64_t, int, const FrameKinOut&, hipStream_t);
template hipError_t launch_frame_kin<float>(const KModel<float>*, int, const void*, const void*, const void*,
                                            const void*, int64_t, int, const FrameKinOut&, hipStream_t);

}  // namespace ikg
