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
// states are assembled in LDS (zeroed once; every matrix writes the same
// non-zero positions) and streamed out with 16-byte coalesced stores.  Storing
// the rows straight from the lanes (8-byte stores 120 B apart across lanes)
// was measured 3.5x slower.
#include <hip/hip_runtime.h>

#include "ikg_launch.hpp"

namespace ikg {

namespace {

#ifndef IKG_FK_TILE
#define IKG_FK_TILE 32
#endif
constexpr int kStatesPerTile = IKG_FK_TILE;
// LDS holds the dense matrices of one slice of the tile at a time and the
// emission pass runs once per slice.  fp64: two slices of 16 states (23 KB,
// 6 workgroups per CU instead of 3) -- measured -18% for the task_space_terms
// output set, -3% for all outputs, +1% for J + dJ; fp32 (23 KB for 32 states
// already): one slice (two measured +6%).
template <typename T>
constexpr int slices() {
  return sizeof(T) == 8 ? 2 : 1;
}

template <typename T>
__device__ inline void cross3(const T* a, const T* b, T* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// sin/cos of a joint angle: ikg_device.hpp cw_sincos (Cody-Waite reduction and
// Taylor polynomials).  It replaced OCML's sincos here first, whose
// Payne-Hanek path for huge arguments dominated the code of the first version.
template <typename T>
__device__ inline void joint_sincos(T x, T* s, T* c) {
  cw_sincos(x, s, c);
}

// R <- R Rot_axis(s, c) and a = the axis column of R (unchanged by the
// rotation).  Compile-time axis: the specialised two-column update; runtime
// axis (SpecGeneric): the branch-free one-hot form R Rot = c R + s R[e]x +
// (1 - c)(R e) e^T (a select chain over a runtime axis index is lowered to
// scratch memory).
template <int AX, typename T>
__device__ inline void col_rot(T* R, int axis, T s, T c, T* a) {
  if constexpr (AX != kAxRuntime) {
    column(R, AX, a);
    rotate_axis(R, AX, s, c);
  } else {
    const T e0 = T(axis == 0), e1 = T(axis == 1), e2 = T(axis == 2);
    const T omc = T(1) - c;
    T Rn[9];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const T r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
      const T u = e0 * r0 + e1 * r1 + e2 * r2;
      a[r] = u;
      Rn[3 * r + 0] = c * r0 + s * (e2 * r1 - e1 * r2) + omc * u * e0;
      Rn[3 * r + 1] = c * r1 + s * (e0 * r2 - e2 * r0) + omc * u * e1;
      Rn[3 * r + 2] = c * r2 + s * (e1 * r0 - e0 * r1) + omc * u * e2;
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = Rn[i];
  }
}

// Walk state along a hand's support chain: body frame (R, o), the velocity o'
// of its origin and the body's angular velocity w.
template <typename T>
struct ChainState {
  T R[9], o[3], od[3], w[3];
};

// Advance the chain across slot k (0 = root, 1..6 = arm joint k-1) given the
// joint's (sin, cos) and rate.  Out: the joint's world axis a and its
// derivative a' = w_parent x a.  The placements come from the arm-structured
// tables: model-wide addresses, so they are scalar loads and each lane selects
// its arm's value (armc) -- no per-lane address arithmetic.  SP
// (ikg_device.hpp Spec) gives the compile-time axis of each slot, the exact
// zero components of the arm offsets and whether joint placements carry
// rotations (Nextage: Z | Z,Y,Y,X,Y,Z, none); SpecGeneric reads them from the
// model (axes are model-wide, so the runtime-axis branches stay uniform).
template <class SP, typename T>
__device__ inline void chain_joint(const KModel<T>* __restrict__ m, bool right, int k, T s, T c, T vj,
                                   ChainState<T>& st, T* a, T* ad) {
  if (k == 0) {
    const bool prot = SP::prot && ((m->rot_mask >> 6) & 1);
#pragma unroll
    for (int i = 0; i < 9; ++i) st.R[i] = prot ? m->root_R[i] : T(i % 4 == 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      st.o[i] = m->root_t[i];
      st.od[i] = T(0);
      st.w[i] = T(0);
    }
    col_rot<SP::axis(0)>(st.R, m->root_axis, s, c, a);
  } else {
    const int ka = k - 1;
    T pt[3], d[3], wd[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) pt[i] = SP::zero_t(ka, i) ? T(0) : armc<T>(right, m->arm_t[0][ka][i], m->arm_t[1][ka][i]);
    matvec3(st.R, pt, d);
    cross3(st.w, d, wd);  // velocity of the new origin: o' + w x (o_new - o)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      st.o[i] += d[i];
      st.od[i] += wd[i];
    }
    if constexpr (SP::prot) {
      if (m->rot_mask & (1 << ka)) {
        T P[9], Rn[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) P[i] = armc<T>(right, m->arm_R[0][ka][i], m->arm_R[1][ka][i]);
        matmul3(st.R, P, Rn);
#pragma unroll
        for (int i = 0; i < 9; ++i) st.R[i] = Rn[i];
      }
    }
    switch (ka) {  // k is a compile-time constant of the unrolled chain loops
      case 0: col_rot<SP::axis(1)>(st.R, m->arm_axis[0], s, c, a); break;
      case 1: col_rot<SP::axis(2)>(st.R, m->arm_axis[1], s, c, a); break;
      case 2: col_rot<SP::axis(3)>(st.R, m->arm_axis[2], s, c, a); break;
      case 3: col_rot<SP::axis(4)>(st.R, m->arm_axis[3], s, c, a); break;
      case 4: col_rot<SP::axis(5)>(st.R, m->arm_axis[4], s, c, a); break;
      default: col_rot<SP::axis(6)>(st.R, m->arm_axis[5], s, c, a); break;
    }
  }
  cross3(st.w, a, ad);
#pragma unroll
  for (int i = 0; i < 3; ++i) st.w[i] += a[i] * vj;
}

// q index of chain slot k (0 = root, 1..6 = arm joints)
template <typename T>
__device__ inline int chain_q(const KModel<T>* __restrict__ m, bool right, int k) {
  return k == 0 ? m->root_q : (right ? m->arm_q[1][k - 1] : m->arm_q[0][k - 1]);
}

template <typename T>
struct FramePass {
  T R[9], p[3], pd[3], w[3];  // effector placement, origin velocity, angular velocity (world)
};

// The state's chain values: (sin, cos, rate) of the root and arm joints and
// their q indices.  All loads are issued together and the chain loops below
// are unrolled over these registers (a rolled loop waits on one global load
// per joint per pass: that exposed latency dominated the first version).
template <typename T>
struct JointVals {
  T s[7], c[7], v[7];
  int j[7];
};

template <typename T>
__device__ inline void load_joints(const KModel<T>* __restrict__ m, bool right, const T* __restrict__ qrow,
                                   const T* __restrict__ vrow, JointVals<T>& jv) {
  T qv[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    jv.j[k] = chain_q(m, right, k);
    qv[k] = qrow[jv.j[k]];
    jv.v[k] = vrow ? vrow[jv.j[k]] : T(0);
  }
#pragma unroll
  for (int k = 0; k < 7; ++k) joint_sincos(qv[k], &jv.s[k], &jv.c[k]);
}

// Forward pass to the effector frame (pin.forwardKinematics first order +
// updateFramePlacements, frame = LARM_EFF / RARM_EFF on the last arm joint).
template <class SP, typename T>
__device__ inline void frame_pass(const KModel<T>* __restrict__ m, bool right, const JointVals<T>& jv,
                                  FramePass<T>& f) {
  ChainState<T> st;
  T a[3], ad[3];
#pragma unroll
  for (int k = 0; k < 7; ++k) chain_joint<SP>(m, right, k, jv.s[k], jv.c[k], jv.v[k], st, a, ad);
  T ht[3], hR[9], d[3], wd[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) ht[i] = armc<T>(right, m->hand_t[0][i], m->hand_t[1][i]);
#pragma unroll
  for (int i = 0; i < 9; ++i) hR[i] = armc<T>(right, m->hand_R[0][i], m->hand_R[1][i]);
  matvec3(st.R, ht, d);
  cross3(st.w, d, wd);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    f.p[i] = st.o[i] + d[i];
    f.pd[i] = st.od[i] + wd[i];
    f.w[i] = st.w[i];
  }
  matmul3(st.R, hR, f.R);
}

// express a LOCAL_WORLD_ALIGNED motion column in RF (WORLD: shift to the world
// origin; LOCAL: rotate into the frame)
template <int RF, typename T>
__device__ inline void to_rf(const FramePass<T>& f, const T* lin, const T* ang, T* out) {
  if constexpr (RF == 2) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      out[i] = lin[i];
      out[3 + i] = ang[i];
    }
  } else if constexpr (RF == 0) {  // v_O = v_p + w x (0 - p) = v_p + p x w
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

// column k of J (WHICH = 0) or dJ (WHICH = 1) in RF from the chain state at
// joint k (axis a, its derivative ad) and the effector pass f
template <int WHICH, int RF, typename T>
__device__ inline void jac_column(const FramePass<T>& f, const ChainState<T>& st, const T* a, const T* ad, T* col) {
  T r[3], lin[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) r[i] = f.p[i] - st.o[i];
  if constexpr (WHICH == 0) {
    cross3(a, r, lin);
    to_rf<RF>(f, lin, a, col);
  } else if constexpr (RF == 0) {  // d/dt [o x a; a] = [o' x a + o x a'; a']
    T t3[3], t4[3];
    cross3(st.od, a, t3);
    cross3(st.o, ad, t4);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      col[i] = t3[i] + t4[i];
      col[3 + i] = ad[i];
    }
  } else {
    T rd[3], t1[3], t2[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) rd[i] = f.pd[i] - st.od[i];
    cross3(ad, r, t1);
    cross3(a, rd, t2);
#pragma unroll
    for (int i = 0; i < 3; ++i) lin[i] = t1[i] + t2[i];
    if constexpr (RF == 1) {  // d/dt (R^T J_lwa) = R^T (dJ_lwa - w x J_lwa)
      T jl[3], wl[3], wa[3], l2[3], a2[3];
      cross3(a, r, jl);
      cross3(f.w, jl, wl);
      cross3(f.w, a, wa);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        l2[i] = lin[i] - wl[i];
        a2[i] = ad[i] - wa[i];
      }
      to_rf<RF>(f, l2, a2, col);
    } else {
      to_rf<RF>(f, lin, ad, col);
    }
  }
}

// Second pass along the chain: write the lane's 6 rows of column j = chain
// joint k into `rows` (row stride nq) and accumulate dJ v (WHICH = 1).
template <int WHICH, int RF, class SP, typename T>
__device__ inline void emit_columns(const KModel<T>* __restrict__ m, bool right, const JointVals<T>& jv,
                                    const FramePass<T>& f, T* rows, int nq, T* acc) {
  ChainState<T> st;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    T a[3], ad[3], col[6];
    chain_joint<SP>(m, right, k, jv.s[k], jv.c[k], jv.v[k], st, a, ad);
    jac_column<WHICH, RF>(f, st, a, ad, col);
#pragma unroll
    for (int i = 0; i < 6; ++i) rows[i * nq + jv.j[k]] = col[i];
    if constexpr (WHICH == 1) {
#pragma unroll
      for (int i = 0; i < 6; ++i) acc[i] += col[i] * jv.v[k];
    }
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

// One tile of 32 states per workgroup.  (A grid-stride loop over tiles let the
// compiler hoist the model-table values out of the loop: more live registers.)
template <typename T, int RF, class SP>
__global__ __launch_bounds__(64) void ikg_frame_kin_kernel(const KModel<T>* __restrict__ m, const T* __restrict__ q,
                                                           const T* __restrict__ v, const T* __restrict__ qd,
                                                           const T* __restrict__ vd, int64_t B, FrameKinOut o) {
  extern __shared__ __align__(16) unsigned char smem[];
  T* tile = reinterpret_cast<T*>(smem);
  constexpr int kSlices = slices<T>();
  constexpr int kSliceStates = kStatesPerTile / kSlices;
  const int nq = m->nq;
  const int per_state = 12 * nq;
  const int lane = threadIdx.x;
  const int arm = lane & 1;
  const bool right = arm != 0;
  const int64_t p0 = (int64_t)blockIdx.x * kStatesPerTile;
  const int ns = (int)min((int64_t)kStatesPerTile, B - p0);
  const int sl = lane >> 1;
  const bool live = sl < ns;
  const int64_t p = p0 + sl;
  if (o.J || o.dJ) {
    for (int i = lane; i < kSliceStates * per_state; i += 64) tile[i] = T(0);  // once: same non-zeros every slice
  }
  JointVals<T> jv;
  FramePass<T> f;
  if (live) {
    load_joints(m, right, q + p * nq, v ? v + p * nq : nullptr, jv);
    frame_pass<SP>(m, right, jv, f);
    if (o.placement) {
      T* out = (T*)o.placement + p * 24 + arm * 12;
#pragma unroll
      for (int i = 0; i < 9; ++i) out[i] = f.R[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) out[9 + i] = f.p[i];
    }
    if (o.velocity) {
      T vf[6];
      to_rf<RF>(f, f.pd, f.w, vf);
      T* out = (T*)o.velocity + p * 12 + arm * 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) out[i] = vf[i];
    }
    if (o.err || o.derr) {  // control.py:314-333 (always LOCAL_WORLD_ALIGNED)
      JointVals<T> jd;
      FramePass<T> fd;
      load_joints(m, right, qd + p * nq, vd ? vd + p * nq : nullptr, jd);
      frame_pass<SP>(m, right, jd, fd);
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
  T* rows = tile + (sl % kSliceStates) * per_state + 6 * arm * nq;
  if (o.J) {
#pragma unroll 1
    for (int h = 0; h < kSlices; ++h) {
      if (live && sl / kSliceStates == h) emit_columns<0, RF, SP>(m, right, jv, f, rows, nq, (T*)nullptr);
      __syncthreads();
      const int nsh = min(max(ns - h * kSliceStates, 0), kSliceStates);
      tile_store(tile, (T*)o.J + (p0 + h * kSliceStates) * per_state, nsh * per_state);
      __syncthreads();
    }
  }
  if (o.dJ || o.dJv) {
    T acc[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
#pragma unroll 1
    for (int h = 0; h < kSlices; ++h) {
      if (live && sl / kSliceStates == h) emit_columns<1, RF, SP>(m, right, jv, f, rows, nq, acc);
      if (o.dJ) {
        __syncthreads();
        const int nsh = min(max(ns - h * kSliceStates, 0), kSliceStates);
        tile_store(tile, (T*)o.dJ + (p0 + h * kSliceStates) * per_state, nsh * per_state);
        if (h + 1 < kSlices) __syncthreads();
      }
    }
    if (live && o.dJv) {
      T* out = (T*)o.dJv + p * 12 + arm * 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) out[i] = acc[i];
    }
  }
}

template <typename T, int RF, class SP>
static hipError_t launch_frame_kin_t(const KModel<T>* dm, int nq, const T* q, const T* v, const T* qd, const T* vd,
                                     int64_t B, const FrameKinOut& o, hipStream_t s) {
  const int64_t ntiles = (B + kStatesPerTile - 1) / kStatesPerTile;
  const size_t lds = (o.J || o.dJ) ? sizeof(T) * (kStatesPerTile / slices<T>()) * 12 * nq : 0;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)ikg_frame_kin_kernel<T, RF, SP>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((ikg_frame_kin_kernel<T, RF, SP>), dim3((unsigned)ntiles), dim3(64), lds, s, dm, q, v, qd, vd,
                     B, o);
  return hipGetLastError();
}

template <typename T, class SP>
static hipError_t launch_frame_kin_sp(const KModel<T>* dm, int nq, const T* q, const T* v, const T* qd, const T* vd,
                                      int64_t B, int rf, const FrameKinOut& o, hipStream_t s) {
  switch (rf) {
    case 0: return launch_frame_kin_t<T, 0, SP>(dm, nq, q, v, qd, vd, B, o, s);
    case 1: return launch_frame_kin_t<T, 1, SP>(dm, nq, q, v, qd, vd, B, o, s);
    default: return launch_frame_kin_t<T, 2, SP>(dm, nq, q, v, qd, vd, B, o, s);
  }
}

template <typename T>
hipError_t launch_frame_kin(const KModel<T>* dm, int nq, int spec, const void* q, const void* v, const void* qd,
                            const void* vd, int64_t B, int rf, const FrameKinOut& o, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if ((B + kStatesPerTile - 1) / kStatesPerTile > 0x7fffffff) return hipErrorInvalidValue;
  const T *tq = (const T*)q, *tv = (const T*)v, *tqd = (const T*)qd, *tvd = (const T*)vd;
  if (spec == kSpecNextage) return launch_frame_kin_sp<T, SpecNextage>(dm, nq, tq, tv, tqd, tvd, B, rf, o, s);
  return launch_frame_kin_sp<T, SpecGeneric>(dm, nq, tq, tv, tqd, tvd, B, rf, o, s);
}

template hipError_t launch_frame_kin<double>(const KModel<double>*, int, int, const void*, const void*, const void*,
                                             const void*, int64_t, int, const FrameKinOut&, hipStream_t);
template hipError_t launch_frame_kin<float>(const KModel<float>*, int, int, const void*, const void*, const void*,
                                            const void*, int64_t, int, const FrameKinOut&, hipStream_t);

}  // namespace ikg
