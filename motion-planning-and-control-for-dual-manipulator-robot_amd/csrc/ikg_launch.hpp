// Host-side launcher declarations shared by ikg_kernels.hip and ikg_capi.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <utility>
#include <vector>

#include "ikg_collision.hpp"
#include "ikg_device.hpp"
#include "ikg_solve.hpp"

namespace ikg {

struct JitKernels;  // ikg_jit.hpp

// Workspaces of captured solves.  Outside a stream capture a
// solve's scratch is stream-ordered: hipMallocAsync / hipFreeAsync.  Inside a
// capture those calls become graph memory nodes, and a 164 MB record buffer
// taken that way read back as zeros in a later replay after a process had
// used the default pool heavily (tests/test_gpu_graph.py with
// IKG_TRAJ_REC=1; the same buffer from hipMalloc passed every replay).  So a
// captured solve takes its scratch from hipMalloc (relaxed capture mode for
// the call) and hands it to the capturing graph as a user object
// (hipGraphRetainUserObject): the buffer lives exactly as long as the graph
// and its executable instantiations.  The user object's destructor may not
// call HIP, so it only queues the buffer on the model's pending list.  A
// later capture takes a pending buffer that is large enough instead of
// allocating (no HIP call), so a workload that recaptures every cycle and
// never solves uncaptured holds a bounded number of buffers; the rest are
// freed by the model's next uncaptured call, ikg_model_trim or
// ikg_model_destroy.  Every instantiation of one captured graph shares its
// scratch, so two of them must not run at the same time (include/ikgrasp.h,
// "Graphs").
struct WsBuf {
  int dev;
  void* p;
  size_t bytes;
  // recorded by the captured work at the buffer's last use (a node of the
  // graph): a later capture reuses the buffer only once it has completed, so
  // a launch of the destroyed graph still in flight keeps its scratch (ADVICE
  // r5: a user object may be released before its exec's last launch ends).
  hipEvent_t done = nullptr;
  bool reuse = true;  // false: the record could not be captured -- never reused
};

struct WsState {
  static constexpr int kDevs = 64;
  std::mutex mu;
  std::vector<WsBuf> pending;     // buffers whose graphs are gone
  std::vector<WsBuf> held;        // buffers of graphs still alive (their completion events)
  int64_t live = 0;               // buffers held by graphs
  hipMemPool_t pool[kDevs] = {};  // the model's scratch pools (ws_pool), per device
};

struct WsOwner {
  std::shared_ptr<WsState> st = std::make_shared<WsState>();
};

struct GraphScratch {  // one captured buffer, owned by its graph's user object
  std::shared_ptr<WsState> st;
  WsBuf b;
};

inline void graph_scratch_release(void* arg) {  // user-object destructor: no HIP calls here
  GraphScratch* g = static_cast<GraphScratch*>(arg);
  {
    std::lock_guard<std::mutex> lock(g->st->mu);
    WsBuf b = g->b;
    for (size_t i = 0; i < g->st->held.size(); ++i)
      if (g->st->held[i].p == b.p) {
        b.done = g->st->held[i].done;
        b.reuse = g->st->held[i].reuse;
        g->st->held.erase(g->st->held.begin() + i);
        break;
      }
    g->st->pending.push_back(b);
    --g->st->live;
  }
  delete g;
}

inline bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusActive;
}

// Free the buffers of graphs destroyed since the last call (never while the
// calling thread's stream is capturing: hipFree is not a capturable call).
inline void ws_drain(WsOwner* owner) {
  if (!owner) return;
  std::vector<WsBuf> v;
  {
    std::lock_guard<std::mutex> lock(owner->st->mu);
    v.swap(owner->st->pending);
  }
  if (v.empty()) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  for (auto& b : v) {
    (void)hipSetDevice(b.dev);
    (void)hipFree(b.p);  // synchronises: every launch that used it has ended
    if (b.done) (void)hipEventDestroy(b.done);
  }
  if (prev >= 0) (void)hipSetDevice(prev);
}

// The smallest pending buffer on `dev` of at least `bytes` whose last use has
// completed (its event, queried outside capture semantics), taken off the
// list for a capture to reuse, or null.
inline void* ws_take_pending(WsState& st, int dev, size_t bytes, size_t* got, hipEvent_t* done) {
  std::lock_guard<std::mutex> lock(st.mu);
  int best = -1;
  for (int i = 0; i < (int)st.pending.size(); ++i) {
    const WsBuf& b = st.pending[i];
    if (b.dev != dev || b.bytes < bytes || (best >= 0 && b.bytes >= st.pending[best].bytes) || !b.done || !b.reuse)
      continue;
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    const hipError_t q = hipEventQuery(b.done);
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (q == hipSuccess) best = i;
    else if (q != hipErrorNotReady) (void)hipGetLastError();
  }
  if (best < 0) return nullptr;
  const WsBuf b = st.pending[best];
  st.pending.erase(st.pending.begin() + best);
  *got = b.bytes;
  *done = b.done;
  return b.p;
}

// How much freed scratch a model's pool keeps mapped across synchronisations
// (its release threshold): 1.25 GiB by default -- a C2 collision solve's
// records (656 MB) and every record-free solve's scratch stay mapped for the
// next solve; anything above goes back to the driver at the next
// synchronisation, so an idle model holds at most 1.25 GiB per device.  A
// larger collision solve maps its records afresh each time: C3 fp32 + collision
// (5.2 GB) 1.82 -> 1.93 ms, the C4 share and C5 + collision within their spread
// (profiles/r06/records/; round 5 kept 6.5 GiB).
// IKG_WS_KEEP_MB overrides (0 = keep nothing, as the device's default pool).
inline uint64_t ws_keep_bytes() {
  static const uint64_t v = [] {
    const char* e = getenv("IKG_WS_KEEP_MB");
    return e ? (uint64_t)strtoull(e, nullptr, 10) << 20 : (uint64_t)1280 << 20;
  }();
  return v;
}

// The model's stream-ordered scratch pool, one per device it solves on, which
// keeps what a solve frees (up to ws_keep_bytes) for the next solve instead of
// returning it to the driver at every synchronisation, as the device's default
// pool does (threshold 0): a collision solve's record buffer (656 MB at C2)
// was otherwise mapped afresh on every call (1-1.5% of a collision solve).
// The pools are the model's: ikg_model_trim returns their unused memory,
// ikg_model_destroy destroys them (ws_pool_release).  IKG_WS_POOL=0: the
// device's default pool (A/B).
inline hipMemPool_t ws_pool(WsOwner* owner) {
  static const bool on = !(getenv("IKG_WS_POOL") && atoi(getenv("IKG_WS_POOL")) == 0);
  if (!on || !owner) return nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= WsState::kDevs) return nullptr;
  WsState& st = *owner->st;
  std::lock_guard<std::mutex> lock(st.mu);
  if (!st.pool[dev]) {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    uint64_t keep = ws_keep_bytes();
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    st.pool[dev] = pool;
  }
  return st.pool[dev];
}

// Every device the model has a pool on, with the pool handles copied out
// under the lock (`take`: and cleared, for ws_pool_release).  The callers
// synchronise and call into HIP outside the lock: graph_scratch_release takes
// the same mutex and may run on a runtime thread while a device synchronises.
inline std::vector<std::pair<int, hipMemPool_t>> ws_pools(WsOwner* owner, bool take) {
  std::vector<std::pair<int, hipMemPool_t>> v;
  if (!owner) return v;
  WsState& st = *owner->st;
  std::lock_guard<std::mutex> lock(st.mu);
  for (int d = 0; d < WsState::kDevs; ++d)
    if (st.pool[d]) {
      v.emplace_back(d, st.pool[d]);
      if (take) st.pool[d] = nullptr;
    }
  return v;
}

// Destroy the model's pools (ikg_model_destroy): each device is synchronised
// first, so the stream-ordered frees of its last solves have run.
inline void ws_pool_release(WsOwner* owner) {
  for (auto& dp : ws_pools(owner, true)) {
    (void)hipSetDevice(dp.first);
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(dp.second);
  }
}

// Return the pools' unused memory to the driver (ikg_model_trim): each device
// is synchronised, then its pool trimmed to nothing kept; the pool stays
// usable.
inline hipError_t ws_pool_trim(WsOwner* owner) {
  hipError_t rc = hipSuccess;
  for (auto& dp : ws_pools(owner, false)) {
    (void)hipSetDevice(dp.first);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemPoolTrimTo(dp.second, 0);
    if (e != hipSuccess && rc == hipSuccess) rc = e;
  }
  return rc;
}

inline hipError_t ws_alloc(WsOwner* owner, void** p, size_t bytes, hipStream_t s) {
  *p = nullptr;
  if (!owner || !stream_capturing(s)) {
    if (hipMemPool_t pool = ws_pool(owner)) return hipMallocFromPoolAsync(p, bytes, pool, s);
    return hipMallocAsync(p, bytes, s);
  }
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamGetCaptureInfo_v2(s, &cst, nullptr, &graph, nullptr, nullptr);
  if (e != hipSuccess || !graph) return e != hipSuccess ? e : hipErrorStreamCaptureInvalidated;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const size_t want = bytes ? bytes : 1;
  size_t got = want;
  hipEvent_t done = nullptr;
  *p = ws_take_pending(*owner->st, dev, want, &got, &done);  // a destroyed graph's buffer, its last launch ended
  if (!*p) {
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    e = hipMalloc(p, want);
    if (e == hipSuccess && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      done = nullptr;
    }
    (void)hipThreadExchangeStreamCaptureMode(&mode);
    if (e != hipSuccess) {
      *p = nullptr;
      return e;
    }
  }
  {
    std::lock_guard<std::mutex> lock(owner->st->mu);
    owner->st->held.push_back(WsBuf{dev, *p, got, done});
  }
  GraphScratch* g = new GraphScratch{owner->st, WsBuf{dev, *p, got}};
  hipUserObject_t uo = nullptr;
  e = hipUserObjectCreate(&uo, g, graph_scratch_release, 1, hipUserObjectNoDestructorSync);
  if (e == hipSuccess) {
    {
      std::lock_guard<std::mutex> lock(owner->st->mu);
      ++owner->st->live;
    }
    e = hipGraphRetainUserObject(graph, uo, 1, hipGraphUserObjectMove);  // the graph takes our reference
    if (e != hipSuccess) (void)hipUserObjectRelease(uo, 1);                // -> destructor queues the buffer
    return e;
  }
  delete g;
  {  // back on the pending list: freed by the next uncaptured call
    std::lock_guard<std::mutex> lock(owner->st->mu);
    for (size_t i = 0; i < owner->st->held.size(); ++i)
      if (owner->st->held[i].p == *p) {
        owner->st->held.erase(owner->st->held.begin() + i);
        break;
      }
    owner->st->pending.push_back(WsBuf{dev, *p, got, done});
  }
  *p = nullptr;
  return e;
}

// the matching free: a captured solve's buffer stays with its graph, and the
// capture records its completion event after the buffer's last use (a failed
// record drops the event: that buffer is then never reused by a capture)
inline hipError_t ws_free(WsOwner* owner, void* p, hipStream_t s) {
  if (!p) return hipSuccess;
  if (owner && stream_capturing(s)) {
    std::lock_guard<std::mutex> lock(owner->st->mu);
    for (auto& b : owner->st->held)
      if (b.p == p && b.done) {
        if (hipEventRecord(b.done, s) != hipSuccess) {
          (void)hipGetLastError();
          b.reuse = false;
        }
        break;
      }
    return hipSuccess;
  }
  return hipFreeAsync(p, s);
}

struct BatchArgs {
  const void* targets;
  const void* q0;
  int64_t q0_stride;
  int64_t B;
  void* q_out;
  uint8_t* converged;
  int32_t* iters;
  void* err_out;
  int ppw;         // problems per 64-lane wave (1..32)
  int64_t S = 1;   // seeds per target (multi-start): problem p = (target p / S, q0 row p % S)
  int variant = 0; // ikg_variant
  // model-specialised pair kernels on this device (ikg_model_specialize), or null
  const JitKernels* jit = nullptr;
  // collision continuation: record buffers offered to the pair kernel (records
  // every iterate from the first passing one on, RecOut); `rec_used` is set
  // when the launch took them
  void* rec = nullptr;
  int32_t* rec_n = nullptr;
  void* ck = nullptr;           // window checkpoints (ikg_solve.hpp kWinOf), ck_per_problem per problem
  bool* rec_used = nullptr;
  // resume launch (the collision scan's windows to regenerate, ikg_collision.hip):
  // listed problems, their count (device) and windows to regenerate per problem
  const int32_t* rec_list = nullptr;
  const int32_t* rec_count = nullptr;
  const uint32_t* rec_wmask = nullptr;
  uint64_t* rec_rmask = nullptr;    // per problem and window, the iterates the resume kernel recorded
  int64_t rec_rbase = 0, rec_rcap = 0;  // list entries [rbase, rbase + rcap) this resume launch regenerates
  int64_t rec_slots = 0;        // records capacity: problems whose records `rec` holds (0: every problem of the launch)
  WsOwner* ws_owner = nullptr;  // scratch of captured solves (ws_alloc)
};

// waves of a resume launch (grid-stride over listed problems x windows)
inline unsigned resume_waves(int64_t B, int nw, int per_wave) {
  const int64_t w = (B * nw + per_wave - 1) / per_wave;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(w, 4096));
}

struct MultiArgs {
  const void* targets;
  int64_t T;
  const void* seeds;
  int64_t S;
  void* q_out;
  uint8_t* converged;
  int32_t* iters;
  void* err_out;
  int32_t* best_seed;
  int nq;
  // workspace for the S x T per-seed results (device, caller-owned)
  void* ws_q;
  uint8_t* ws_conv;
  int32_t* ws_iters;
  void* ws_err;
  // KCollision<T>* (device) when params.check_collision: the seeds' results
  // go through the collision continuation before the best-seed reduction
  const void* collision = nullptr;
  int n_geoms = 0;
  int variant = 0;  // ikg_variant of the per-seed solves
  const JitKernels* jit = nullptr;
  WsOwner* ws_owner = nullptr;
  // collision continuation records for the S x T per-seed problems (BatchArgs::rec)
  void* rec = nullptr;
  int32_t* rec_n = nullptr;
  void* ck = nullptr;
  bool* rec_used = nullptr;
  int64_t rec_slots = 0;  // BatchArgs::rec_slots
  int64_t rec_chunk = 0;  // targets per launch when the records of all T x S problems exceed the budget (0: all)
};

// Debug knob IKG_POISON=1 (read per call): every stream-ordered workspace is
// filled right after its allocation, so a read of memory the solve did not
// write gives a wrong answer on the first run instead of stale data from an
// earlier solve or graph replay.  Integer arrays (counts, indices, flags) get
// 0xFF bytes (-1: "nothing recorded", never an index that is used); floating
// arrays get 0x7F bytes (1.4e306 / 3.4e38: finite, so no -ffinite-math-only
// code sees a NaN, but absurd as a joint angle or an error norm).
inline bool ws_poison() {
  const char* e = getenv("IKG_POISON");
  return e && atoi(e) != 0;
}
inline void poison_int(void* p, size_t bytes, hipStream_t s) {
  if (p && bytes && ws_poison()) (void)hipMemsetAsync(p, 0xFF, bytes, s);
}
inline void poison_float(void* p, size_t bytes, hipStream_t s) {
  if (p && bytes && ws_poison()) (void)hipMemsetAsync(p, 0x7F, bytes, s);
}

// Debug knob IKG_WS_TRACE=1: every stream-ordered workspace allocation and
// free is printed (address range, whether the stream is capturing).
inline void ws_trace(const char* what, const void* p, size_t bytes, hipStream_t s) {
  const char* e = getenv("IKG_WS_TRACE");
  if (!(e && atoi(e) != 0)) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &st);
  fprintf(stderr, "[ikg ws] %s %p +%zu -> %p%s\n", what, p, bytes, (const void*)((const char*)p + bytes),
          st == hipStreamCaptureStatusActive ? " (capturing)" : "");
}

// kernel specialisation chosen at model creation (ikg_model_build.hpp)
constexpr int kSpecGeneric = 0;
constexpr int kSpecNextage = 1;
constexpr int kSpecGenericWrist = 2;  // generic tables, spherical-wrist solve

template <typename T>
hipError_t launch_pair_batch(const KModel<T>* dmodel, const KParams<T>& prm, const BatchArgs& a, int spec,
                             hipStream_t s);

// the concrete layout (IKG_VARIANT_PAIR / PACKED / QUAD) launch_pair_batch runs for B problems
template <typename T>
int resolve_variant(const KParams<T>& prm, int spec, int variant, int64_t B, bool rec);

// pair layout, Nextage specialisation, lambda = 0, built with the max-ILP
// scheduler for launches of at most one wave per SIMD (ikg_pair_ilp.hip)
hipError_t launch_pair_ilp(const KModel<float>* dmodel, const KParams<float>& prm, const BatchArgs& a, bool med,
                           size_t lds, hipStream_t s);

// packed fp32 layout, Nextage specialisation (ikg_packed.hip)
hipError_t launch_packed_batch(const KModel<float>* dmodel, const KParams<float>& prm, const BatchArgs& a,
                               hipStream_t s);

// quad layout (8 lanes per problem), Nextage specialisation (ikg_quad.hip)
template <typename T>
hipError_t launch_quad_batch(const KModel<T>* dmodel, const KParams<T>& prm, const BatchArgs& a, hipStream_t s);

template <typename T>
hipError_t launch_multistart(const KModel<T>* dmodel, const KParams<T>& prm, const MultiArgs& a, int spec,
                             hipStream_t s);

template <typename T>
hipError_t launch_fk(const KModel<T>* dmodel, const void* q, int64_t B, void* hands, hipStream_t s);

template <typename T>
hipError_t launch_log6(const void* M, int64_t B, void* out, hipStream_t s);

template <typename T>
hipError_t launch_pair_state(const KModel<T>* dm, const void* targets, const void* q0, int64_t stride, int64_t B,
                             void* out, hipStream_t s);


template <typename T>
hipError_t launch_collision(const KModel<T>* dm, const KCollision<T>* dc, const void* q, const void* targets,
                            int64_t B, uint8_t* out, hipStream_t s);

// nq / ng: model joints and scene geometries (size the per-problem LDS slices)
template <typename T>
hipError_t launch_collide_continue(const KModel<T>* dm, const KCollision<T>* dc, const KParams<T>& prm,
                                   const BatchArgs& a, int spec, int nq, int ng, hipStream_t s);

// planner queries: distance over a pair subset; target geometry
// against world-fixed geometries
template <typename T>
hipError_t launch_distance(const KModel<T>* dm, const KCollision<T>* dc, const void* q, const void* targets,
                           int64_t B, const int32_t* pair_idx, int n_idx, void* out, hipStream_t s);
template <typename T>
hipError_t launch_target_env(const KCollision<T>* dc, const void* targets, int64_t B, const int32_t* geoms,
                             int n_geoms, uint8_t* out, hipStream_t s);

// controller kinematics (ikg_control.hip): optional outputs
struct FrameKinOut {
  void* placement;  // [B,2,12]
  void* velocity;   // [B,2,6]
  void* J;          // [B,12,nq]
  void* dJ;         // [B,12,nq]
  void* dJv;        // [B,12]
  void* err;        // [B,12]
  void* derr;       // [B,12]
};
template <typename T>
hipError_t launch_frame_kin(const KModel<T>* dm, int nq, int spec, const void* q, const void* v, const void* qd,
                            const void* vd,
                            int64_t B, int rf, const FrameKinOut& o, hipStream_t s);

}  // namespace ikg
