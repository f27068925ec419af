// C-ABI of libikgrasp.so (include/ikgrasp.h).
//
// Owns model validation / upload, argument checking, optional host staging
// and kernel dispatch.  No exception or exit crosses the boundary: every
// failure returns a negative code and leaves a message in ikg_last_error().
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "ikg_device.hpp"
#include "ikg_jit.hpp"
#include "ikg_solve.hpp"
#include "ikg_launch.hpp"
#include "ikg_model_build.hpp"
#include "ikgrasp.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(IKG_EHIP, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace

struct ikg_model {
  ikg_model_desc desc;
  ikg::KModel<double> k64;
  ikg::KModel<float> k32;
  int spec = ikg::kSpecGeneric;
  std::mutex mu;
  std::vector<void*> dev64;  // per device
  std::vector<void*> dev32;
  // collision scene (ikg_model_set_collision)
  bool has_collision = false;
  ikg::KCollision<double> c64;
  ikg::KCollision<float> c32;
  std::vector<void*> col64;
  std::vector<void*> col32;
  // model-specialised pair kernels (ikg_model_specialize): code objects per
  // dtype (0 = f64, 1 = f32), loaded modules per device
  std::vector<char> jit_code[2];
  std::vector<ikg::JitKernels*> jit[2];
  // scratch of solves captured into graphs (ikg_launch.hpp ws_alloc), freed here
  ikg::WsOwner ws;

  template <typename T>
  const ikg::JitKernels* jit_kernels(int device) {
    std::lock_guard<std::mutex> lock(mu);
    const auto& v = jit[sizeof(T) == 8 ? 0 : 1];
    return device < (int)v.size() ? v[device] : nullptr;
  }

  // Upload `bytes` of `src` to `slot[device]` once; the slot is reused after.
  int upload(std::vector<void*>& slot, int device, const void* src, size_t bytes, const void** out) {
    std::lock_guard<std::mutex> lock(mu);
    if ((int)slot.size() <= device) slot.resize(device + 1, nullptr);
    if (!slot[device]) {
      void* p = nullptr;
      hipError_t e = hipMalloc(&p, bytes);
      if (e != hipSuccess) return fail(IKG_ENOMEM, "hipMalloc(model tables): %s", hipGetErrorString(e));
      e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        (void)hipFree(p);
        return hip_fail(e, "hipMemcpy(model tables)");
      }
      slot[device] = p;
    }
    *out = slot[device];
    return IKG_OK;
  }

  template <typename T>
  int device_tables(int device, const ikg::KModel<T>** out) {
    const bool d = sizeof(T) == 8;
    return upload(d ? dev64 : dev32, device, d ? (const void*)&k64 : (const void*)&k32, sizeof(ikg::KModel<T>),
                  (const void**)out);
  }

  template <typename T>
  int collision_tables(int device, const ikg::KCollision<T>** out) {
    if (!has_collision) return fail(IKG_EINVAL, "no collision scene attached (ikg_model_set_collision)");
    const bool d = sizeof(T) == 8;
    return upload(d ? col64 : col32, device, d ? (const void*)&c64 : (const void*)&c32, sizeof(ikg::KCollision<T>),
                  (const void**)out);
  }
};

namespace {

// Select and restore the current device around a call.
struct DeviceGuard {
  int prev = -1;
  int rc = IKG_OK;
  explicit DeviceGuard(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
      rc = hip_fail(e, "hipGetDeviceCount");
      return;
    }
    if (device < 0 || device >= n) {
      rc = fail(IKG_ENODEV, "device %d out of range (%d visible)", device, n);
      return;
    }
    (void)hipGetDevice(&prev);
    e = hipSetDevice(device);
    if (e != hipSuccess) rc = hip_fail(e, "hipSetDevice");
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Stages host buffers through device scratch when IKG_FLAG_HOST_POINTERS is set.
struct Staging {
  std::vector<void*> allocs;
  hipStream_t s;
  int rc = IKG_OK;
  explicit Staging(hipStream_t st) : s(st) {}
  ~Staging() {
    for (void* p : allocs) (void)hipFree(p);
  }
  void* in(const void* host, size_t bytes) {
    if (!host || rc) return nullptr;
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes ? bytes : 1);
    if (e != hipSuccess) {
      rc = fail(IKG_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
      return nullptr;
    }
    allocs.push_back(d);
    if (bytes) {
      e = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync(H2D)");
    }
    return d;
  }
  void* out(size_t bytes) { return in_alloc(bytes); }
  void* in_alloc(size_t bytes) {
    if (rc) return nullptr;
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes ? bytes : 1);
    if (e != hipSuccess) {
      rc = fail(IKG_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
      return nullptr;
    }
    allocs.push_back(d);
    return d;
  }
  int back(void* host, const void* dev, size_t bytes) {
    if (!host || !dev || rc) return rc;
    hipError_t e = hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s);
    if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync(D2H)");
    return rc;
  }
};

void free_slots(std::vector<void*>& slot) {
  for (size_t i = 0; i < slot.size(); ++i)
    if (slot[i]) {
      (void)hipSetDevice((int)i);
      (void)hipFree(slot[i]);
      slot[i] = nullptr;
    }
}

// Problems per wave.  Full 32-problem waves are fastest at every batch size
// measured (B = 4k..131k, fp32/fp64): spreading a small batch over more,
// sparser waves was 1.3-3x SLOWER (profiles/r01/ppw_sweep.txt).
int auto_ppw(int /*device*/, int64_t /*B*/) { return 32; }

// One-wave-per-problem kernels (collision query, pre-screen, continuation,
// distance, best-seed) launch one 64-lane workgroup per unit; HIP caps a grid at
// 2^32 - 1 work items, so a launch holds at most this many waves.
constexpr int64_t kMaxWaves = (int64_t)0xFFFFFFFFu / 64;

int check_params(const ikg_params* p) {
  if (!p) return fail(IKG_EINVAL, "params is NULL");
  if (!(p->eps > 0) || !std::isfinite(p->eps)) return fail(IKG_EINVAL, "eps must be > 0");
  if (!std::isfinite(p->dt)) return fail(IKG_EINVAL, "dt must be finite");
  if (p->max_iters < 0) return fail(IKG_EINVAL, "max_iters must be >= 0");
  if (!(p->lambda >= 0) || !std::isfinite(p->lambda)) return fail(IKG_EINVAL, "lambda must be >= 0");
  if (p->variant != IKG_VARIANT_AUTO && p->variant != IKG_VARIANT_PAIR && p->variant != IKG_VARIANT_PACKED &&
      p->variant != IKG_VARIANT_QUAD)
    return fail(IKG_EINVAL, "variant %d not available in this build", p->variant);
  if (p->problems_per_wave < 0 || p->problems_per_wave > 32)
    return fail(IKG_EINVAL, "problems_per_wave must be in [0, 32]");
  if (p->check_collision != 0 && p->check_collision != 1) return fail(IKG_EINVAL, "check_collision must be 0 or 1");
  return IKG_OK;
}

// Host-pointer inputs are checked for finiteness before staging: the device
// code is compiled with -ffinite-math-only, so a NaN/inf target, q0 row or seed
// would be undefined there.  Device-pointer callers own that contract
// (include/ikgrasp.h "Conventions").
template <typename T>
int check_finite(const void* p, int64_t n, const char* what) {
  const T* x = static_cast<const T*>(p);
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(x[i])) return fail(IKG_EINVAL, "%s[%lld] is not finite", what, (long long)i);
  return IKG_OK;
}

template <typename T>
ikg::KParams<T> kparams(const ikg_params* p) {
  return ikg::make_kparams<T>(p);
}

// Records in the batch kernel for the collision continuation (the default
// since round 3: C2 with the collision term 1.62 -> 1.30 ms; IKG_TRAJ_REC=0
// selects the trajectory kernel, which recomputes the updates past the first
// passing iterate).  Its round-2 graph-replay mismatch was the graph memory
// node the records came from (ws_alloc, ikg_launch.hpp).  Up
// to rec_budget() bytes of records per solve.
static bool rec_in_batch() {
  const char* e = getenv("IKG_TRAJ_REC");
  return !(e && atoi(e) == 0);
}
// Memory of a collision solve (round 6, window checkpoints, ikg_solve.hpp):
//  * checkpoints, one area per problem of a launch (ck_per_problem: 34 slots,
//    17 KB in fp64, 8.7 KB in fp32 at max_iters 1,000: C2 71 MB, C3 570 MB,
//    C4's 131,072-problem fp64 share 2.3 GB).  A batch whose checkpoints exceed
//    the checkpoint budget (16 GiB, IKG_CK_BUDGET_MB) is solved in chunks of
//    equal size that fit, one launch sequence per chunk (fixed slots carry no
//    shared state, so a problem's answer does not depend on the chunking);
//  * the regenerated records of the problems the scan lists, (max_iters + 1)
//    records per problem, for as many problems as the records budget holds
//    (1 GiB, IKG_REC_BUDGET_MB: 6,700 fp64 / 13,400 fp32 problems); the resume
//    kernel and the records scan run in rounds of that many list entries
//    (ikg_collision.hip launch_collide_continue).
// Round 5 held every problem's records (C3 fp32 5.2 GB, the C4 share 21 GB)
// under a 24 GiB budget; the model's pool keeps 1.25 GiB between solves
// (ikg_launch.hpp ws_keep_bytes).
constexpr size_t kRecBudgetMB = 1024, kCkBudgetMB = 16384;
static size_t rec_budget() {
  if (const char* e = getenv("IKG_REC_BUDGET_MB")) return std::max<size_t>(1, (size_t)atoll(e)) << 20;
  return kRecBudgetMB << 20;
}
static size_t ck_budget() {
  if (const char* e = getenv("IKG_CK_BUDGET_MB")) return std::max<size_t>(1, (size_t)atoll(e)) << 20;
  return kCkBudgetMB << 20;
}

// the final record (record layout) fits a checkpoint slot (ikg_solve.hpp kCkSlot)
static bool rec_fits(int nq) {
  return ikg::rec_len(std::max(0, nq - 1 - 2 * ikg::kArmDof)) <= ikg::kCkSlot;
}

// bytes of one problem's regenerated records, and of its checkpoints
template <typename T>
static size_t rec_records_bytes(const ikg_params& params, int nq) {
  const size_t rl = (size_t)ikg::rec_len(std::max(0, nq - 1 - 2 * ikg::kArmDof));
  return sizeof(T) * rl * ((size_t)params.max_iters + 1);
}
template <typename T>
static size_t rec_ck_bytes(const ikg_params& params) {
  return sizeof(T) * (size_t)ikg::ck_per_problem<T>(params.max_iters);
}

// units (problems, or multi-start targets of `per_unit` problems each) per
// launch: all of them when their checkpoints fit the budget, else the fewest
// equal chunks that do (at least one unit)
template <typename T>
static int64_t rec_chunk(const ikg_params& params, int64_t units, int64_t per_unit) {
  const size_t unit_bytes = rec_ck_bytes<T>(params) * (size_t)per_unit;
  const int64_t cap = std::max<int64_t>(1, (int64_t)(ck_budget() / std::max<size_t>(1, unit_bytes)));
  if (units <= cap) return units;
  const int64_t n = (units + cap - 1) / cap;
  return (units + n - 1) / n;
}

// Checkpoints and records of the collision continuation for `n` problems (one
// chunk, see solve_batch_t): checkpoints for all n, records for the records
// budget's capacity (a.rec_slots).  Null when the allocation fails (the
// continuation then runs without them).
template <typename T>
void* offer_records(ikg_model* model, ikg::BatchArgs& a, const ikg_params& params, int64_t n, int nq, hipStream_t s,
                    bool* rec_used) {
  const int64_t slots = std::min<int64_t>(n, std::max<int64_t>(1, (int64_t)(rec_budget() / rec_records_bytes<T>(params, nq))));
  const size_t b_rec = (rec_records_bytes<T>(params, nq) * (size_t)slots + 255) & ~(size_t)255;
  const size_t b_ck = (rec_ck_bytes<T>(params) * (size_t)n + 255) & ~(size_t)255;
  const size_t b_n = (sizeof(int32_t) * (size_t)n + 255) & ~(size_t)255;
  void* rec = nullptr;
  if (ikg::ws_alloc(&model->ws, &rec, b_rec + b_ck + b_n, s) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  a.rec = rec;
  a.ck = (char*)rec + b_rec;
  a.rec_n = (int32_t*)((char*)rec + b_rec + b_ck);
  a.rec_slots = slots;
  ikg::ws_trace("alloc rec", rec, b_rec + b_ck + b_n, s);
  ikg::poison_float(rec, b_rec + b_ck, s);
  ikg::poison_int(a.rec_n, sizeof(int32_t) * (size_t)n, s);
  a.rec_used = rec_used;
  return rec;
}

// chunk [off, off + n) of a batch's arguments (device pointers)
template <typename T>
static ikg::BatchArgs batch_slice(const ikg::BatchArgs& a, int64_t off, int64_t n, int nq) {
  ikg::BatchArgs c = a;
  c.B = n;
  c.targets = (const T*)a.targets + off * 12;
  if (a.q0_stride) c.q0 = (const T*)a.q0 + off * a.q0_stride;
  c.q_out = (T*)a.q_out + off * nq;
  if (a.converged) c.converged = a.converged + off;
  if (a.iters) c.iters = a.iters + off;
  if (a.err_out) c.err_out = (T*)a.err_out + off * 2;
  return c;
}

template <typename T>
int solve_batch_t(ikg_model* model, int device, const void* targets, const void* q0, int64_t q0_stride, int64_t B,
                  const ikg_params* params, void* q_out, uint8_t* converged, int32_t* iters, void* err_out,
                  hipStream_t s, uint32_t flags) {
  if (!ikg::stream_capturing(s)) ikg::ws_drain(&model->ws);  // scratch of destroyed graphs
  const ikg::KModel<T>* dm = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc) return rc;
  const ikg::KCollision<T>* dc = nullptr;
  if (params->check_collision && (rc = model->collision_tables<T>(device, &dc))) return rc;
  const int nq = model->desc.nq;
  ikg::BatchArgs a{targets, q0, q0_stride, B, q_out, converged, iters, err_out, 32};
  a.ws_owner = &model->ws;
  a.ppw = params->problems_per_wave > 0 ? params->problems_per_wave : auto_ppw(device, B);
  a.variant = params->variant;
  if (params->variant == IKG_VARIANT_PACKED && (sizeof(T) != 4 || model->spec != ikg::kSpecNextage || params->lambda > 0))
    return fail(IKG_EINVAL, "variant PACKED needs fp32, a Nextage-class model and lambda = 0");
  if (params->variant == IKG_VARIANT_QUAD && (model->spec != ikg::kSpecNextage || params->lambda > 0))
    return fail(IKG_EINVAL, "variant QUAD needs a Nextage-class model and lambda = 0");
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  if (host) {
    const int64_t q0_rows = q0_stride == 0 ? 1 : B;
    if ((rc = check_finite<T>(targets, 12 * B, "targets"))) return rc;
    for (int64_t r = 0; r < q0_rows; ++r)
      if ((rc = check_finite<T>(static_cast<const T*>(q0) + r * q0_stride, nq, "q0 row"))) return rc;
    a.targets = st.in(targets, sizeof(T) * 12 * B);
    a.q0 = st.in(q0, sizeof(T) * (q0_stride == 0 ? nq : q0_stride * (q0_rows - 1) + nq));
    a.q_out = st.out(sizeof(T) * nq * B);
    a.converged = converged ? (uint8_t*)st.out(B) : nullptr;
    a.iters = iters ? (int32_t*)st.out(sizeof(int32_t) * B) : nullptr;
    a.err_out = err_out ? st.out(sizeof(T) * 2 * B) : nullptr;
    if (st.rc) return st.rc;
  }
  if (dc) {  // the continuation reads and rewrites every per-problem output
    if (!a.converged) a.converged = (uint8_t*)st.out(B);
    if (!a.iters) a.iters = (int32_t*)st.out(sizeof(int32_t) * B);
    if (!a.err_out) a.err_out = st.out(sizeof(T) * 2 * B);
    if (st.rc) return st.rc;
  }
  a.jit = model->jit_kernels<T>(device);
  // collision term, pair layout, Nextage loop: the batch kernel itself records
  // every iterate from the first passing one on, for the continuation's scan
  // (ikg_collision.hip), whatever the q0 layout; the records
  // take (max_iters + 1) x rec_len values per problem, offered up to the budget
  bool rec_used = false;
  void* rec = nullptr;
  int64_t chunk = B;
  const ikg::KParams<T> kp = kparams<T>(params);
  if (dc && model->spec == ikg::kSpecNextage && !(params->lambda > 0) && !a.jit && rec_in_batch() &&
      rec_fits(nq) && ikg::resolve_variant<T>(kp, model->spec, a.variant, B, true) != IKG_VARIANT_QUAD) {
    chunk = rec_chunk<T>(*params, B, 1);
    rec = offer_records<T>(model, a, *params, chunk, nq, s, &rec_used);
    if (!rec) chunk = B;
    // every chunk runs the layout the whole batch would
    if (chunk < B) a.variant = ikg::resolve_variant<T>(kp, model->spec, a.variant, B, true);
  }
  hipError_t e = hipSuccess;
  for (int64_t off = 0; off < B && e == hipSuccess; off += chunk) {
    const ikg::BatchArgs c = chunk < B ? batch_slice<T>(a, off, std::min(chunk, B - off), nq) : a;
    e = ikg::launch_pair_batch<T>(dm, kp, c, model->spec, s);
    if (e != hipSuccess) {
      if (rec) {
        ikg::ws_trace("free rec", rec, 0, s);
        (void)ikg::ws_free(&model->ws, rec, s);
      }
      return hip_fail(e, "ikg pair kernel launch");
    }
    if (dc) e = ikg::launch_collide_continue<T>(dm, dc, kp, c, model->spec, nq, model->c64.n_geoms, s);
  }
  if (rec) {
    ikg::ws_trace("free rec", rec, 0, s);
    const hipError_t ef = ikg::ws_free(&model->ws, rec, s);
    if (e == hipSuccess) e = ef;
  }
  if (e != hipSuccess) return hip_fail(e, "ikg collision continuation launch");
  if (host) {
    st.back(q_out, a.q_out, sizeof(T) * nq * B);
    st.back(converged, a.converged, B);
    st.back(iters, a.iters, sizeof(int32_t) * B);
    st.back(err_out, a.err_out, sizeof(T) * 2 * B);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

template <typename T>
int solve_multi_t(ikg_model* model, int device, const void* targets, int64_t T_, const void* seeds, int64_t S,
                  const ikg_params* params, void* q_out, uint8_t* converged, int32_t* iters, void* err_out,
                  int32_t* best_seed, hipStream_t s, uint32_t flags) {
  if (!ikg::stream_capturing(s)) ikg::ws_drain(&model->ws);  // scratch of destroyed graphs
  const ikg::KModel<T>* dm = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc) return rc;
  const int nq = model->desc.nq;
  ikg::MultiArgs a{targets, T_, seeds, S, q_out, converged, iters, err_out, best_seed, nq,
                   nullptr, nullptr, nullptr, nullptr};
  a.variant = params->variant;
  a.jit = model->jit_kernels<T>(device);
  a.ws_owner = &model->ws;
  if (params->variant == IKG_VARIANT_PACKED && (sizeof(T) != 4 || model->spec != ikg::kSpecNextage || params->lambda > 0))
    return fail(IKG_EINVAL, "variant PACKED needs fp32, a Nextage-class model and lambda = 0");
  if (params->variant == IKG_VARIANT_QUAD && (model->spec != ikg::kSpecNextage || params->lambda > 0))
    return fail(IKG_EINVAL, "variant QUAD needs a Nextage-class model and lambda = 0");
  if (params->check_collision) {
    const ikg::KCollision<T>* dc = nullptr;
    if ((rc = model->collision_tables<T>(device, &dc))) return rc;
    a.collision = dc;
    a.n_geoms = model->c64.n_geoms;
  }
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  if (host) {
    if ((rc = check_finite<T>(targets, 12 * T_, "targets")) || (rc = check_finite<T>(seeds, nq * S, "seeds")))
      return rc;
    a.targets = st.in(targets, sizeof(T) * 12 * T_);
    a.seeds = st.in(seeds, sizeof(T) * nq * S);
    a.q_out = st.out(sizeof(T) * nq * T_);
    a.converged = converged ? (uint8_t*)st.out(T_) : nullptr;
    a.iters = iters ? (int32_t*)st.out(sizeof(int32_t) * T_) : nullptr;
    a.err_out = err_out ? st.out(sizeof(T) * 2 * T_) : nullptr;
    a.best_seed = best_seed ? (int32_t*)st.out(sizeof(int32_t) * T_) : nullptr;
    if (st.rc) return st.rc;
  }
  // per-seed workspace, stream-ordered (capturable) allocation
  const int64_t n = T_ * S;
  const size_t b_q = sizeof(T) * nq * n, b_err = sizeof(T) * 2 * n, b_it = sizeof(int32_t) * n;
  char* ws = nullptr;
  hipError_t e = ikg::ws_alloc(&model->ws, (void**)&ws, b_q + b_err + b_it + n + 64, s);
  if (e != hipSuccess) return fail(IKG_ENOMEM, "multistart workspace allocation: %s", hipGetErrorString(e));
  ikg::ws_trace("alloc multistart", ws, b_q + b_err + b_it + n + 64, s);
  ikg::poison_float(ws, b_q + b_err, s);
  ikg::poison_int(ws + b_q + b_err, b_it + n, s);
  a.ws_q = ws;
  a.ws_err = ws + b_q;
  a.ws_iters = (int32_t*)(ws + b_q + b_err);
  a.ws_conv = (uint8_t*)(ws + b_q + b_err + b_it);
  // the collision continuation's records, as solve_batch_t (same values for a
  // seed whatever call solves it)
  bool rec_used = false;
  void* rec = nullptr;
  if (a.collision && model->spec == ikg::kSpecNextage && !(params->lambda > 0) && !a.jit && rec_in_batch() &&
      rec_fits(nq) && params->variant != IKG_VARIANT_QUAD) {
    ikg::BatchArgs tmp{};
    a.rec_chunk = rec_chunk<T>(*params, T_, S);  // targets per launch (each with its S seeds)
    rec = offer_records<T>(model, tmp, *params, a.rec_chunk * S, nq, s, &rec_used);
    a.rec = tmp.rec;
    a.rec_n = tmp.rec_n;
    a.ck = tmp.ck;
    a.rec_slots = tmp.rec_slots;
    a.rec_used = tmp.rec_used;
    if (!rec) a.rec_chunk = 0;
  }
  e = ikg::launch_multistart<T>(dm, kparams<T>(params), a, model->spec, s);
  if (rec) {
    ikg::ws_trace("free rec", rec, 0, s);
    const hipError_t ef = ikg::ws_free(&model->ws, rec, s);
    if (e == hipSuccess) e = ef;
  }
  ikg::ws_trace("free multistart", ws, 0, s);
  hipError_t e2 = ikg::ws_free(&model->ws, ws, s);
  if (e != hipSuccess) return hip_fail(e, "ikg multistart kernel launch");
  if (e2 != hipSuccess) return hip_fail(e2, "multistart workspace free");
  if (host) {
    st.back(q_out, a.q_out, sizeof(T) * nq * T_);
    st.back(converged, a.converged, T_);
    st.back(iters, a.iters, sizeof(int32_t) * T_);
    st.back(err_out, a.err_out, sizeof(T) * 2 * T_);
    st.back(best_seed, a.best_seed, sizeof(int32_t) * T_);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

template <typename T>
int fk_t(ikg_model* model, int device, const void* q, int64_t B, void* hands, hipStream_t s, uint32_t flags) {
  const ikg::KModel<T>* dm = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc) return rc;
  const int nq = model->desc.nq;
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void* dq = q;
  void* dh = hands;
  if (host) {
    dq = st.in(q, sizeof(T) * nq * B);
    dh = st.out(sizeof(T) * 24 * B);
    if (st.rc) return st.rc;
  }
  hipError_t e = ikg::launch_fk<T>(dm, dq, B, dh, s);
  if (e != hipSuccess) return hip_fail(e, "ikg fk kernel launch");
  if (host) {
    st.back(hands, dh, sizeof(T) * 24 * B);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

template <typename T>
int collision_t(ikg_model* model, int device, const void* q, const void* targets, int64_t B, uint8_t* out,
                hipStream_t s, uint32_t flags) {
  const ikg::KModel<T>* dm = nullptr;
  const ikg::KCollision<T>* dc = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc || (rc = model->collision_tables<T>(device, &dc))) return rc;
  const int nq = model->desc.nq;
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void* dq = q;
  const void* dt = targets;
  uint8_t* dout = out;
  if (host) {
    dq = st.in(q, sizeof(T) * nq * B);
    dt = st.in(targets, sizeof(T) * 12 * B);
    dout = (uint8_t*)st.out(B);
    if (st.rc) return st.rc;
  }
  hipError_t e = ikg::launch_collision<T>(dm, dc, dq, dt, B, dout, s);
  if (e != hipSuccess) return hip_fail(e, "ikg collision kernel launch");
  if (host) {
    st.back(out, dout, B);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

template <typename T>
int log6_t(const void* M, int64_t B, void* out, hipStream_t s, uint32_t flags) {
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void* dm = M;
  void* dout = out;
  if (host) {
    dm = st.in(M, sizeof(T) * 12 * B);
    dout = st.out(sizeof(T) * 6 * B);
    if (st.rc) return st.rc;
  }
  hipError_t e = ikg::launch_log6<T>(dm, B, dout, s);
  if (e != hipSuccess) return hip_fail(e, "ikg log6 kernel launch");
  if (host) {
    st.back(out, dout, sizeof(T) * 6 * B);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

template <typename T>
int pair_state_t(ikg_model* model, int device, const void* targets, const void* q0, int64_t B, void* out) {
  const ikg::KModel<T>* dm = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc) return rc;
  Staging st(0);
  const void* dt = st.in(targets, sizeof(T) * 12 * B);
  const void* dq = st.in(q0, sizeof(T) * model->desc.nq);
  void* dout = st.out(sizeof(T) * 62 * B);
  if (st.rc) return st.rc;
  hipError_t e = ikg::launch_pair_state<T>(dm, dt, dq, 0, B, dout, 0);
  if (e != hipSuccess) return hip_fail(e, "pair state kernel");
  st.back(out, dout, sizeof(T) * 62 * B);
  if (st.rc) return st.rc;
  e = hipStreamSynchronize(0);
  return e == hipSuccess ? IKG_OK : hip_fail(e, "hipStreamSynchronize");
}

}  // namespace

extern "C" {

// Diagnostic (not in include/ikgrasp.h): per-lane iteration-0 state of the
// pair kernel, host pointers, q0 broadcast; out [B,2,31].
int ikg_debug_pair_state(const ikg_model* model, int device, int dtype, const void* targets, const void* q0,
                         int64_t B, void* out) {
  g_err[0] = 0;
  if (!model || B < 0) return fail(IKG_EINVAL, "bad arguments");
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  ikg_model* m = const_cast<ikg_model*>(model);
  return dtype == IKG_F64 ? pair_state_t<double>(m, device, targets, q0, B, out)
                          : pair_state_t<float>(m, device, targets, q0, B, out);
}

int ikg_log6_batch(int device, int dtype, const void* M, int64_t B, void* out, void* stream, uint32_t flags) {
  g_err[0] = 0;
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (B > 0 && (!M || !out)) return fail(IKG_EINVAL, "M and out are required");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? log6_t<double>(M, B, out, s, flags) : log6_t<float>(M, B, out, s, flags);
}

const char* ikg_last_error(void) { return g_err; }

// Diagnostic (not in include/ikgrasp.h): scratch buffers held by captured
// graphs (live) and those whose graphs are gone (pending: reused by the next
// capture, freed by the model's next uncaptured solve or ikg_model_trim).
// tests/test_gpu_graph.py.
int ikg_debug_ws_count(const ikg_model* model, int64_t* live, int64_t* pending) {
  if (!model || !live || !pending) return fail(IKG_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lock(model->ws.st->mu);
  *live = model->ws.st->live;
  *pending = (int64_t)model->ws.st->pending.size();
  return IKG_OK;
}

// Diagnostic (not in include/ikgrasp.h): bytes the model's scratch pools
// hold from the runtime (reserved) and hand out at the moment (used), summed
// over devices (hipMemPoolAttrReservedMemCurrent / UsedMemCurrent).
// tests/test_gpu_memory.py.
int ikg_debug_ws_pool(const ikg_model* model, int64_t* reserved, int64_t* used) {
  if (!model || !reserved || !used) return fail(IKG_EINVAL, "bad arguments");
  *reserved = *used = 0;
  for (auto& dp : ikg::ws_pools(const_cast<ikg::WsOwner*>(&model->ws), false)) {
    uint64_t r = 0, u = 0;
    if (hipMemPoolGetAttribute(dp.second, hipMemPoolAttrReservedMemCurrent, &r) != hipSuccess ||
        hipMemPoolGetAttribute(dp.second, hipMemPoolAttrUsedMemCurrent, &u) != hipSuccess)
      return fail(IKG_EHIP, "hipMemPoolGetAttribute failed");
    *reserved += (int64_t)r;
    *used += (int64_t)u;
  }
  return IKG_OK;
}

const char* ikg_version(void) { return "ikgrasp 0.1.0 (gfx950, pair kernel)"; }

void ikg_params_default(ikg_params* p) {
  if (!p) return;
  p->eps = 1e-3;       // config.py:22
  p->dt = 1e-2;        // inverse_geometry.py:54
  p->max_iters = 1000;  // inverse_geometry.py:53
  p->variant = IKG_VARIANT_AUTO;
  p->lambda = 0.0;      // np.linalg.pinv semantics
  p->problems_per_wave = 0;
  p->check_collision = 0;
}

int ikg_model_create(const ikg_model_desc* d, ikg_model** out) {
  g_err[0] = 0;
  if (!d || !out) return fail(IKG_EINVAL, "NULL argument");
  *out = nullptr;
  if (d->nq <= 0 || d->nq > IKG_MAX_NQ) return fail(IKG_EINVAL, "nq=%d outside [1,%d]", d->nq, IKG_MAX_NQ);
  for (int q = 0; q < d->nq; ++q) {
    if (d->axis[q] < 0 || d->axis[q] > 2) return fail(IKG_EINVAL, "joint %d: axis must be 0/1/2", q);
    if (d->parent[q] < -1 || d->parent[q] >= q)
      return fail(IKG_EINVAL, "joint %d: parent %d must precede it (Pinocchio order)", q, d->parent[q]);
    if (!(d->lower[q] <= d->upper[q])) return fail(IKG_EINVAL, "joint %d: lower > upper", q);
  }
  const int r = d->root_q;
  if (r < 0 || r >= d->nq || d->parent[r] != -1) return fail(IKG_EINVAL, "root_q must be a joint under the universe");
  bool used[IKG_MAX_NQ] = {};
  used[r] = true;
  for (int a = 0; a < 2; ++a) {
    int prev = r;
    for (int j = 0; j < IKG_ARM_DOF; ++j) {
      const int q = d->arm_q[a][j];
      if (q < 0 || q >= d->nq || used[q]) return fail(IKG_EINVAL, "arm %d joint %d: bad or repeated q index", a, j);
      if (d->parent[q] != prev) return fail(IKG_EINVAL, "arm %d joint %d: not a serial chain from the root", a, j);
      used[q] = true;
      prev = q;
    }
  }
  for (int j = 0; j < IKG_ARM_DOF; ++j)
    if (d->axis[d->arm_q[0][j]] != d->axis[d->arm_q[1][j]])
      return fail(IKG_EINVAL, "arm joint %d: left/right axes differ (unsupported)", j);
  ikg_model* m = new (std::nothrow) ikg_model();
  if (!m) return fail(IKG_ENOMEM, "out of host memory");
  m->desc = *d;
  ikg::build_kmodel<double>(*d, m->k64);
  ikg::build_kmodel<float>(*d, m->k32);
  m->spec = ikg::choose_spec(m->k64);
  *out = m;
  return IKG_OK;
}

void ikg_model_destroy(ikg_model* m) {
  if (!m) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  free_slots(m->dev64);
  free_slots(m->dev32);
  free_slots(m->col64);
  free_slots(m->col32);
  for (auto& v : m->jit)
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]) {
        (void)hipSetDevice((int)i);
        ikg::jit_unload(*v[i]);
        delete v[i];
      }
  // scratch of captured graphs destroyed by now (a graph still alive keeps
  // its buffer: graphs must be destroyed before the model, whose tables they
  // also reference -- include/ikgrasp.h "Graphs")
  ikg::ws_drain(&m->ws);
  ikg::ws_pool_release(&m->ws);
  if (prev >= 0) (void)hipSetDevice(prev);
  delete m;
}

int ikg_model_trim(ikg_model* m) {
  g_err[0] = 0;
  if (!m) return fail(IKG_EINVAL, "model is NULL");
  int prev = -1;
  (void)hipGetDevice(&prev);
  ikg::ws_drain(&m->ws);  // buffers of destroyed graphs
  const hipError_t e = ikg::ws_pool_trim(&m->ws);
  if (prev >= 0) (void)hipSetDevice(prev);
  return e == hipSuccess ? IKG_OK : hip_fail(e, "ikg_model_trim");
}

int ikg_solve_batch(const ikg_model* model, int device, int dtype, const void* targets, const void* q0,
                    int64_t q0_stride, int64_t B, const ikg_params* params, void* q_out, uint8_t* converged,
                    int32_t* iters, void* err_out, void* stream, uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (B > 0 && (!targets || !q0 || !q_out)) return fail(IKG_EINVAL, "targets, q0 and q_out are required");
  if (q0_stride != 0 && q0_stride < model->desc.nq) return fail(IKG_EINVAL, "q0_stride must be 0 or >= nq");
  if (int rc = check_params(params)) return rc;
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  {
    const int ppw = params->problems_per_wave > 0 ? params->problems_per_wave : 32;
    if ((B + ppw - 1) / ppw > kMaxWaves) return fail(IKG_EINVAL, "B=%lld too large for one launch", (long long)B);
  }
  if (params->check_collision && B > kMaxWaves)
    return fail(IKG_EINVAL, "B=%lld too large for the collision launch (at most %lld)", (long long)B,
                (long long)kMaxWaves);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? solve_batch_t<double>(m, device, targets, q0, q0_stride, B, params, q_out, converged,
                                                  iters, err_out, s, flags)
                          : solve_batch_t<float>(m, device, targets, q0, q0_stride, B, params, q_out, converged,
                                                 iters, err_out, s, flags);
}

int ikg_solve_multistart(const ikg_model* model, int device, int dtype, const void* targets, int64_t T,
                         const void* seeds, int64_t S, const ikg_params* params, void* q_out, uint8_t* converged,
                         int32_t* iters, void* err_out, int32_t* best_seed, void* stream, uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (T < 0 || S <= 0) return fail(IKG_EINVAL, "need T >= 0 and S >= 1");
  if (S > (int64_t)1 << 24) return fail(IKG_EINVAL, "S=%lld seeds per target is too many", (long long)S);
  if (T > 0 && (!targets || !seeds || !q_out)) return fail(IKG_EINVAL, "targets, seeds and q_out are required");
  if (int rc = check_params(params)) return rc;
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (T > kMaxWaves || (T * S + 31) / 32 > kMaxWaves)
    return fail(IKG_EINVAL, "T=%lld x S=%lld too large for one launch", (long long)T, (long long)S);
  if (params->check_collision && T * S > kMaxWaves)
    return fail(IKG_EINVAL, "T*S=%lld too large for the collision launch (at most %lld)", (long long)(T * S),
                (long long)kMaxWaves);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (T == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? solve_multi_t<double>(m, device, targets, T, seeds, S, params, q_out, converged, iters,
                                                  err_out, best_seed, s, flags)
                          : solve_multi_t<float>(m, device, targets, T, seeds, S, params, q_out, converged, iters,
                                                 err_out, best_seed, s, flags);
}

int ikg_fk_batch(const ikg_model* model, int device, int dtype, const void* q, int64_t B, void* hands, void* stream,
                 uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (B > 0 && (!q || !hands)) return fail(IKG_EINVAL, "q and hands are required");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? fk_t<double>(m, device, q, B, hands, s, flags)
                          : fk_t<float>(m, device, q, B, hands, s, flags);
}

int ikg_model_set_collision(ikg_model* m, const ikg_collision_desc* d) {
  g_err[0] = 0;
  if (!m || !d) return fail(IKG_EINVAL, "NULL argument");
  if (d->n_geoms < 1 || d->n_geoms > IKG_MAX_GEOMS)
    return fail(IKG_EINVAL, "n_geoms=%d outside [1,%d]", d->n_geoms, IKG_MAX_GEOMS);
  if (d->n_pairs < 0 || d->n_pairs > IKG_MAX_PAIRS)
    return fail(IKG_EINVAL, "n_pairs=%d outside [0,%d]", d->n_pairs, IKG_MAX_PAIRS);
  if (d->target_geom < -1 || d->target_geom >= d->n_geoms) return fail(IKG_EINVAL, "target_geom out of range");
  for (int g = 0; g < d->n_geoms; ++g) {
    if (d->kind[g] < IKG_GEOM_SPHERE || d->kind[g] > IKG_GEOM_MESHBOX)
      return fail(IKG_EINVAL, "geometry %d: unknown kind %d", g, d->kind[g]);
    if (d->joint[g] < -1 || d->joint[g] >= m->desc.nq)
      return fail(IKG_EINVAL, "geometry %d: joint %d out of range", g, d->joint[g]);
    for (int i = 0; i < 3; ++i)
      if (!(d->dims[g][i] >= 0) || !std::isfinite(d->dims[g][i]))
        return fail(IKG_EINVAL, "geometry %d: dims must be finite and >= 0", g);
  }
  for (int k = 0; k < d->n_pairs; ++k) {
    const int a = d->pairs[k][0], b = d->pairs[k][1];
    if (a < 0 || b < 0 || a >= d->n_geoms || b >= d->n_geoms || a == b)
      return fail(IKG_EINVAL, "pair %d: bad geometry indices (%d, %d)", k, a, b);
  }
  std::lock_guard<std::mutex> lock(m->mu);
  int prev = -1;
  (void)hipGetDevice(&prev);
  free_slots(m->col64);  // re-uploaded lazily; callers must not race a solve
  free_slots(m->col32);
  if (prev >= 0) (void)hipSetDevice(prev);
  ikg::build_kcollision<double>(*d, m->c64);
  ikg::build_kcollision<float>(*d, m->c32);
  m->has_collision = true;
  return IKG_OK;
}

int ikg_collision_batch(const ikg_model* model, int device, int dtype, const void* q, const void* targets, int64_t B,
                        uint8_t* in_collision, void* stream, uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (B > 0 && (!q || !targets || !in_collision)) return fail(IKG_EINVAL, "q, targets and in_collision are required");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (!model->has_collision) return fail(IKG_EINVAL, "no collision scene attached (ikg_model_set_collision)");
  if (B > kMaxWaves) return fail(IKG_EINVAL, "B=%lld too large for one launch (at most %lld)", (long long)B, (long long)kMaxWaves);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? collision_t<double>(m, device, q, targets, B, in_collision, s, flags)
                          : collision_t<float>(m, device, q, targets, B, in_collision, s, flags);
}

}  // extern "C"

// Small index arrays of the planner queries: host -> device each call.
template <typename T>
int distance_t(ikg_model* model, int device, const void* q, const void* targets, int64_t B, const int32_t* idx,
               int32_t n, void* out, hipStream_t s, uint32_t flags) {
  const ikg::KModel<T>* dm = nullptr;
  const ikg::KCollision<T>* dc = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc || (rc = model->collision_tables<T>(device, &dc))) return rc;
  const int nq = model->desc.nq;
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void* dq = q;
  const void* dt = targets;
  void* dout = out;
  const int32_t* didx = (const int32_t*)st.in(idx, sizeof(int32_t) * n);
  if (host) {
    dq = st.in(q, sizeof(T) * nq * B);
    dt = st.in(targets, sizeof(T) * 12 * B);
    dout = st.out(sizeof(T) * B);
  }
  if (st.rc) return st.rc;
  hipError_t e = ikg::launch_distance<T>(dm, dc, dq, dt, B, didx, n, dout, s);
  if (e != hipSuccess) return hip_fail(e, "ikg distance kernel launch");
  if (host) st.back(out, dout, sizeof(T) * B);
  if (st.rc) return st.rc;
  e = hipStreamSynchronize(s);  // the staged index array is freed on return
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return IKG_OK;
}

template <typename T>
int target_env_t(ikg_model* model, int device, const void* targets, int64_t B, const int32_t* geoms, int32_t n,
                 uint8_t* out, hipStream_t s, uint32_t flags) {
  const ikg::KCollision<T>* dc = nullptr;
  int rc = model->collision_tables<T>(device, &dc);
  if (rc) return rc;
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void* dt = targets;
  uint8_t* dout = out;
  const int32_t* dg = (const int32_t*)st.in(geoms, sizeof(int32_t) * n);
  if (host) {
    dt = st.in(targets, sizeof(T) * 12 * B);
    dout = (uint8_t*)st.out(B);
  }
  if (st.rc) return st.rc;
  hipError_t e = ikg::launch_target_env<T>(dc, dt, B, dg, n, dout, s);
  if (e != hipSuccess) return hip_fail(e, "ikg target/env kernel launch");
  if (host) st.back(out, dout, B);
  if (st.rc) return st.rc;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return IKG_OK;
}

extern "C" {

int ikg_distance_batch(const ikg_model* model, int device, int dtype, const void* q, const void* targets,
                       int64_t B, const int32_t* pair_idx, int32_t n_pairs, void* dist, void* stream,
                       uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (n_pairs < 1 || !pair_idx) return fail(IKG_EINVAL, "pair_idx must list at least one pair");
  if (B > 0 && (!q || !targets || !dist)) return fail(IKG_EINVAL, "q, targets and dist are required");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (!model->has_collision) return fail(IKG_EINVAL, "no collision scene attached (ikg_model_set_collision)");
  for (int32_t k = 0; k < n_pairs; ++k)
    if (pair_idx[k] < 0 || pair_idx[k] >= model->c64.n_pairs)
      return fail(IKG_EINVAL, "pair_idx[%d] = %d outside [0, %d)", k, pair_idx[k], model->c64.n_pairs);
  if (B > kMaxWaves) return fail(IKG_EINVAL, "B=%lld too large for one launch (at most %lld)", (long long)B, (long long)kMaxWaves);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? distance_t<double>(m, device, q, targets, B, pair_idx, n_pairs, dist, s, flags)
                          : distance_t<float>(m, device, q, targets, B, pair_idx, n_pairs, dist, s, flags);
}

int ikg_target_env_batch(const ikg_model* model, int device, int dtype, const void* targets, int64_t B,
                         const int32_t* geoms, int32_t n_geoms, uint8_t* in_collision, void* stream,
                         uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (n_geoms < 1 || !geoms) return fail(IKG_EINVAL, "geoms must list at least one geometry");
  if (B > 0 && (!targets || !in_collision)) return fail(IKG_EINVAL, "targets and in_collision are required");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (!model->has_collision) return fail(IKG_EINVAL, "no collision scene attached (ikg_model_set_collision)");
  for (int32_t k = 0; k < n_geoms; ++k)
    if (geoms[k] < 0 || geoms[k] >= model->c64.n_geoms || geoms[k] == model->c64.target_geom)
      return fail(IKG_EINVAL, "geoms[%d] = %d is not a scene geometry other than the target", k, geoms[k]);
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? target_env_t<double>(m, device, targets, B, geoms, n_geoms, in_collision, s, flags)
                          : target_env_t<float>(m, device, targets, B, geoms, n_geoms, in_collision, s, flags);
}

}  // extern "C"

// ------------------------------------------------------------ controller kinematics
template <typename T>
int frame_kin_t(ikg_model* model, int device, const void* q, const void* v, const void* qd, const void* vd, int64_t B,
                int rf, const ikg_frame_kin_out& out, hipStream_t s, uint32_t flags) {
  const ikg::KModel<T>* dm = nullptr;
  int rc = model->device_tables<T>(device, &dm);
  if (rc) return rc;
  const int nq = model->desc.nq;
  const size_t sz[7] = {24, 12, (size_t)12 * nq, (size_t)12 * nq, 12, 12, 12};  // per state
  void* host_out[7] = {out.placement, out.velocity, out.J, out.dJ, out.dJv, out.err, out.derr};
  void* dev_out[7];
  Staging st(s);
  const bool host = flags & IKG_FLAG_HOST_POINTERS;
  const void *dq = q, *dv = v, *dqd = qd, *dvd = vd;
  const bool des = out.err || out.derr;
  if (host) {
    dq = st.in(q, sizeof(T) * nq * B);
    dv = st.in(v, sizeof(T) * nq * B);
    if (des) {
      dqd = st.in(qd, sizeof(T) * nq * B);
      dvd = st.in(vd, sizeof(T) * nq * B);
    }
  }
  for (int i = 0; i < 7; ++i) dev_out[i] = host && host_out[i] ? st.out(sizeof(T) * sz[i] * B) : host_out[i];
  if (st.rc) return st.rc;
  ikg::FrameKinOut o{dev_out[0], dev_out[1], dev_out[2], dev_out[3], dev_out[4], dev_out[5], dev_out[6]};
  hipError_t e = ikg::launch_frame_kin<T>(dm, nq, model->spec, dq, dv, des ? dqd : nullptr, des ? dvd : nullptr, B, rf, o, s);
  if (e != hipSuccess) return hip_fail(e, "ikg frame kinematics kernel launch");
  if (host) {
    for (int i = 0; i < 7; ++i)
      if (host_out[i]) st.back(host_out[i], dev_out[i], sizeof(T) * sz[i] * B);
    if (st.rc) return st.rc;
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  }
  return IKG_OK;
}

extern "C" {

int ikg_frame_kinematics_batch(const ikg_model* model, int device, int dtype, const void* q, const void* v,
                               const void* q_des, const void* v_des, int64_t B, int rf,
                               const ikg_frame_kin_out* out, void* stream, uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (!out) return fail(IKG_EINVAL, "out is NULL");
  if (B < 0) return fail(IKG_EINVAL, "B must be >= 0");
  if (rf < IKG_WORLD || rf > IKG_LOCAL_WORLD_ALIGNED) return fail(IKG_EINVAL, "rf %d unknown", rf);
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (B > 0 && !q) return fail(IKG_EINVAL, "q is required");
  if (B > 0 && (out->err || out->derr) && !q_des) return fail(IKG_EINVAL, "err/derr need q_des");
  if (B > (int64_t)1 << 40) return fail(IKG_EINVAL, "B too large");
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  if (B == 0) return IKG_OK;
  ikg_model* m = const_cast<ikg_model*>(model);
  hipStream_t s = (hipStream_t)stream;
  return dtype == IKG_F64 ? frame_kin_t<double>(m, device, q, v, q_des, v_des, B, rf, *out, s, flags)
                          : frame_kin_t<float>(m, device, q, v, q_des, v_des, B, rf, *out, s, flags);
}

}  // extern "C"

// ------------------------------------------------------------ model-specialised kernels
namespace {

// Compile (once per model and dtype) the pair kernels against this model's
// tables; the caller holds m->mu.
int jit_code_locked(ikg_model* m, int dtype) {
  std::vector<char>& code = m->jit_code[dtype == IKG_F64 ? 0 : 1];
  if (!code.empty()) return IKG_OK;
  const std::string src = dtype == IKG_F64 ? ikg::jit_source(m->k64) : ikg::jit_source(m->k32);
  const std::string err = ikg::jit_compile(src, code);
  if (!err.empty()) {
    code.clear();
    return fail(IKG_EHIP, "model specialisation: %s", err.c_str());
  }
  return IKG_OK;
}

}  // namespace

extern "C" {

int ikg_model_specialize(ikg_model* model, int device, int dtype, uint32_t flags) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  if (flags & ~IKG_SPECIALIZE_IF_GENERIC) return fail(IKG_EINVAL, "flags must be 0 or IKG_SPECIALIZE_IF_GENERIC");
  if ((flags & IKG_SPECIALIZE_IF_GENERIC) && model->spec == ikg::kSpecNextage) return IKG_OK;
  DeviceGuard g(device);
  if (g.rc) return g.rc;
  std::lock_guard<std::mutex> lock(model->mu);
  auto& slot = model->jit[dtype == IKG_F64 ? 0 : 1];
  if ((int)slot.size() > device && slot[device]) return IKG_OK;
  if (int rc = jit_code_locked(model, dtype)) return rc;
  ikg::JitKernels* k = new (std::nothrow) ikg::JitKernels();
  if (!k) return fail(IKG_ENOMEM, "out of host memory");
  const hipError_t e = ikg::jit_load(model->jit_code[dtype == IKG_F64 ? 0 : 1], *k);
  if (e != hipSuccess) {
    delete k;
    return hip_fail(e, "hipModuleLoadData(specialised kernels)");
  }
  if ((int)slot.size() <= device) slot.resize(device + 1, nullptr);
  slot[device] = k;
  return IKG_OK;
}

int ikg_model_is_specialized(const ikg_model* model, int device, int dtype) {
  if (!model || device < 0 || (dtype != IKG_F64 && dtype != IKG_F32)) return 0;
  ikg_model* m = const_cast<ikg_model*>(model);
  return dtype == IKG_F64 ? m->jit_kernels<double>(device) != nullptr : m->jit_kernels<float>(device) != nullptr;
}

// Diagnostic (not in include/ikgrasp.h; no GPU needed): run the specialising
// compile and report the code object's size; with `path`, also write the code
// object there (llvm-objdump -d for the ISA).
int ikg_debug_jit_compile(const ikg_model* model, int dtype, const char* path, size_t* code_size) {
  g_err[0] = 0;
  if (!model) return fail(IKG_EINVAL, "model is NULL");
  if (dtype != IKG_F64 && dtype != IKG_F32) return fail(IKG_EINVAL, "dtype %d unknown", dtype);
  ikg_model* m = const_cast<ikg_model*>(model);
  std::lock_guard<std::mutex> lock(m->mu);
  if (int rc = jit_code_locked(m, dtype)) return rc;
  const std::vector<char>& code = m->jit_code[dtype == IKG_F64 ? 0 : 1];
  if (code_size) *code_size = code.size();
  if (path) {
    FILE* f = fopen(path, "wb");
    if (!f) return fail(IKG_EINVAL, "cannot open %s", path);
    const size_t n = fwrite(code.data(), 1, code.size(), f);
    fclose(f);
    if (n != code.size()) return fail(IKG_EINVAL, "short write to %s", path);
  }
  return IKG_OK;
}

}  // extern "C"
