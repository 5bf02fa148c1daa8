// lorb_internal.h -- shared internals of liblorb.so (HIP runtime for gfx950 / MI355X).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/lorb_c.h"

struct lorb_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  hipEvent_t ev[64] = {};
  // grow-only device scratch buffers, one per slot
  static constexpr int kScratch = 128;
  void* scratch[kScratch] = {};
  size_t scratch_sz[kScratch] = {};
  // host copy of the bytes last uploaded into a slot (lorb::upload); an identical re-upload of
  // per-call constants (problem offsets, scan tiles) is skipped.  Cleared whenever the slot is
  // handed out as kernel-written scratch.
  std::vector<unsigned char> up_mirror[kScratch];
  // per-kernel event timing
  bool ktime = false;
  std::vector<hipEvent_t> kev_pool;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> kev[LORB_K_COUNT];
  // S_BF_TKEY entries known to hold all-ones (0: re-fill before use), for the buffer tkey_buf
  size_t tkey_ready = 0;
  void* tkey_buf = nullptr;
  void* done_buf = nullptr;  // S_BF_DONE as last zeroed
  // pinned host staging
  void* pinned = nullptr;
  size_t pinned_sz = 0;
  // spin_sync's event (no timing)
  hipEvent_t spin_ev = nullptr;
  // lorb_ctx_ba_solver's solver (destroyed with the ctx)
  lorb_ba_solver* solver = nullptr;
  // pinned (coherent, mapped) staging of lorb::InPack / OutPack and its device-side addresses
  void* io_in = nullptr;
  void* io_in_dev = nullptr;
  size_t io_in_sz = 0;
  void* io_out = nullptr;
  void* io_out_dev = nullptr;
  size_t io_out_sz = 0;
  bool io_pending = false;  // an InPack pull may still read the staging (cleared by OutPack::fetch)
};

namespace lorb {
// Wait for the stream by polling an event from the host instead of a blocking synchronize: the
// device plan build's one readback sits on the step's critical path, and a blocked host thread
// wakes up tens of microseconds after the copy lands.
inline hipError_t spin_sync(lorb_ctx* ctx) {
  hipError_t e = hipEventRecord(ctx->spin_ev, ctx->stream);
  if (e != hipSuccess) return e;
  while ((e = hipEventQuery(ctx->spin_ev)) == hipErrorNotReady) {
  }
  return e;
}
}  // namespace lorb

// multi-GPU communicator (lorb_comm.hip): RCCL over xGMI, or a host callback transport
struct lorb_comm {
  lorb_ctx* ctx = nullptr;
  int nranks = 1, rank = 0;
  bool rccl = false;
  void* nccl = nullptr;                    // ncclComm_t
  lorb_host_allreduce_fn fn = nullptr;     // host transport
  void* user = nullptr;
  double* pinned = nullptr;                // host staging for the callback transport
  size_t pinned_n = 0;
  double* dbuf = nullptr;                  // device staging of comm_allreduce_host (RCCL; grow-only)
  size_t dbuf_n = 0;
};

namespace lorb {

int set_error(lorb_ctx* ctx, int code, const char* fmt, ...);
// stream-ordered all-reduce of device doubles on comm->ctx->stream (send may equal recv)
int comm_allreduce(lorb_comm* comm, const double* d_send, double* d_recv, size_t n, int op);
// blocking all-reduce of a host array (plan construction)
int comm_allreduce_host(lorb_comm* comm, double* h_buf, size_t n, int op);

#define LORB_HIP(ctx, call)                                                              \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      return ::lorb::set_error((ctx), LORB_E_DEVICE, "%s failed: %s (%s:%d)", #call,    \
                               hipGetErrorString(e_), __FILE__, __LINE__);               \
  } while (0)

#define LORB_CHECK_LAUNCH(ctx) LORB_HIP(ctx, hipGetLastError())

#define LORB_TRY(expr)          \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != LORB_OK) return rc_; \
  } while (0)

// device-built plan (lorb_ba_plan_create_dev): the solution in double, caller camera order, plus
// the LM summary, into d_out = [poses 6C | points 3P | iterations, successful, termination, initial
// cost, final cost] (async on the plan's stream)
int ba_plan_result64_dev(lorb_ba_plan* P, double* d_out);
// the same as lorb_ba_plan_result_dev with the poses written into a keyframe ring (pose c of the
// window to slot (t0 + c) mod R, 6 floats each) instead of a pose array
int ba_plan_result_ring_dev(lorb_ba_plan* P, float* ring, int R, int t0, float* d_point_out);
// a device-built plan whose callers keep the observation slots sorted by point (stably, no unused
// slots) builds without the counting sort; slots found out of order fall back to it (same result)
void ba_plan_sorted_hint(lorb_ba_plan* P, bool sorted);
// the window's live point / observation counts as the last lorb_ba_plan_update_dev read them
void ba_plan_window_counts(const lorb_ba_plan* P, int* n_points, int* n_obs);
// the last device build's per-point observation offsets (point-sorted slots), device pointer
const int* ba_plan_point_offsets(const lorb_ba_plan* P);

// crossCheck keys of ONE brute-force problem (lorb_bf_match_dev without its finalisation): per
// query (dist << 32 | train) or all-ones; *qkey_out is ctx scratch valid until the next matcher call
int match1_keys_dev(lorb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                    unsigned long long** qkey_out, hipStream_t stream = nullptr);  // null: ctx->stream
// the same into caller-owned buffers: qkey (nq entries), tkey (nt entries, all-ones on entry and
// again once the call's kernels have run), on stream st
int match1_keys_into(lorb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                     unsigned long long* qkey, uint32_t* tkey, hipStream_t st);

// grow-only scratch: returns device pointer in *out
int scratch(lorb_ctx* ctx, int slot, size_t bytes, void** out);
template <typename T>
int scratch_t(lorb_ctx* ctx, int slot, size_t count, T** out) {
  void* p = nullptr;
  int rc = scratch(ctx, slot, count * sizeof(T) + 16, &p);
  *out = static_cast<T*>(p);
  return rc;
}

// H2D into scratch slot (sync w.r.t. host buffer: uses hipMemcpyAsync + stream sync at end
// of the calling API).
int upload(lorb_ctx* ctx, int slot, const void* host, size_t bytes, void** dev);
template <typename T>
int upload_t(lorb_ctx* ctx, int slot, const T* host, size_t count, T** dev) {
  void* p = nullptr;
  if (host == nullptr || count == 0) { *dev = nullptr; return scratch(ctx, slot, 16, &p) == LORB_OK ? (*dev = nullptr, LORB_OK) : LORB_E_DEVICE; }
  int rc = upload(ctx, slot, host, count * sizeof(T), &p);
  *dev = static_cast<T*>(p);
  return rc;
}

// Host-array entry points (the per-frame calls a host caller issues, e.g. SearchByProjection on the
// live tracking path): every input array is packed into ONE pinned staging buffer that ONE pull
// kernel on the ctx stream copies into a device block (a kernel reading the mapped host buffer: an
// SDMA copy would cost the engine-to-queue hand-off, ~10 us on the tracking path); the outputs live
// in ONE block: device memory that ONE device-to-host copy brings back, or (alloc(true)) the mapped
// pinned buffer itself, written by the call's last kernel with plain stores (no atomics, no reads).
// Usage: InPack::add() per input (before commit), commit() (pack + pull), dev<T>(i) per input;
// OutPack::add() per output, alloc(direct), dev<T>(i), fetch() (copy if needed + wait), then
// host<T>(i).  One of each per ctx is in use at a time (calls on one ctx are serialized).
class InPack {
 public:
  explicit InPack(lorb_ctx* c) : ctx(c) {}
  int add(const void* host, size_t bytes) {  // returns the part index
    parts.push_back({host, bytes, total});
    total += (bytes + 255) & ~size_t(255);
    return (int)parts.size() - 1;
  }
  template <typename T>
  int add_t(const T* host, size_t count) { return add(host, host ? count * sizeof(T) : 0); }
  // mapped: no pull -- dev<T>() then addresses the mapped staging itself (for a kernel that reads
  // each input once: one PCIe round trip instead of a pull launch and its hand-off)
  int commit(bool mapped = false);
  template <typename T>
  T* dev(int i) const { return parts[i].bytes ? reinterpret_cast<T*>(static_cast<unsigned char*>(base) + parts[i].off) : nullptr; }

 private:
  struct Part { const void* host; size_t bytes, off; };
  lorb_ctx* ctx;
  std::vector<Part> parts;
  size_t total = 0;
  void* base = nullptr;
};
class OutPack {
 public:
  explicit OutPack(lorb_ctx* c) : ctx(c) {}
  int add(size_t bytes) {
    parts.push_back({bytes, total});
    total += (bytes + 255) & ~size_t(255);
    return (int)parts.size() - 1;
  }
  int alloc(bool direct = false);
  int fetch();  // one D2H copy into pinned memory (unless direct), then waits for the stream
  template <typename T>
  T* dev(int i) const { return reinterpret_cast<T*>(static_cast<unsigned char*>(dbase) + parts[i].off); }
  template <typename T>
  const T* host(int i) const { return reinterpret_cast<const T*>(static_cast<const unsigned char*>(hbase) + parts[i].off); }

 private:
  struct Part { size_t bytes, off; };
  lorb_ctx* ctx;
  std::vector<Part> parts;
  size_t total = 0;
  void* dbase = nullptr;
  void* hbase = nullptr;
  bool direct = false;
};

// brackets one kernel launch with events when ctx->ktime is set
struct KernelTimer {
  lorb_ctx* ctx; int k; hipEvent_t b = nullptr, e = nullptr;
  KernelTimer(lorb_ctx* c, int kid);
  ~KernelTimer();
};

inline unsigned ceil_div(size_t a, size_t b) { return static_cast<unsigned>((a + b - 1) / b); }

// Exclusive scan of one int per thread across a 1024-thread workgroup (16 wavefronts): wave
// inclusive scan with DPP-lowered shuffles, then the 16 wave totals from LDS.  Returns the
// exclusive prefix of this thread; *total = the workgroup sum.  wsum: __shared__ int[16].
// Every thread of the workgroup must call it (two barriers).
__device__ __forceinline__ int block_excl_scan_1024(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const int s = wsum[w];
    pre += w < wv ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// The same for any workgroup size NT (a multiple of 64); wsum: __shared__ int[NT / 64].
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* wsum, int* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  int pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int s = wsum[w];
    pre += w < wv ? s : 0;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + incl - v;
}

// Exclusive prefix sums of one tile in[0 .. n), n <= kScanTile, into out by ONE 1024-thread
// workgroup, plus `carry`: coalesced 16-byte loads into LDS (one pad word per 16 so that each
// thread's 16 consecutive values are conflict-free), a 16-value serial scan per thread, the
// workgroup scan of the thread sums, coalesced stores.  s_tile: __shared__ int[kScanTileLds].
// Returns the tile sum; *mx (optional) gets this thread's max of its values.
constexpr int kScanTile = 16384, kScanTileLds = kScanTile + kScanTile / 16;
__device__ __forceinline__ int wg_scan_tile(const int* __restrict__ in, int* __restrict__ out, int n, int carry,
                                            int* s_tile, int* wsum, int* mx = nullptr) {
  const int t = threadIdx.x;
  auto pad = [](int i) { return i + (i >> 4); };
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = 4 * (t + 1024 * u);
    int4 v = make_int4(0, 0, 0, 0);
    if (i + 3 < n && ((reinterpret_cast<size_t>(in) & 15) == 0)) {
      v = *reinterpret_cast<const int4*>(in + i);
    } else {
      v.x = i < n ? in[i] : 0; v.y = i + 1 < n ? in[i + 1] : 0;
      v.z = i + 2 < n ? in[i + 2] : 0; v.w = i + 3 < n ? in[i + 3] : 0;
    }
    s_tile[pad(i)] = v.x; s_tile[pad(i + 1)] = v.y; s_tile[pad(i + 2)] = v.z; s_tile[pad(i + 3)] = v.w;
  }
  __syncthreads();
  int v[16], loc = 0, m = 0;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    v[u] = s_tile[17 * t + u];
    m = max(m, v[u]);
    loc += v[u];
  }
  int tot;
  int run = carry + block_excl_scan_1024(loc, wsum, &tot);
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    s_tile[17 * t + u] = run;
    run += v[u];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = 4 * (t + 1024 * u);
    const int4 r = make_int4(s_tile[pad(i)], s_tile[pad(i + 1)], s_tile[pad(i + 2)], s_tile[pad(i + 3)]);
    if (i + 3 < n && ((reinterpret_cast<size_t>(out) & 15) == 0)) {
      *reinterpret_cast<int4*>(out + i) = r;
    } else {
      if (i < n) out[i] = r.x;
      if (i + 1 < n) out[i + 1] = r.y;
      if (i + 2 < n) out[i + 2] = r.z;
      if (i + 3 < n) out[i + 3] = r.w;
    }
  }
  __syncthreads();  // s_tile is reused by the next tile
  if (mx) *mx = max(*mx, m);
  return tot;
}

// The same over any n, tile after tile (one workgroup).  Returns the total.
__device__ __forceinline__ int wg_excl_scan(const int* __restrict__ in, int* __restrict__ out, int n, int* s_tile,
                                            int* wsum, int* mx = nullptr) {
  int carry = 0;
  for (int base = 0; base < n; base += kScanTile)
    carry += wg_scan_tile(in + base, out + base, min(n - base, kScanTile), carry, s_tile, wsum, mx);
  return carry;
}

// Exclusive max-scan (identity `lo`) across an NT-thread workgroup; wmax: __shared__ int[NT / 64].
template <int NT>
__device__ __forceinline__ int block_excl_max(int v, int lo, int* wmax) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl = max(incl, u);
  }
  int ex = __shfl_up(incl, 1, 64);
  if (lane == 0) ex = lo;
  if (lane == 63) wmax[wv] = incl;
  __syncthreads();
  int pre = lo;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) pre = w < wv ? max(pre, wmax[w]) : pre;
  __syncthreads();
  return max(pre, ex);
}

// A 4x4 float matrix passed by value as a kernel argument (no upload).
struct Mat4f {
  float v[16];
};

// Frame::UnprojectStereo for one keypoint with depth z > 0 (src/frame.cpp:335-356): camera
// coordinates in float, then Twc * [x y z 1] accumulated in double as cv::Mat's float gemm does.
// Shared by k_unproject and the LocalMapping append (compiled -ffp-contract=off: same bits).
__device__ __forceinline__ void unproject_point(float fx, float fy, float cx, float cy, const Mat4f& Twc, float u,
                                                float v, float z, float* out) {
  const float xx = (u - cx) * z / fx;
  const float yy = (v - cy) * z / fy;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const double s = (double)Twc.v[4 * r] * xx + (double)Twc.v[4 * r + 1] * yy + (double)Twc.v[4 * r + 2] * z +
                     (double)Twc.v[4 * r + 3] * 1.0f;
    out[r] = (float)s;
  }
}
// cv::Mat::inv() of a 4x4 CV_32F (hal::LU32f), host side (lorb_window.hip)
bool inv4_lu32f(const float* A, float* out);

// Four counters (plain POD: HIP's int4 member proxies are avoided in arithmetic-heavy code).
struct I4 {
  int v[4];
};

// Exclusive scan of four counters at once across an NT-thread workgroup; wsum: __shared__ I4[NT / 64].
template <int NT>
__device__ __forceinline__ I4 block_excl_scan4(const I4& v, I4* wsum, I4* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  I4 incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = __shfl_up(incl.v[q], o, 64);
      if (lane >= o) incl.v[q] += u;
    }
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  I4 pre = {{0, 0, 0, 0}}, tot = {{0, 0, 0, 0}};
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const I4 s = wsum[w];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      pre.v[q] += w < wv ? s.v[q] : 0;
      tot.v[q] += s.v[q];
    }
  }
  __syncthreads();
  *total = tot;
  I4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) r.v[q] = pre.v[q] + incl.v[q] - v.v[q];
  return r;
}

}  // namespace lorb

// scratch slot plan (per API family; calls on one ctx are serialized)
enum {
  S_BF_Q = 0, S_BF_T, S_BF_TL, S_BF_TILES, S_BF_K1, S_BF_K2, S_BF_QKEY, S_BF_OUT0, S_BF_OUT1,
  S_BF_OUT2, S_BF_OUT3, S_BF_OUT4, S_BF_OUT5, S_BF_OFF,
  S_W0 = 14, S_W1, S_W2, S_W3, S_W4, S_W5, S_W6, S_W7, S_W8, S_W9,
  S_KP = 24,   /* 10 slots: keypoint upload + grid */
  S_WX = 34,   /* 8 slots: windowed-matcher scratch */
  S_BF_TKEY = 120, /* crossCheck per-train keys: all-ones between calls (the merge resets them) */
  S_IO_IN = 121,   /* InPack device block */
  S_IO_OUT = 122,  /* OutPack device block */
  S_BF_DONE = 123  /* k_bf_cc1's workgroup counter: zero between calls (the last workgroup resets it) */
};
