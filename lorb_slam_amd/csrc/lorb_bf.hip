// lorb_bf.hip -- brute-force ORB Hamming matching on gfx950 (MI355X).
//
// Replaces cv::BFMatcher(NORM_HAMMING, crossCheck=true).match (src/matcher.cpp:36-39, 342-345)
// and the best/second-best scan of Matcher::SearchByProjection (src/matcher.cpp:289-311) for an
// unbounded window (BASELINE config "2000x2000 random 256-bit descriptors, ratio test").
//
// Design (CDNA4-first, integer VALU bound -- no GEMM reshaping):
//   * One "scan" kernel: each lane owns one descriptor of the LANE side (8 VGPRs), the wave
//     walks the UNIFORM side in order.  Uniform descriptors are wave-uniform addresses, so they
//     arrive through the scalar cache (s_load) straight into SGPRs -- no LDS traffic at all.
//   * Distance: 8 x v_xor_b32 + 8 x v_bcnt_u32_b32 (popcount-accumulate).
//   * Tie semantics are folded into one 32-bit key = (dist << 23) | uniform_index, so
//     "strict <, first index wins" == unsigned min.  Top-2 of keys costs v_min + v_med3
//     per pair; top-1 (cross-check reverse pass) costs one v_min.
//   * Large problems are split into uniform-side chunks (more workgroups) and merged by a
//     tiny deterministic merge kernel (top-2 of keys is associative).
//   * Cross-check: the reverse pass (lanes = trains, uniform = queries) yields each train's
//     nearest query; a 64-bit atomicMin of (dist<<32 | train) per query reproduces OpenCV's
//     ascending-train "if (d < dist[q])" resolution exactly; a per-problem block then applies
//     the reference's minDist / max(2*minDist, 30) filter.
#include "lorb_internal.h"

#include <cstdlib>

namespace {

constexpr uint32_t kIdxBits = 23;
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1u;
constexpr uint32_t kSentinel = 256u << kIdxBits;  // "dist 256, index 0": never beaten by d=256

struct BfTile {
  int32_t lane_base;   // first lane descriptor (global index into the lane array)
  int32_t lane_count;  // <= 256
  int32_t uni_base;    // first uniform descriptor (global index)
  int32_t uni_count;   // uniform descriptors in this chunk
  int32_t uni_local0;  // problem-local index of uni_base (goes into the key)
  int32_t out_base;    // partial-output index of lane 0 (chunk-major)
};

__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  // not volatile: a pure value, so the scheduler may interleave independent pairs' chains
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// popcount-accumulate chain: one v_xor_b32 + one v_bcnt_u32_b32 per 32-bit word (16 VALU/pair)
// (written as asm: from __builtin_popcount(x) + acc the compiler emits v_bcnt x, 0 plus v_add3
// trees, 12% slower here)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}

// (dist << kIdxBits) + idx as ONE v_lshl_add_u32 with the index in an SGPR: the index goes through
// an opaque scalar move (written as plain C++, the compiler folds the step offset into an immediate
// and splits all but one key per step into v_lshlrev + v_add3)
__device__ __forceinline__ uint32_t make_key(uint32_t d, uint32_t idx) {
  asm("s_mov_b32 %0, %0" : "+s"(idx));
  return (d << kIdxBits) + idx;
}
static_assert(kIdxBits == 23, "make_key's shift");

__device__ __forceinline__ uint32_t hamming256(const uint4& a0, const uint4& a1, const uint4& b0,
                                               const uint4& b1) {
  uint32_t d = __builtin_popcount(a0.x ^ b0.x);
  d = bcnt_acc(a0.y ^ b0.y, d);
  d = bcnt_acc(a0.z ^ b0.z, d);
  d = bcnt_acc(a0.w ^ b0.w, d);
  d = bcnt_acc(a1.x ^ b1.x, d);
  d = bcnt_acc(a1.y ^ b1.y, d);
  d = bcnt_acc(a1.z ^ b1.z, d);
  d = bcnt_acc(a1.w ^ b1.w, d);
  return d;
}

// QPL = lane-side descriptors per thread (1, 2 or 4; LORB_BF_QPL): a block covers 256*QPL lane items; every
// uniform descriptor loaded into SGPRs feeds QPL distance chains.
// ATOM (top-1 only): the chunk's key is combined into k1_out[lane item] by atomicMin (one key per
// lane item for all chunks, no partial array and no serial merge over chunks)
template <bool TOP2, int QPL, bool ATOM = false>
__device__ __forceinline__ void scan_tile(const uint4* __restrict__ lane_desc, const uint4* __restrict__ uni_desc,
                                          const BfTile& tl, uint32_t* __restrict__ k1_out,
                                          uint32_t* __restrict__ k2_out) {
  uint4 a[QPL][2];
  uint32_t k1[QPL], k2[QPL];
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    const int l = threadIdx.x + 256 * r;
    a[r][0] = a[r][1] = make_uint4(0, 0, 0, 0);
    if (l < tl.lane_count) {
      a[r][0] = lane_desc[2 * (size_t)(tl.lane_base + l)];
      a[r][1] = lane_desc[2 * (size_t)(tl.lane_base + l) + 1];
    }
    k1[r] = kSentinel;
    k2[r] = kSentinel;
  }
  const uint4* __restrict__ u = uni_desc + 2 * (size_t)tl.uni_base;
  const uint32_t kb = (uint32_t)tl.uni_local0;
  const int n = tl.uni_count;
  int j = 0;
  // 4 train descriptors per step in SGPRs (s_load); the next step's are requested before this
  // step's 18 x 4 x QPL VALU ops, so the scalar-cache / L2 latency hides behind them.  Two steps
  // per iteration on two register sets, so no set is copied into the other between steps.
  auto step = [&](const uint4 (&b)[8], int js) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int r = 0; r < QPL; ++r) {
        const uint32_t key = make_key(hamming256(a[r][0], a[r][1], b[2 * s], b[2 * s + 1]), kb + (uint32_t)(js + s));
        if (TOP2) k2[r] = umed3(k1[r], key, k2[r]);
        k1[r] = min(k1[r], key);
      }
    }
  };
  uint4 bA[8], bB[8];
  if (n >= 4) {  // bA: the descriptors of step j whenever j + 4 <= n at the loop head
#pragma unroll
    for (int s = 0; s < 8; ++s) bA[s] = u[s];
  }
  for (; j + 8 <= n; j += 8) {
#pragma unroll
    for (int s = 0; s < 8; ++s) bB[s] = u[2 * (j + 4) + s];
    step(bA, j);
    if (j + 12 <= n) {
#pragma unroll
      for (int s = 0; s < 8; ++s) bA[s] = u[2 * (j + 8) + s];
    }
    step(bB, j + 4);
  }
  if (j + 4 <= n) {
    step(bA, j);
    j += 4;
  }
  for (; j < n; ++j) {
    const uint4 b0 = u[2 * j], b1 = u[2 * j + 1];
#pragma unroll
    for (int r = 0; r < QPL; ++r) {
      const uint32_t key = make_key(hamming256(a[r][0], a[r][1], b0, b1), kb + (uint32_t)j);
      if (TOP2) k2[r] = umed3(k1[r], key, k2[r]);
      k1[r] = min(k1[r], key);
    }
  }
#pragma unroll
  for (int r = 0; r < QPL; ++r) {
    const int l = threadIdx.x + 256 * r;
    if (l < tl.lane_count) {
      if (ATOM) {
        if (k1[r] < kSentinel) atomicMin(&k1_out[tl.lane_base + l], k1[r]);
      } else {
        k1_out[tl.out_base + l] = k1[r];
        if (TOP2) k2_out[tl.out_base + l] = k2[r];
      }
    }
  }
}

template <bool TOP2, int QPL>
__global__ __launch_bounds__(256) void k_bf_scan(const uint4* __restrict__ lane_desc,
                                                 const uint4* __restrict__ uni_desc,
                                                 const BfTile* __restrict__ tiles,
                                                 uint32_t* __restrict__ k1_out,
                                                 uint32_t* __restrict__ k2_out) {
  scan_tile<TOP2, QPL>(lane_desc, uni_desc, tiles[blockIdx.x], k1_out, k2_out);
}

// One problem (the LocalMapping step's SearchLocalPoints): the tile of workgroup b is computed,
// not read from an uploaded table -- chunk c = b / lane_tiles, lane tile b % lane_tiles, the order
// of build_tiles -- and the crossCheck query keys (kinit) are set to all-ones on the way.
struct BfGrid1 {
  int nl, nu, n_chunks, lt, lane_tiles;
};
__device__ __forceinline__ BfTile scan1_tile_of(const BfGrid1& g) {
  const int c = blockIdx.x / g.lane_tiles, t = (blockIdx.x - c * g.lane_tiles) * g.lt;
  const int a = (int)((int64_t)g.nu * c / g.n_chunks), b = (int)((int64_t)g.nu * (c + 1) / g.n_chunks);
  BfTile tl;
  tl.lane_base = t;
  tl.lane_count = min(g.lt, g.nl - t);
  tl.uni_base = a;
  tl.uni_count = b - a;
  tl.uni_local0 = a;
  tl.out_base = c * g.nl + t;
  return tl;
}
template <int QPL>
__device__ __forceinline__ void scan1_tile(const uint4* __restrict__ lane_desc, const uint4* __restrict__ uni_desc,
                                           const BfGrid1& g, uint32_t* __restrict__ k1_out) {
  scan_tile<false, QPL, true>(lane_desc, uni_desc, scan1_tile_of(g), k1_out, nullptr);
}
template <bool TOP2, int QPL>
__global__ __launch_bounds__(256) void k_bf_scan1(const uint4* __restrict__ lane_desc,
                                                  const uint4* __restrict__ uni_desc, BfGrid1 g,
                                                  uint32_t* __restrict__ k1_out, uint32_t* __restrict__ k2_out,
                                                  unsigned long long* __restrict__ kinit, int n_init) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n_init; i += gridDim.x * 256) kinit[i] = ~0ull;
  scan_tile<TOP2, QPL, !TOP2>(lane_desc, uni_desc, scan1_tile_of(g), k1_out, k2_out);
}

// One problem, crossCheck: each train's nearest query (the scan's atomicMin over the chunks) offered
// to that query (k_cc_scatter's atomicMin); the train key is reset to all-ones for the next call
__global__ __launch_bounds__(256) void k_cc_merge1(uint32_t* __restrict__ tkey, int nt,
                                                   unsigned long long* __restrict__ qkey) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;
  const uint32_t k = tkey[t];
  if (k >= kSentinel) return;
  tkey[t] = 0xffffffffu;
  const unsigned long long v = ((unsigned long long)(k >> kIdxBits) << 32) | (unsigned)t;
  atomicMin(&qkey[k & kIdxMask], v);
}

// merge chunk partials: part[c * n + i] -> out[i]
template <bool TOP2>
__global__ __launch_bounds__(256) void k_bf_merge(const uint32_t* __restrict__ k1p,
                                                  const uint32_t* __restrict__ k2p, int n,
                                                  int n_chunks, uint32_t* __restrict__ k1o,
                                                  uint32_t* __restrict__ k2o,
                                                  unsigned long long* __restrict__ kinit, int n_init) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_init) kinit[i] = ~0ull;  // crossCheck query keys, folded in instead of a fill launch
  if (i >= n) return;
  uint32_t k1 = kSentinel, k2 = kSentinel;
  for (int c = 0; c < n_chunks; ++c) {
    const uint32_t a = k1p[(size_t)c * n + i];
    if (TOP2) k2 = umed3(k1, a, k2);
    k1 = min(k1, a);
    if (TOP2) {
      const uint32_t b = k2p[(size_t)c * n + i];
      k2 = umed3(k1, b, k2);
      k1 = min(k1, b);
    }
  }
  k1o[i] = k1;
  if (TOP2) k2o[i] = k2;
}

__device__ __forceinline__ int find_problem(const int32_t* __restrict__ off, int np, int i) {
  int lo = 0, hi = np - 1;  // largest p with off[p] <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// decode top-2 keys + level-gated ratio test (src/matcher.cpp:305-311)
__global__ __launch_bounds__(256) void k_top2_finalize(
    const uint32_t* __restrict__ k1, const uint32_t* __restrict__ k2, int nq,
    const int32_t* __restrict__ q_off, const int32_t* __restrict__ t_off, int np,
    const int32_t* __restrict__ t_level, int32_t* __restrict__ best_idx,
    int32_t* __restrict__ best_dist, int32_t* __restrict__ best_level,
    int32_t* __restrict__ second_dist, int32_t* __restrict__ second_level,
    uint8_t* __restrict__ accepted) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq) return;
  const int p = find_problem(q_off, np, i);
  const int tb = t_off[p];
  const bool has_t = t_off[p + 1] > tb;
  const uint32_t a = has_t ? k1[i] : kSentinel, b = has_t ? k2[i] : kSentinel;
  const int d1 = (int)(a >> kIdxBits), d2 = (int)(b >> kIdxBits);
  const int i1 = d1 < 256 ? (int)(a & kIdxMask) : -1;
  const int i2 = d2 < 256 ? (int)(b & kIdxMask) : -1;
  const int l1 = i1 >= 0 ? (t_level ? t_level[tb + i1] : 0) : -1;
  const int l2 = i2 >= 0 ? (t_level ? t_level[tb + i2] : 0) : -1;
  int acc = 0;
  if (d1 <= LORB_TH_HIGH) {
    acc = 1;
    if (l1 == l2 && (double)d1 > 0.8 * (double)d2) acc = 0;
  }
  best_idx[i] = i1;
  best_dist[i] = d1;
  best_level[i] = l1;
  second_dist[i] = d2;
  second_level[i] = l2;
  accepted[i] = (uint8_t)acc;
}

// cross-check resolution: per train, offer (dist, train) to its nearest query
// (sharded rows: keys carry GLOBAL query numbers, q_base[p] = this rank's first query of
// problem p; only trains whose nearest query is local are offered)
__global__ __launch_bounds__(256) void k_cc_scatter(const uint32_t* __restrict__ tkey, int nt,
                                                    const int32_t* __restrict__ q_off,
                                                    const int32_t* __restrict__ t_off, int np,
                                                    const int32_t* __restrict__ q_base,
                                                    unsigned long long* __restrict__ qkey) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;
  const int p = find_problem(t_off, np, t);
  const uint32_t k = tkey[t];
  if (k >= kSentinel) return;  // no query anywhere
  uint32_t q = k & kIdxMask;
  const uint32_t d = k >> kIdxBits;
  if (q_base) {
    if ((int)q < q_base[p] || (int)q >= q_base[p] + (q_off[p + 1] - q_off[p])) return;
    q -= (uint32_t)q_base[p];
  } else if (q_off[p + 1] == q_off[p]) {
    return;
  }
  const unsigned long long v = ((unsigned long long)d << 32) | (unsigned)(t - t_off[p]);
  atomicMin(&qkey[q_off[p] + q], v);
}

// one workgroup per problem: DMatch list + minDist filter (src/matcher.cpp:42-56)
// MODE 0: whole problem on this device.  Sharded rows: MODE 1 writes the local DMatches and the
// local minDist (ex[p], as double) for an all-reduce(min); MODE 2 filters with the global
// minDist and writes the local count (ex[np + p]) for an all-reduce(sum).
template <int MODE>
__device__ __forceinline__ void cc_finalize_body(int p, const unsigned long long* __restrict__ qkey,
                                                 const int32_t* __restrict__ q_off, const int32_t* __restrict__ t_off,
                                                 int32_t* __restrict__ cc_train, int32_t* __restrict__ cc_dist,
                                                 int32_t* __restrict__ match_train, int32_t* __restrict__ n_matches,
                                                 double* __restrict__ ex, int np, int nq1, int nt1) {
  // q_off == nullptr: one problem with nq1 queries and nt1 trains (offsets passed by value)
  const int q0 = q_off ? q_off[p] : 0, q1 = q_off ? q_off[p + 1] : nq1;
  const bool has_t = q_off ? t_off[p + 1] > t_off[p] : nt1 > 0;
  __shared__ int s_min[256];
  __shared__ int s_cnt[256];
  int mn = 0x7fffffff;
  if (MODE != 2) {
  for (int q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const unsigned long long v = has_t ? qkey[q] : ~0ull;
    if (v != ~0ull) {
      const int d = (int)(v >> 32);
      cc_train[q] = (int)(v & 0xffffffffu);
      cc_dist[q] = d;
      mn = min(mn, d);
    } else {
      cc_train[q] = -1;
      cc_dist[q] = 0;
    }
  }
  s_min[threadIdx.x] = mn;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) s_min[threadIdx.x] = min(s_min[threadIdx.x], s_min[threadIdx.x + s]);
    __syncthreads();
  }
  }
  if (MODE == 1) {
    if (threadIdx.x == 0) ex[p] = (double)s_min[0];
    return;
  }
  const int minDist = MODE == 2 ? (int)ex[p] : s_min[0];
  // d > max(2*minDist, 30.0) rejects (exact in integers); no key at all: 2 * INT_MAX is not formed
  const int thr = minDist >= (1 << 30) ? 30 : max(2 * minDist, 30);
  int cnt = 0;
  for (int q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const unsigned long long v = has_t ? qkey[q] : ~0ull;
    int m = -1;
    if (v != ~0ull && (int)(v >> 32) <= thr) { m = (int)(v & 0xffffffffu); cnt++; }
    match_train[q] = m;
  }
  s_cnt[threadIdx.x] = cnt;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) s_cnt[threadIdx.x] += s_cnt[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (MODE == 2) ex[np + p] = (double)s_cnt[0];
    else n_matches[p] = s_cnt[0];
  }
}
template <int MODE>
__global__ __launch_bounds__(256) void k_cc_finalize(const unsigned long long* __restrict__ qkey,
                                                     const int32_t* __restrict__ q_off,
                                                     const int32_t* __restrict__ t_off,
                                                     int32_t* __restrict__ cc_train,
                                                     int32_t* __restrict__ cc_dist,
                                                     int32_t* __restrict__ match_train,
                                                     int32_t* __restrict__ n_matches,
                                                     double* __restrict__ ex, int np, int nq1 = 0, int nt1 = 0) {
  cc_finalize_body<MODE>(blockIdx.x, qkey, q_off, t_off, cc_train, cc_dist, match_train, n_matches, ex, np, nq1, nt1);
}

// The one-problem crossCheck (lorb_bf_match, np == 1) in ONE launch: k_bf_scan1<false>'s tiles, then
// the workgroup that finishes last (a device-scope counter) runs k_cc_merge1 and k_cc_finalize<0> for
// the problem.  Every workgroup's key atomics and query-key initialisation are released (agent-scope
// fence) before its count; the last one acquires before reading them and resets the counter.
template <int QPL>
__global__ __launch_bounds__(256) void k_bf_cc1(const uint4* __restrict__ lane_desc, const uint4* __restrict__ uni_desc,
                                                BfGrid1 g, uint32_t* __restrict__ tkey,
                                                unsigned long long* __restrict__ qkey, unsigned* __restrict__ done,
                                                int32_t* __restrict__ cc_train, int32_t* __restrict__ cc_dist,
                                                int32_t* __restrict__ match_train, int32_t* __restrict__ n_matches) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < g.nu; i += gridDim.x * 256) qkey[i] = ~0ull;
  scan1_tile<QPL>(lane_desc, uni_desc, g, tkey);
  __shared__ int s_last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(done, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  for (int t = threadIdx.x; t < g.nl; t += 256) {  // k_cc_merge1
    const uint32_t k = __hip_atomic_load(&tkey[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k >= kSentinel) continue;
    tkey[t] = 0xffffffffu;
    atomicMin(&qkey[k & kIdxMask], ((unsigned long long)(k >> kIdxBits) << 32) | (unsigned)t);
  }
  __threadfence();
  __syncthreads();
  cc_finalize_body<0>(0, qkey, nullptr, nullptr, cc_train, cc_dist, match_train, n_matches, nullptr, 1, g.nu, g.nl);
  if (threadIdx.x == 0) *done = 0u;
}

// train keys <-> doubles for the all-reduce(min) (keys < 2^32 are exact in double); trains of
// problems without local queries were not scanned and offer the sentinel
__global__ void k_u32_f64(const uint32_t* __restrict__ a, double* __restrict__ b, int n, int dir,
                          uint32_t* __restrict__ c, const int32_t* __restrict__ q_off,
                          const int32_t* __restrict__ t_off, int np) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (dir == 0) {
    const int p = find_problem(t_off, np, i);
    b[i] = q_off[p + 1] > q_off[p] ? (double)a[i] : (double)kSentinel;
  } else {
    c[i] = (uint32_t)b[i];
  }
}
__global__ void k_counts_out(const double* __restrict__ ex, int np, int32_t* __restrict__ n_matches) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < np) n_matches[p] = (int32_t)ex[np + p];
}


// MapPoint::ComputeDescriptor (src/map_point.cpp:69-129), one wavefront per map point: lane i
// owns candidate descriptor i (rows i, i+64, ... for long lists).  The median of row i of the
// all-pairs Hamming matrix (self-distance 0 included, element floor((n-1)/2) of the sorted row,
// src/map_point.cpp:115-118) is found by a 9-step binary search over the value range [0, 256]
// counting #{j : d(i, j) <= v}; the other candidates are wave-uniform loads (scalar cache).
// The smallest median wins, first index on ties (strict '<', :119).
__global__ __launch_bounds__(256) void k_compute_descriptor(const uint4* __restrict__ desc,
                                                            const int32_t* __restrict__ d_off,
                                                            int np, int32_t* __restrict__ best,
                                                            uint4* __restrict__ out_desc) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  const int lane = threadIdx.x & 63;
  const int o0 = d_off[p], n = d_off[p + 1] - o0;
  if (n <= 0) {
    if (lane == 0) best[p] = -1;
    return;
  }
  const int k = (n - 1) / 2;  // vDist[0.5 * (n - 1)]: the double index truncates
  const uint4* __restrict__ D = desc + 2 * (size_t)o0;
  unsigned long long bestkey = ~0ull;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const bool act = i < n;
    const uint4 a0 = act ? D[2 * i] : make_uint4(0, 0, 0, 0), a1 = act ? D[2 * i + 1] : make_uint4(0, 0, 0, 0);
    // the median is the smallest v in [0, 256] with #{j : d(i, j) <= v} > k (at most 9 steps)
    int lo = 0, hi = act ? 256 : 0;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      int cnt = 0;
      for (int j = 0; j < n; ++j) cnt += (int)(hamming256(a0, a1, D[2 * j], D[2 * j + 1]) <= (uint32_t)mid);
      if (cnt > k) hi = mid;
      else lo = mid + 1;
    }
    if (act) {
      const unsigned long long key = ((unsigned long long)lo << 32) | (unsigned)i;
      bestkey = key < bestkey ? key : bestkey;
    }
  }
  // first index with the smallest median: min over (median, index)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(bestkey, off, 64);
    bestkey = o < bestkey ? o : bestkey;
  }
  const int bi = (int)(bestkey & 0xffffffffu);
  if (lane == 0) best[p] = bi;
  if (out_desc && lane < 2) out_desc[2 * (size_t)p + lane] = D[2 * bi + lane];
}

// Host: tile table for "lanes = L side, uniform = U side" with a fixed number of U chunks.
int build_tiles(lorb_ctx* ctx, int np, const int32_t* l_off, const int32_t* u_off, int lt,
                std::vector<BfTile>& tiles, int* n_chunks_out, const int32_t* u_base = nullptr) {
  const int64_t nl_total = l_off[np] - l_off[0];
  int64_t max_u = 0, lane_tiles = 0;
  for (int p = 0; p < np; p++) {
    const int64_t nl = l_off[p + 1] - l_off[p], nu = u_off[p + 1] - u_off[p];
    if (nl < 0 || nu < 0) return lorb::set_error(ctx, LORB_E_INVALID, "offsets not monotone at problem %d", p);
    if (nu > (int64_t)kIdxMask) return lorb::set_error(ctx, LORB_E_INVALID, "problem %d: %lld uniform items > 2^23-1", p, (long long)nu);
    if (nu > 0) lane_tiles += (nl + lt - 1) / lt;
    max_u = std::max<int64_t>(max_u, nu);
  }
  // Uniform-range chunks per lane tile.  With >= 256 lane tiles the chip is filled already: aim
  // at ~8 workgroups per CU (latency hiding), >= 128 uniform items per chunk (measured best for
  // C2).  With fewer tiles the scan is VALU-bound on a partly filled chip and workgroups sharing
  // a CU share its SIMDs: a CU's time is (workgroups on it) x (uniform items per chunk), so pick
  // the count minimising ceil(tiles x chunks / CUs) x ceil(max_u / chunks) (+ chunks: the merge
  // reads one key per chunk), >= 32 uniform items per chunk, at most 64 chunks.
  int n_chunks = 1;
  constexpr int64_t kCUs = 256;  // MI355X: 8 XCDs x 32 CUs
  if (lane_tiles >= kCUs) {
    const int64_t want = (2048 + lane_tiles - 1) / lane_tiles;
    const int64_t cap = std::max<int64_t>(1, max_u / 128);
    n_chunks = (int)std::max<int64_t>(1, std::min<int64_t>(want, std::min<int64_t>(cap, 64)));
  } else if (lane_tiles > 0) {
    const int64_t cap = std::max<int64_t>(1, std::min<int64_t>(64, max_u / 32));
    int64_t best = -1;
    for (int64_t nc = 1; nc <= cap; ++nc) {
      const int64_t cost = (lane_tiles * nc + kCUs - 1) / kCUs * ((max_u + nc - 1) / nc) + nc;
      if (best < 0 || cost < best) { best = cost; n_chunks = (int)nc; }
    }
  }
  tiles.clear();
  for (int p = 0; p < np; p++) {
    const int l0 = l_off[p] - l_off[0], nl = l_off[p + 1] - l_off[p];
    const int u0 = u_off[p] - u_off[0], nu = u_off[p + 1] - u_off[p];
    if (nu == 0 || nl == 0) continue;
    for (int c = 0; c < n_chunks; c++) {
      const int a = (int)((int64_t)nu * c / n_chunks), b = (int)((int64_t)nu * (c + 1) / n_chunks);
      for (int t = 0; t < nl; t += lt) {
        BfTile tl;
        tl.lane_base = l0 + t;
        tl.lane_count = std::min(lt, nl - t);
        tl.uni_base = u0 + a;
        tl.uni_count = b - a;
        tl.uni_local0 = a + (u_base ? u_base[p] : 0);
        tl.out_base = (int)((int64_t)c * nl_total + l0 + t);
        tiles.push_back(tl);
      }
    }
  }
  *n_chunks_out = n_chunks;
  return LORB_OK;
}

// scan + merge; final keys land in k1/k2 (n_lanes entries)
// kinit (n_init entries) is set to all-ones by the merge when one runs (*kinit_done = true);
// otherwise the caller initialises it.
template <bool TOP2>
int scan(lorb_ctx* ctx, int np, const uint8_t* d_lane, const int32_t* l_off, const uint8_t* d_uni,
         const int32_t* u_off, uint32_t** k1_final, uint32_t** k2_final, const int32_t* u_base = nullptr,
         unsigned long long* kinit = nullptr, int n_init = 0, bool* kinit_done = nullptr) {
  if (kinit_done) *kinit_done = false;
  std::vector<BfTile> tiles;
  int n_chunks = 1;
  static const int qpl = [] {
    const char* e = getenv("LORB_BF_QPL");
    const int v = e ? atoi(e) : 2;
    return v == 1 || v == 4 ? v : 2;
  }();
  LORB_TRY(build_tiles(ctx, np, l_off, u_off, 256 * qpl, tiles, &n_chunks, u_base));
  const int nl = l_off[np] - l_off[0];
  BfTile* d_tiles = nullptr;
  uint32_t *k1 = nullptr, *k2 = nullptr, *m1 = nullptr, *m2 = nullptr;
  LORB_TRY(lorb::scratch_t(ctx, S_BF_K1, (size_t)nl * n_chunks, &k1));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_K2, (size_t)nl * (TOP2 ? n_chunks : 1), &k2));
  if (!tiles.empty()) {
    LORB_TRY(lorb::upload_t(ctx, S_BF_TILES, tiles.data(), tiles.size(), &d_tiles));
    lorb::KernelTimer kt(ctx, TOP2 ? LORB_K_BF_SCAN_TOP2 : LORB_K_BF_SCAN_TOP1);
    if (qpl == 2)
      hipLaunchKernelGGL((k_bf_scan<TOP2, 2>), dim3((unsigned)tiles.size()), dim3(256), 0, ctx->stream,
                         reinterpret_cast<const uint4*>(d_lane), reinterpret_cast<const uint4*>(d_uni),
                         d_tiles, k1, k2);
    else if (qpl == 4)
      hipLaunchKernelGGL((k_bf_scan<TOP2, 4>), dim3((unsigned)tiles.size()), dim3(256), 0, ctx->stream,
                         reinterpret_cast<const uint4*>(d_lane), reinterpret_cast<const uint4*>(d_uni),
                         d_tiles, k1, k2);
    else
      hipLaunchKernelGGL((k_bf_scan<TOP2, 1>), dim3((unsigned)tiles.size()), dim3(256), 0, ctx->stream,
                         reinterpret_cast<const uint4*>(d_lane), reinterpret_cast<const uint4*>(d_uni),
                         d_tiles, k1, k2);
    LORB_CHECK_LAUNCH(ctx);
  }
  if (n_chunks > 1 && nl > 0) {
    LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT4, (size_t)nl, &m1));
    LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT5, (size_t)nl, &m2));
    const int ni = kinit ? n_init : 0;
    hipLaunchKernelGGL(k_bf_merge<TOP2>, dim3(lorb::ceil_div(std::max(nl, ni), 256)), dim3(256), 0, ctx->stream,
                       k1, k2, nl, n_chunks, m1, m2, kinit, ni);
    LORB_CHECK_LAUNCH(ctx);
    if (kinit_done) *kinit_done = ni > 0;
    *k1_final = m1;
    *k2_final = m2;
  } else {
    *k1_final = k1;
    *k2_final = k2;
  }
  return LORB_OK;
}

}  // namespace

namespace {
// grid of the one-problem scan (k_bf_scan1 / k_bf_cc1).  Chunks of the query range: the chunks'
// keys meet in one atomicMin per train, so chunks are cheap -- aim at ~6 workgroups per CU
// (latency hiding on the VALU-bound scan), >= 32 queries per chunk (LORB_BF_NC overrides:
// diagnostics).  qpl: LORB_BF_QPL (1, 2 or 4).
BfGrid1 grid1_of(int nq, int nt, int* qpl_out) {
  static const int qpl = [] {
    const char* e = getenv("LORB_BF_QPL");
    const int v = e ? atoi(e) : 2;
    return v == 1 || v == 4 ? v : 2;
  }();
  const int lt = 256 * qpl, lane_tiles = (nt + lt - 1) / lt;
  static const int nc_env = [] { const char* e = getenv("LORB_BF_NC"); return e ? atoi(e) : 0; }();
  int n_chunks = std::max(1, std::min((1536 + lane_tiles - 1) / lane_tiles, nq / 32));
  if (nc_env > 0) n_chunks = std::min(nc_env, nq);
  *qpl_out = qpl;
  return BfGrid1{nt, nq, n_chunks, lt, lane_tiles};
}
// the per-train keys (all-ones between calls; a fresh or grown buffer is set once)
int tkeys1(lorb_ctx* ctx, int nt, hipStream_t st, uint32_t** tkey) {
  LORB_TRY(lorb::scratch_t(ctx, S_BF_TKEY, (size_t)nt, tkey));
  if (ctx->tkey_buf != (void*)*tkey || ctx->tkey_ready < (size_t)nt) {
    LORB_HIP(ctx, hipMemsetAsync(*tkey, 0xff, sizeof(uint32_t) * (ctx->scratch_sz[S_BF_TKEY] / sizeof(uint32_t)), st));
    ctx->tkey_ready = ctx->scratch_sz[S_BF_TKEY] / sizeof(uint32_t);
    ctx->tkey_buf = *tkey;
  }
  return LORB_OK;
}
}  // namespace

// The crossCheck keys of ONE problem: per query (dist << 32 | train) of the train whose nearest
// query it is, all-ones where none (lorb_bf_match_dev up to the finalisation, which the caller does:
// k_cc_finalize<0>, or the LocalMapping append).  Nothing is uploaded: the scan computes its tiles and
// clears the keys, the chunk merge and the scatter are one launch.
int lorb::match1_keys_dev(lorb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                          unsigned long long** qkey_out, hipStream_t stream) {
  hipStream_t st = stream ? stream : ctx->stream;
  unsigned long long* qkey = nullptr;
  LORB_TRY(lorb::scratch_t(ctx, S_BF_QKEY, (size_t)std::max(nq, 1), &qkey));
  uint32_t* tkey = nullptr;
  size_t ready = 0;
  if (nt > 0 && nq > 0) {
    LORB_TRY(tkeys1(ctx, nt, st, &tkey));
    ready = ctx->tkey_ready;
    ctx->tkey_ready = 0;  // until the merge has been enqueued (it restores the all-ones)
  }
  LORB_TRY(lorb::match1_keys_into(ctx, d_q, nq, d_t, nt, qkey, tkey, st));
  if (tkey) ctx->tkey_ready = ready;
  *qkey_out = qkey;
  return LORB_OK;
}

// The same into caller-owned buffers: qkey (nq entries) and tkey (nt entries, all-ones on entry;
// the merge restores the all-ones).  The LocalMapping step owns its pair, so its side-stream match
// shares no scratch with matcher calls on the ctx stream.
int lorb::match1_keys_into(lorb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                           unsigned long long* qkey, uint32_t* tkey, hipStream_t st) {
  if (nt > 0 && nq > 0) {
    // reverse pass: lanes = trains, uniform = queries -> nearest query per train
    if (nq > (int)kIdxMask) return lorb::set_error(ctx, LORB_E_INVALID, "problem 0: %d uniform items > 2^23-1", nq);
    int qpl = 2;
    const BfGrid1 g = grid1_of(nq, nt, &qpl);
    const unsigned nb = (unsigned)(g.lane_tiles * g.n_chunks);
    {
      lorb::KernelTimer kt(ctx, LORB_K_BF_SCAN_TOP1);
      if (qpl == 2)
        hipLaunchKernelGGL((k_bf_scan1<false, 2>), dim3(nb), dim3(256), 0, st, reinterpret_cast<const uint4*>(d_t),
                           reinterpret_cast<const uint4*>(d_q), g, tkey, (uint32_t*)nullptr, qkey, nq);
      else if (qpl == 4)
        hipLaunchKernelGGL((k_bf_scan1<false, 4>), dim3(nb), dim3(256), 0, st, reinterpret_cast<const uint4*>(d_t),
                           reinterpret_cast<const uint4*>(d_q), g, tkey, (uint32_t*)nullptr, qkey, nq);
      else
        hipLaunchKernelGGL((k_bf_scan1<false, 1>), dim3(nb), dim3(256), 0, st, reinterpret_cast<const uint4*>(d_t),
                           reinterpret_cast<const uint4*>(d_q), g, tkey, (uint32_t*)nullptr, qkey, nq);
    }
    hipLaunchKernelGGL(k_cc_merge1, dim3(lorb::ceil_div(nt, 256)), dim3(256), 0, st, tkey, nt, qkey);
    LORB_CHECK_LAUNCH(ctx);
  } else if (nq > 0) {
    LORB_HIP(ctx, hipMemsetAsync(qkey, 0xff, sizeof(unsigned long long) * nq, st));
  }
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

namespace {

// lorb_bf_match_dev for ONE problem: the keys (match1_keys_dev) and the finalisation with the offsets
// passed by value.  Same outputs, bit for bit, as the general path.
int match1_dev(lorb_ctx* ctx, const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int32_t* d_cc_train,
               int32_t* d_cc_dist, int32_t* d_match_train, int32_t* d_n_matches) {
  if (nq > 0 && nt > 0 && nq <= (int)kIdxMask) {  // scan + merge + finalize in one launch (k_bf_cc1)
    int qpl = 2;
    const BfGrid1 g = grid1_of(nq, nt, &qpl);
    uint32_t* tkey = nullptr;
    unsigned long long* qkey = nullptr;
    unsigned* done = nullptr;
    LORB_TRY(tkeys1(ctx, nt, ctx->stream, &tkey));
    LORB_TRY(lorb::scratch_t(ctx, S_BF_QKEY, (size_t)nq, &qkey));
    LORB_TRY(lorb::scratch_t(ctx, S_BF_DONE, 1, &done));
    if (ctx->done_buf != (void*)done) {
      LORB_HIP(ctx, hipMemsetAsync(done, 0, sizeof(unsigned), ctx->stream));
      ctx->done_buf = done;
    }
    const size_t ready = ctx->tkey_ready;
    ctx->tkey_ready = 0;  // until the launch is enqueued (its last workgroup restores the all-ones)
    ctx->done_buf = nullptr;
    const unsigned nb = (unsigned)(g.lane_tiles * g.n_chunks);
    const uint4* lt = reinterpret_cast<const uint4*>(d_t);
    const uint4* ut = reinterpret_cast<const uint4*>(d_q);
    {
      lorb::KernelTimer kt(ctx, LORB_K_BF_SCAN_TOP1);
      if (qpl == 2)
        hipLaunchKernelGGL(k_bf_cc1<2>, dim3(nb), dim3(256), 0, ctx->stream, lt, ut, g, tkey, qkey, done, d_cc_train,
                           d_cc_dist, d_match_train, d_n_matches);
      else if (qpl == 4)
        hipLaunchKernelGGL(k_bf_cc1<4>, dim3(nb), dim3(256), 0, ctx->stream, lt, ut, g, tkey, qkey, done, d_cc_train,
                           d_cc_dist, d_match_train, d_n_matches);
      else
        hipLaunchKernelGGL(k_bf_cc1<1>, dim3(nb), dim3(256), 0, ctx->stream, lt, ut, g, tkey, qkey, done, d_cc_train,
                           d_cc_dist, d_match_train, d_n_matches);
    }
    LORB_CHECK_LAUNCH(ctx);
    ctx->tkey_ready = ready;
    ctx->done_buf = done;
    return LORB_OK;
  }
  unsigned long long* qkey = nullptr;
  LORB_TRY(lorb::match1_keys_dev(ctx, d_q, nq, d_t, nt, &qkey));
  hipLaunchKernelGGL(k_cc_finalize<0>, dim3(1), dim3(256), 0, ctx->stream, qkey, (const int32_t*)nullptr,
                     (const int32_t*)nullptr, d_cc_train, d_cc_dist, d_match_train, d_n_matches, (double*)nullptr, 1, nq, nt);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int check_offsets(lorb_ctx* ctx, int np, const int32_t* a, const int32_t* b) {
  if (!ctx) return LORB_E_INVALID;
  if (np < 0 || (np > 0 && (!a || !b))) return lorb::set_error(ctx, LORB_E_INVALID, "bad problem offsets");
  if (np > 0 && (a[0] != 0 || b[0] != 0)) return lorb::set_error(ctx, LORB_E_INVALID, "offsets must start at 0");
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_bf_top2_dev(lorb_ctx* ctx, int32_t np, const uint8_t* d_q, const int32_t* q_off,
                     const uint8_t* d_t, const int32_t* t_off, const int32_t* d_t_level,
                     int32_t* d_best_idx, int32_t* d_best_dist, int32_t* d_best_level,
                     int32_t* d_second_dist, int32_t* d_second_level, uint8_t* d_accepted) {
  LORB_TRY(check_offsets(ctx, np, q_off, t_off));
  if (np == 0 || q_off[np] == 0) return LORB_OK;
  uint32_t *k1 = nullptr, *k2 = nullptr;
  LORB_TRY(scan<true>(ctx, np, d_q, q_off, d_t, t_off, &k1, &k2));
  int32_t* d_off = nullptr;
  std::vector<int32_t> offs(q_off, q_off + np + 1);
  offs.insert(offs.end(), t_off, t_off + np + 1);
  LORB_TRY(lorb::upload_t(ctx, S_BF_OFF, offs.data(), offs.size(), &d_off));
  const int nq = q_off[np];
  hipLaunchKernelGGL(k_top2_finalize, dim3(lorb::ceil_div(nq, 256)), dim3(256), 0, ctx->stream, k1,
                     k2, nq, d_off, d_off + np + 1, np, d_t_level, d_best_idx, d_best_dist,
                     d_best_level, d_second_dist, d_second_level, d_accepted);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int lorb_bf_top2(lorb_ctx* ctx, int32_t np, const uint8_t* q, const int32_t* q_off,
                 const uint8_t* t, const int32_t* t_off, const int32_t* t_level,
                 int32_t* best_idx, int32_t* best_dist, int32_t* best_level, int32_t* second_dist,
                 int32_t* second_level, uint8_t* accepted) {
  LORB_TRY(check_offsets(ctx, np, q_off, t_off));
  if (np == 0) return LORB_OK;
  const int nq = q_off[np], nt = t_off[np];
  if (nq == 0) return LORB_OK;
  uint8_t *dq = nullptr, *dt = nullptr;
  int32_t *dl = nullptr, *o = nullptr;
  uint8_t* dacc = nullptr;
  LORB_TRY(lorb::upload_t(ctx, S_BF_Q, q, (size_t)nq * 32, &dq));
  if (nt > 0) LORB_TRY(lorb::upload_t(ctx, S_BF_T, t, (size_t)nt * 32, &dt));
  if (t_level && nt > 0) LORB_TRY(lorb::upload_t(ctx, S_BF_TL, t_level, (size_t)nt, &dl));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT0, (size_t)nq * 5, &o));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT1, (size_t)nq, &dacc));
  LORB_TRY(lorb_bf_top2_dev(ctx, np, dq, q_off, dt, t_off, dl, o, o + nq, o + 2 * nq, o + 3 * nq,
                            o + 4 * nq, dacc));
  int32_t* outs[5] = {best_idx, best_dist, best_level, second_dist, second_level};
  for (int k = 0; k < 5; k++)
    LORB_HIP(ctx, hipMemcpyAsync(outs[k], o + (size_t)k * nq, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(accepted, dacc, nq, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_bf_match_dev(lorb_ctx* ctx, int32_t np, const uint8_t* d_q, const int32_t* q_off,
                      const uint8_t* d_t, const int32_t* t_off, int32_t* d_cc_train,
                      int32_t* d_cc_dist, int32_t* d_match_train, int32_t* d_n_matches) {
  LORB_TRY(check_offsets(ctx, np, q_off, t_off));
  if (np == 0) return LORB_OK;
  const int nq = q_off[np], nt = t_off[np];
  if (np == 1) return match1_dev(ctx, d_q, nq, d_t, nt, d_cc_train, d_cc_dist, d_match_train, d_n_matches);
  uint32_t *k1 = nullptr, *k2 = nullptr;
  unsigned long long* qkey = nullptr;
  int32_t* d_off = nullptr;
  std::vector<int32_t> offs(q_off, q_off + np + 1);
  offs.insert(offs.end(), t_off, t_off + np + 1);
  LORB_TRY(lorb::upload_t(ctx, S_BF_OFF, offs.data(), offs.size(), &d_off));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_QKEY, (size_t)std::max(nq, 1), &qkey));
  bool keyed = false;
  if (nt > 0 && nq > 0) {
    // reverse pass: lanes = trains, uniform = queries  -> nearest query per train
    LORB_TRY(scan<false>(ctx, np, d_t, t_off, d_q, q_off, &k1, &k2, nullptr, qkey, nq, &keyed));
    if (!keyed) LORB_HIP(ctx, hipMemsetAsync(qkey, 0xff, sizeof(unsigned long long) * nq, ctx->stream));
    hipLaunchKernelGGL(k_cc_scatter, dim3(lorb::ceil_div(nt, 256)), dim3(256), 0, ctx->stream, k1,
                       nt, d_off, d_off + np + 1, np, (const int32_t*)nullptr, qkey);
    LORB_CHECK_LAUNCH(ctx);
  } else if (nq > 0) {
    LORB_HIP(ctx, hipMemsetAsync(qkey, 0xff, sizeof(unsigned long long) * nq, ctx->stream));
  }
  hipLaunchKernelGGL(k_cc_finalize<0>, dim3(np), dim3(256), 0, ctx->stream, qkey, d_off,
                     d_off + np + 1, d_cc_train, d_cc_dist, d_match_train, d_n_matches, (double*)nullptr, np);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

// Query rows sharded over ranks: reverse pass over the LOCAL queries with global
// query numbers in the keys, all-reduce(min) of the per-train keys, local resolution, then the
// global minDist (min) and match count (sum).  Three exchanges of Nt + 2 np doubles in total.
int lorb_bf_match_sharded_dev(lorb_ctx* ctx, lorb_comm* comm, int32_t np, const uint8_t* d_q,
                              const int32_t* q_off, const int32_t* q_base, const uint8_t* d_t,
                              const int32_t* t_off, int32_t* d_cc_train, int32_t* d_cc_dist,
                              int32_t* d_match_train, int32_t* d_n_matches) {
  LORB_TRY(check_offsets(ctx, np, q_off, t_off));
  if (!comm || !q_base || comm->ctx != ctx) return lorb::set_error(ctx, LORB_E_INVALID, "bad communicator / q_base");
  for (int p = 0; p < np; ++p)
    if (q_base[p] < 0 || (int64_t)q_base[p] + (q_off[p + 1] - q_off[p]) > (int64_t)kIdxMask)
      return lorb::set_error(ctx, LORB_E_INVALID, "problem %d: global query index out of range", p);
  if (np == 0) return LORB_OK;
  const int nq = q_off[np], nt = t_off[np];
  uint32_t *k1 = nullptr, *k2 = nullptr, *kt = nullptr;
  unsigned long long* qkey = nullptr;
  int32_t* d_off = nullptr;
  double *kd = nullptr, *ex = nullptr;
  std::vector<int32_t> offs(q_off, q_off + np + 1);
  offs.insert(offs.end(), t_off, t_off + np + 1);
  offs.insert(offs.end(), q_base, q_base + np);
  LORB_TRY(lorb::upload_t(ctx, S_BF_OFF, offs.data(), offs.size(), &d_off));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_QKEY, (size_t)std::max(nq, 1), &qkey));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT2, (size_t)std::max(nt, 1), &kd));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT3, (size_t)std::max(nt, 1), &kt));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT1, (size_t)2 * np, &ex));
  if (nq > 0) LORB_HIP(ctx, hipMemsetAsync(qkey, 0xff, sizeof(unsigned long long) * nq, ctx->stream));
  if (nt > 0) {
    if (nq > 0) {
      LORB_TRY(scan<false>(ctx, np, d_t, t_off, d_q, q_off, &k1, &k2, q_base));
      hipLaunchKernelGGL(k_u32_f64, dim3(lorb::ceil_div(nt, 256)), dim3(256), 0, ctx->stream, k1, kd, nt, 0,
                         (uint32_t*)nullptr, (const int32_t*)d_off, (const int32_t*)(d_off + np + 1), np);
    } else {
      std::vector<double> sent(nt, (double)kSentinel);
      LORB_HIP(ctx, hipMemcpyAsync(kd, sent.data(), sizeof(double) * nt, hipMemcpyHostToDevice, ctx->stream));
      LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    LORB_TRY(lorb::comm_allreduce(comm, kd, kd, (size_t)nt, LORB_OP_MIN));
    hipLaunchKernelGGL(k_u32_f64, dim3(lorb::ceil_div(nt, 256)), dim3(256), 0, ctx->stream, (const uint32_t*)nullptr, kd, nt, 1,
                       kt, (const int32_t*)d_off, (const int32_t*)(d_off + np + 1), np);
    hipLaunchKernelGGL(k_cc_scatter, dim3(lorb::ceil_div(nt, 256)), dim3(256), 0, ctx->stream, kt, nt, d_off,
                       d_off + np + 1, np, (const int32_t*)(d_off + 2 * np + 2), qkey);
    LORB_CHECK_LAUNCH(ctx);
  }
  hipLaunchKernelGGL(k_cc_finalize<1>, dim3(np), dim3(256), 0, ctx->stream, qkey, d_off, d_off + np + 1, d_cc_train,
                     d_cc_dist, d_match_train, d_n_matches, ex, np);
  LORB_TRY(lorb::comm_allreduce(comm, ex, ex, (size_t)np, LORB_OP_MIN));
  hipLaunchKernelGGL(k_cc_finalize<2>, dim3(np), dim3(256), 0, ctx->stream, qkey, d_off, d_off + np + 1, d_cc_train,
                     d_cc_dist, d_match_train, d_n_matches, ex, np);
  LORB_TRY(lorb::comm_allreduce(comm, ex + np, ex + np, (size_t)np, LORB_OP_SUM));
  hipLaunchKernelGGL(k_counts_out, dim3(lorb::ceil_div(np, 256)), dim3(256), 0, ctx->stream, ex, np, d_n_matches);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int lorb_compute_descriptor_dev(lorb_ctx* ctx, int32_t n_points, const int32_t* d_off,
                                const uint8_t* d_desc, int32_t* d_best, uint8_t* d_out_desc) {
  if (!ctx || n_points < 0 || (n_points > 0 && (!d_off || !d_best))) return LORB_E_INVALID;
  if (n_points == 0) return LORB_OK;
  hipLaunchKernelGGL(k_compute_descriptor, dim3(lorb::ceil_div(n_points, 4)), dim3(256), 0, ctx->stream,
                     reinterpret_cast<const uint4*>(d_desc), d_off, n_points, d_best,
                     reinterpret_cast<uint4*>(d_out_desc));
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int lorb_compute_descriptor(lorb_ctx* ctx, int32_t n_points, const int32_t* d_off_h,
                            const uint8_t* desc, int32_t* best, uint8_t* out_desc) {
  if (!ctx || n_points < 0 || (n_points > 0 && (!d_off_h || !best))) return LORB_E_INVALID;
  if (n_points == 0) return LORB_OK;
  const int nd = d_off_h[n_points];
  for (int p = 0; p < n_points; ++p)
    if (d_off_h[p + 1] < d_off_h[p]) return lorb::set_error(ctx, LORB_E_INVALID, "offsets not monotone at point %d", p);
  if (d_off_h[0] != 0) return lorb::set_error(ctx, LORB_E_INVALID, "offsets must start at 0");
  int32_t *doff = nullptr, *dbest = nullptr;
  uint8_t *dd = nullptr, *dout = nullptr;
  LORB_TRY(lorb::upload_t(ctx, S_BF_OFF, d_off_h, (size_t)n_points + 1, &doff));
  if (nd > 0) LORB_TRY(lorb::upload_t(ctx, S_BF_Q, desc, (size_t)nd * 32, &dd));
  LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT0, (size_t)n_points, &dbest));
  if (out_desc) LORB_TRY(lorb::scratch_t(ctx, S_BF_OUT1, (size_t)n_points * 32, &dout));
  LORB_TRY(lorb_compute_descriptor_dev(ctx, n_points, doff, dd, dbest, dout));
  LORB_HIP(ctx, hipMemcpyAsync(best, dbest, sizeof(int32_t) * n_points, hipMemcpyDeviceToHost, ctx->stream));
  if (out_desc) LORB_HIP(ctx, hipMemcpyAsync(out_desc, dout, (size_t)n_points * 32, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (out_desc)  // points without candidates keep whatever the caller had: mark them unchanged
    for (int p = 0; p < n_points; ++p)
      if (best[p] < 0) memset(out_desc + 32 * (size_t)p, 0, 32);
  return LORB_OK;
}

int lorb_bf_match(lorb_ctx* ctx, int32_t np, const uint8_t* q, const int32_t* q_off,
                  const uint8_t* t, const int32_t* t_off, int32_t* cc_train, int32_t* cc_dist,
                  int32_t* match_train, int32_t* n_matches) {
  LORB_TRY(check_offsets(ctx, np, q_off, t_off));
  if (np == 0) return LORB_OK;
  const int nq = q_off[np], nt = t_off[np];
  // both descriptor sets in one pull, the four outputs stored straight into pinned memory
  lorb::InPack in(ctx);
  const int iq = in.add(q, (size_t)nq * 32), it = in.add(t, (size_t)nt * 32);
  LORB_TRY(in.commit());
  lorb::OutPack out(ctx);
  const int io = out.add(sizeof(int32_t) * ((size_t)nq * 3 + np));
  LORB_TRY(out.alloc(true));  // the finalize kernels write the four outputs with plain stores
  int32_t* o = out.dev<int32_t>(io);
  LORB_TRY(lorb_bf_match_dev(ctx, np, in.dev<uint8_t>(iq), q_off, in.dev<uint8_t>(it), t_off, o, o + nq, o + 2 * nq,
                             o + 3 * nq));
  LORB_TRY(out.fetch());
  const int32_t* h = out.host<int32_t>(io);
  if (nq > 0) {
    memcpy(cc_train, h, sizeof(int32_t) * nq);
    memcpy(cc_dist, h + nq, sizeof(int32_t) * nq);
    memcpy(match_train, h + 2 * nq, sizeof(int32_t) * nq);
  }
  memcpy(n_matches, h + 3 * nq, sizeof(int32_t) * np);
  return LORB_OK;
}

}  // extern "C"
