// lorb_window.hip -- windowed (projection) ORB matching on gfx950 + its frame-side callees.
//
// (a4) Matcher::SearchByProjection(Frame*, Frame*, th)          src/matcher.cpp:64-218
// (a5) Matcher::SearchByProjection(Frame*, set<MapPoint*>, th)  src/matcher.cpp:220-316
// (a7) Frame::AssignFeaturesToGrid / GetFeaturesInArea          src/frame.cpp:87-115, 370-423
// (a8) Frame::IsInFrustum + MapPoint::PredictScale              src/frame.cpp:425-494, map_point.cpp:267-284
// (a20) Frame::UnprojectStereo                                  src/frame.cpp:335-356
//
// The reference resolves map points sequentially: a keypoint slot already holding a map point
// with mnObs>0 is skipped by every LATER point (src/matcher.cpp:149-151, 273-275).  That order
// dependence is reproduced exactly and in parallel by a Jacobi fixpoint:
//   round r: every point picks best/second over its candidate list, skipping slots that were
//            locked before the call or claimed (accepted + mnObs>0) by an EARLIER point in
//            round r-1's results;  claims = min point index per slot.
// Point 0 is exact in round 1, point j depends only on points < j, so after round k points
// 0..k-1 are final; a round with no change is the unique sequential answer.  Rounds are bounded
// by n+1 and in practice end after a handful.  All float expressions follow the reference's
// operation order (built with -ffp-contract=off) so candidate sets are bit-identical.
#include "lorb_internal.h"

#include <cmath>

namespace {

constexpr int kCells = LORB_GRID_COLS * LORB_GRID_ROWS;
constexpr uint32_t kNoClaim = 0x7fffffff;

struct WinParams {  // per-call scalars (device copy of lorb_frame_params)
  lorb_frame_params fp;
  float th;
  int mode_forward, mode_backward;  // a4 only
  float Rcw[9], tcw[3];             // a4 only
};

__device__ __forceinline__ int hamming(const uint4* a, const uint4* b) {
  const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Frame::PosInGrid: the cell of a keypoint, or -1 outside the grid
__device__ __forceinline__ int pos_in_grid(float x, float y, const lorb_frame_params& fp) {
  const int px = (int)roundf((x - fp.min_x) * fp.grid_w_inv);
  const int py = (int)roundf((y - fp.min_y) * fp.grid_h_inv);
  if (px < 0 || px >= LORB_GRID_COLS || py < 0 || py >= LORB_GRID_ROWS) return -1;
  return px * LORB_GRID_ROWS + py;
}

// The grid of n <= kGridLds keypoints built by one NT-thread workgroup in its own LDS (off: kCells + 1,
// cur: kCells, idx: n), lists in keypoint order: the candidate kernels of the host-array calls build
// it per workgroup instead of reading a grid built by a launch of its own.
template <int NT>
__device__ __forceinline__ void grid_lds(const float* __restrict__ x, const float* __restrict__ y, int n,
                                         const lorb_frame_params& fp, int* off, int* cur, int* idx) {
  constexpr int CPT = kCells / NT;  // consecutive cells per thread in the scan
  static_assert(kCells % NT == 0, "cells per thread");
  __shared__ int wsum[NT / 64];
  const int t = threadIdx.x;
  for (int c = t; c < kCells; c += NT) off[c] = 0;
  __syncthreads();
  for (int i = t; i < n; i += NT) {
    const int c = pos_in_grid(x[i], y[i], fp);
    if (c >= 0) atomicAdd(&off[c], 1);
  }
  __syncthreads();
  int v[CPT], sum = 0;
#pragma unroll
  for (int k = 0; k < CPT; ++k) { v[k] = off[CPT * t + k]; sum += v[k]; }
  int tot;
  int run = lorb::block_excl_scan<NT>(sum, wsum, &tot);
#pragma unroll
  for (int k = 0; k < CPT; ++k) { off[CPT * t + k] = run; cur[CPT * t + k] = run; run += v[k]; }
  if (t == NT - 1) off[kCells] = tot;
  __syncthreads();
  for (int i = t; i < n; i += NT) {
    const int c = pos_in_grid(x[i], y[i], fp);
    if (c >= 0) idx[atomicAdd(&cur[c], 1)] = i;
  }
  __syncthreads();
  for (int c = t; c < kCells; c += NT) {  // insertion (keypoint) order inside every cell
    const int a = off[c], b = off[c + 1];
    for (int i = a + 1; i < b; ++i) {
      const int w = idx[i];
      int j = i;
      while (j > a) {
        const int u = idx[j - 1];
        if (u <= w) break;
        idx[j] = u;
        --j;
      }
      idx[j] = w;
    }
  }
  __syncthreads();
}

// (a7) grid: one workgroup; cell = PosInGrid; per-cell lists in keypoint (insertion) order.  The
// offsets and (up to kGridLds keypoints) the lists are built in LDS and stored once, coalesced.
constexpr int kGridLds = 6144;
// scatter keypoints into their cells' lists (atomics: any order), then restore insertion (index)
// order inside every cell (cells hold a handful of entries); indices only, never a pointer below a
// cell's first entry
__device__ __forceinline__ void grid_place(int* idx, const int* off, int* cur, const int* __restrict__ kp_cell,
                                           int n, int t) {
  for (int i = t; i < n; i += 1024) {
    const int c = kp_cell[i];
    if (c >= 0) idx[atomicAdd(&cur[c], 1)] = i;
  }
  __syncthreads();
  for (int c = t; c < kCells; c += 1024) {
    const int a = off[c], b = off[c + 1];
    for (int i = a + 1; i < b; ++i) {
      const int v = idx[i];
      int j = i;
      while (j > a) {
        const int u = idx[j - 1];
        if (u <= v) break;
        idx[j] = u;
        --j;
      }
      idx[j] = v;
    }
  }
}
__global__ __launch_bounds__(1024) void k_grid_build(const float* __restrict__ x, const float* __restrict__ y,
                                                     int n, lorb_frame_params fp,
                                                     int* __restrict__ cell_off,  // kCells+1
                                                     int* __restrict__ cell_idx, int* __restrict__ kp_cell) {
  __shared__ int off[kCells + 1];  // counts, then offsets
  __shared__ int cur[kCells];
  __shared__ int s_idx[kGridLds];
  const bool lds = n <= kGridLds;
  const int t = threadIdx.x;
  for (int c = t; c < kCells; c += 1024) off[c] = 0;
  __syncthreads();
  for (int i = t; i < n; i += 1024) {
    const int c = pos_in_grid(x[i], y[i], fp);
    kp_cell[i] = c;
    if (c >= 0) atomicAdd(&off[c], 1);
  }
  __syncthreads();
  {  // 3072-entry exclusive scan: three consecutive cells per thread
    static_assert(kCells == 3 * 1024, "grid scan assumes 64 x 48 cells");
    __shared__ int wsum[16];
    const int c0 = 3 * t;
    const int a = off[c0], b = off[c0 + 1], c = off[c0 + 2];
    int tot;
    const int ex = lorb::block_excl_scan_1024(a + b + c, wsum, &tot);
    off[c0] = ex; off[c0 + 1] = ex + a; off[c0 + 2] = ex + a + b;
    cur[c0] = ex; cur[c0 + 1] = ex + a; cur[c0 + 2] = ex + a + b;
    if (t == 1023) off[kCells] = tot;
  }
  __syncthreads();
  // separate instantiations for the LDS and the global list: a pointer that may be either is a flat
  // pointer, and the sort's walk below a cell's first entry must not be formed on the LDS aperture
  if (lds) grid_place(s_idx, off, cur, kp_cell, n, t);
  else grid_place(cell_idx, off, cur, kp_cell, n, t);
  for (int c = t; c <= kCells; c += 1024) cell_off[c] = off[c];
  if (lds) {
    __syncthreads();
    const int tot = off[kCells];
    for (int i = t; i < tot; i += 1024) cell_idx[i] = s_idx[i];
  }
}

struct FeatArea {  // Frame::GetFeaturesInArea window
  int x0, x1, y0, y1;
  bool empty;
};
__device__ __forceinline__ FeatArea feat_area(const lorb_frame_params& fp, float x, float y, float r) {
  FeatArea a;
  a.empty = true;
  a.x0 = max(0, (int)floorf((x - fp.min_x - r) * fp.grid_w_inv));
  if (a.x0 >= LORB_GRID_COLS) return a;
  a.x1 = min(LORB_GRID_COLS - 1, (int)ceilf((x - fp.min_x + r) * fp.grid_w_inv));
  if (a.x1 < 0) return a;
  a.y0 = max(0, (int)floorf((y - fp.min_y - r) * fp.grid_h_inv));
  if (a.y0 >= LORB_GRID_ROWS) return a;
  a.y1 = min(LORB_GRID_ROWS - 1, (int)ceilf((y - fp.min_y + r) * fp.grid_h_inv));
  if (a.y1 < 0) return a;
  a.empty = false;
  return a;
}

struct KpDev {
  const float *x, *y, *angle, *uR;
  const int* octave;
  const uint4* desc;
  const uint8_t* slot_state;
  const int *cell_off, *cell_idx;
  int n;
};

// The candidate kernels of the host-array calls (k_cand_*<., true>, n <= kStageKps keypoints) build
// the frame's grid in their own LDS instead of reading one built by a launch of its own.  (Staging
// the keypoints' coordinates, octaves and descriptors into LDS as well measured slower: 11.5 ->
// 12.2 us per a4 launch.)
constexpr int kStageKps = 1024;
struct KpLds {
  int off[kCells + 1], cur[kCells], idx[kStageKps];
};
template <int NT>
__device__ __forceinline__ KpDev stage_grid(const KpDev& G, const lorb_frame_params& fp, KpLds& L) {
  grid_lds<NT>(G.x, G.y, G.n, fp, L.off, L.cur, L.idx);  // ends with a barrier
  KpDev K = G;
  K.cell_off = L.off;
  K.cell_idx = L.idx;
  return K;
}


// Walk GetFeaturesInArea in reference order (ix outer, iy inner, cell insertion order) and apply
// the level / window / stereo filters -- one WAVEFRONT per query.  The window's cells are taken 64
// at a time (lane = cell); a wave scan of their sizes flattens the cell lists into one entry
// sequence in reference order, the entries are taken 64 at a time (lane = entry, owner cell by a
// 6-step binary search over the scanned sizes), and survivors are compacted with a ballot, so
// candidate k of the query is the k-th survivor of the reference's loop.  WRITE=false counts,
// WRITE=true emits (keypoint, distance | octave << 16).  All arguments are wave-uniform; returns the count.
template <bool WRITE>
__device__ __forceinline__ int walk_candidates_wave(const KpDev& K, const lorb_frame_params& fp, float x,
                                                    float y, float r, int minLevel, int maxLevel,
                                                    float stereo_u, float stereo_r, const uint4* qdesc,
                                                    int2* out) {
  const FeatArea a = feat_area(fp, x, y, r);
  if (a.empty) return 0;
  const int lane = threadIdx.x & 63;
  const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  const int ny = a.y1 - a.y0 + 1;
  const int ncell = (a.x1 - a.x0 + 1) * ny;
  const unsigned long long lt = (1ull << lane) - 1ull;
  int n = 0;
  for (int cb = 0; cb < ncell; cb += 64) {
    const int ci = cb + lane;
    int beg = 0, len = 0;
    if (ci < ncell) {
      const int c = (a.x0 + ci / ny) * LORB_GRID_ROWS + (a.y0 + ci % ny);
      beg = K.cell_off[c];
      len = K.cell_off[c + 1] - beg;
    }
    int incl = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    const int ex = incl - len;
    const int total = __shfl(incl, 63, 64);
    for (int eb = 0; eb < total; eb += 64) {
      const int e = eb + lane;
      int src = 0;  // last lane (cell) whose first entry is <= e: the owner (ex is non-decreasing)
#pragma unroll
      for (int st = 32; st >= 1; st >>= 1) {
        const int cand = src + st;
        const int exc = __shfl(ex, cand & 63, 64);
        if (cand < 64 && exc <= e) src = cand;
      }
      const int sbeg = __shfl(beg, src, 64), sex = __shfl(ex, src, 64);
      bool pass = false;
      int j = 0, oc = 0;
      if (e < total) {
        j = K.cell_idx[sbeg + (e - sex)];
        oc = K.octave[j];
        // slots locked before the call (mnObs > 0) are skipped by every point (src/matcher.cpp:
        // 149-151, 273-275): a pure filter, applied here once instead of in every resolver round
        pass = K.slot_state[j] != LORB_SLOT_LOCKED;
        pass = pass && !(bCheckLevels && (oc < minLevel || (maxLevel >= 0 && oc > maxLevel)));
        const float distx = K.x[j] - x;
        const float disty = K.y[j] - y;
        pass = pass && (fabsf(distx) < r && fabsf(disty) < r);
        if (pass && K.uR) {  // stereo consistency (checked after occupancy in the reference;
                             // both are pure filters so the order is immaterial)
          const float uRj = K.uR[j];
          if (uRj > 0) pass = !(fabsf(stereo_u - uRj) > stereo_r);
        }
      }
      const unsigned long long m = __ballot(pass);
      if (WRITE && pass) out[n + __popcll(m & lt)] = make_int2(j, hamming(qdesc, K.desc + 2 * (size_t)j) | (oc << 16));
      n += __popcll(m);
    }
  }
  return n;
}

constexpr int kCandWaves = 4;  // queries (wavefronts) per 256-thread workgroup

// (a5) candidates of each local map point, one wavefront per point
template <bool WRITE, bool GRID = false>
__global__ __launch_bounds__(64 * kCandWaves) void k_cand_local(KpDev K, WinParams P, int np,
                                                    const uint8_t* __restrict__ in_view,
                                                    const uint8_t* __restrict__ is_bad,
                                                    const float* __restrict__ px, const float* __restrict__ py,
                                                    const float* __restrict__ pxr, const int* __restrict__ plev,
                                                    const float* __restrict__ vcos, const uint4* __restrict__ pdesc,
                                                    int* __restrict__ cand_cnt, const int* __restrict__ cand_off,
                                                    int2* __restrict__ cand, int stride = 0) {
  const int m = blockIdx.x * kCandWaves + (threadIdx.x >> 6);
  // the query's scalars requested first (GRID: they arrive while the keypoints are staged)
  const int mq = min(m, np - 1);
  const bool act = in_view[mq] && !(is_bad && is_bad[mq]);
  const int lev = plev[mq];
  const float vc = vcos[mq], qx = px[mq], qy = py[mq], qxr = pxr[mq];
  if constexpr (GRID) {
    __shared__ KpLds L;
    K = stage_grid<64 * kCandWaves>(K, P.fp, L);
  }
  if (m >= np) return;
  int cnt = 0;
  if (act) {
    float r = ((double)vc > 0.998) ? 2.5f : 4.0f;  // RadiusByViewingCos
    if (P.th != 1.0f) r *= P.th;
    const float rs = r * P.fp.scale_factors[lev];
    cnt = walk_candidates_wave<WRITE>(K, P.fp, qx, qy, rs, lev - 1, lev, qxr, rs, pdesc + 2 * (size_t)m,
                                      WRITE ? cand + (stride > 0 ? (size_t)m * stride : (size_t)cand_off[m]) : nullptr);
  }
  if ((!WRITE || stride > 0) && (threadIdx.x & 63) == 0) cand_cnt[m] = cnt;
}

// (a4) projection of last-frame map points + candidates, one wavefront per point
__device__ __forceinline__ float gemv3(const float* R, float a, float b, float c, float t) {
  const double s = (double)R[0] * (double)a + (double)R[1] * (double)b + (double)R[2] * (double)c;
  return (float)(s + (double)t);
}
// WRITE: emit at cand_off[i] (two passes: count, scan, write); STRIDE > 0: one pass, emit at
// i * STRIDE and write the count (STRIDE bounds a query's candidates: the frame's keypoint count)
// the candidates of last-frame point i (one wavefront; returns the count, written at `out` if WRITE)
struct FrameQuery {  // a last-frame point's inputs
  bool act;          // has a map point and is not an outlier
  float X, Y, Z;
  int o;             // octave
};
__device__ __forceinline__ FrameQuery frame_query(int i, const uint8_t* __restrict__ has_mp,
                                                  const uint8_t* __restrict__ outlier, const float* __restrict__ pos,
                                                  const int* __restrict__ loct) {
  FrameQuery q;
  q.act = has_mp[i] && !(outlier && outlier[i]);
  q.X = pos[3 * i]; q.Y = pos[3 * i + 1]; q.Z = pos[3 * i + 2];
  q.o = loct[i];
  return q;
}
template <bool WRITE>
__device__ __forceinline__ int cand_frame_one(const KpDev& K, const WinParams& P, const FrameQuery& q,
                                              const uint4* qdesc, int2* out) {
  int cnt = 0;
  if (q.act) {
    const float X = q.X, Y = q.Y, Z = q.Z;
    const float xc = gemv3(P.Rcw + 0, X, Y, Z, P.tcw[0]);
    const float yc = gemv3(P.Rcw + 3, X, Y, Z, P.tcw[1]);
    const float zc = gemv3(P.Rcw + 6, X, Y, Z, P.tcw[2]);
    const float invzc = (float)(1.0 / (double)zc);
    if (!(invzc < 0)) {
      const float u = P.fp.fx * xc * invzc + P.fp.cx;
      const float v = P.fp.fy * yc * invzc + P.fp.cy;
      if (!(u < P.fp.min_x || u > P.fp.max_x) && !(v < P.fp.min_y || v > P.fp.max_y)) {
        const int o = q.o;
        const float radius = P.th * P.fp.scale_factors[o];
        int mn, mx;
        if (P.mode_forward) { mn = o; mx = -1; }
        else if (P.mode_backward) { mn = 0; mx = o; }
        else { mn = o - 1; mx = o + 1; }
        const float ur = u - P.fp.bf * invzc;
        cnt = walk_candidates_wave<WRITE>(K, P.fp, u, v, radius, mn, mx, ur, radius, qdesc, out);
      }
    }
  }
  return cnt;
}
template <bool WRITE, bool GRID = false>
__global__ __launch_bounds__(64 * kCandWaves) void k_cand_frame(KpDev K, WinParams P, int nl,
                                                    const uint8_t* __restrict__ has_mp,
                                                    const uint8_t* __restrict__ outlier,
                                                    const float* __restrict__ pos,
                                                    const int* __restrict__ loct,
                                                    const uint4* __restrict__ ldesc,
                                                    int* __restrict__ cand_cnt, const int* __restrict__ cand_off,
                                                    int2* __restrict__ cand, int stride = 0) {
  const int i = blockIdx.x * kCandWaves + (threadIdx.x >> 6);
  // the query's inputs requested first (GRID: they arrive while the keypoints are staged)
  const FrameQuery q = frame_query(min(i, nl - 1), has_mp, outlier, pos, loct);
  if constexpr (GRID) {
    __shared__ KpLds L;
    K = stage_grid<64 * kCandWaves>(K, P.fp, L);
  }
  if (i >= nl) return;
  const int cnt = cand_frame_one<WRITE>(
      K, P, q, ldesc + 2 * (size_t)i,
      WRITE ? cand + (stride > 0 ? (size_t)i * stride : (size_t)cand_off[i]) : nullptr);
  if ((!WRITE || stride > 0) && (threadIdx.x & 63) == 0) cand_cnt[i] = cnt;
}

// exclusive scan of candidate counts (one workgroup, chunked)
__global__ __launch_bounds__(1024) void k_scan(const int* __restrict__ cnt, int n, int* __restrict__ off) {
  __shared__ int wsum[16];
  int carry = 0;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + (int)threadIdx.x;
    const int v = i < n ? cnt[i] : 0;
    int tot;
    const int ex = lorb::block_excl_scan_1024(v, wsum, &tot);
    if (i < n) off[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) off[n] = carry;
}

// one-pass candidate lists of the host-array matchers (a4, a5): up to this many entries (n_queries *
// nk) the candidates go to a fixed stride per query
constexpr size_t kCandStrided = size_t(1) << 20;

// Candidate list of a windowed match: a query has at most nk candidates, so `bound` = n_queries *
// nk entries always suffice.  Up to kCandBound entries that bound is allocated and the call needs
// no host round trip; past it the exact total (d_total, written by k_scan) is read back.
int alloc_candidates(lorb_ctx* ctx, const int* d_total, size_t bound, int2** cand) {
  constexpr size_t kCandBound = size_t(8) << 20;
  size_t cap = bound;
  if (cap > kCandBound) {
    int total = 0;
    LORB_HIP(ctx, hipMemcpyAsync(&total, d_total, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    cap = (size_t)total;
  }
  return lorb::scratch_t(ctx, S_W9, std::max<size_t>(cap, 1), cand);
}

// Jacobi fixpoint resolver (one workgroup per call).  MODE 0 = a5 (best/second + ratio test),
// MODE 1 = a4 (best only + rotation histogram / ComputeThreeMaxima null-out).  out != null: assign
// and the count are also copied there (nk + 1 ints) at the end.
template <int MODE>
__device__ __forceinline__ void resolve_run(int np, int nk, const int* cand_off, const int2* __restrict__ cand,
                                            const uint8_t* __restrict__ pt_locked,
                                            const float* __restrict__ last_angle,
                                            const float* cur_angle,
                                            int* res,      // np: accepted slot or -1
                                            int* claim,    // nk
                                            int* assign,   // nk: the working assignment
                                            int* bins,     // np scratch (MODE 1)
                                            int* nulls,    // nk scratch (MODE 1)
                                            int* __restrict__ assign_g,  // nk: where the assignment goes (or null)
                                            int* __restrict__ nmatches, int stride, int* __restrict__ out) {
  __shared__ int s_changed;
  __shared__ int hist[LORB_HISTO_LENGTH];
  __shared__ int s_ind[3];
  __shared__ int s_acc, s_rej;
  const int t = threadIdx.x;
  // np <= 1024 (one query per thread): the first kRegCand candidates of the thread's query, its lock
  // flag and (MODE 1) its angle are loaded once, all together, into registers; every round then reads
  // them (and their claims, from LDS) without a global round trip.  Later candidates, if any, come
  // from global.
  constexpr int kRegCand = 8;
  const bool regc = np <= 1024;
  int2 rc[kRegCand];
  int rn = 0;
  bool lk_t = false;
  float la_t = 0.0f;
  if (regc && t < np) {
    lk_t = pt_locked[t];
    if (MODE == 1) la_t = last_angle[t];
    if (stride > 0) {
      // strided lists: the first slots are requested together with the count (one round trip)
      const int a = t * stride, kmax = min(kRegCand, stride);
#pragma unroll
      for (int k = 0; k < kRegCand; ++k) rc[k] = cand[a + min(k, kmax - 1)];
      rn = min(cand_off[t], kmax);
    } else {
      const int a = cand_off[t], b = cand_off[t + 1];
      rn = min(b - a, kRegCand);
      if (rn > 0) {
#pragma unroll
        for (int k = 0; k < kRegCand; ++k) rc[k] = cand[a + min(k, rn - 1)];
      }
    }
  }
  for (int c = t; c < nk; c += 1024) claim[c] = kNoClaim;
  for (int m = t; m < np; m += 1024) res[m] = -2;  // "never computed"
  if (t == 0) { s_acc = 0; s_rej = 0; }
  __syncthreads();
  for (int round = 0; round <= np; ++round) {
    if (t == 0) s_changed = 0;
    __syncthreads();
    for (int m = t; m < np; m += 1024) {
      // stride > 0: query m's candidates at [m stride, m stride + count), cand_off holds the counts
      const int a = stride > 0 ? m * stride : cand_off[m], b = stride > 0 ? a + cand_off[m] : cand_off[m + 1];
      int bestDist = 256, bestIdx = -1;
      int bestLevel = -1, bestDist2 = 256, bestLevel2 = -1;
      // candidates in list order (ties keep the first, as the reference's loop)
      auto consider = [&](const int2 cd) {  // (slot, distance | octave << 16); pre-call locked slots removed
        const int j = cd.x;
        if ((int)claim[j] < m) return;  // locked by an earlier point during this call
        const int dist = cd.y & 0xffff;
        if (MODE == 0) {
          const int oc = cd.y >> 16;
          if (dist < bestDist) {
            bestDist2 = bestDist; bestDist = dist;
            bestLevel2 = bestLevel; bestLevel = oc; bestIdx = j;
          } else if (dist < bestDist2) {
            bestLevel2 = oc; bestDist2 = dist;
          }
        } else {
          if (dist < bestDist) { bestDist = dist; bestIdx = j; }
        }
      };
      int e0 = a;
      if (regc) {
#pragma unroll
        for (int k = 0; k < kRegCand; ++k)
          if (k < rn) consider(rc[k]);
        e0 = a + rn;
      }
      for (int e = e0; e < b; ++e) consider(cand[e]);
      int r = -1;
      if (bestDist <= LORB_TH_HIGH) {
        r = bestIdx;
        if (MODE == 0 && bestLevel == bestLevel2 && (double)bestDist > 0.8 * (double)bestDist2) r = -1;
      }
      if (r != res[m]) { res[m] = r; s_changed = 1; }
    }
    __syncthreads();
    if (!s_changed) break;
    for (int c = t; c < nk; c += 1024) claim[c] = kNoClaim;
    __syncthreads();
    for (int m = t; m < np; m += 1024)
      if (res[m] >= 0 && (regc ? lk_t : pt_locked[m] != 0)) atomicMin(&claim[res[m]], m);
    __syncthreads();
  }
  // final slot assignment: last accepted writer per slot
  for (int c = t; c < nk; c += 1024) { assign[c] = LORB_ASSIGN_UNCHANGED; if (MODE == 1) nulls[c] = 0; }
  if (MODE == 1 && t < LORB_HISTO_LENGTH) hist[t] = 0;
  __syncthreads();
  for (int m = t; m < np; m += 1024) {
    const int r = res[m];
    if (r >= 0) {
      atomicMax(&assign[r], m);
      atomicAdd(&s_acc, 1);
      if (MODE == 1) {
        float rot = (regc ? la_t : last_angle[m]) - cur_angle[r];
        if (rot < 0.0) rot += 360.0f;
        const float factor = LORB_HISTO_LENGTH / 360.0f;
        int bin = (int)roundf(rot * factor);
        if (bin == LORB_HISTO_LENGTH) bin = 0;
        bins[m] = bin;
        atomicAdd(&hist[bin], 1);
      }
    }
  }
  __syncthreads();
  if (MODE == 1) {
    if (t < 64) {  // Matcher::ComputeThreeMaxima, src/matcher.cpp:387-428, on one wavefront
      // The reference's insertion loop (strict >, bins in order, counts starting at 0) keeps the
      // three largest non-zero counts, ties to the lower bin.  Lane = bin; three wave argmax rounds
      // over the key count * 64 + (63 - bin) (largest count, then lowest bin) give the same bins.
      static_assert(LORB_HISTO_LENGTH <= 64, "one bin per lane");
      const int cnt = t < LORB_HISTO_LENGTH ? hist[t] : 0;
      int key = cnt > 0 ? cnt * 64 + (63 - t) : -1;
      int ind[3], mx[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        int k = key;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) k = max(k, __shfl_xor(k, o, 64));
        ind[r] = k >= 0 ? 63 - (k & 63) : -1;
        mx[r] = k >= 0 ? k >> 6 : 0;
        if (k >= 0 && t == ind[r]) key = -1;  // taken
      }
      if ((float)mx[1] < 0.1f * (float)mx[0]) { ind[1] = -1; ind[2] = -1; }
      else if ((float)mx[2] < 0.1f * (float)mx[0]) { ind[2] = -1; }
      if (t == 0) { s_ind[0] = ind[0]; s_ind[1] = ind[1]; s_ind[2] = ind[2]; }
    }
    __syncthreads();
    for (int m = t; m < np; m += 1024) {
      const int r = res[m];
      if (r >= 0) {
        const int b = bins[m];
        if (b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) { nulls[r] = 1; atomicAdd(&s_rej, 1); }
      }
    }
    __syncthreads();
    for (int c = t; c < nk; c += 1024)
      if (nulls[c]) assign[c] = LORB_ASSIGN_NULL;
  }
  __syncthreads();
  if (t == 0) *nmatches = s_acc - s_rej;
  for (int c = t; c < nk; c += 1024) {
    const int v = assign[c];
    if (assign_g && assign_g != assign) assign_g[c] = v;
    if (out) out[c] = v;  // the host-array calls: the mapped result block, plain stores
  }
  if (out && t == 0) out[nk] = s_acc - s_rej;
}
// LDS modes of k_resolve: 1 = claim and res (nk + np ints); 2 = also the working assignment, the
// MODE-1 bins / nulls and a copy of the current frame's keypoint angles (4 nk + 2 np words).
inline int resolve_lds_mode(int np, int nk, size_t* bytes) {
  const size_t b2 = sizeof(int) * (4 * (size_t)nk + 2 * (size_t)np), b1 = sizeof(int) * ((size_t)np + (size_t)nk);
  if (b2 <= 120 * 1024) { *bytes = b2; return 2; }
  if (b1 <= 120 * 1024) { *bytes = b1; return 1; }
  *bytes = 0;
  return 0;
}
template <int MODE>
__global__ __launch_bounds__(1024) void k_resolve(int np, int nk, const int* __restrict__ cand_off,
                                                  const int2* __restrict__ cand,
                                                  const uint8_t* __restrict__ pt_locked,
                                                  const float* __restrict__ last_angle,
                                                  const float* __restrict__ cur_angle,
                                                  int* __restrict__ res, int* __restrict__ claim,
                                                  int* __restrict__ assign, int* __restrict__ bins,
                                                  int* __restrict__ nulls, int* __restrict__ nmatches, int lds_mode,
                                                  int stride = 0, int* __restrict__ out = nullptr) {
  // the working set in LDS (dynamic shared memory) as far as it fits (resolve_lds_mode), else global
  extern __shared__ int s_dyn[];
  int* wassign = assign;
  const float* ca = cur_angle;
  if (lds_mode >= 1) { claim = s_dyn; res = s_dyn + nk; }
  if (lds_mode == 2) {
    wassign = res + np;
    nulls = wassign + nk;
    bins = nulls + nk;
    float* s_ca = reinterpret_cast<float*>(bins + np);
    if (MODE == 1)
      for (int c = threadIdx.x; c < nk; c += 1024) s_ca[c] = cur_angle[c];
    ca = s_ca;  // resolve_run's first barrier orders these stores before any read
  }
  resolve_run<MODE>(np, nk, cand_off, cand, pt_locked, last_angle, ca, res, claim, wassign, bins, nulls, assign,
                    nmatches, stride, out);
}

// (a8) Frame::IsInFrustum + PredictScale, one thread per map point
__global__ __launch_bounds__(256) void k_frustum(lorb_frame_params fp, const float* __restrict__ T,
                                                 const float* __restrict__ Ow, int n,
                                                 const float* __restrict__ pos, const float* __restrict__ nrm,
                                                 const float* __restrict__ maxd, const float* __restrict__ mind,
                                                 float cos_limit, uint8_t* __restrict__ in_view,
                                                 float* __restrict__ ox, float* __restrict__ oy,
                                                 float* __restrict__ oxr, int* __restrict__ olev,
                                                 float* __restrict__ ocos,
                                                 const uint8_t* __restrict__ skip_a,
                                                 const uint8_t* __restrict__ skip_b) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  in_view[m] = 0;
  // EstimatePoseLocal skips points already matched in the frame and bad points before calling
  // IsInFrustum (src/visual_odometry.cpp:181-184); they leave tracking with mbTrackInView false
  if ((skip_a && skip_a[m]) || (skip_b && skip_b[m])) return;
  const float P0 = pos[3 * m], P1 = pos[3 * m + 1], P2 = pos[3 * m + 2];
  float Pc[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const double s = (double)T[4 * r] * P0 + (double)T[4 * r + 1] * P1 + (double)T[4 * r + 2] * P2 + (double)T[4 * r + 3] * 1.0f;
    Pc[r] = (float)s;
  }
  if (Pc[2] < 0.0f) return;
  const float invz = 1.0f / Pc[2];
  const float u = fp.fx * Pc[0] * invz + fp.cx;
  const float v = fp.fy * Pc[1] * invz + fp.cy;
  if (u < fp.min_x || u > fp.max_x) return;
  if (v < fp.min_y || v > fp.max_y) return;
  const float maxDistance = 1.2f * maxd[m];
  const float minDistance = 0.8f * mind[m];
  const float PO0 = P0 - Ow[0], PO1 = P1 - Ow[1], PO2 = P2 - Ow[2];
  const float dist = (float)sqrt((double)PO0 * PO0 + (double)PO1 * PO1 + (double)PO2 * PO2);
  if (dist < minDistance || dist > maxDistance) return;
  const float dot = PO0 * nrm[3 * m] + PO1 * nrm[3 * m + 1] + PO2 * nrm[3 * m + 2];
  const float viewCos = dot / dist;
  if (viewCos < cos_limit) return;
  const float ratio = maxd[m] / dist;
  int nScale = (int)ceilf((float)log((double)ratio) / fp.log_scale_factor);
  if (nScale < 0) nScale = 0;
  else if (nScale >= fp.n_levels) nScale = fp.n_levels - 1;
  in_view[m] = 1;
  ox[m] = u;
  oxr[m] = u - fp.bf * invz;
  oy[m] = v;
  olev[m] = nScale;
  ocos[m] = viewCos;
}

// (a20) Frame::UnprojectStereo, one thread per keypoint; Twc = mTcw.inv() given
__global__ __launch_bounds__(256) void k_unproject(lorb_frame_params fp, lorb::Mat4f Twc, int n,
                                                   const float* __restrict__ x, const float* __restrict__ y,
                                                   const float* __restrict__ depth, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float z = depth[i];
  if (z > 0) {
    lorb::unproject_point(fp.fx, fp.fy, fp.cx, fp.cy, Twc, x[i], y[i], z, out + 3 * i);
  } else {
    out[3 * i] = 0.0f; out[3 * i + 1] = 0.0f; out[3 * i + 2] = 0.0f;
  }
}

}  // namespace

// cv::Mat::inv() for 4x4 CV_32F: hal::LU32f (partial pivoting, float), host side
bool lorb::inv4_lu32f(const float* Ain, float* out) {
  float A[16], b[16];
  memcpy(A, Ain, sizeof(A));
  for (int i = 0; i < 16; i++) b[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  const float eps = 1.1920928955078125e-07f * 10;
  for (int i = 0; i < 4; i++) {
    int k = i;
    for (int j = i + 1; j < 4; j++)
      if (std::fabs(A[j * 4 + i]) > std::fabs(A[k * 4 + i])) k = j;
    if (std::fabs(A[k * 4 + i]) < eps) { memset(out, 0, 16 * sizeof(float)); return false; }
    if (k != i) {
      for (int j = i; j < 4; j++) std::swap(A[i * 4 + j], A[k * 4 + j]);
      for (int j = 0; j < 4; j++) std::swap(b[i * 4 + j], b[k * 4 + j]);
    }
    const float dd = -1 / A[i * 4 + i];
    for (int j = i + 1; j < 4; j++) {
      const float alpha = A[j * 4 + i] * dd;
      for (int kk = i + 1; kk < 4; kk++) A[j * 4 + kk] += alpha * A[i * 4 + kk];
      for (int kk = 0; kk < 4; kk++) b[j * 4 + kk] += alpha * b[i * 4 + kk];
    }
  }
  for (int i = 3; i >= 0; i--)
    for (int j = 0; j < 4; j++) {
      float s = b[i * 4 + j];
      for (int k = i + 1; k < 4; k++) s -= A[i * 4 + k] * b[k * 4 + j];
      b[i * 4 + j] = s / A[i * 4 + i];
    }
  memcpy(out, b, sizeof(b));
  return true;
}

namespace {
using lorb::inv4_lu32f;

// a frame's keypoints (Frame::mvKeysUn, mDescriptors, slot states) for the host-array entry points:
// packed into their InPack (one pull for every input), then the device grid built
struct KpParts {
  int x, y, ang, oc, desc, ur, ss;
  std::vector<uint8_t> zeros;
};
void kps_add(lorb::InPack& in, const lorb_keypoints* k, const uint8_t* slot_state, KpParts& p) {
  const size_t n = (size_t)k->n;
  p.x = in.add_t(k->x, n); p.y = in.add_t(k->y, n); p.ang = in.add_t(k->angle, n);
  p.oc = in.add_t(k->octave, n); p.desc = in.add_t(k->desc, n * 32); p.ur = in.add_t(k->u_right, n);
  if (!slot_state) { p.zeros.assign(n, 0); slot_state = p.zeros.data(); }
  p.ss = in.add_t(slot_state, n);
}
// grid = false: the candidate kernel builds the grid in its own LDS (k_cand_*<., true>)
int kps_finish(lorb_ctx* ctx, const lorb::InPack& in, const KpParts& p, int n, int slot0, KpDev* K,
               const lorb_frame_params* fp, bool grid = true) {
  const float* x = in.dev<float>(p.x);
  const float* y = in.dev<float>(p.y);
  K->x = x; K->y = y; K->angle = in.dev<float>(p.ang); K->uR = in.dev<float>(p.ur); K->octave = in.dev<int>(p.oc);
  K->desc = in.dev<const uint4>(p.desc); K->slot_state = in.dev<uint8_t>(p.ss);
  K->cell_off = nullptr; K->cell_idx = nullptr; K->n = n;
  if (!grid) return LORB_OK;
  int *cell_off, *cell_idx, *kp_cell;
  LORB_TRY(lorb::scratch_t(ctx, slot0 + 7, kCells + 1, &cell_off));
  LORB_TRY(lorb::scratch_t(ctx, slot0 + 8, (size_t)std::max(n, 1), &cell_idx));
  LORB_TRY(lorb::scratch_t(ctx, slot0 + 9, (size_t)std::max(n, 1), &kp_cell));
  hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), 0, ctx->stream, x, y, n, *fp, cell_off, cell_idx, kp_cell);
  LORB_CHECK_LAUNCH(ctx);
  K->cell_off = cell_off; K->cell_idx = cell_idx;
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_search_by_projection_local(lorb_ctx* ctx, const lorb_frame_params* frame, const lorb_keypoints* kps,
                                    const uint8_t* slot_state, const lorb_local_points* pts, float th,
                                    int32_t* assign, int32_t* nmatches) {
  if (!ctx || !frame || !kps || !pts || !assign || !nmatches) return LORB_E_INVALID;
  const int nk = kps->n, np = pts->n;
  if (nk < 0 || np < 0) return lorb::set_error(ctx, LORB_E_INVALID, "negative sizes");
  if (nk == 0) { *nmatches = 0; return LORB_OK; }
  for (int i = 0; i < np; ++i)
    if (pts->track_in_view[i] && !(pts->is_bad && pts->is_bad[i]) &&
        (pts->pred_level[i] < 0 || pts->pred_level[i] >= LORB_MAX_LEVELS))
      return lorb::set_error(ctx, LORB_E_INVALID, "point %d: predicted level %d out of range", i, pts->pred_level[i]);
  // every input in one pull, the result stored straight into pinned memory by k_resolve
  lorb::InPack in(ctx);
  KpParts kp;
  kps_add(in, kps, slot_state, kp);
  const int i_iv = in.add_t(pts->track_in_view, np), i_bad = in.add_t(pts->is_bad, np), i_lk = in.add_t(pts->locked, np),
            i_px = in.add_t(pts->proj_x, np), i_py = in.add_t(pts->proj_y, np), i_pxr = in.add_t(pts->proj_xr, np),
            i_pl = in.add_t(pts->pred_level, np), i_vc = in.add_t(pts->view_cos, np),
            i_pd = in.add_t(pts->desc, (size_t)np * 32);
  LORB_TRY(in.commit());
  const bool strided = (size_t)np * (size_t)nk <= kCandStrided;  // as lorb_search_by_projection_frame
  const bool lds_grid = strided && nk <= kStageKps;  // the candidate kernel builds the grid itself
  KpDev K;
  LORB_TRY(kps_finish(ctx, in, kp, nk, S_KP, &K, frame, !lds_grid));
  const uint8_t *iv = in.dev<uint8_t>(i_iv), *bad = in.dev<uint8_t>(i_bad), *lk = in.dev<uint8_t>(i_lk);
  const float *px = in.dev<float>(i_px), *py = in.dev<float>(i_py), *pxr = in.dev<float>(i_pxr), *vc = in.dev<float>(i_vc);
  const int* pl = in.dev<int>(i_pl);
  const uint8_t* pd = in.dev<uint8_t>(i_pd);
  WinParams P{};
  P.fp = *frame;
  P.th = th;
  int *cnt, *off, *res, *claim, *dassign, *dnm;
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 0, (size_t)np + 1, &cnt));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 1, (size_t)np + 1, &off));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 2, (size_t)np + 1, &res));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 3, (size_t)nk + 1, &claim));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 4, (size_t)nk + 1, &dassign));
  dnm = dassign + nk;
  lorb::OutPack out(ctx);
  const int o_as = out.add(sizeof(int) * ((size_t)nk + 1));
  LORB_TRY(out.alloc(true));  // k_resolve writes assign + count into the mapped block
  const unsigned g = lorb::ceil_div(std::max(np, 1), kCandWaves);
  int2* cand;
  if (strided) {
    LORB_TRY(lorb::scratch_t(ctx, S_W9, std::max<size_t>((size_t)np * nk, 1), &cand));
    if (np > 0) {
      lorb::KernelTimer kt(ctx, LORB_K_WINDOW_CAND);
      if (lds_grid)
        hipLaunchKernelGGL((k_cand_local<true, true>), dim3(g), dim3(256), 0, ctx->stream, K, P, np, iv, bad, px, py, pxr,
                           pl, vc, reinterpret_cast<const uint4*>(pd), cnt, (const int*)nullptr, cand, nk);
      else
        hipLaunchKernelGGL(k_cand_local<true>, dim3(g), dim3(256), 0, ctx->stream, K, P, np, iv, bad, px, py, pxr, pl,
                           vc, reinterpret_cast<const uint4*>(pd), cnt, (const int*)nullptr, cand, nk);
    }
  } else {
    if (np > 0) {
      lorb::KernelTimer kt(ctx, LORB_K_WINDOW_CAND);
      hipLaunchKernelGGL(k_cand_local<false>, dim3(g), dim3(256), 0, ctx->stream, K, P, np, iv, bad, px, py, pxr, pl, vc,
                         reinterpret_cast<const uint4*>(pd), cnt, (const int*)nullptr, (int2*)nullptr, 0);
    }
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, cnt, np, off);
    LORB_TRY(alloc_candidates(ctx, off + np, (size_t)np * (size_t)nk, &cand));
    if (np > 0)
      hipLaunchKernelGGL(k_cand_local<true>, dim3(g), dim3(256), 0, ctx->stream, K, P, np, iv, bad, px, py, pxr, pl, vc,
                         reinterpret_cast<const uint4*>(pd), cnt, off, cand, 0);
  }
  size_t rlds = 0;
  const int rmode = resolve_lds_mode(np, nk, &rlds);
  hipLaunchKernelGGL(k_resolve<0>, dim3(1), dim3(1024), rlds, ctx->stream, np, nk,
                     strided ? (const int*)cnt : (const int*)off, cand, lk,
                     (const float*)nullptr, (const float*)nullptr, res, claim, dassign, (int*)nullptr, (int*)nullptr, dnm,
                     rmode, strided ? nk : 0, out.dev<int>(o_as));
  LORB_CHECK_LAUNCH(ctx);
  LORB_TRY(out.fetch());
  memcpy(assign, out.host<int>(o_as), sizeof(int) * nk);
  *nmatches = out.host<int>(o_as)[nk];
  return LORB_OK;
}

int lorb_search_by_projection_frame(lorb_ctx* ctx, const lorb_frame_params* cur, const float cur_Tcw[16],
                                    const lorb_keypoints* cur_kps, const uint8_t* cur_slot_state,
                                    const lorb_last_frame* last, float th, int32_t* assign, int32_t* nmatches) {
  if (!ctx || !cur || !cur_Tcw || !cur_kps || !last || !assign || !nmatches) return LORB_E_INVALID;
  const int nk = cur_kps->n, nl = last->n;
  if (nk < 0 || nl < 0) return lorb::set_error(ctx, LORB_E_INVALID, "negative sizes");
  if (nk == 0) { *nmatches = 0; return LORB_OK; }
  for (int i = 0; i < nl; ++i)
    if (last->has_mp[i] && (last->octave[i] < 0 || last->octave[i] >= LORB_MAX_LEVELS))
      return lorb::set_error(ctx, LORB_E_INVALID, "last keypoint %d: octave %d out of range", i, last->octave[i]);
  // src/matcher.cpp:74-87: motion direction from the two poses (cv::gemm: double accumulation)
  WinParams P{};
  P.fp = *cur;
  P.th = th;
  const float* T = cur_Tcw;
  const float Rcw[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
  const float tcw[3] = {T[3], T[7], T[11]};
  memcpy(P.Rcw, Rcw, sizeof(Rcw));
  memcpy(P.tcw, tcw, sizeof(tcw));
  float twc[3];
  for (int i = 0; i < 3; i++) {
    const double s = (double)Rcw[i] * tcw[0] + (double)Rcw[3 + i] * tcw[1] + (double)Rcw[6 + i] * tcw[2];
    twc[i] = (float)(-s);
  }
  const float* L = last->Tcw;
  const double s2 = (double)L[8] * twc[0] + (double)L[9] * twc[1] + (double)L[10] * twc[2];
  const float tlc2 = (float)(s2 + (double)L[11]);
  P.mode_forward = tlc2 > cur->b;
  P.mode_backward = -tlc2 > cur->b;
  // every input in one pull, the result stored straight into pinned memory by k_resolve
  lorb::InPack in(ctx);
  KpParts kp;
  kps_add(in, cur_kps, cur_slot_state, kp);
  const int i_hm = in.add_t(last->has_mp, nl), i_ol = in.add_t(last->outlier, nl), i_lk = in.add_t(last->mp_locked, nl),
            i_pos = in.add_t(last->mp_pos, (size_t)nl * 3), i_ld = in.add_t(last->mp_desc, (size_t)nl * 32),
            i_lo = in.add_t(last->octave, nl), i_la = in.add_t(last->angle, nl);
  LORB_TRY(in.commit());
  // a query has at most nk candidates: up to kCandStrided entries one pass writes them at i * nk
  // (no count pass, no scan); past it the count / scan / write passes size the list exactly
  const bool strided = (size_t)nl * (size_t)nk <= kCandStrided;
  const bool lds_grid = strided && nk <= kStageKps;  // the candidate kernel builds the grid itself
  KpDev K;
  LORB_TRY(kps_finish(ctx, in, kp, nk, S_KP, &K, cur, !lds_grid));
  const uint8_t *hm = in.dev<uint8_t>(i_hm), *ol = in.dev<uint8_t>(i_ol), *lk = in.dev<uint8_t>(i_lk),
                *ld = in.dev<uint8_t>(i_ld);
  const float *pos = in.dev<float>(i_pos), *la = in.dev<float>(i_la);
  const int* lo = in.dev<int>(i_lo);
  int *cnt, *off, *res, *claim, *dassign, *dnm, *bins, *nulls;
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 0, (size_t)nl + 1, &cnt));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 1, (size_t)nl + 1, &off));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 2, (size_t)nl + 1, &res));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 3, (size_t)nk + 1, &claim));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 5, (size_t)nl + 1, &bins));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 6, (size_t)nk + 1, &nulls));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 4, (size_t)nk + 1, &dassign));
  dnm = dassign + nk;
  lorb::OutPack out(ctx);
  const int o_as = out.add(sizeof(int) * ((size_t)nk + 1));
  LORB_TRY(out.alloc(true));  // k_resolve writes assign + count into the mapped block
  const unsigned g = lorb::ceil_div(std::max(nl, 1), kCandWaves);
  int2* cand;
  if (strided) {
    LORB_TRY(lorb::scratch_t(ctx, S_W9, std::max<size_t>((size_t)nl * nk, 1), &cand));
    if (nl > 0) {
      lorb::KernelTimer kt(ctx, LORB_K_WINDOW_CAND);
      if (lds_grid)
        hipLaunchKernelGGL((k_cand_frame<true, true>), dim3(g), dim3(256), 0, ctx->stream, K, P, nl, hm, ol, pos, lo,
                           reinterpret_cast<const uint4*>(ld), cnt, (const int*)nullptr, cand, nk);
      else
        hipLaunchKernelGGL(k_cand_frame<true>, dim3(g), dim3(256), 0, ctx->stream, K, P, nl, hm, ol, pos, lo,
                           reinterpret_cast<const uint4*>(ld), cnt, (const int*)nullptr, cand, nk);
    }
  } else {
    if (nl > 0) {
      lorb::KernelTimer kt(ctx, LORB_K_WINDOW_CAND);
      hipLaunchKernelGGL(k_cand_frame<false>, dim3(g), dim3(256), 0, ctx->stream, K, P, nl, hm, ol, pos, lo,
                         reinterpret_cast<const uint4*>(ld), cnt, (const int*)nullptr, (int2*)nullptr, 0);
    }
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, cnt, nl, off);
    LORB_TRY(alloc_candidates(ctx, off + nl, (size_t)nl * (size_t)nk, &cand));
    if (nl > 0)
      hipLaunchKernelGGL(k_cand_frame<true>, dim3(g), dim3(256), 0, ctx->stream, K, P, nl, hm, ol, pos, lo,
                         reinterpret_cast<const uint4*>(ld), cnt, off, cand, 0);
  }
  size_t rlds = 0;
  const int rmode = resolve_lds_mode(nl, nk, &rlds);
  hipLaunchKernelGGL(k_resolve<1>, dim3(1), dim3(1024), rlds, ctx->stream, nl, nk,
                     strided ? (const int*)cnt : (const int*)off, cand, lk,
                     la, K.angle, res, claim, dassign, bins, nulls, dnm,
                     rmode, strided ? nk : 0, out.dev<int>(o_as));
  LORB_CHECK_LAUNCH(ctx);
  LORB_TRY(out.fetch());
  memcpy(assign, out.host<int>(o_as), sizeof(int) * nk);
  *nmatches = out.host<int>(o_as)[nk];
  return LORB_OK;
}

int lorb_is_in_frustum(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                       const lorb_frustum_points* pts, float viewing_cos_limit, uint8_t* in_view,
                       float* proj_x, float* proj_y, float* proj_xr, int32_t* pred_level, float* view_cos) {
  if (!ctx || !frame || !Tcw || !pts) return LORB_E_INVALID;
  const int n = pts->n;
  if (n <= 0) return LORB_OK;
  float Twc[16];
  inv4_lu32f(Tcw, Twc);
  const float Ow[3] = {Twc[3], Twc[7], Twc[11]};
  float *dT, *dO, *pos, *nrm, *mx, *mn, *outf;
  uint8_t* iv;
  int* lev;
  LORB_TRY(lorb::upload_t(ctx, S_W0, Tcw, 16, &dT));
  LORB_TRY(lorb::upload_t(ctx, S_W1, Ow, 3, &dO));
  LORB_TRY(lorb::upload_t(ctx, S_W2, pts->pos, (size_t)n * 3, &pos));
  LORB_TRY(lorb::upload_t(ctx, S_W3, pts->normal, (size_t)n * 3, &nrm));
  LORB_TRY(lorb::upload_t(ctx, S_W4, pts->max_dist, n, &mx));
  LORB_TRY(lorb::upload_t(ctx, S_W5, pts->min_dist, n, &mn));
  LORB_TRY(lorb::scratch_t(ctx, S_W6, (size_t)n * 4, &outf));
  LORB_TRY(lorb::scratch_t(ctx, S_W7, (size_t)n, &iv));
  LORB_TRY(lorb::scratch_t(ctx, S_W8, (size_t)n, &lev));
  hipLaunchKernelGGL(k_frustum, dim3(lorb::ceil_div(n, 256)), dim3(256), 0, ctx->stream, *frame, dT, dO, n, pos, nrm, mx,
                     mn, viewing_cos_limit, iv, outf, outf + n, outf + 2 * n, lev, outf + 3 * n,
                     (const uint8_t*)nullptr, (const uint8_t*)nullptr);
  LORB_CHECK_LAUNCH(ctx);
  LORB_HIP(ctx, hipMemcpyAsync(in_view, iv, n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(proj_x, outf, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(proj_y, outf + n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(proj_xr, outf + 2 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(view_cos, outf + 3 * n, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(pred_level, lev, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

// the tracking sequence of VisualOdometry::EstimatePoseLocal
// (src/visual_odometry.cpp:173-201) on device-resident frame and map data: IsInFrustum for every
// local map point not already in the frame and not bad, then SearchByProjection(F, localMPs, th).
int lorb_track_local_map_dev(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                             const lorb_keypoints* d_kps, const uint8_t* d_slot_state,
                             const lorb_map_points_dev* pts, float viewing_cos_limit, float th,
                             uint8_t* d_in_view, float* d_track, int32_t* d_level,
                             int32_t* d_assign, int32_t* d_nmatches) {
  if (!ctx || !frame || !Tcw || !d_kps || !pts || !d_in_view || !d_track || !d_level || !d_assign || !d_nmatches)
    return LORB_E_INVALID;
  const int nk = d_kps->n, np = pts->n;
  if (nk < 0 || np < 0) return lorb::set_error(ctx, LORB_E_INVALID, "negative sizes");
  if (frame->n_levels < 1 || frame->n_levels > LORB_MAX_LEVELS)
    return lorb::set_error(ctx, LORB_E_INVALID, "n_levels %d out of range", frame->n_levels);
  float Twc[16];
  inv4_lu32f(Tcw, Twc);
  const float TO[19] = {Tcw[0], Tcw[1], Tcw[2], Tcw[3], Tcw[4], Tcw[5], Tcw[6], Tcw[7], Tcw[8], Tcw[9],
                        Tcw[10], Tcw[11], Tcw[12], Tcw[13], Tcw[14], Tcw[15], Twc[3], Twc[7], Twc[11]};
  float* dTO;
  LORB_TRY(lorb::upload_t(ctx, S_WX + 7, TO, 19, &dTO));
  if (np > 0)
    hipLaunchKernelGGL(k_frustum, dim3(lorb::ceil_div(np, 256)), dim3(256), 0, ctx->stream, *frame, dTO, dTO + 16, np,
                       pts->pos, pts->normal, pts->max_dist, pts->min_dist, viewing_cos_limit, d_in_view, d_track,
                       d_track + np, d_track + 2 * np, d_level, d_track + 3 * np, pts->in_frame, pts->is_bad);
  if (nk == 0) {
    LORB_HIP(ctx, hipMemsetAsync(d_nmatches, 0, sizeof(int32_t), ctx->stream));
    LORB_CHECK_LAUNCH(ctx);
    return LORB_OK;
  }
  // keypoint grid of the frame, from the device keypoints (src/frame.cpp:87-115)
  KpDev K;
  int *cell_off, *cell_idx, *kp_cell;
  LORB_TRY(lorb::scratch_t(ctx, S_KP + 7, kCells + 1, &cell_off));
  LORB_TRY(lorb::scratch_t(ctx, S_KP + 8, (size_t)nk, &cell_idx));
  LORB_TRY(lorb::scratch_t(ctx, S_KP + 9, (size_t)nk, &kp_cell));
  hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), 0, ctx->stream, d_kps->x, d_kps->y, nk, *frame, cell_off, cell_idx,
                     kp_cell);
  uint8_t* ss = const_cast<uint8_t*>(d_slot_state);
  if (!ss) {
    LORB_TRY(lorb::scratch_t(ctx, S_KP + 6, (size_t)nk, &ss));
    LORB_HIP(ctx, hipMemsetAsync(ss, 0, nk, ctx->stream));
  }
  K.x = d_kps->x; K.y = d_kps->y; K.angle = d_kps->angle; K.uR = d_kps->u_right; K.octave = d_kps->octave;
  K.desc = reinterpret_cast<const uint4*>(d_kps->desc); K.slot_state = ss;
  K.cell_off = cell_off; K.cell_idx = cell_idx; K.n = nk;
  WinParams P{};
  P.fp = *frame;
  P.th = th;
  int *cnt, *off, *res, *claim;
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 0, (size_t)np + 1, &cnt));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 1, (size_t)np + 1, &off));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 2, (size_t)np + 1, &res));
  LORB_TRY(lorb::scratch_t(ctx, S_WX + 3, (size_t)nk + 1, &claim));
  const unsigned g = lorb::ceil_div(std::max(np, 1), kCandWaves);
  const float* tx = d_track;
  if (np > 0) {
    lorb::KernelTimer kt(ctx, LORB_K_WINDOW_CAND);
    hipLaunchKernelGGL(k_cand_local<false>, dim3(g), dim3(256), 0, ctx->stream, K, P, np, d_in_view, pts->is_bad, tx,
                       tx + np, tx + 2 * np, d_level, tx + 3 * np, reinterpret_cast<const uint4*>(pts->desc), cnt,
                       (const int*)nullptr, (int2*)nullptr);
  }
  hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, ctx->stream, cnt, np, off);
  int2* cand;
  LORB_TRY(alloc_candidates(ctx, off + np, (size_t)np * (size_t)nk, &cand));
  if (np > 0)
    hipLaunchKernelGGL(k_cand_local<true>, dim3(g), dim3(256), 0, ctx->stream, K, P, np, d_in_view, pts->is_bad, tx,
                       tx + np, tx + 2 * np, d_level, tx + 3 * np, reinterpret_cast<const uint4*>(pts->desc), cnt, off,
                       cand);
  size_t rlds = 0;
  const int rmode = resolve_lds_mode(np, nk, &rlds);
  hipLaunchKernelGGL(k_resolve<0>, dim3(1), dim3(1024), rlds, ctx->stream, np, nk, off, cand,
                     pts->locked, (const float*)nullptr, (const float*)nullptr, res, claim, d_assign, (int*)nullptr,
                     (int*)nullptr, d_nmatches, rmode);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int lorb_track_local_map(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16], const lorb_keypoints* kps,
                         const uint8_t* slot_state, const lorb_map_points_dev* pts, float viewing_cos_limit, float th,
                         uint8_t* in_view, float* track, int32_t* level, int32_t* assign, int32_t* nmatches) {
  if (!ctx || !frame || !Tcw || !kps || !pts || !nmatches) return LORB_E_INVALID;
  const int nk = kps->n, np = pts->n;
  if (nk < 0 || np < 0) return lorb::set_error(ctx, LORB_E_INVALID, "negative sizes");
  if ((np > 0 && (!in_view || !track || !level || !pts->pos || !pts->normal || !pts->max_dist || !pts->min_dist ||
                  !pts->desc || !pts->locked)) ||
      (nk > 0 && (!assign || !kps->x || !kps->y || !kps->octave || !kps->angle || !kps->desc)))
    return lorb::set_error(ctx, LORB_E_INVALID, "null array");
  enum { S_TL = 64 };  // 64 .. 87: staging of this call
  lorb_keypoints K{};
  lorb_map_points_dev M{};
  K.n = nk; M.n = np;
  LORB_TRY(lorb::upload_t(ctx, S_TL + 0, kps->x, (size_t)nk, const_cast<float**>(&K.x)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 1, kps->y, (size_t)nk, const_cast<float**>(&K.y)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 2, kps->octave, (size_t)nk, const_cast<int32_t**>(&K.octave)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 3, kps->angle, (size_t)nk, const_cast<float**>(&K.angle)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 4, kps->u_right, kps->u_right ? (size_t)nk : 0, const_cast<float**>(&K.u_right)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 5, kps->desc, (size_t)nk * 32, const_cast<uint8_t**>(&K.desc)));
  uint8_t* dss;
  LORB_TRY(lorb::upload_t(ctx, S_TL + 6, slot_state, slot_state ? (size_t)nk : 0, &dss));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 7, pts->pos, (size_t)np * 3, const_cast<float**>(&M.pos)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 8, pts->normal, (size_t)np * 3, const_cast<float**>(&M.normal)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 9, pts->max_dist, (size_t)np, const_cast<float**>(&M.max_dist)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 10, pts->min_dist, (size_t)np, const_cast<float**>(&M.min_dist)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 11, pts->desc, (size_t)np * 32, const_cast<uint8_t**>(&M.desc)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 12, pts->locked, (size_t)np, const_cast<uint8_t**>(&M.locked)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 13, pts->is_bad, pts->is_bad ? (size_t)np : 0, const_cast<uint8_t**>(&M.is_bad)));
  LORB_TRY(lorb::upload_t(ctx, S_TL + 14, pts->in_frame, pts->in_frame ? (size_t)np : 0,
                          const_cast<uint8_t**>(&M.in_frame)));
  uint8_t* div;
  float* dtr;
  int32_t *dlv, *das, *dnm;
  LORB_TRY(lorb::scratch_t(ctx, S_TL + 15, (size_t)std::max(np, 1), &div));
  LORB_TRY(lorb::scratch_t(ctx, S_TL + 16, (size_t)std::max(np, 1) * 4, &dtr));
  LORB_TRY(lorb::scratch_t(ctx, S_TL + 17, (size_t)std::max(np, 1), &dlv));
  LORB_TRY(lorb::scratch_t(ctx, S_TL + 18, (size_t)std::max(nk, 1), &das));
  LORB_TRY(lorb::scratch_t(ctx, S_TL + 19, 1, &dnm));
  LORB_TRY(lorb_track_local_map_dev(ctx, frame, Tcw, &K, dss, &M, viewing_cos_limit, th, div, dtr, dlv, das, dnm));
  if (np > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(in_view, div, (size_t)np, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(track, dtr, sizeof(float) * 4 * np, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(level, dlv, sizeof(int32_t) * np, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (nk > 0) LORB_HIP(ctx, hipMemcpyAsync(assign, das, sizeof(int32_t) * nk, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(nmatches, dnm, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_unproject_stereo_dev(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16], int32_t n,
                              const float* d_x, const float* d_y, const float* d_depth, float* d_out) {
  if (!ctx || !frame || !Tcw) return LORB_E_INVALID;
  if (n <= 0) return LORB_OK;
  float Twc[16];
  inv4_lu32f(Tcw, Twc);
  lorb::Mat4f T;
  memcpy(T.v, Twc, sizeof(T.v));
  hipLaunchKernelGGL(k_unproject, dim3(lorb::ceil_div(n, 256)), dim3(256), 0, ctx->stream, *frame, T, n, d_x, d_y,
                     d_depth, d_out);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int lorb_unproject_stereo(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16], int32_t n,
                          const float* x, const float* y, const float* depth, float* out_xyz) {
  if (!ctx || !frame || !Tcw) return LORB_E_INVALID;
  if (n <= 0) return LORB_OK;
  float Twc[16];
  inv4_lu32f(Tcw, Twc);
  float *dx, *dy, *dd, *o;
  lorb::Mat4f T;
  memcpy(T.v, Twc, sizeof(T.v));
  LORB_TRY(lorb::upload_t(ctx, S_W1, x, n, &dx));
  LORB_TRY(lorb::upload_t(ctx, S_W2, y, n, &dy));
  LORB_TRY(lorb::upload_t(ctx, S_W3, depth, n, &dd));
  LORB_TRY(lorb::scratch_t(ctx, S_W4, (size_t)n * 3, &o));
  hipLaunchKernelGGL(k_unproject, dim3(lorb::ceil_div(n, 256)), dim3(256), 0, ctx->stream, *frame, T, n, dx, dy, dd, o);
  LORB_CHECK_LAUNCH(ctx);
  LORB_HIP(ctx, hipMemcpyAsync(out_xyz, o, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

}  // extern "C"
