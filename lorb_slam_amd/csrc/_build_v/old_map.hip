// lorb_map.hip -- the device-resident local map and its chained LocalMapping step (SURVEY §8 a17
// "full step" mode, §7 item 8).
//
// The reference's designed-but-disabled step (src/local_mapping.cpp:24-33, 55-76):
//   1. the new keyframe's matches become observations: for every slot with a map point that the
//      frame is not yet in, MapPoint::AddObservation(frame, slot)  (src/local_mapping.cpp:57-70);
//      the matches come from Matcher::SearchLocalPoints -- BFMatcher(NORM_HAMMING, crossCheck) of
//      the keyframe's descriptors against the window's map points (src/matcher.cpp:319-366);
//   2. the keyframe's unmatched keypoints with a stereo depth become new map points at
//      Frame::UnprojectStereo (src/frame.cpp:335-356), observed by the keyframe, with the
//      keypoint's descriptor (the VisualOdometry::UpdateFrame pattern, src/visual_odometry.cpp:214-230);
//   3. Map::AddFrame (src/local_mapping.cpp:76) -- the keyframe joins the window; the window
//      keeps the newest W keyframes (the oldest leaves; KeyFramesCulling is empty in the reference,
//      src/local_mapping.cpp:110-113, so this is the step's sliding-window policy);
//   4. BA::LocalPoseOptimization over the window (src/local_mapping.cpp:32; src/bundle_adjust.cpp:207-330):
//      points = those with an observation by a window keyframe, observations by the F keyframes
//      before the window are MPCost residuals (fixed poses), and the float write-back of poses and
//      points (src/bundle_adjust.cpp:317-329).
//
// Everything stays in HBM: map points (position, descriptor), observations (point, keyframe id, uv),
// a ring of keyframe poses.  One step = matcher + unprojection + append (one workgroup, block scans
// in keypoint order) + cull/compaction (flags, one-launch scans, stable gathers) + the device-built BA
// plan (lorb_ba_plan_update_dev: its one small readback is the step's only host synchronisation)
// + the LM solve (hipGraph per iteration) + the float write-back.
#include <algorithm>
#include <chrono>
#include <cstdlib>

#include "lorb_internal.h"

namespace {

struct MapDev {
  float* pos; uint8_t* desc; int* obs_pt; int* obs_kf; float* obs_uv;        // current buffers
  float* pos2; uint8_t* desc2; int* obs_pt2; int* obs_kf2; float* obs_uv2;   // compaction targets
  int* obs_frame;                                                            // BA slot of each observation
  int* cnt;      // [0] points, [1] observations, [2] error flags, [3] new points, [4] new observations, [5] matches
  int* flag_pt; int* newid; int* flag_obs; int* newpos;  // newid / newpos: scans within kScanTile tiles
  int* flag_new; int* newnew;  // points that got an observation this step, and their scan
  int* tile_tot;  // tile sums of the three scans: [0, ntP) kept points, [ntP, 2 ntP) new-observation
                  // points, then observations
  float* ring;   // R x 6 keyframe poses, slot = kf mod R
  float* pose_init; float* fixed;
  int P_cap, K_cap, W, F, R;
};

struct Pose6 { float v[6]; };

__device__ __forceinline__ int ring_slot(int kf, int R) { const int r = kf % R; return r < 0 ? r + R : r; }

// step 1 + 2: one workgroup, keypoints in order.  First the matcher's finalisation (k_cc_finalize's
// work on the crossCheck keys: the DMatches, minDist and the d <= max(2 minDist, 30) filter,
// src/matcher.cpp:342-362) into mt.  A matched keypoint adds an observation of its map point; an
// unmatched one with depth > 0 adds a new point at Frame::UnprojectStereo (src/frame.cpp:335-356,
// lorb::unproject_point) and its observation.  Observations and new points are appended in keypoint
// order: thread t owns a run of consecutive keypoints, one block scan of three counters
// (observations, new points, matches) places every run.  RM > 0 (n <= 1024 RM): every input of the
// thread's keypoints is loaded in one batch up front and stays in registers, so the kernel pays one
// memory round trip instead of one per phase; RM = 0 re-reads them (any n).
template <int RM>
__global__ __launch_bounds__(1024) void k_map_append(MapDev m, int n, int kf, Pose6 pose,
                                                     const unsigned long long* __restrict__ qkey, int has_t,
                                                     int* __restrict__ mt, lorb::Mat4f Twc, float fx, float fy,
                                                     float cx, float cy, const uint8_t* __restrict__ kdesc,
                                                     const float* __restrict__ x, const float* __restrict__ y,
                                                     const float* __restrict__ depth) {
  __shared__ lorb::I4 wsum[16];
  __shared__ int s_min[16];
  const int t = threadIdx.x;
  const int P0 = m.cnt[0], K0 = m.cnt[1];
  const int R = RM > 0 ? RM : (n + 1023) / 1024, q0 = min(t * R, n), q1 = min(q0 + R, n);
  constexpr int RA = RM > 0 ? RM : 1;
  unsigned long long kv[RA];
  float xv[RA], yv[RA], zv[RA];
  uint4 d0[RA], d1[RA];
  int mv[RA];
  if constexpr (RM > 0) {
#pragma unroll
    for (int u = 0; u < RM; ++u) {
      const int q = q0 + u;
      const bool ok = q < q1;
      kv[u] = ok && has_t ? qkey[q] : ~0ull;
      xv[u] = ok ? x[q] : 0.0f; yv[u] = ok ? y[q] : 0.0f; zv[u] = ok ? depth[q] : 0.0f;
      d0[u] = d1[u] = make_uint4(0, 0, 0, 0);
      if (ok) {
        const uint4* sd = reinterpret_cast<const uint4*>(kdesc + 32 * (size_t)q);
        d0[u] = sd[0]; d1[u] = sd[1];
      }
    }
  }
  auto key_of = [&](int u, int q) -> unsigned long long {
    if constexpr (RM > 0) return kv[u];
    else return has_t ? qkey[q] : ~0ull;
  };
  auto depth_of = [&](int u, int q) -> float {
    if constexpr (RM > 0) return zv[u];
    else return depth[q];
  };
  {
    int mn = 0x7fffffff;
#pragma unroll RA
    for (int u = 0; u < (RM > 0 ? RM : 1 << 30); ++u) {
      const int q = q0 + u;
      if (q >= q1) break;
      const unsigned long long v = key_of(u, q);
      if (v != ~0ull) mn = min(mn, (int)(v >> 32));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mn = min(mn, __shfl_xor(mn, o, 64));
    if ((t & 63) == 0) s_min[t >> 6] = mn;
    __syncthreads();
    mn = s_min[0];
#pragma unroll
    for (int w = 1; w < 16; ++w) mn = min(mn, s_min[w]);
    // d > max(2 * minDist, 30.0) rejects (exact in integers); no crossCheck key at all: no
    // threshold is compared, and 2 * INT_MAX is not formed
    const int thr = mn == 0x7fffffff ? 30 : max(2 * mn, 30);
#pragma unroll RA
    for (int u = 0; u < (RM > 0 ? RM : 1 << 30); ++u) {
      const int q = q0 + u;
      if (q >= q1) break;
      const unsigned long long v = key_of(u, q);
      const int a = (v != ~0ull && (int)(v >> 32) <= thr) ? (int)(v & 0xffffffffu) : -1;
      mt[q] = a;
      if constexpr (RM > 0) mv[u] = a;
    }
  }
  auto match_of = [&](int u, int q) -> int {
    if constexpr (RM > 0) return mv[u];
    else return mt[q];
  };
  lorb::I4 c = {{0, 0, 0, 0}};
#pragma unroll RA
  for (int u = 0; u < (RM > 0 ? RM : 1 << 30); ++u) {
    const int q = q0 + u;
    if (q >= q1) break;
    const bool mat = match_of(u, q) >= 0;
    const bool nw = !mat && depth_of(u, q) > 0.0f;
    c.v[0] += mat || nw; c.v[1] += nw; c.v[2] += mat;
  }
  lorb::I4 tot;
  const lorb::I4 ex = lorb::block_excl_scan4<1024>(c, wsum, &tot);
  const bool ok = (P0 + tot.v[1] <= m.P_cap) && (K0 + tot.v[0] <= m.K_cap);
  if (t == 0) {
    m.cnt[2] = ok ? 0 : 1;  // this step's capacity flag (no separate clear)
    if (!ok) { m.cnt[3] = 0; m.cnt[4] = 0; m.cnt[5] = tot.v[2]; }  // the attempt appended nothing
  }
  if (!ok) return;  // the map is left exactly as it was (the host stops the step here)
  if (t < 6) m.ring[6 * ring_slot(kf, m.R) + t] = pose.v[t];
  int ko = K0 + ex.v[0], pn = P0 + ex.v[1];
#pragma unroll RA
  for (int u = 0; u < (RM > 0 ? RM : 1 << 30); ++u) {
    const int q = q0 + u;
    if (q >= q1) break;
    const int a = match_of(u, q);
    const float z = depth_of(u, q);
    const bool mat = a >= 0, nw = !mat && z > 0.0f;
    if (!(mat || nw)) continue;
    float xq, yq;
    if constexpr (RM > 0) { xq = xv[u]; yq = yv[u]; }
    else { xq = x[q]; yq = y[q]; }
    int p = a;
    if (nw) {
      p = pn++;
      float X[3];
      lorb::unproject_point(fx, fy, cx, cy, Twc, xq, yq, z, X);
      m.pos[3 * p + 0] = X[0]; m.pos[3 * p + 1] = X[1]; m.pos[3 * p + 2] = X[2];
      uint4* dd = reinterpret_cast<uint4*>(m.desc + 32 * (size_t)p);
      if constexpr (RM > 0) { dd[0] = d0[u]; dd[1] = d1[u]; }
      else {
        const uint4* sd = reinterpret_cast<const uint4*>(kdesc + 32 * (size_t)q);
        dd[0] = sd[0]; dd[1] = sd[1];
      }
    }
    const int k = ko++;
    m.obs_pt[k] = p;
    m.flag_new[p] = 1;  // at most one per point: crossCheck matches are one-to-one
    m.obs_kf[k] = kf;
    m.obs_uv[2 * k + 0] = xq;
    m.obs_uv[2 * k + 1] = yq;
  }
  if (t == 0) {
    m.cnt[0] = P0 + tot.v[1]; m.cnt[1] = K0 + tot.v[0];
    m.cnt[3] = tot.v[1]; m.cnt[4] = tot.v[0]; m.cnt[5] = tot.v[2];
  }
}

// cull, one launch: a point stays while a window keyframe (id >= t0) observes it; an observation
// stays while its point stays and its keyframe is in the window or among the F fixed keyframes
// before it; flags beyond the count are 0 (scan tail).  Slots [0, K0) are sorted by point: each
// thread finds its point's run inside its wavefront from two ballots (run starts, window
// keyframes) and ORs the run's window bits; a run that crosses the wavefront's edge also walks the
// slots beyond it.  The step's new observations (slots >= K0, keyframe = the newest, in the
// window) keep themselves and their points (flag_new marks a point that got one).
__global__ __launch_bounds__(256) void k_map_cull(MapDev m, int Kb, int K0, int t0) {
  const int k = blockIdx.x * 256 + threadIdx.x, lane = threadIdx.x & 63;
  const int kc = min(m.cnt[1], Kb), k0 = min(K0, kc);
  const bool old = k < k0;
  int p = -1, kfv = 0, pprev = -1;
  if (k < kc) { p = m.obs_pt[k]; kfv = m.obs_kf[k]; }
  if (old && k > 0) pprev = m.obs_pt[k - 1];
  const bool start = old && (k == 0 || pprev != p);
  // every slot that is not an earlier one ends the runs before it
  const unsigned long long B = __ballot(start || !old), Wb = __ballot(old && kfv >= t0);
  if (k > Kb) return;
  if (k >= kc) { m.flag_obs[k] = 0; return; }
  if (!old) {
    m.flag_obs[k] = kfv >= t0 - m.F;  // (a new observation: its keyframe is the newest)
    if (kfv >= t0) m.flag_pt[p] = 1;
    return;
  }
  const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1;
  const unsigned long long below = B & upto, above = B & ~upto;
  const int s0 = below ? 63 - __builtin_clzll(below) : 0;   // run's first lane in this wavefront
  const int e0 = above ? __builtin_ctzll(above) : 64;       // one past its last lane
  const unsigned long long run = (e0 == 64 ? ~0ull : (1ull << e0) - 1) & ~((1ull << s0) - 1);
  bool keep = (Wb & run) != 0 || m.flag_new[p] != 0;
  const int wbase = k - lane;
  if (!below)  // the run began in an earlier wavefront
    for (int j = wbase - 1; !keep && j >= 0 && m.obs_pt[j] == p; --j) keep = m.obs_kf[j] >= t0;
  if (!above)  // the run goes on past this wavefront
    for (int j = wbase + 64; !keep && j < k0 && m.obs_pt[j] == p; ++j) keep = m.obs_kf[j] >= t0;
  m.flag_obs[k] = keep && kfv >= t0 - m.F;
  if (start && keep) m.flag_pt[p] = 1;
}

// the flag scans are tile-local (one workgroup per tile, all tiles of both arrays in one launch);
// a consumer adds the sums of the tiles before its own (few: kScanTile = 16 k entries each)
__device__ __forceinline__ int tile_base(const int* tot, int tile) {
  int s = 0;
  for (int k = 0; k < tile; ++k) s += tot[k];
  return s;
}
__device__ __forceinline__ int new_id(const MapDev& m, int i) {
  return m.newid[i] + tile_base(m.tile_tot, i / lorb::kScanTile);
}
__device__ __forceinline__ int new_pos(const MapDev& m, int ntP, int i) {
  return m.newpos[i] + tile_base(m.tile_tot + 2 * ntP, i / lorb::kScanTile);
}
// observations this step added to points with (pre-compaction) id < p
__device__ __forceinline__ int new_before(const MapDev& m, int ntP, int p) {
  return m.newnew[p] + tile_base(m.tile_tot + ntP, p / lorb::kScanTile);
}

// stable gathers into the alternate buffers; observation slots as lorb_ba_window_dev wants them.
// The observations stay sorted by point (stably): slots [0, K0) hold the earlier ones, sorted; the
// step's new ones (slots >= K0, keypoint order, one per point at most) go after their point's
// earlier ones.  A kept earlier observation moves to (kept ones before it) + (new ones of points
// before its point); a new one of point p to (kept earlier ones of points <= p: the kept count
// before the first earlier slot of a point > p) + (new ones of points before p).  That slot is
// pt_off[p + 1] of the BA plan built on the earlier slots (its per-point offsets, points [0, P0)),
// or a binary search over them when there is no such plan.
// Workgroup 0 also writes the new counts and the window's initial / fixed poses from the ring.
__global__ __launch_bounds__(256) void k_map_compact(MapDev m, int Pb, int Kb, int K0, int P0, int t0, int ntP,
                                                     const int* __restrict__ pt_off) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0) {
    if (i == 0) { m.cnt[0] = new_id(m, Pb); m.cnt[1] = new_pos(m, ntP, Kb); }
    for (int j = i; j < 6 * m.W; j += 256) m.pose_init[j] = m.ring[6 * ring_slot(t0 + j / 6, m.R) + j % 6];
    for (int j = i; j < 6 * m.F; j += 256) m.fixed[j] = m.ring[6 * ring_slot(t0 - 1 - j / 6, m.R) + j % 6];
  }
  const int fp = i < Pb ? m.flag_pt[i] : 0;
  if (i < Pb && m.flag_new[i]) m.flag_new[i] = 0;  // cleared for the next slide (scanned already)
  if (fp) {
    m.flag_pt[i] = 0;  // cleared for the next slide (only this thread reads it here)
    const int d = new_id(m, i);
    m.pos2[3 * d + 0] = m.pos[3 * i + 0];
    m.pos2[3 * d + 1] = m.pos[3 * i + 1];
    m.pos2[3 * d + 2] = m.pos[3 * i + 2];
    const uint4* s = reinterpret_cast<const uint4*>(m.desc + 32 * (size_t)i);
    uint4* o = reinterpret_cast<uint4*>(m.desc2 + 32 * (size_t)d);
    o[0] = s[0]; o[1] = s[1];
  }
  if (i < Kb && m.flag_obs[i]) {
    const int p = m.obs_pt[i], kf = m.obs_kf[i];
    int d;
    if (i < K0) {
      d = new_pos(m, ntP, i) + new_before(m, ntP, p);
    } else {
      int lo = 0, hi = K0;  // first earlier slot of a point > p
      if (pt_off) {
        lo = pt_off[min(p + 1, P0)];
      } else {
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (m.obs_pt[mid] <= p) lo = mid + 1; else hi = mid;
        }
      }
      d = new_pos(m, ntP, lo) + new_before(m, ntP, p);
    }
    m.obs_pt2[d] = new_id(m, p);
    m.obs_kf2[d] = kf;
    m.obs_uv2[2 * d + 0] = m.obs_uv[2 * i + 0];
    m.obs_uv2[2 * d + 1] = m.obs_uv[2 * i + 1];
    m.obs_frame[d] = kf >= t0 ? kf - t0 : -1 - (t0 - 1 - kf);
  }
}

// the three compaction scans, tile-local: workgroups [0, ntP) the kept-point flags, [ntP, 2 ntP)
// the new-observation flags of the points, the rest the observation flags
__global__ __launch_bounds__(1024) void k_map_scans(MapDev m, int Pb, int Kb, int ntP) {
  __shared__ int wsum[16];
  __shared__ int s_tile[lorb::kScanTileLds];
  const int seg = (int)blockIdx.x < ntP ? 0 : (int)blockIdx.x < 2 * ntP ? 1 : 2;
  const int tile = blockIdx.x - seg * ntP;
  const int n = seg < 2 ? Pb + 1 : Kb + 1, base = tile * lorb::kScanTile;
  const int* in = seg == 0 ? m.flag_pt : seg == 1 ? m.flag_new : m.flag_obs;
  int* out = seg == 0 ? m.newid : seg == 1 ? m.newnew : m.newpos;
  const int tot = lorb::wg_scan_tile(in + base, out + base, min(n - base, lorb::kScanTile), 0, s_tile, wsum);
  if (threadIdx.x == 0) m.tile_tot[blockIdx.x] = tot;
}

}  // namespace

struct lorb_map {
  lorb_ctx* ctx = nullptr;
  MapDev m{};
  int t0 = 0;            // id of the oldest window keyframe
  int h_P = 0, h_K = 0;  // counts after the last step (host mirror)
  int n_cap = 0, last_n = 0;
  float fx = 0, fy = 0, cx = 0, cy = 0;
  // LORB_MAP_PROFILE=1: host wall time per phase with a stream sync after each (diagnostics only)
  bool prof = false;
  double prof_ms[8] = {};
  int prof_n = 0;
  int* mt = nullptr;
  // the step's crossCheck keys: per-query keys and per-train keys (all-ones between steps), owned by
  // the map so that its side-stream match shares no scratch with matcher calls on the ctx stream
  unsigned long long* qkey = nullptr;
  uint32_t* tkey = nullptr;
  int* pinned = nullptr;
  lorb_ba_plan* plan = nullptr;
  bool plan_ok = false;  // plan built on the current slots (its point offsets serve the compaction)
  bool broken = false;   // a failed step whose counts could not be re-read: the map is unusable
  // Overlap (lorb_map_set_overlap, default off): a step's match and append touch only the map's
  // point descriptors, its new slots / points and counts, its own key buffers -- nothing the previous
  // step's LM solve and write-back read or write -- so they run on a side stream as soon as the
  // previous step's plan build has read the map (ev_built), concurrently with that solve; the slide
  // waits for both.  The caller's keyframe arrays must be complete when the step is called (the side
  // stream is not ordered after work the caller still has queued, lorb_c.h).
  bool overlap = false;
  hipStream_t side = nullptr;
  hipEvent_t ev_built = nullptr, ev_app = nullptr;
  bool built = false;  // ev_built recorded by the previous step
  int n_overlapped = 0;  // steps whose match + append ran on the side stream
  std::vector<void*> allocs;
  ~lorb_map() {
    if (prof && prof_n)
      fprintf(stderr, "lorb_map profile over %d steps (ms/step): match %.3f unproject %.3f append %.3f slide %.3f "
              "plan %.3f solve %.3f writeback %.3f\n", prof_n, prof_ms[0] / prof_n, prof_ms[1] / prof_n,
              prof_ms[2] / prof_n, prof_ms[3] / prof_n, prof_ms[4] / prof_n, prof_ms[5] / prof_n, prof_ms[6] / prof_n);
    if (side) (void)hipStreamSynchronize(side);
    if (plan) (void)lorb_ba_plan_destroy(plan);
    if (pinned) (void)hipHostFree(pinned);
    if (ev_built) (void)hipEventDestroy(ev_built);
    if (ev_app) (void)hipEventDestroy(ev_app);
    if (side) (void)hipStreamDestroy(side);
    for (void* p : allocs) (void)hipFree(p);
  }
};

namespace {

template <typename T>
int malloc_n(lorb_map* M, size_t n, T** out) {
  void* p = nullptr;
  LORB_HIP(M->ctx, hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
  M->allocs.push_back(p);
  *out = static_cast<T*>(p);
  return LORB_OK;
}

int map_alloc(lorb_map* M, const lorb_map_init* in) {
  MapDev& m = M->m;
  m.P_cap = in->max_points; m.K_cap = in->max_obs; m.W = in->n_window; m.F = in->n_fixed;
  m.R = in->n_window + in->n_fixed + 1;
  const size_t P = (size_t)m.P_cap, K = (size_t)m.K_cap;
  LORB_TRY(malloc_n(M, 3 * P, &m.pos)); LORB_TRY(malloc_n(M, 3 * P, &m.pos2));
  LORB_TRY(malloc_n(M, 32 * P, &m.desc)); LORB_TRY(malloc_n(M, 32 * P, &m.desc2));
  LORB_TRY(malloc_n(M, K, &m.obs_pt)); LORB_TRY(malloc_n(M, K, &m.obs_pt2));
  LORB_TRY(malloc_n(M, K, &m.obs_kf)); LORB_TRY(malloc_n(M, K, &m.obs_kf2));
  LORB_TRY(malloc_n(M, 2 * K, &m.obs_uv)); LORB_TRY(malloc_n(M, 2 * K, &m.obs_uv2));
  LORB_TRY(malloc_n(M, K, &m.obs_frame));
  LORB_TRY(malloc_n(M, (size_t)8, &m.cnt));
  LORB_TRY(malloc_n(M, P + 1, &m.flag_pt)); LORB_TRY(malloc_n(M, P + 1, &m.newid));
  // point flags start clear and are cleared again by the compaction that consumes them
  LORB_HIP(M->ctx, hipMemsetAsync(m.flag_pt, 0, sizeof(int) * ((size_t)P + 1), M->ctx->stream));
  LORB_TRY(malloc_n(M, P + 1, &m.flag_new)); LORB_TRY(malloc_n(M, P + 1, &m.newnew));
  LORB_HIP(M->ctx, hipMemsetAsync(m.flag_new, 0, sizeof(int) * ((size_t)P + 1), M->ctx->stream));
  LORB_TRY(malloc_n(M, K + 1, &m.flag_obs)); LORB_TRY(malloc_n(M, K + 1, &m.newpos));
  LORB_TRY(malloc_n(M, 2 * (P + 1) / lorb::kScanTile + (K + 1) / lorb::kScanTile + 4, &m.tile_tot));
  LORB_TRY(malloc_n(M, 6 * (size_t)m.R, &m.ring));
  LORB_TRY(malloc_n(M, 6 * (size_t)m.W, &m.pose_init));
  LORB_TRY(malloc_n(M, 6 * (size_t)std::max(m.F, 1), &m.fixed));
  const size_t n = (size_t)std::max(in->max_keypoints, 1);
  M->n_cap = (int)n;
  LORB_TRY(malloc_n(M, n, &M->mt));
  LORB_TRY(malloc_n(M, n, &M->qkey));
  LORB_TRY(malloc_n(M, P, &M->tkey));
  LORB_HIP(M->ctx, hipMemsetAsync(M->tkey, 0xff, sizeof(uint32_t) * std::max<size_t>(P, 1), M->ctx->stream));
  LORB_HIP(M->ctx, hipHostMalloc(reinterpret_cast<void**>(&M->pinned), sizeof(int) * 8));
  return LORB_OK;
}

lorb_ba_window_dev window_of(const lorb_map* M) {
  const MapDev& m = M->m;
  lorb_ba_window_dev w{};
  w.n_poses = m.W; w.n_fixed = m.F; w.max_points = m.P_cap; w.max_obs = m.K_cap;
  w.d_n_points = m.cnt; w.d_n_obs = m.cnt + 1;
  w.fx = M->fx; w.fy = M->fy; w.cx = M->cx; w.cy = M->cy;
  w.d_pose_init = m.pose_init; w.d_fixed_pose = m.fixed; w.d_point_init = m.pos;
  w.d_obs_point = m.obs_pt; w.d_obs_frame = m.obs_frame; w.d_obs_uv = m.obs_uv;
  return w;
}

// slide to window [t0, t0 + W): cull points no window keyframe observes, drop observations by
// keyframes older than the fixed ones, compact (stable), rebuild the BA slots and window poses
int map_slide(lorb_map* M, int t0, int Pb, int Kb, int K0, int P0, const int* pt_off) {
  lorb_ctx* ctx = M->ctx;
  hipStream_t s = ctx->stream;
  MapDev& m = M->m;
  hipLaunchKernelGGL(k_map_cull, dim3(lorb::ceil_div(Kb + 1, 256)), dim3(256), 0, s, m, Kb, std::min(K0, Kb), t0);
  const int ntP = lorb::ceil_div(Pb + 1, lorb::kScanTile), ntK = lorb::ceil_div(Kb + 1, lorb::kScanTile);
  hipLaunchKernelGGL(k_map_scans, dim3(2 * ntP + ntK), dim3(1024), 0, s, m, Pb, Kb, ntP);
  const int nmax = std::max(std::max(Pb, Kb), 1);
  hipLaunchKernelGGL(k_map_compact, dim3(lorb::ceil_div(nmax, 256)), dim3(256), 0, s, m, Pb, Kb, std::min(K0, Kb), P0, t0,
                     ntP, pt_off);
  LORB_CHECK_LAUNCH(ctx);
  std::swap(m.pos, m.pos2); std::swap(m.desc, m.desc2); std::swap(m.obs_pt, m.obs_pt2);
  std::swap(m.obs_kf, m.obs_kf2); std::swap(m.obs_uv, m.obs_uv2);
  M->t0 = t0;
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_map_create(lorb_ctx* ctx, const lorb_map_init* in, lorb_map** out) {
  if (!ctx || !in || !out) return LORB_E_INVALID;
  *out = nullptr;
  if (in->n_window < 1 || in->n_fixed < 0 || in->n_points < 0 || in->n_obs < 0 || in->max_keypoints < 0 ||
      in->n_points > in->max_points || in->n_obs > in->max_obs || !in->pose ||
      (in->n_fixed > 0 && !in->fixed_pose) ||
      (in->n_points > 0 && (!in->point || !in->point_desc)) ||
      (in->n_obs > 0 && (!in->obs_point || !in->obs_kf || !in->obs_uv)))
    return lorb::set_error(ctx, LORB_E_INVALID, "lorb_map_create: bad sizes or missing arrays");
  const int W = in->n_window, F = in->n_fixed;
  for (int k = 0; k < in->n_obs; ++k) {
    if (in->obs_point[k] < 0 || in->obs_point[k] >= in->n_points)
      return lorb::set_error(ctx, LORB_E_INVALID, "observation %d: point %d outside [0, %d)", k, in->obs_point[k], in->n_points);
    if (in->obs_kf[k] < -F || in->obs_kf[k] >= W)
      return lorb::set_error(ctx, LORB_E_INVALID, "observation %d: keyframe %d outside [-%d, %d)", k, in->obs_kf[k], F, W);
  }
  lorb_map* M = new (std::nothrow) lorb_map();
  if (!M) return LORB_E_NOMEM;
  M->ctx = ctx;
  {
    const char* e = getenv("LORB_MAP_PROFILE");
    M->prof = e && e[0] == '1';
  }
  M->fx = in->fx; M->fy = in->fy; M->cx = in->cx; M->cy = in->cy;
  int rc = map_alloc(M, in);
  if (rc == LORB_OK) {
    hipStream_t s = ctx->stream;
    MapDev& m = M->m;
    std::vector<float> ring(6 * (size_t)m.R, 0.0f);
    for (int j = 0; j < W; ++j)
      for (int q = 0; q < 6; ++q) ring[6 * (size_t)(j % m.R) + q] = in->pose[6 * (size_t)j + q];
    for (int j = 0; j < F; ++j)
      for (int q = 0; q < 6; ++q) ring[6 * (size_t)(((-1 - j) % m.R + m.R) % m.R) + q] = in->fixed_pose[6 * (size_t)j + q];
    const int cnt[8] = {in->n_points, in->n_obs, 0, 0, 0, 0, 0, 0};
    auto up = [&](void* d, const void* h, size_t bytes) -> int {
      if (bytes) LORB_HIP(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
      return LORB_OK;
    };
    rc = up(m.ring, ring.data(), sizeof(float) * ring.size());
    if (rc == LORB_OK) rc = up(m.cnt, cnt, sizeof(cnt));
    if (rc == LORB_OK) rc = up(m.pos, in->point, sizeof(float) * 3 * (size_t)in->n_points);
    if (rc == LORB_OK) rc = up(m.desc, in->point_desc, 32 * (size_t)in->n_points);
    // the map keeps its observations sorted by point (stably): sort the initial ones once
    std::vector<int> ord(in->n_obs);
    for (int k = 0; k < in->n_obs; ++k) ord[k] = k;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return in->obs_point[a] < in->obs_point[b]; });
    std::vector<int> op(in->n_obs), ok(in->n_obs);
    std::vector<float> ouv(2 * (size_t)in->n_obs);
    for (int k = 0; k < in->n_obs; ++k) {
      op[k] = in->obs_point[ord[k]]; ok[k] = in->obs_kf[ord[k]];
      ouv[2 * k] = in->obs_uv[2 * ord[k]]; ouv[2 * k + 1] = in->obs_uv[2 * ord[k] + 1];
    }
    if (rc == LORB_OK) rc = up(m.obs_pt, op.data(), sizeof(int) * (size_t)in->n_obs);
    if (rc == LORB_OK) rc = up(m.obs_kf, ok.data(), sizeof(int) * (size_t)in->n_obs);
    if (rc == LORB_OK) rc = up(m.obs_uv, ouv.data(), sizeof(float) * 2 * (size_t)in->n_obs);
    if (rc == LORB_OK) {
      // the initial window [0, W): obs slots / window poses, no culling of a consistent input
      rc = map_slide(M, 0, in->n_points, in->n_obs, in->n_obs, in->n_points, nullptr);
      M->h_P = in->n_points; M->h_K = in->n_obs;  // upper bounds until the first readback
    }
    if (rc == LORB_OK) {
      const lorb_ba_window_dev w = window_of(M);
      rc = lorb_ba_plan_create_dev(ctx, &w, &M->plan);
      // the map keeps its observations sorted by point: later builds skip the counting sort
      if (rc == LORB_OK) lorb::ba_plan_sorted_hint(M->plan, true);
      M->plan_ok = rc == LORB_OK;
    }
    if (rc == LORB_OK) {
      LORB_HIP(ctx, hipMemcpyAsync(M->pinned, m.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, s));
      LORB_HIP(ctx, hipStreamSynchronize(s));
      M->h_P = M->pinned[0]; M->h_K = M->pinned[1];
    }
  }
  if (rc != LORB_OK) { delete M; return rc; }
  *out = M;
  return LORB_OK;
}

int lorb_map_step_dev(lorb_map* M, const lorb_frame_params* frame, const float pose[6], const float Tcw[16], int32_t n,
                      const uint8_t* d_desc, const float* d_x, const float* d_y, const float* d_depth,
                      const lorb_lm_options* opt) {
  if (!M || !frame || !pose || !Tcw || !opt || n < 0) return LORB_E_INVALID;
  lorb_ctx* ctx = M->ctx;
  if (n > M->n_cap) return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints > the map's max_keypoints %d", n, M->n_cap);
  if (n > 0 && (!d_desc || !d_x || !d_y || !d_depth)) return LORB_E_INVALID;
  if (M->broken) return lorb::set_error(ctx, LORB_E_DEVICE, "the map is unusable after an earlier failed step");
  hipStream_t s = ctx->stream;
  MapDev& m = M->m;
  const int kf = M->t0 + m.W;  // the new keyframe's id
  auto clk = std::chrono::steady_clock::now();
  auto mark = [&](int i) -> int {
    if (!M->prof) return LORB_OK;
    LORB_HIP(ctx, hipStreamSynchronize(s));
    const auto now = std::chrono::steady_clock::now();
    M->prof_ms[i] += std::chrono::duration<double, std::milli>(now - clk).count();
    clk = now;
    return LORB_OK;
  };
  LORB_TRY(mark(7));
  const bool ovl = M->overlap && M->built && !M->prof && !ctx->ktime;
  if (ovl && !M->side) {
    LORB_HIP(ctx, hipStreamCreateWithFlags(&M->side, hipStreamNonBlocking));
    LORB_HIP(ctx, hipEventCreateWithFlags(&M->ev_app, hipEventDisableTiming));
  }
  hipStream_t ms = ovl ? M->side : s;  // the match + append stream
  M->n_overlapped += ovl;
  if (ovl) LORB_HIP(ctx, hipStreamWaitEvent(ms, M->ev_built, 0));
  // 1. SearchLocalPoints: the keyframe's descriptors against the map's points -- the crossCheck keys
  //    here, the finalisation (minDist filter) inside the append
  unsigned long long* qkey = nullptr;
  const bool has_t = M->h_P > 0;
  if (n > 0 && has_t) {
    // the per-train keys are restored to all-ones by the append's merge (k_cc_merge1); a failure
    // between the scan and that merge would leave stale keys for the next step: reset them here, or
    // mark the map unusable when even that fails
    if (const int rc = lorb::match1_keys_into(ctx, d_desc, n, m.desc, M->h_P, M->qkey, M->tkey, ms); rc != LORB_OK) {
      if (hipMemsetAsync(M->tkey, 0xff, sizeof(uint32_t) * std::max<size_t>(m.P_cap, 1), ms) != hipSuccess) M->broken = true;
      return rc;
    }
    qkey = M->qkey;
  }
  LORB_TRY(mark(0));
  LORB_TRY(mark(1));
  // 2 + 3. AddObservation / new points at UnprojectStereo (Twc = mTcw.inv(), src/frame.cpp:350),
  // keyframe pose into the ring
  Pose6 p6;
  for (int q = 0; q < 6; ++q) p6.v[q] = pose[q];
  lorb::Mat4f Twc;
  lorb::inv4_lu32f(Tcw, Twc.v);
#define LORB_APPEND(RM)                                                                                       \
  hipLaunchKernelGGL(k_map_append<RM>, dim3(1), dim3(1024), 0, ms, m, n, kf, p6, (const unsigned long long*)qkey, \
                     (int)(has_t && qkey), M->mt, Twc, frame->fx, frame->fy, frame->cx, frame->cy, d_desc, d_x, d_y, \
                     d_depth)
  if (n <= 1024) LORB_APPEND(1);
  else if (n <= 2048) LORB_APPEND(2);
  else if (n <= 4096) LORB_APPEND(4);
  else LORB_APPEND(0);
#undef LORB_APPEND
  if (hipGetLastError() != hipSuccess) {  // the append did not run: the map's counts are unknown
    M->broken = true;
    return lorb::set_error(ctx, LORB_E_DEVICE, "k_map_append launch failed; the map is unusable");
  }
  if (ovl) {  // the rest of the step follows the previous step's write-back on the main stream
    LORB_HIP(ctx, hipEventRecord(M->ev_app, ms));
    LORB_HIP(ctx, hipStreamWaitEvent(s, M->ev_app, 0));
  }
  M->last_n = n;
  // Capacity: n keypoints add at most n points and n observations.  When that bound does not fit,
  // read the append's verdict before anything else changes: a refused append leaves the map as it
  // was (no ring write, no slide, no cull), so the map stays usable after the error.
  if (M->h_P + n > m.P_cap || M->h_K + n > m.K_cap) {
    LORB_HIP(ctx, hipMemcpyAsync(M->pinned, m.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, s));
    LORB_HIP(ctx, hipStreamSynchronize(s));
    if (M->pinned[2] & 1)
      return lorb::set_error(ctx, LORB_E_NOMEM, "map capacity exceeded (points %d + %d new / %d, observations %d + %d new / %d)",
                             M->h_P, n, m.P_cap, M->h_K, n, m.K_cap);
  }
  LORB_TRY(mark(2));
  // 4. slide the window by one keyframe; cull and compact
  LORB_TRY(map_slide(M, M->t0 + 1, std::min(M->h_P + n, m.P_cap), std::min(M->h_K + n, m.K_cap), M->h_K, M->h_P,
                      M->plan_ok ? lorb::ba_plan_point_offsets(M->plan) : nullptr));
  LORB_TRY(mark(3));
  // 5. BA plan of the slid window; its one readback carries the window's live counts too
  const lorb_ba_window_dev w = window_of(M);
  M->plan_ok = false;
  if (const int rc = lorb_ba_plan_update_dev(M->plan, &w); rc != LORB_OK) {
    M->built = false;  // the next step's match waits for this step's kernels on the main stream
    // the append and the slide have run: the live counts are the device's now, and the next slide
    // takes h_K as the end of the point-sorted slots -- re-read them, or mark the map unusable
    if (hipMemcpyAsync(M->pinned, m.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess) {
      M->h_P = M->pinned[0]; M->h_K = M->pinned[1];
    } else {
      M->broken = true;
    }
    return rc;
  }
  M->plan_ok = true;
  // the plan build has read the map: the next step's match and append may start (see `side`)
  if (!M->ev_built) LORB_HIP(ctx, hipEventCreateWithFlags(&M->ev_built, hipEventDisableTiming));
  LORB_HIP(ctx, hipEventRecord(M->ev_built, s));
  M->built = true;
  LORB_TRY(mark(4));
  lorb::ba_plan_window_counts(M->plan, &M->h_P, &M->h_K);
  // 6. LocalPoseOptimization + float write-back of poses (ring) and points (map)
  LORB_TRY(lorb_ba_plan_solve(M->plan, opt));
  LORB_TRY(mark(5));
  // float write-back: poses straight into the ring (Frame::SetPose), points into the map
  LORB_TRY(lorb::ba_plan_result_ring_dev(M->plan, m.ring, m.R, M->t0, m.pos));
  LORB_TRY(mark(6));
  if (M->prof) M->prof_n++;
  return LORB_OK;
}

int lorb_map_set_overlap(lorb_map* M, int32_t enable) {
  if (!M || (enable != 0 && enable != 1)) return LORB_E_INVALID;
  M->overlap = enable == 1;
  if (!M->overlap && M->side) {  // later steps run on the ctx stream only: drain the side stream's work
    LORB_HIP(M->ctx, hipStreamSynchronize(M->side));
  }
  return LORB_OK;
}

int lorb_map_counts(lorb_map* M, int32_t* out, int32_t n) {
  if (!M || !out || n < 0) return LORB_E_INVALID;
  lorb_ctx* ctx = M->ctx;
  LORB_HIP(ctx, hipMemcpyAsync(M->pinned, M->m.cnt, sizeof(int) * 8, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const int32_t v[9] = {M->pinned[0], M->pinned[1], M->t0, M->last_n, M->pinned[3], M->pinned[4], M->pinned[5], M->m.W,
                        M->n_overlapped};
  for (int i = 0; i < n && i < 9; ++i) out[i] = v[i];
  return LORB_OK;
}

int lorb_map_read(lorb_map* M, const lorb_map_state* st) {
  if (!M || !st) return LORB_E_INVALID;
  lorb_ctx* ctx = M->ctx;
  hipStream_t s = ctx->stream;
  const MapDev& m = M->m;
  int32_t c[8];
  LORB_TRY(lorb_map_counts(M, c, 8));
  const size_t P = (size_t)c[0], K = (size_t)c[1];
  auto down = [&](void* h, const void* d, size_t bytes) -> int {
    if (h && bytes) LORB_HIP(ctx, hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s));
    return LORB_OK;
  };
  LORB_TRY(down(st->point, m.pos, sizeof(float) * 3 * P));
  LORB_TRY(down(st->point_desc, m.desc, 32 * P));
  LORB_TRY(down(st->obs_point, m.obs_pt, sizeof(int) * K));
  LORB_TRY(down(st->obs_kf, m.obs_kf, sizeof(int) * K));
  LORB_TRY(down(st->obs_uv, m.obs_uv, sizeof(float) * 2 * K));
  LORB_TRY(down(st->obs_frame, m.obs_frame, sizeof(int) * K));
  LORB_TRY(down(st->match_train, M->mt, sizeof(int) * (size_t)M->last_n));
  std::vector<float> ring(6 * (size_t)m.R);
  LORB_TRY(down(ring.data(), m.ring, sizeof(float) * ring.size()));
  LORB_HIP(ctx, hipStreamSynchronize(s));
  auto slot = [&](int kf) { return ((kf % m.R) + m.R) % m.R; };
  if (st->pose)
    for (int j = 0; j < m.W; ++j)
      for (int q = 0; q < 6; ++q) st->pose[6 * j + q] = ring[6 * (size_t)slot(M->t0 + j) + q];
  if (st->fixed_pose)
    for (int j = 0; j < m.F; ++j)
      for (int q = 0; q < 6; ++q) st->fixed_pose[6 * j + q] = ring[6 * (size_t)slot(M->t0 - 1 - j) + q];
  if (st->summary && M->plan) LORB_TRY(lorb_ba_plan_read(M->plan, nullptr, nullptr, st->summary));
  return LORB_OK;
}

int lorb_map_plan(lorb_map* M, lorb_ba_plan** out) {
  if (!M || !out) return LORB_E_INVALID;
  *out = M->plan;
  return LORB_OK;
}

int lorb_map_destroy(lorb_map* M) {
  if (!M) return LORB_E_INVALID;
  (void)hipStreamSynchronize(M->ctx->stream);
  delete M;
  return LORB_OK;
}

}  // extern "C"
