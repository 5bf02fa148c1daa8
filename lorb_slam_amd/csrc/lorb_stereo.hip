// lorb_stereo.hip -- Frame::ComputeStereoMatches (src/frame.cpp:125-333), SURVEY §8f row 2.
//
// Three launches on the ctx stream:
//   k_st_rows    one workgroup: the row table vRowIndices (:140-161) as CSR in LDS-counted rows;
//                row lists are unordered -- the Hamming search below takes the lexicographic
//                minimum of (distance, iR), which is what the reference's ascending-iR scan with a
//                strict '<' selects, so list order does not matter;
//   k_st_match   one wavefront per left keypoint: band Hamming search (:195-225), 11x11 SAD sweep
//                over +-5 columns on the keypoint's pyramid level (:230-273, 121 row-sums spread
//                over the 64 lanes), parabola fit and disparity checks (:275-313);
//   k_st_reject  one workgroup: the median of the accepted SAD minima by a two-byte radix
//                select (SAD < 2^16: 121 * 510 = 61710), then the 1.5*1.4*median cut (:319-332).
// Edge cases the reference leaves undefined are defined as in oracle/stereo.c (header comment).
#include <algorithm>

#include "lorb_internal.h"

namespace {

constexpr int kStMaxRows = 4096;   // LDS row table bound (level-0 image rows)
constexpr int kStWaves = 4;        // waves (left keypoints) per workgroup in k_st_match

struct Pyr {
  const uint8_t* data;
  int64_t offset[LORB_MAX_LEVELS];
  int rows[LORB_MAX_LEVELS], cols[LORB_MAX_LEVELS], step[LORB_MAX_LEVELS];
  int n_levels;
};

struct Keys {
  const float* x;
  const float* y;
  const int* octave;
  const uint4* desc;
  int n;
};

__device__ __forceinline__ int desc_dist(const uint4* a, const uint4* b) {
  const uint4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

struct Scales { float sf[LORB_MAX_LEVELS]; };

constexpr int kStBandKeys = 8192;  // right keypoints whose band is kept in LDS between the passes

// band [lo, hi] of right keypoint (octave o, row y) clipped to [0, nRows) (:155-160); lo > hi => empty
__device__ __forceinline__ int band_packed(int o, float kpY, const float* s_sf, int n_levels, int nRows) {
  if (o < 0 || o >= n_levels) return 1;  // lo = 1, hi = 0
  const float r = 2.0f * s_sf[o];
  int hi = (int)ceilf(kpY + r), lo = (int)floorf(kpY - r);
  lo = lo < 0 ? 0 : lo;
  hi = hi > nRows - 1 ? nRows - 1 : hi;
  if (lo > hi) return 1;
  return lo | (hi << 16);
}

__global__ __launch_bounds__(1024) void k_st_rows(Keys R, Scales S, int n_levels, int nRows, int* __restrict__ row_off,
                                                  int* __restrict__ row_list) {
  __shared__ int cnt[kStMaxRows + 1];
  __shared__ int s_band[kStBandKeys];
  __shared__ float s_sf[LORB_MAX_LEVELS];
  __shared__ int wsum[16];
  const int t = threadIdx.x;
  if (t < LORB_MAX_LEVELS) s_sf[t] = S.sf[t];
  for (int i = t; i <= nRows; i += 1024) cnt[i] = 0;
  __syncthreads();
  // pass 1: bands (four keypoints per thread per sweep, loads issued together) and row counts
  for (int base = 0; base < R.n; base += 4096) {
    int o[4];
    float y[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int i = base + t + 1024 * k;
      o[k] = i < R.n ? R.octave[i] : -1;
      y[k] = i < R.n ? R.y[i] : 0.0f;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int i = base + t + 1024 * k;
      if (i >= R.n) continue;
      const int bp = band_packed(o[k], y[k], s_sf, n_levels, nRows);
      if (i < kStBandKeys) s_band[i] = bp;
      for (int yi = bp & 0xffff; yi <= (bp >> 16); yi++) atomicAdd(&cnt[yi], 1);
    }
  }
  __syncthreads();
  // exclusive scan of cnt[0..nRows) in place: each thread owns a contiguous chunk
  const int per = (nRows + 1023) / 1024;
  const int b0 = t * per, b1 = min(b0 + per, nRows);
  int s = 0;
  for (int i = b0; i < b1; i++) s += cnt[i];
  int tot;
  int run = lorb::block_excl_scan_1024(s, wsum, &tot);
  for (int i = b0; i < b1; i++) { const int c = cnt[i]; cnt[i] = run; row_off[i] = run; run += c; }
  if (t == 1023) row_off[nRows] = tot;
  __syncthreads();
  // pass 2: fill (row lists are unordered, see the header)
  for (int iR = t; iR < R.n; iR += 1024) {
    const int bp = iR < kStBandKeys ? s_band[iR] : band_packed(R.octave[iR], R.y[iR], s_sf, n_levels, nRows);
    for (int yi = bp & 0xffff; yi <= (bp >> 16); yi++) row_list[atomicAdd(&cnt[yi], 1)] = iR;
  }
}

__device__ __forceinline__ int px(const Pyr& P, int lv, int r, int c) {
  return P.data[P.offset[lv] + (int64_t)r * P.step[lv] + c];
}

__global__ __launch_bounds__(64 * kStWaves) void k_st_match(Keys L, Keys R, Pyr PL, Pyr PR, Scales S, float bf, float b,
                                                            const int* __restrict__ row_off,
                                                            const int* __restrict__ row_list, float* __restrict__ u_right,
                                                            float* __restrict__ depth, int* __restrict__ sad_out) {
  __shared__ int rs[kStWaves][128];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int iL = blockIdx.x * kStWaves + wv;
  if (iL >= L.n) return;
  float ur_o = -1.0f, dp_o = -1.0f;
  int sad_o = -1;
  const int nRows = PL.rows[0];
  const int levelL = L.octave[iL];
  const float vL = L.y[iL], uL = L.x[iL];
  const float minZ = b, minD = 0;
  const float maxD = bf / minZ;
  const float minU = uL - maxD, maxU = uL - minD;
  bool go = levelL >= 0 && levelL < PL.n_levels && vL >= 0.0f && vL < (float)nRows && !(maxU < 0);
  unsigned long long key = (unsigned long long)LORB_TH_HIGH << 32;
  if (go) {
    const int row = (int)vL;
    const int c0 = row_off[row], c1 = row_off[row + 1];
    const uint4* dL = L.desc + 2 * (size_t)iL;
    for (int c = c0 + lane; c < c1; c += 64) {
      const int iR = row_list[c];
      const int o = R.octave[iR];
      if (o < levelL - 1 || o > levelL + 1) continue;
      const float uR = R.x[iR];
      if (uR >= minU && uR <= maxU) {
        const unsigned long long k = ((unsigned long long)desc_dist(dL, R.desc + 2 * (size_t)iR) << 32) | (unsigned)iR;
        key = k < key ? k : key;
      }
    }
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long v = __shfl_xor(key, o, 64);
      key = v < key ? v : key;
    }
  }
  const int bestDist = (int)(key >> 32), bestIdxR = (int)(key & 0xffffffffu);
  go = go && bestDist < (LORB_TH_HIGH + LORB_TH_LOW) / 2;                     // :230
  float scaleduR0 = 0;
  int cu = 0, cv = 0, cr = 0;
  if (go) {
    const float uR0 = R.x[bestIdxR];                                         // :234-238
    const float scaleFactor = 1.0f / S.sf[levelL];
    const float scaleduL = roundf(uL * scaleFactor);
    const float scaledvL = roundf(vL * scaleFactor);
    scaleduR0 = roundf(uR0 * scaleFactor);
    cu = (int)scaleduL; cv = (int)scaledvL; cr = (int)scaleduR0;
    const float iniu = scaleduR0 + 5 - 5, endu = scaleduR0 + 5 + 5 + 1;      // :253-256
    const bool il_in = cv - 5 >= 0 && cu - 5 >= 0 && cv + 6 <= PL.rows[levelL] && cu + 6 <= PL.cols[levelL];
    const bool ir_in = cv - 5 >= 0 && cr - 10 >= 0 && cv + 6 <= PR.rows[levelL] && cr + 11 <= PR.cols[levelL];
    go = il_in && !(iniu < 0 || endu >= PR.cols[levelL]) && ir_in;
  }
  if (go) {
    // 121 row sums: task t -> (incR = t / 11 - 5, dy = t % 11 - 5)
    const int cL = px(PL, levelL, cv, cu);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int t = lane + 64 * h;
      if (t < 121) {
        const int inc = t / 11 - 5, dy = t % 11 - 5;
        const int cR = px(PR, levelL, cv, cr + inc);
        const uint8_t* pl = PL.data + PL.offset[levelL] + (int64_t)(cv + dy) * PL.step[levelL] + (cu - 5);
        const uint8_t* pr = PR.data + PR.offset[levelL] + (int64_t)(cv + dy) * PR.step[levelL] + (cr + inc - 5);
        int s = 0;
#pragma unroll
        for (int dx = 0; dx < 11; dx++) s += abs(((int)pl[dx] - cL) - ((int)pr[dx] - cR));
        rs[wv][t] = s;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int sad = 0;
    if (lane < 11) {
#pragma unroll
      for (int dy = 0; dy < 11; dy++) sad += rs[wv][lane * 11 + dy];
    }
    float vD[11];
#pragma unroll
    for (int i = 0; i < 11; i++) vD[i] = (float)__shfl(sad, i, 64);
    if (lane == 0) {
      int bestSad = INT32_MAX, bestincR = 0;                                  // :246-273
#pragma unroll
      for (int i = 0; i < 11; i++)
        if (vD[i] < (float)bestSad) { bestSad = (int)vD[i]; bestincR = i - 5; }
      if (bestincR != -5 && bestincR != 5) {                                  // :275
        float dist1 = 0, dist2 = 0, dist3 = 0;
#pragma unroll
        for (int i = 1; i < 10; i++)
          if (i == bestincR + 5) { dist1 = vD[i - 1]; dist2 = vD[i]; dist3 = vD[i + 1]; }
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));  // :286
        if (!(deltaR < -1 || deltaR > 1)) {
          float bestuR = S.sf[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);   // :296
          float disparity = (uL - bestuR);
          if (disparity >= minD && disparity < maxD) {                        // :301-313
            if (disparity <= 0) {
              disparity = (float)0.01;
              bestuR = (float)((double)uL - 0.01);
            }
            dp_o = bf / disparity;
            ur_o = bestuR;
            sad_o = bestSad;
          }
        }
      }
    }
  }
  if (lane == 0) { u_right[iL] = ur_o; depth[iL] = dp_o; sad_out[iL] = sad_o; }
}

// wave 0: the 256-bin histogram bucket b holding 0-based rank k, and the rank r within it
__device__ __forceinline__ void select_bucket(const int* hist, int k, int& b, int& r) {
  const int lane = threadIdx.x & 63;
  const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2], h3 = hist[4 * lane + 3];
  const int s = h0 + h1 + h2 + h3;
  int incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  const int ex = incl - s;
  // the owning lane: ex <= k < incl (exactly one lane)
  const unsigned long long m = __ballot(ex <= k && k < incl);
  const int src = __ffsll((long long)m) - 1;
  int kk = k - ex, bb = 4 * lane;
  if (kk >= h0) { kk -= h0; bb++; if (kk >= h1) { kk -= h1; bb++; if (kk >= h2) { kk -= h2; bb++; } } }
  b = __shfl(bb, src, 64);
  r = __shfl(kk, src, 64);
}

__global__ __launch_bounds__(1024) void k_st_reject(int n, const int* __restrict__ sad, float* __restrict__ u_right,
                                                    float* __restrict__ depth) {
  __shared__ int hist[256];
  __shared__ int s_n, s_hi, s_rank, s_med;
  const int t = threadIdx.x;
  if (t < 256) hist[t] = 0;
  if (t == 0) s_n = 0;
  __syncthreads();
  int nloc = 0;
  for (int i = t; i < n; i += 1024) {
    const int v = sad[i];
    if (v >= 0) { nloc++; atomicAdd(&hist[(v >> 8) & 255], 1); }
  }
  atomicAdd(&s_n, nloc);
  __syncthreads();
  const int cnt = s_n;
  if (cnt == 0) return;                                                       // empty: no rejection
  if (t < 64) {  // :320 vDistIdx[size/2]: the bucket holding rank cnt/2
    int b, r;
    select_bucket(hist, cnt / 2, b, r);
    if (t == 0) { s_hi = b; s_rank = r; }
  }
  __syncthreads();
  if (t < 256) hist[t] = 0;
  __syncthreads();
  const int hsel = s_hi;
  for (int i = t; i < n; i += 1024) {
    const int v = sad[i];
    if (v >= 0 && (v >> 8) == hsel) atomicAdd(&hist[v & 255], 1);
  }
  __syncthreads();
  if (t < 64) {
    int b, r;
    select_bucket(hist, s_rank, b, r);
    if (t == 0) s_med = (hsel << 8) | b;
  }
  __syncthreads();
  const float median = (float)s_med;
  const float thDist = 1.5f * 1.4f * median;                                  // :321
  for (int i = t; i < n; i += 1024) {
    const int v = sad[i];
    if (v >= 0 && !((float)v < thDist)) { u_right[i] = -1.0f; depth[i] = -1.0f; }
  }
}

Keys keys_of(const lorb_stereo_keys* k) {
  return Keys{k->x, k->y, k->octave, reinterpret_cast<const uint4*>(k->desc), k->n};
}

Pyr pyr_of(const lorb_image_pyramid* p, const uint8_t* data) {
  Pyr P{};
  P.data = data;
  P.n_levels = p->n_levels;
  for (int l = 0; l < LORB_MAX_LEVELS; l++) {
    P.offset[l] = p->offset[l]; P.rows[l] = p->rows[l]; P.cols[l] = p->cols[l]; P.step[l] = p->step[l];
  }
  return P;
}

int check_pyr(lorb_ctx* ctx, const lorb_image_pyramid* p, int n_levels, const char* side) {
  if (!p || p->n_levels < n_levels || p->n_levels > LORB_MAX_LEVELS || (!p->data && p->n_levels > 0))
    return lorb::set_error(ctx, LORB_E_INVALID, "%s pyramid: n_levels %d < frame levels %d (or no data)", side,
                           p ? p->n_levels : -1, n_levels);
  for (int l = 0; l < p->n_levels; l++)
    if (p->rows[l] < 0 || p->cols[l] < 0 || p->step[l] < p->cols[l] || p->offset[l] < 0)
      return lorb::set_error(ctx, LORB_E_INVALID, "%s pyramid level %d: bad geometry", side, l);
  return LORB_OK;
}

int64_t pyr_bytes(const lorb_image_pyramid* p) {
  int64_t e = 0;
  for (int l = 0; l < p->n_levels; l++)
    if (p->rows[l] > 0) e = std::max<int64_t>(e, p->offset[l] + (int64_t)(p->rows[l] - 1) * p->step[l] + p->cols[l]);
  return e;
}

enum { S_ST = 48 };  // scratch slots S_ST .. S_ST+15

int enqueue_stereo(lorb_ctx* ctx, const lorb_frame_params* fp, const Keys& L, const Keys& R, const Pyr& PL,
                   const Pyr& PR, float* d_ur, float* d_dp) {
  const int nRows = PL.rows[0];
  if (nRows > kStMaxRows)
    return lorb::set_error(ctx, LORB_E_INVALID, "image rows %d > %d", nRows, kStMaxRows);
  Scales S{};
  for (int l = 0; l < LORB_MAX_LEVELS; l++) S.sf[l] = fp->scale_factors[l];
  int *row_off, *row_list, *sad;
  // each right keypoint covers at most ceil(y+r) - floor(y-r) + 1 rows
  float rmax = 0;
  for (int l = 0; l < fp->n_levels; l++) rmax = std::max(rmax, 2.0f * fp->scale_factors[l]);
  const size_t per = (size_t)(2.0f * rmax) + 3;
  LORB_TRY(lorb::scratch_t(ctx, S_ST + 0, (size_t)nRows + 1, &row_off));
  LORB_TRY(lorb::scratch_t(ctx, S_ST + 1, std::max<size_t>((size_t)R.n * per, 1), &row_list));
  LORB_TRY(lorb::scratch_t(ctx, S_ST + 2, std::max<size_t>((size_t)L.n, 1), &sad));
  hipLaunchKernelGGL(k_st_rows, dim3(1), dim3(1024), 0, ctx->stream, R, S, fp->n_levels, nRows, row_off, row_list);
  {
    lorb::KernelTimer kt(ctx, LORB_K_STEREO);
    hipLaunchKernelGGL(k_st_match, dim3(lorb::ceil_div(L.n, kStWaves)), dim3(64 * kStWaves), 0, ctx->stream, L, R, PL,
                       PR, S, fp->bf, fp->b, row_off, row_list, d_ur, d_dp, sad);
  }
  hipLaunchKernelGGL(k_st_reject, dim3(1), dim3(1024), 0, ctx->stream, L.n, sad, d_ur, d_dp);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

int check_args(lorb_ctx* ctx, const lorb_frame_params* fp, const lorb_stereo_keys* l, const lorb_stereo_keys* r,
               const lorb_image_pyramid* pl, const lorb_image_pyramid* pr) {
  if (!fp || !l || !r || !pl || !pr) return lorb::set_error(ctx, LORB_E_INVALID, "null argument");
  if (l->n < 0 || r->n < 0) return lorb::set_error(ctx, LORB_E_INVALID, "negative keypoint count");
  if (fp->n_levels < 1 || fp->n_levels > LORB_MAX_LEVELS)
    return lorb::set_error(ctx, LORB_E_INVALID, "n_levels %d out of range", fp->n_levels);
  if ((l->n && (!l->x || !l->y || !l->octave || !l->desc)) || (r->n && (!r->x || !r->y || !r->octave || !r->desc)))
    return lorb::set_error(ctx, LORB_E_INVALID, "keypoint arrays missing");
  LORB_TRY(check_pyr(ctx, pl, fp->n_levels, "left"));
  LORB_TRY(check_pyr(ctx, pr, fp->n_levels, "right"));
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_compute_stereo_matches_dev(lorb_ctx* ctx, const lorb_frame_params* frame, const lorb_stereo_keys* d_left,
                                    const lorb_stereo_keys* d_right, const lorb_image_pyramid* d_left_pyr,
                                    const lorb_image_pyramid* d_right_pyr, float* d_u_right, float* d_depth) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_args(ctx, frame, d_left, d_right, d_left_pyr, d_right_pyr));
  if (d_left->n == 0) return LORB_OK;
  if (!d_u_right || !d_depth) return lorb::set_error(ctx, LORB_E_INVALID, "null output");
  return enqueue_stereo(ctx, frame, keys_of(d_left), keys_of(d_right), pyr_of(d_left_pyr, d_left_pyr->data),
                        pyr_of(d_right_pyr, d_right_pyr->data), d_u_right, d_depth);
}

int lorb_compute_stereo_matches(lorb_ctx* ctx, const lorb_frame_params* frame, const lorb_stereo_keys* left,
                                const lorb_stereo_keys* right, const lorb_image_pyramid* left_pyr,
                                const lorb_image_pyramid* right_pyr, float* u_right, float* depth) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_args(ctx, frame, left, right, left_pyr, right_pyr));
  const int nL = left->n, nR = right->n;
  if (nL == 0) return LORB_OK;
  if (!u_right || !depth) return lorb::set_error(ctx, LORB_E_INVALID, "null output");
  Keys L{}, R{};
  L.n = nL; R.n = nR;
  uint8_t *dl, *dr;
  LORB_TRY(lorb::upload_t(ctx, S_ST + 3, left->x, nL, const_cast<float**>(&L.x)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 4, left->y, nL, const_cast<float**>(&L.y)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 5, left->octave, nL, const_cast<int**>(&L.octave)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 6, left->desc, (size_t)nL * 32, &dl));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 7, right->x, nR, const_cast<float**>(&R.x)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 8, right->y, nR, const_cast<float**>(&R.y)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 9, right->octave, nR, const_cast<int**>(&R.octave)));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 10, right->desc, (size_t)nR * 32, &dr));
  L.desc = reinterpret_cast<const uint4*>(dl);
  R.desc = reinterpret_cast<const uint4*>(dr);
  uint8_t *pl, *pr;
  LORB_TRY(lorb::upload_t(ctx, S_ST + 11, left_pyr->data, (size_t)pyr_bytes(left_pyr), &pl));
  LORB_TRY(lorb::upload_t(ctx, S_ST + 12, right_pyr->data, (size_t)pyr_bytes(right_pyr), &pr));
  float *dur, *ddp;
  LORB_TRY(lorb::scratch_t(ctx, S_ST + 13, (size_t)nL, &dur));
  LORB_TRY(lorb::scratch_t(ctx, S_ST + 14, (size_t)nL, &ddp));
  LORB_TRY(enqueue_stereo(ctx, frame, L, R, pyr_of(left_pyr, pl), pyr_of(right_pyr, pr), dur, ddp));
  LORB_HIP(ctx, hipMemcpyAsync(u_right, dur, sizeof(float) * nL, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(depth, ddp, sizeof(float) * nL, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

}  // extern "C"
