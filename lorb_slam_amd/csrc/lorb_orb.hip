// lorb_orb.hip -- the descriptor stage of ORBextractor::operator() (src/ORBextractor.cpp:1087-1154),
// SURVEY §8f row 3:
//   k_orb_blur  GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) of every pyramid level
//               (:1131-1132), OpenCV 3.1's 8U fixed-point separable smoothing (integer taps =
//               round(256 k), integer row and column passes, (s + 2^15) >> 16, saturate); one
//               workgroup per 64 x 16 output tile, the 70 x 22 input tile and the row pass in LDS;
//   k_orb_desc  one wavefront per keypoint: IC_Angle on the raw level (:79-107; lane = patch
//               column, integer moments reduced across the wave) with cv::fastAtan2, then the
//               rBRIEF test pairs on the blurred level (:110-150; lane = four pairs, nibbles
//               merged by a lane shuffle).  The 256-pair pattern is the caller's (the reference's
//               bit_pattern_31_), staged in LDS.
// Integer sums make the blur and the moments order-independent, so results are bit-exact with
// oracle/orb.c; the float expressions follow the reference's order (-ffp-contract=off).
#include <algorithm>
#include <cfloat>
#include <vector>
#include <cmath>

#include "lorb_internal.h"

namespace {

constexpr int kHalfPatch = 15;
constexpr int kTileW = 64, kTileH = 16;

struct OrbPyr {
  const uint8_t* data;
  uint8_t* blur;  // same layout (offsets / steps) as data
  int64_t offset[LORB_MAX_LEVELS];
  int rows[LORB_MAX_LEVELS], cols[LORB_MAX_LEVELS], step[LORB_MAX_LEVELS];
  int tile_off[LORB_MAX_LEVELS + 1];  // first tile of each level
  int tiles_x[LORB_MAX_LEVELS];
  int n_levels;
  int k[7];                           // fixed-point Gaussian taps
  int umax[kHalfPatch + 1];
};

__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

__global__ __launch_bounds__(256) void k_orb_blur(OrbPyr P) {
  __shared__ int in[kTileH + 6][kTileW + 6 + 1];
  __shared__ int rowp[kTileH + 6][kTileW + 1];
  const int b = blockIdx.x, t = threadIdx.x;
  int l = 0;
  while (l + 1 < P.n_levels && b >= P.tile_off[l + 1]) ++l;
  const int tb = b - P.tile_off[l];
  const int x0 = (tb % P.tiles_x[l]) * kTileW, y0 = (tb / P.tiles_x[l]) * kTileH;
  const int rows = P.rows[l], cols = P.cols[l], step = P.step[l];
  const uint8_t* src = P.data + P.offset[l];
  for (int e = t; e < (kTileH + 6) * (kTileW + 6); e += 256) {
    const int r = e / (kTileW + 6), c = e - r * (kTileW + 6);
    const int yy = reflect101(y0 + r - 3, rows), xx = reflect101(x0 + c - 3, cols);
    in[r][c] = src[(int64_t)yy * step + xx];
  }
  __syncthreads();
  for (int e = t; e < (kTileH + 6) * kTileW; e += 256) {  // row pass (every staged row)
    const int r = e / kTileW, c = e - r * kTileW;
    int s = 0;
#pragma unroll
    for (int d = 0; d < 7; ++d) s += P.k[d] * in[r][c + d];
    rowp[r][c] = s;
  }
  __syncthreads();
  uint8_t* dst = P.blur + P.offset[l];
  for (int e = t; e < kTileH * kTileW; e += 256) {  // column pass
    const int r = e / kTileW, c = e - r * kTileW;
    const int y = y0 + r, x = x0 + c;
    if (y >= rows || x >= cols) continue;
    int s = 0;
#pragma unroll
    for (int d = 0; d < 7; ++d) s += P.k[d] * rowp[r + d][c];
    const int v = (s + (1 << 15)) >> 16;
    dst[(int64_t)y * step + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
  }
}

// cv::fastAtan2 (OpenCV 3.1), degrees
__device__ __forceinline__ float fast_atan2(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / 3.1415926535897932384626433832795);
  const float p3 = -0.3258083974640975f * (float)(180 / 3.1415926535897932384626433832795);
  const float p5 = 0.1555786518463281f * (float)(180 / 3.1415926535897932384626433832795);
  const float p7 = -0.04432655554792128f * (float)(180 / 3.1415926535897932384626433832795);
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + (float)DBL_EPSILON);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + (float)DBL_EPSILON);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kDescWaves = 4;

__global__ __launch_bounds__(64 * kDescWaves) void k_orb_desc(OrbPyr P, int n, const float* __restrict__ kx,
                                                              const float* __restrict__ ky,
                                                              const int* __restrict__ klev,
                                                              const int* __restrict__ pattern,
                                                              float* __restrict__ angle_out,
                                                              uint8_t* __restrict__ desc_out) {
  __shared__ int s_pat[1024];
  for (int e = threadIdx.x; e < 1024; e += 64 * kDescWaves) s_pat[e] = pattern[e];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * kDescWaves + (threadIdx.x >> 6);
  if (i >= n) return;
  const int l = klev[i];
  if (l < 0 || l >= P.n_levels) return;  // validated on the host for the host entry point
  const int step = P.step[l];
  const int cx = __float2int_rn(kx[i]), cy = __float2int_rn(ky[i]);  // cvRound
  // IC_Angle: lane u + 15 (u in [-15, 15]) sums column u over the disc, rows split in two halves
  int m10 = 0, m01 = 0;
  {
    const uint8_t* center = P.data + P.offset[l] + (int64_t)cy * step + cx;
    const int u = (lane & 31) - kHalfPatch;
    const bool half = lane >= 32;  // rows v > 0 for the upper half-wave, v <= 0 for the lower
    if ((lane & 31) < 2 * kHalfPatch + 1) {
      for (int k = 0; k <= kHalfPatch; ++k) {
        const int v = half ? k + 1 : -k;
        if (v > kHalfPatch) break;
        const int av = v < 0 ? -v : v;
        if ((u < 0 ? -u : u) <= P.umax[av]) {
          const int val = center[u + v * step];
          m10 += u * val;
          m01 += v * val;
        }
      }
    }
    m10 = wave_isum(m10);
    m01 = wave_isum(m01);
  }
  const float ang = fast_atan2((float)m01, (float)m10);
  // computeOrbDescriptor on the blurred level
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  const float angle = ang * factorPI;
  const float a = (float)cos((double)angle), b = (float)sin((double)angle);
  const uint8_t* center = P.blur + P.offset[l] + (int64_t)cy * step + cx;
  int nib = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int* p0 = s_pat + 4 * (4 * lane + k);  // pair 4 lane + k = bit (4 lane + k) & 7 of byte lane / 2
    const int t0 = center[__float2int_rn(p0[0] * b + p0[1] * a) * step + __float2int_rn(p0[0] * a - p0[1] * b)];
    const int t1 = center[__float2int_rn(p0[2] * b + p0[3] * a) * step + __float2int_rn(p0[2] * a - p0[3] * b)];
    nib |= (t0 < t1) << k;
  }
  const int hi = __shfl_down(nib, 1, 64);
  if ((lane & 1) == 0) desc_out[32 * (size_t)i + (lane >> 1)] = (uint8_t)(nib | (hi << 4));
  if (lane == 0) angle_out[i] = ang;
}

// cv::getGaussianKernel(7, 2, CV_32F) * 256, rounded (convertTo CV_32S, float arithmetic)
void gauss_taps(int* k7) {
  float cf[7];
  double sum = 0;
  const double sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX);
  for (int i = 0; i < 7; i++) {
    const double x = i - (7 - 1) * 0.5;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) cf[i] = (float)(cf[i] * sum);
  for (int i = 0; i < 7; i++) k7[i] = (int)std::nearbyint(cf[i] * 256.f);
}

// ORBextractor::ORBextractor, src/ORBextractor.cpp:469-483
void orb_umax(int* umax) {
  int v, v0;
  const int vmax = (int)std::floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
  const int vmin = (int)std::ceil(kHalfPatch * std::sqrt(2.f) / 2);
  const double hp2 = kHalfPatch * kHalfPatch;
  for (v = 0; v <= vmax; ++v) umax[v] = (int)std::nearbyint(std::sqrt(hp2 - v * v));
  for (v = kHalfPatch, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
}

int64_t pyr_extent(const lorb_image_pyramid* p) {
  int64_t e = 0;
  for (int l = 0; l < p->n_levels; l++)
    if (p->rows[l] > 0) e = std::max<int64_t>(e, p->offset[l] + (int64_t)(p->rows[l] - 1) * p->step[l] + p->cols[l]);
  return e;
}

int check_orb(lorb_ctx* ctx, const lorb_image_pyramid* p, int n) {
  if (!p || n < 0) return lorb::set_error(ctx, LORB_E_INVALID, "null pyramid or negative count");
  if (p->n_levels < 1 || p->n_levels > LORB_MAX_LEVELS || !p->data)
    return lorb::set_error(ctx, LORB_E_INVALID, "pyramid n_levels %d out of range (or no data)", p->n_levels);
  for (int l = 0; l < p->n_levels; l++)
    if (p->rows[l] < 1 || p->cols[l] < 1 || p->step[l] < p->cols[l] || p->offset[l] < 0)
      return lorb::set_error(ctx, LORB_E_INVALID, "pyramid level %d: bad geometry", l);
  return LORB_OK;
}

enum { S_ORB = 48 };  // shares the stereo family's slots (calls on one ctx are serialized)

int enqueue_orb(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const uint8_t* d_data, int n, const float* d_x,
                const float* d_y, const int* d_lev, const int* d_pat, float* d_ang, uint8_t* d_desc) {
  OrbPyr P{};
  P.data = d_data;
  P.n_levels = pyr->n_levels;
  int tiles = 0;
  for (int l = 0; l < pyr->n_levels; l++) {
    P.offset[l] = pyr->offset[l]; P.rows[l] = pyr->rows[l]; P.cols[l] = pyr->cols[l]; P.step[l] = pyr->step[l];
    P.tile_off[l] = tiles;
    P.tiles_x[l] = (pyr->cols[l] + kTileW - 1) / kTileW;
    tiles += P.tiles_x[l] * ((pyr->rows[l] + kTileH - 1) / kTileH);
  }
  P.tile_off[pyr->n_levels] = tiles;
  gauss_taps(P.k);
  orb_umax(P.umax);
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 0, (size_t)pyr_extent(pyr), &P.blur));
  hipLaunchKernelGGL(k_orb_blur, dim3(tiles), dim3(256), 0, ctx->stream, P);
  if (n > 0)
    hipLaunchKernelGGL(k_orb_desc, dim3(lorb::ceil_div(n, kDescWaves)), dim3(64 * kDescWaves), 0, ctx->stream, P, n,
                       d_x, d_y, d_lev, d_pat, d_ang, d_desc);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
}

// ---- detection stage (src/ORBextractor.cpp:898-1000): per-cell cv::FAST ------------------

constexpr int kOff16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                               {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

struct FastCell {
  int level, ini_x, ini_y, w, h, out_base;
};

// cornerScore<16> (OpenCV 3.1 fast_score.cpp) on the LDS cell image (row stride w)
__device__ __forceinline__ int fast_score(const uint8_t* ptr, const int* pixel, int threshold) {
  int d[25];
  const int v = ptr[0];
#pragma unroll
  for (int k = 0; k < 25; k++) d[k] = v - ptr[pixel[k]];
  int a0 = threshold;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int a = min(d[k + 1], d[k + 2]);
    a = min(a, d[k + 3]);
    if (a <= a0) continue;
#pragma unroll
    for (int m = 4; m <= 8; m++) a = min(a, d[k + m]);
    a0 = max(a0, min(a, d[k]));
    a0 = max(a0, min(a, d[k + 9]));
  }
  int b0 = -a0;
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    int b = max(d[k + 1], d[k + 2]);
#pragma unroll
    for (int m = 3; m <= 5; m++) b = max(b, d[k + m]);
    if (b >= b0) continue;
#pragma unroll
    for (int m = 6; m <= 8; m++) b = max(b, d[k + m]);
    b0 = min(b0, max(b, d[k]));
    b0 = min(b0, max(b, d[k + 9]));
  }
  return -b0 - 1;
}

// One 1024-thread workgroup per cell: the cell image in LDS, FAST_t<16> detection + score for
// every inner pixel, 3x3 non-maximum suppression, the iniThFAST -> minThFAST fallback when at
// most 3 corners survive, and the survivors written in FAST's row-major order (block scan).
__global__ __launch_bounds__(1024) void k_orb_fast(const uint8_t* __restrict__ data, OrbPyr P,
                                                   const FastCell* __restrict__ cells, int ini_th, int min_th,
                                                   float* __restrict__ ox, float* __restrict__ oy,
                                                   float* __restrict__ oresp, int* __restrict__ ocount) {
  extern __shared__ uint8_t lds[];
  __shared__ int s_count, wsum[16];
  __shared__ int pixel[25];
  const FastCell c = cells[blockIdx.x];
  const int w = c.w, h = c.h, n = w * h, t = threadIdx.x;
  uint8_t* img = lds;
  uint8_t* score = lds + n;
  uint8_t* corner = lds + 2 * n;
  const uint8_t* src = data + P.offset[c.level] + (int64_t)c.ini_y * P.step[c.level] + c.ini_x;
  const int step = P.step[c.level];
  for (int p0 = t; p0 < n; p0 += 1024 * 8) {  // eight loads in flight per thread
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int p = p0 + 1024 * u;
      const int i = p / w, j = p - i * w;
      v[u] = p < n ? src[(int64_t)i * step + j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (p0 + 1024 * u < n) img[p0 + 1024 * u] = v[u];
  }
  if (t < 25) pixel[t] = kOff16[t & 15][0] + kOff16[t & 15][1] * w;
  for (int pass = 0; pass < 2; ++pass) {
    const int th = min(max(pass ? min_th : ini_th, 0), 255);
    for (int p = t; p < n; p += 1024) { score[p] = 0; corner[p] = 0; }
    if (t == 0) s_count = 0;
    __syncthreads();
    for (int p = t; p < n; p += 1024) {
      const int i = p / w, j = p - i * w;
      if (i < 3 || i >= h - 3 || j < 3 || j >= w - 3) continue;
      const uint8_t* ptr = img + p;
      const int v = ptr[0];
      auto cat = [&](int k) { const int e = ptr[pixel[k]] - v; return e < -th ? 1 : (e > th ? 2 : 0); };
      int d = cat(0) | cat(8);
      if (d == 0) continue;
      d &= cat(2) | cat(10);
      d &= cat(4) | cat(12);
      d &= cat(6) | cat(14);
      if (d == 0) continue;
      d &= cat(1) | cat(9);
      d &= cat(3) | cat(11);
      d &= cat(5) | cat(13);
      d &= cat(7) | cat(15);
      bool is = false;
      if (d & 1) {
        const int vt = v - th;
        int count = 0;
        for (int k = 0; k < 25; k++) {
          if (ptr[pixel[k]] < vt) { if (++count > 8) { is = true; break; } }
          else count = 0;
        }
      }
      if (!is && (d & 2)) {
        const int vt = v + th;
        int count = 0;
        for (int k = 0; k < 25; k++) {
          if (ptr[pixel[k]] > vt) { if (++count > 8) { is = true; break; } }
          else count = 0;
        }
      }
      if (is) { corner[p] = 1; score[p] = (uint8_t)fast_score(ptr, pixel, th); }
    }
    __syncthreads();
    int mine = 0;
    for (int p = t; p < n; p += 1024) {
      if (!corner[p]) continue;
      const int s = score[p];
      mine += s > score[p - w - 1] && s > score[p - w] && s > score[p - w + 1] && s > score[p - 1] && s > score[p + 1] &&
              s > score[p + w - 1] && s > score[p + w] && s > score[p + w + 1];
    }
    if (mine) atomicAdd(&s_count, mine);
    __syncthreads();
    if (pass == 0 && s_count > 3) break;  // uniform: s_count is read by every thread after the barrier
    __syncthreads();
  }
  int run = 0;
  for (int base = 0; base < n; base += 1024) {
    const int p = base + t;
    bool keep = false;
    if (p < n && corner[p]) {
      const int s = score[p];
      keep = s > score[p - w - 1] && s > score[p - w] && s > score[p - w + 1] && s > score[p - 1] && s > score[p + 1] &&
             s > score[p + w - 1] && s > score[p + w] && s > score[p + w + 1];
    }
    int tot;
    const int ex = lorb::block_excl_scan_1024(keep ? 1 : 0, wsum, &tot);
    if (keep) {
      const int i = p / w, j = p - i * w;
      const int o = c.out_base + run + ex;
      ox[o] = (float)(j + c.ini_x); oy[o] = (float)(i + c.ini_y); oresp[o] = (float)score[p];
    }
    run += tot;
  }
  if (t == 0) ocount[blockIdx.x] = run;
}

// the cell grid of one level, src/ORBextractor.cpp:903-990 (see oracle/fast.c)
int orb_cells(int rows, int cols, int n_desired, float image_ratio, std::vector<int>& cells) {
  const int EDGE = 19;
  const int levelCols = (int)std::sqrt((float)n_desired / (5 * image_ratio));
  const int levelRows = (int)(image_ratio * levelCols);
  if (levelCols < 1 || levelRows < 1) return -1;
  const int minBorderX = EDGE, minBorderY = EDGE, maxBorderX = cols - EDGE, maxBorderY = rows - EDGE;
  const int W = maxBorderX - minBorderX, H = maxBorderY - minBorderY;
  const int cellW = (int)std::ceil((float)W / levelCols), cellH = (int)std::ceil((float)H / levelRows);
  cells.assign(4 * (size_t)levelRows * levelCols, 0);
  float hY = (float)(cellH + 6);
  for (int i = 0; i < levelRows; i++) {
    const float iniY = (float)(minBorderY + i * cellH - 3);
    bool skip_row = false;
    if (i == levelRows - 1) {
      hY = maxBorderY + 3 - iniY;
      if (hY <= 0) skip_row = true;
    }
    float hX = (float)(cellW + 6);
    for (int j = 0; j < levelCols; j++) {
      const float iniX = (float)(minBorderX + j * cellW - 3);
      int* c = &cells[4 * (size_t)(i * levelCols + j)];
      c[0] = (int)iniX; c[1] = (int)iniY;
      if (skip_row) continue;
      if (j == levelCols - 1) {
        hX = maxBorderX + 3 - iniX;
        if (hX <= 0) continue;
      }
      c[2] = (int)hX; c[3] = (int)hY;
    }
  }
  return levelRows * levelCols;
}

// ---- ComputePyramid (src/ORBextractor.cpp:1157-1184): OpenCV 3.1 8U INTER_LINEAR resize ----
// Host: the tap tables exactly as imgwarp.cpp builds them (double -> float coordinates,
// cvRound(c * 2048) as short).  Device: one thread per destination pixel, the two source rows'
// integer horizontal taps, then the vertical combine -- SSE2 VResizeLinearVec_32s8u arithmetic for
// columns < xs and the scalar FixedPtCast for the rest (oracle/orb.c states the formulas).
__device__ __forceinline__ int sat16d(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

__global__ __launch_bounds__(256) void k_orb_resize(const uint8_t* __restrict__ src, int sh, int sw, int sstep,
                                                    uint8_t* __restrict__ dst, int dh, int dw, int dstep,
                                                    const int* __restrict__ xofs, const short2* __restrict__ ia,
                                                    const int* __restrict__ yofs, const short2* __restrict__ ib,
                                                    int xmax, int xs) {
  const int dx = blockIdx.x * 64 + (threadIdx.x & 63);
  const int dy = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (dx >= dw || dy >= dh) return;
  const int sx = xofs[dx];
  const short2 a = ia[dx];
  int r[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    int sy = yofs[dy] + k;
    sy = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
    const uint8_t* S = src + (int64_t)sy * sstep;
    r[k] = dx < xmax ? S[sx] * a.x + S[sx + 1] * a.y : S[sx] * 2048;
  }
  const short2 b = ib[dy];
  int v;
  if (dx < xs) {
    const int x0 = sat16d(r[0] >> 4), y0 = sat16d(r[1] >> 4);
    const int m0 = (x0 * b.x) >> 16, m1 = (y0 * b.y) >> 16;
    const int sum = sat16d(m0 + m1);
    v = sat16d(sum + 2) >> 2;
  } else {
    v = (r[0] * b.x + r[1] * b.y + (1 << 21)) >> 22;
  }
  dst[(int64_t)dy * dstep + dx] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

short sat16h(int v) { return (short)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

void resize_tabs(int ssize, int dsize, std::vector<int>& ofs, std::vector<short2>& a, int* xmax_out, bool clamp) {
  const double inv_scale = (double)dsize / ssize, scale = 1. / inv_scale;
  int xmax = dsize;
  ofs.resize(dsize); a.resize(dsize);
  for (int dx = 0; dx < dsize; dx++) {
    float f = (float)((dx + 0.5) * scale - 0.5);
    int s = (int)std::floor(f);
    f -= s;
    if (clamp) {
      if (s < 0) { f = 0; s = 0; }
      if (s + 1 >= ssize) {
        xmax = std::min(xmax, dx);
        if (s >= ssize - 1) { f = 0; s = ssize - 1; }
      }
    }
    ofs[dx] = s;
    a[dx].x = sat16h((int)std::nearbyint((1.f - f) * 2048));
    a[dx].y = sat16h((int)std::nearbyint(f * 2048));
  }
  if (xmax_out) *xmax_out = xmax;
}

int simd_cols(int width) {
  int x = 0;
  while (x <= width - 16) x += 16;
  while (x < width - 4) x += 4;
  return x;
}

int pyramid_layout(int rows, int cols, int n_levels, const float* sf, lorb_image_pyramid* P) {
  std::memset(P, 0, sizeof(*P));
  P->n_levels = n_levels;
  int64_t off = 0;
  for (int l = 0; l < n_levels; l++) {
    const float inv = 1.0f / sf[l];
    P->cols[l] = (int)std::nearbyint((float)cols * inv);
    P->rows[l] = (int)std::nearbyint((float)rows * inv);
    P->step[l] = P->cols[l];
    P->offset[l] = off;
    off += (int64_t)P->rows[l] * P->cols[l];
  }
  return (int)std::min<int64_t>(off, INT32_MAX);
}

int enqueue_pyramid(lorb_ctx* ctx, const uint8_t* d_img, int rows, int cols, int step, const lorb_image_pyramid& P,
                    uint8_t* d_out) {
  LORB_HIP(ctx, hipMemcpy2DAsync(d_out, P.cols[0], d_img, step, P.cols[0], P.rows[0], hipMemcpyDeviceToDevice,
                                 ctx->stream));
  // the tap tables stay alive until the stream has consumed them (synchronised below)
  std::vector<std::vector<int>> keep_i(2 * P.n_levels);
  std::vector<std::vector<short2>> keep_s(2 * P.n_levels);
  for (int l = 1; l < P.n_levels; l++) {
    std::vector<int>& xofs = keep_i[2 * l];
    std::vector<int>& yofs = keep_i[2 * l + 1];
    std::vector<short2>& ia = keep_s[2 * l];
    std::vector<short2>& ib = keep_s[2 * l + 1];
    int xmax;
    resize_tabs(P.cols[l - 1], P.cols[l], xofs, ia, &xmax, true);
    resize_tabs(P.rows[l - 1], P.rows[l], yofs, ib, nullptr, false);
    int *dxo, *dyo;
    short2 *dia, *dib;
    LORB_TRY(lorb::upload_t(ctx, S_ORB + 8 + 4 * (l & 1), xofs.data(), xofs.size(), &dxo));
    LORB_TRY(lorb::upload_t(ctx, S_ORB + 9 + 4 * (l & 1), ia.data(), ia.size(), &dia));
    LORB_TRY(lorb::upload_t(ctx, S_ORB + 10 + 4 * (l & 1), yofs.data(), yofs.size(), &dyo));
    LORB_TRY(lorb::upload_t(ctx, S_ORB + 11 + 4 * (l & 1), ib.data(), ib.size(), &dib));
    const dim3 grid(lorb::ceil_div(P.cols[l], 64), lorb::ceil_div(P.rows[l], 4));
    hipLaunchKernelGGL(k_orb_resize, grid, dim3(256), 0, ctx->stream, d_out + P.offset[l - 1], P.rows[l - 1],
                       P.cols[l - 1], P.step[l - 1], d_out + P.offset[l], P.rows[l], P.cols[l], P.step[l], dxo, dia, dyo,
                       dib, xmax, simd_cols(P.cols[l]));
  }
  LORB_CHECK_LAUNCH(ctx);
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_orb_describe_dev(lorb_ctx* ctx, const lorb_image_pyramid* d_pyr, int32_t n, const float* d_x,
                          const float* d_y, const int32_t* d_level, const int32_t* d_pattern, float* d_angle,
                          uint8_t* d_desc) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, d_pyr, n));
  if (n > 0 && (!d_x || !d_y || !d_level || !d_pattern || !d_angle || !d_desc))
    return lorb::set_error(ctx, LORB_E_INVALID, "null keypoint / pattern / output array");
  return enqueue_orb(ctx, d_pyr, d_pyr->data, n, d_x, d_y, d_level, d_pattern, d_angle, d_desc);
}

int lorb_orb_describe(lorb_ctx* ctx, const lorb_image_pyramid* pyr, int32_t n, const float* x, const float* y,
                      const int32_t* level, const int32_t* pattern, float* angle, uint8_t* desc) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, n));
  if (n > 0 && (!x || !y || !level || !pattern || !angle || !desc))
    return lorb::set_error(ctx, LORB_E_INVALID, "null keypoint / pattern / output array");
  // the defined domain: every patch and test pair inside the level (the extractor keeps keypoints
  // EDGE_THRESHOLD = 19 pixels from each level border, src/ORBextractor.cpp:76, 912-915)
  for (int i = 0; i < n; i++) {
    const int l = level[i];
    if (l < 0 || l >= pyr->n_levels)
      return lorb::set_error(ctx, LORB_E_INVALID, "keypoint %d: level %d out of range", i, l);
    const long cx = std::lrint(x[i]), cy = std::lrint(y[i]);
    if (cx < 19 || cy < 19 || cx > pyr->cols[l] - 20 || cy > pyr->rows[l] - 20)
      return lorb::set_error(ctx, LORB_E_INVALID, "keypoint %d (%g, %g) closer than 19 px to level %d border", i,
                             (double)x[i], (double)y[i], l);
  }
  uint8_t* dd;
  float *dx, *dy, *dang;
  int *dl, *dp;
  uint8_t* ddesc;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 1, pyr->data, (size_t)pyr_extent(pyr), &dd));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 2, x, (size_t)n, &dx));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 3, y, (size_t)n, &dy));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 4, level, (size_t)n, &dl));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 5, pattern, (size_t)1024, &dp));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 6, (size_t)std::max(n, 1), &dang));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 7, (size_t)std::max(n, 1) * 32, &ddesc));
  LORB_TRY(enqueue_orb(ctx, pyr, dd, n, dx, dy, dl, dp, dang, ddesc));
  if (n > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(angle, dang, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(desc, ddesc, (size_t)32 * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}


int lorb_orb_fast_cells(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired, int32_t ini_th,
                        int32_t min_th, int32_t max_keypoints, float* x, float* y, float* response, int32_t max_cells,
                        int32_t* cell_base, int32_t* cell_off, int32_t* n_keypoints) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, 0));
  if (!n_desired || !cell_base || !cell_off || !n_keypoints || max_keypoints < 0 || max_cells < 0)
    return lorb::set_error(ctx, LORB_E_INVALID, "null argument");
  const float ratio = (float)pyr->cols[0] / pyr->rows[0];
  std::vector<FastCell> hc;       // launched cells
  std::vector<int> slot;          // launched cell -> global cell index
  int nc = 0, cap_total = 0;
  std::vector<int> cells;
  for (int l = 0; l < pyr->n_levels; l++) {
    const int ncl = orb_cells(pyr->rows[l], pyr->cols[l], n_desired[l], ratio, cells);
    if (ncl < 0) return lorb::set_error(ctx, LORB_E_INVALID, "level %d: degenerate cell grid (%d features)", l, n_desired[l]);
    if (nc + ncl > max_cells) return lorb::set_error(ctx, LORB_E_INVALID, "more than max_cells = %d cells", max_cells);
    cell_base[l] = nc;
    for (int c = 0; c < ncl; c++) {
      const int* g = &cells[4 * (size_t)c];
      if (g[2] <= 0 || g[3] <= 0) continue;
      if (g[0] < 0 || g[1] < 0 || g[0] + g[2] > pyr->cols[l] || g[1] + g[3] > pyr->rows[l])
        return lorb::set_error(ctx, LORB_E_INVALID, "level %d cell %d outside the image", l, c);
      if (3 * g[2] * g[3] > 96 * 1024)
        return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "cell %d x %d exceeds the LDS tile", g[2], g[3]);
      hc.push_back(FastCell{l, g[0], g[1], g[2], g[3], cap_total});
      slot.push_back(nc + c);
      cap_total += ((g[2] + 1) / 2) * ((g[3] + 1) / 2);  // 3x3 maxima are never 8-adjacent
    }
    nc += ncl;
  }
  cell_base[pyr->n_levels] = nc;
  OrbPyr P{};
  for (int l = 0; l < pyr->n_levels; l++) { P.offset[l] = pyr->offset[l]; P.step[l] = pyr->step[l]; }
  uint8_t* dd;
  FastCell* dcells;
  float *dx, *dy, *dr;
  int* dcnt;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 1, pyr->data, (size_t)pyr_extent(pyr), &dd));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 2, hc.data(), hc.size(), &dcells));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 3, (size_t)std::max(cap_total, 1), &dx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 4, (size_t)std::max(cap_total, 1), &dy));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 5, (size_t)std::max(cap_total, 1), &dr));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 6, std::max<size_t>(hc.size(), 1), &dcnt));
  int max_lds = 0;
  for (const FastCell& f : hc) max_lds = std::max(max_lds, 3 * f.w * f.h);
  if (!hc.empty())
    hipLaunchKernelGGL(k_orb_fast, dim3((unsigned)hc.size()), dim3(1024), (size_t)max_lds, ctx->stream, dd, P,
                       dcells, ini_th, min_th, dx, dy, dr, dcnt);
  LORB_CHECK_LAUNCH(ctx);
  std::vector<int> cnt(hc.size());
  std::vector<float> hx(cap_total), hy(cap_total), hr(cap_total);
  if (!hc.empty()) {
    LORB_HIP(ctx, hipMemcpyAsync(cnt.data(), dcnt, sizeof(int) * hc.size(), hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hx.data(), dx, sizeof(float) * cap_total, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hy.data(), dy, sizeof(float) * cap_total, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hr.data(), dr, sizeof(float) * cap_total, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // compact in level / cell order; cell_off of level l, cell c at cell_base[l] + l + c
  std::vector<int> per_cell(nc, 0), src_of(nc, -1);
  for (size_t k = 0; k < hc.size(); k++) { per_cell[slot[k]] = cnt[k]; src_of[slot[k]] = (int)k; }
  int nk = 0;
  for (int l = 0; l < pyr->n_levels; l++) {
    const int b = cell_base[l], e = cell_base[l + 1];
    for (int g = b; g < e; g++) {
      cell_off[g + l] = nk;
      const int k = src_of[g];
      if (k >= 0) {
        for (int q = 0; q < cnt[k]; q++) {
          if (nk + q < max_keypoints) {
            x[nk + q] = hx[hc[k].out_base + q]; y[nk + q] = hy[hc[k].out_base + q]; response[nk + q] = hr[hc[k].out_base + q];
          }
        }
        nk += cnt[k];
      }
    }
    cell_off[e + l] = nk;
  }
  *n_keypoints = nk;
  if (nk > max_keypoints)
    return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints exceed max_keypoints = %d", nk, max_keypoints);
  return LORB_OK;
}


// Detection + retention (src/ORBextractor.cpp:898-1067).  The FAST cells run on the device
// (lorb_orb_fast_cells); the retention is sequential bookkeeping over a few hundred keypoints per
// cell and runs here on the host with the very std::nth_element / std::partition that
// KeyPointsFilter::retainBest (OpenCV 3.1) calls, so equal responses are resolved exactly as in
// the reference build.
namespace {
struct OrbKp {
  float x, y, size, resp;
  int octave;
};
void retain_best(std::vector<OrbKp>& k, int n_points) {  // KeyPointsFilter::retainBest
  if (n_points >= 0 && k.size() > (size_t)n_points) {
    if (n_points == 0) { k.clear(); return; }
    std::nth_element(k.begin(), k.begin() + n_points, k.end(),
                     [](const OrbKp& a, const OrbKp& b) { return a.resp > b.resp; });
    const float amb = k[n_points - 1].resp;
    auto e = std::partition(k.begin() + n_points, k.end(), [amb](const OrbKp& a) { return a.resp >= amb; });
    k.resize(e - k.begin());
  }
}
}  // namespace

int lorb_orb_detect(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired,
                    const float* scale_factors, int32_t ini_th, int32_t min_th, int32_t max_keypoints, float* x,
                    float* y, int32_t* octave, float* size, float* response, int32_t* level_off,
                    int32_t* n_keypoints) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, 0));
  if (!n_desired || !scale_factors || !level_off || !n_keypoints || max_keypoints < 0)
    return lorb::set_error(ctx, LORB_E_INVALID, "null argument");
  const int L = pyr->n_levels;
  int max_cells = 0, cap = 0;
  const float ratio = (float)pyr->cols[0] / pyr->rows[0];
  std::vector<int> cells;
  for (int l = 0; l < L; l++) {
    const int ncl = orb_cells(pyr->rows[l], pyr->cols[l], n_desired[l], ratio, cells);
    if (ncl < 0) return lorb::set_error(ctx, LORB_E_INVALID, "level %d: degenerate cell grid (%d features)", l, n_desired[l]);
    max_cells += ncl;
    for (int c = 0; c < ncl; c++) cap += ((cells[4 * c + 2] + 1) / 2) * ((cells[4 * c + 3] + 1) / 2);
  }
  std::vector<float> fx(cap + 1), fy(cap + 1), fr(cap + 1);
  std::vector<int32_t> base(L + 1), coff(max_cells + L + 1);
  int32_t nf = 0;
  LORB_TRY(lorb_orb_fast_cells(ctx, pyr, n_desired, ini_th, min_th, cap, fx.data(), fy.data(), fr.data(), max_cells,
                               base.data(), coff.data(), &nf));
  int out = 0;
  for (int l = 0; l < L; l++) {
    level_off[l] = out;
    const int nd = n_desired[l];
    const int levelCols = (int)std::sqrt((float)nd / (5 * ratio));
    const int levelRows = (int)(ratio * levelCols);
    const int nCells = levelRows * levelCols;
    orb_cells(pyr->rows[l], pyr->cols[l], nd, ratio, cells);
    const int nfeaturesCell = (int)std::ceil((float)nd / nCells);
    std::vector<int> nToRetain(nCells, 0), nTotal(nCells, 0);
    std::vector<char> bNoMore(nCells, 0);
    int nNoMore = 0, nToDistribute = 0;
    const int32_t* co = coff.data() + base[l] + l;
    for (int c = 0; c < nCells; c++) {  // :983-1003
      if (cells[4 * c + 2] <= 0 || cells[4 * c + 3] <= 0) continue;
      const int nKeys = co[c + 1] - co[c];
      nTotal[c] = nKeys;
      if (nKeys > nfeaturesCell) { nToRetain[c] = nfeaturesCell; bNoMore[c] = 0; }
      else { nToRetain[c] = nKeys; nToDistribute += nfeaturesCell - nKeys; bNoMore[c] = 1; nNoMore++; }
    }
    while (nToDistribute > 0 && nNoMore < nCells) {  // :1010-1035
      const int nNew = (int)(nfeaturesCell + std::ceil((float)nToDistribute / (nCells - nNoMore)));
      nToDistribute = 0;
      for (int c = 0; c < nCells; c++)
        if (!bNoMore[c]) {
          if (nTotal[c] > nNew) { nToRetain[c] = nNew; bNoMore[c] = 0; }
          else { nToRetain[c] = nTotal[c]; nToDistribute += nNew - nTotal[c]; bNoMore[c] = 1; nNoMore++; }
        }
    }
    const int scaledPatchSize = (int)(31 * scale_factors[l]);  // PATCH_SIZE * mvScaleFactor (:1040)
    std::vector<OrbKp> level;
    std::vector<OrbKp> cell;
    for (int c = 0; c < nCells; c++) {  // :1043-1060
      cell.clear();
      for (int k = co[c]; k < co[c + 1]; k++)
        cell.push_back(OrbKp{fx[k] - (float)cells[4 * c], fy[k] - (float)cells[4 * c + 1], 7.f, fr[k], 0});
      retain_best(cell, nToRetain[c]);
      if ((int)cell.size() > nToRetain[c]) cell.resize(nToRetain[c]);
      for (OrbKp& kp : cell) {
        kp.x += (float)cells[4 * c]; kp.y += (float)cells[4 * c + 1];
        kp.octave = l; kp.size = (float)scaledPatchSize;
        level.push_back(kp);
      }
    }
    if ((int)level.size() > nd) {  // :1063-1067
      retain_best(level, nd);
      level.resize(nd);
    }
    for (const OrbKp& kp : level) {
      if (out < max_keypoints) {
        x[out] = kp.x; y[out] = kp.y; octave[out] = kp.octave; size[out] = kp.size; response[out] = kp.resp;
      }
      out++;
    }
  }
  level_off[L] = out;
  *n_keypoints = out;
  if (out > max_keypoints)
    return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints exceed max_keypoints = %d", out, max_keypoints);
  return LORB_OK;
}


int lorb_orb_pyramid(lorb_ctx* ctx, const uint8_t* image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                     const float* scale_factors, uint8_t* out, int64_t out_bytes, lorb_image_pyramid* layout) {
  if (!ctx) return LORB_E_INVALID;
  if (!image || !scale_factors || !out || !layout || rows < 1 || cols < 1 || step < cols || n_levels < 1 ||
      n_levels > LORB_MAX_LEVELS)
    return lorb::set_error(ctx, LORB_E_INVALID, "bad image / level arguments");
  const int64_t need = pyramid_layout(rows, cols, n_levels, scale_factors, layout);
  for (int l = 0; l < n_levels; l++)
    if (layout->rows[l] < 2 || layout->cols[l] < 2)
      return lorb::set_error(ctx, LORB_E_INVALID, "level %d smaller than 2 x 2", l);
  if (out_bytes < need) return lorb::set_error(ctx, LORB_E_INVALID, "out holds %lld bytes, %lld needed",
                                               (long long)out_bytes, (long long)need);
  uint8_t *dimg, *dout;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 16, image, (size_t)(rows - 1) * step + cols, &dimg));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 17, (size_t)need, &dout));
  LORB_TRY(enqueue_pyramid(ctx, dimg, rows, cols, step, *layout, dout));
  LORB_HIP(ctx, hipMemcpyAsync(out, dout, (size_t)need, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  layout->data = out;
  return LORB_OK;
}

int lorb_orb_pyramid_dev(lorb_ctx* ctx, const uint8_t* d_image, int32_t rows, int32_t cols, int32_t step,
                         int32_t n_levels, const float* scale_factors, uint8_t* d_out, int64_t out_bytes,
                         lorb_image_pyramid* layout) {
  if (!ctx) return LORB_E_INVALID;
  if (!d_image || !scale_factors || !d_out || !layout || rows < 1 || cols < 1 || step < cols || n_levels < 1 ||
      n_levels > LORB_MAX_LEVELS)
    return lorb::set_error(ctx, LORB_E_INVALID, "bad image / level arguments");
  const int64_t need = pyramid_layout(rows, cols, n_levels, scale_factors, layout);
  for (int l = 0; l < n_levels; l++)
    if (layout->rows[l] < 2 || layout->cols[l] < 2)
      return lorb::set_error(ctx, LORB_E_INVALID, "level %d smaller than 2 x 2", l);
  if (out_bytes < need) return lorb::set_error(ctx, LORB_E_INVALID, "out holds %lld bytes, %lld needed",
                                               (long long)out_bytes, (long long)need);
  LORB_TRY(enqueue_pyramid(ctx, d_image, rows, cols, step, *layout, d_out));
  layout->data = d_out;
  return LORB_OK;
}

}  // extern "C"
