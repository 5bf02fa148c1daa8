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
#include "lorb_sincosf.h"

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

__global__ __launch_bounds__(64 * kDescWaves) void k_orb_desc(OrbPyr P, int n, const int* __restrict__ d_n,
                                                              const float* __restrict__ kx,
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
  if (d_n) n = min(n, *d_n);  // device-side count (extraction pipeline); < 0 = failed upstream
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
  const float a = lorb_cosf(angle), b = lorb_sinf(angle);  // std::cos(float) = libm cosf (:115)
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

int enqueue_orb(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const uint8_t* d_data, int n, const int* d_n, const float* d_x,
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
    hipLaunchKernelGGL(k_orb_desc, dim3(lorb::ceil_div(n, kDescWaves)), dim3(64 * kDescWaves), 0, ctx->stream, P, n, d_n,
                       d_x, d_y, d_lev, d_pat, d_ang, d_desc);
  LORB_CHECK_LAUNCH(ctx);
  return LORB_OK;
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

// ---- keypoint stage: ComputeKeyPointsOctTree (src/ORBextractor.cpp:799-897) --------------
// Per level, 30-pixel cells with a 6-pixel overlap inside the EDGE_THRESHOLD-3 border (:803-847);
// per cell cv::FAST(iniThFAST, nonmax) re-run with minThFAST only when the cell found nothing
// (:849-859); then DistributeOctTree (:554-797).  Keypoints travel relative to the level's
// (minBorderX, minBorderY) = (16, 16), as vToDistributeKeys does.

constexpr int kOff16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                               {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
constexpr int kBorder = 19 - 3;       // EDGE_THRESHOLD - 3 (:808)
constexpr int kCellMax = 66;          // cells are < 60 + 6 pixels on a side (wCell = ceil(w / floor(w / 30)))
constexpr int kFastThreads = 256;

struct FastCell {
  int level, ini_x, ini_y, w, h, out_base, rel_x, rel_y;  // rel = (j wCell, i hCell), :865-866
};

// cornerScore<16> (OpenCV 3.1 fast_score.cpp) from the 16 circle pixels in registers
__device__ __forceinline__ int fast_score(int v, const int (&ring)[16], int threshold) {
  int d[25];
#pragma unroll
  for (int k = 0; k < 25; k++) d[k] = v - ring[k & 15];
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

// One 256-thread workgroup per cell: the cell image in LDS, FAST_t<16> detection + score of every
// inner pixel, 3x3 non-maximum suppression, the minThFAST re-run when no corner survives, and the
// survivors written in FAST's row-major order (block scan) relative to the level border.
__global__ __launch_bounds__(kFastThreads) void k_orb_fast(const uint8_t* __restrict__ data, OrbPyr P,
                                                           const FastCell* __restrict__ cells, int ini_th, int min_th,
                                                           float* __restrict__ ox, float* __restrict__ oy,
                                                           float* __restrict__ oresp, int* __restrict__ ocount) {
  __shared__ uint8_t img[kCellMax * kCellMax], score[kCellMax * kCellMax], corner[kCellMax * kCellMax];
  __shared__ int s_count, wsum[kFastThreads / 64];
  const FastCell c = cells[blockIdx.x];
  const int w = c.w, h = c.h, n = w * h, t = threadIdx.x;
  const uint8_t* src = data + P.offset[c.level] + (int64_t)c.ini_y * P.step[c.level] + c.ini_x;
  const int step = P.step[c.level];
  for (int p0 = t; p0 < n; p0 += kFastThreads * 8) {  // eight loads in flight per thread
    uint8_t v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int p = p0 + kFastThreads * u;
      const int i = p / w, j = p - i * w;
      v[u] = p < n ? src[(int64_t)i * step + j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; u++)
      if (p0 + kFastThreads * u < n) img[p0 + kFastThreads * u] = v[u];
  }
  for (int pass = 0; pass < 2; ++pass) {
    const int th = min(max(pass ? min_th : ini_th, 0), 255);
    for (int p = t; p < n; p += kFastThreads) { score[p] = 0; corner[p] = 0; }
    if (t == 0) s_count = 0;
    __syncthreads();
    for (int p = t; p < n; p += kFastThreads) {
      const int i = p / w, j = p - i * w;
      if (i < 3 || i >= h - 3 || j < 3 || j >= w - 3) continue;
      const uint8_t* ptr = img + p;
      const int v = ptr[0];
      // the 16 circle pixels, all loads issued together (no dependent LDS chains)
      int ring[16];
#pragma unroll
      for (int k = 0; k < 16; k++) ring[k] = ptr[kOff16[k][0] + kOff16[k][1] * w];
      // FAST_t<16>'s test: 9 contiguous circle pixels all darker than v - th, or all brighter than
      // v + th, along k = 0 .. 24 (indices mod 16) -- i.e. a circular run of 9 in the 16-bit masks.
      // (OpenCV's quick tests on pixels 0/8, 2/10, ... are necessary conditions of this: they
      // only skip work and never change the answer.)
      unsigned dk = 0, br = 0;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        dk |= (unsigned)(ring[k] < v - th) << k;
        br |= (unsigned)(ring[k] > v + th) << k;
      }
      auto run9 = [](unsigned m) {
        unsigned x = m | (m << 16), r = x;
#pragma unroll
        for (int s2 = 1; s2 < 9; s2++) r &= x >> s2;
        return (r & 0xffffu) != 0u;
      };
      if (run9(dk) || run9(br)) { corner[p] = 1; score[p] = (uint8_t)fast_score(v, ring, th); }
    }
    __syncthreads();
    int mine = 0;
    for (int p = t; p < n; p += kFastThreads) {
      if (!corner[p]) continue;
      const int s = score[p];
      mine += s > score[p - w - 1] && s > score[p - w] && s > score[p - w + 1] && s > score[p - 1] && s > score[p + 1] &&
              s > score[p + w - 1] && s > score[p + w] && s > score[p + w + 1];
    }
    if (mine) atomicAdd(&s_count, mine);
    __syncthreads();
    if (pass == 0 && s_count > 0) break;  // uniform: s_count is read by every thread after the barrier
    __syncthreads();
  }
  int run = 0;
  for (int base = 0; base < n; base += kFastThreads) {
    const int p = base + t;
    bool keep = false;
    if (p < n && corner[p]) {
      const int s = score[p];
      keep = s > score[p - w - 1] && s > score[p - w] && s > score[p - w + 1] && s > score[p - 1] && s > score[p + 1] &&
             s > score[p + w - 1] && s > score[p + w] && s > score[p + w + 1];
    }
    int tot;
    const int ex = lorb::block_excl_scan<kFastThreads>(keep ? 1 : 0, wsum, &tot);
    if (keep) {
      const int i = p / w, j = p - i * w;
      const int o = c.out_base + run + ex;
      ox[o] = (float)(j + c.rel_x); oy[o] = (float)(i + c.rel_y); oresp[o] = (float)score[p];
    }
    run += tot;
  }
  if (t == 0) ocount[blockIdx.x] = run;
}

// the cell grid of one level, src/ORBextractor.cpp:803-847 (see oracle/fast.c)
int orb_cells(int rows, int cols, std::vector<int>& cells, int* ncols, int* nrows) {
  const float W = 30;
  const int minBorderX = kBorder, minBorderY = kBorder, maxBorderX = cols - kBorder, maxBorderY = rows - kBorder;
  const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
  const int nCols = (int)(width / W), nRows = (int)(height / W);
  if (nCols < 1 || nRows < 1) return -1;
  const int wCell = (int)std::ceil(width / (float)nCols), hCell = (int)std::ceil(height / (float)nRows);
  cells.assign(6 * (size_t)nRows * nCols, 0);
  for (int i = 0; i < nRows; i++) {
    const float iniY = (float)(minBorderY + i * hCell);
    float maxY = iniY + (float)hCell + 6;
    const bool skip_row = iniY >= (float)(maxBorderY - 3);
    if (maxY > (float)maxBorderY) maxY = (float)maxBorderY;
    for (int j = 0; j < nCols; j++) {
      const float iniX = (float)(minBorderX + j * wCell);
      float maxX = iniX + (float)wCell + 6;
      int* c = &cells[6 * (size_t)(i * nCols + j)];
      c[0] = (int)iniX; c[1] = (int)iniY; c[4] = j * wCell; c[5] = i * hCell;
      if (skip_row || iniX >= (float)(maxBorderX - 6)) continue;
      if (maxX > (float)maxBorderX) maxX = (float)maxBorderX;
      c[2] = (int)maxX - (int)iniX; c[3] = (int)maxY - (int)iniY;
    }
  }
  *ncols = nCols; *nrows = nRows;
  return nRows * nCols;
}

// ---- DistributeOctTree (src/ORBextractor.cpp:496-797) on the device ----------------------
// One 1024-thread workgroup per level.  The reference's std::list<ExtractorNode> is kept as an
// array of nodes in LIST ORDER (front first); every key is owned by exactly one live node, and each
// node owns a contiguous segment of the level's key permutation `perm`, in the order of its vKeys.
// A division pass (main loop :632-698, or one iteration of the focused loop :709-770):
//   * owner of each permutation position = a max-scan over the positions where segments start;
//   * child class (n1..n4 of DivideNode, :527-541) of every key of a dividing node; four
//     exclusive scans of the one-hot classes give each key's rank among its siblings, i.e. a
//     stable in-place 4-way partition of the parent's segment (the children's vKeys orders);
//   * the new list: push_front of the non-empty children of the dividing nodes in processing
//     order (the last processed parent's children first, each group n4 n3 n2 n1), then the
//     surviving nodes in their old order -- two scans over the nodes;
//   * the focused loop processes vPrevSizeAndPointerToNode in descending (size, creation) order
//     (pointer-order model, oracle/fast.c) and stops after the division that reaches N nodes: a
//     scan of (children - 1) in processing order finds that division.
// The strongest key of each final node (strict >, first in vKeys order, :778-794) is the output.
struct OctNode {
  int x0, y0, x1, y1;  // UL = (x0, y0), BR = (x1, y1)
  int beg, end;        // segment of perm
  int cre;             // creation order (pointer-order model)
  int pend;            // in vSizeAndPointerToNode (a child with > 1 key created by the last pass)
};

struct OctLevel {
  int N, n_ini, node_cap, key_cap;
  int key_base, node_base, cell_begin, cell_end;
  int wd, ht;          // maxX - minX, maxY - minY
  float hx;            // (maxX - minX) / nIni
  float size;          // PATCH_SIZE * mvScaleFactor[l] truncated to int (:881)
  float scale;         // mvScaleFactor[l]
};

struct OctArgs {
  OctLevel lv[LORB_MAX_LEVELS];
  int n_levels;
  const FastCell* cells;
  const int* cell_cnt;
  const float *fx, *fy, *fr;         // FAST output (cell slots)
  float *kx, *ky, *kr;               // compact keys per level (key_base)
  int *perm, *perm2, *cls, *own, *hd;
  lorb::I4* ex;                      // key_cap + 1 per level: key_base + l
  OctNode *na, *nb;                  // two node buffers (node_base)
  int *act, *rank, *ech, *tmp, *surv;
  lorb::I4* cnt;
  int* out_key;                      // kept key per final node (node_base)
  int* out_cnt;                      // nodes per level, -1: failure (capacity / iteration cap)
  int* trace;                        // diagnostics (nullable): per level 8 ints per pass, 64 passes
};

constexpr int kOctThreads = 1024;
constexpr int kOctMaxPasses = 1 << 14;
constexpr int kOctKeyChunk = 2048;

__device__ __forceinline__ int oct_class(float x, float y, const OctNode& nd) {
  const int mx = nd.x0 + (int)ceilf((float)(nd.x1 - nd.x0) / 2);  // DivideNode halfX / halfY (:498-499)
  const int my = nd.y0 + (int)ceilf((float)(nd.y1 - nd.y0) / 2);
  if (x < (float)mx) return y < (float)my ? 0 : 2;
  return y < (float)my ? 1 : 3;
}

__device__ __forceinline__ OctNode oct_child(const OctNode& p, int c, int beg, int n, int cre) {
  const int mx = p.x0 + (int)ceilf((float)(p.x1 - p.x0) / 2);
  const int my = p.y0 + (int)ceilf((float)(p.y1 - p.y0) / 2);
  OctNode r;
  r.x0 = (c & 1) ? mx : p.x0;
  r.x1 = (c & 1) ? p.x1 : mx;
  r.y0 = (c & 2) ? my : p.y0;
  r.y1 = (c & 2) ? p.y1 : my;
  r.beg = beg; r.end = beg + n; r.cre = cre; r.pend = n > 1;
  return r;
}

// in-place exclusive scan of a[0, n) by the whole workgroup (chunked); returns the total
__device__ int oct_scan(int* a, int n, int* wsum) {
  const int t = threadIdx.x, per = (n + kOctThreads - 1) / kOctThreads;
  const int b = min(n, t * per), e = min(n, b + per);
  int s = 0;
  for (int i = b; i < e; i++) s += a[i];
  int tot;
  int pre = lorb::block_excl_scan<kOctThreads>(s, wsum, &tot);
  for (int i = b; i < e; i++) { const int v = a[i]; a[i] = pre; pre += v; }
  __syncthreads();
  return tot;
}

// Shared LDS of k_orb_octree: the small scalars, and (fast path) the node list in LDS.
struct OctSh {
  int wsum[kOctThreads / 64];
  lorb::I4 wsum4[kOctThreads / 64];
  int L, mode, state, cm, E;
};
// The general path: every per-key and per-node array in global memory (any key / node count).
__device__ __forceinline__ void oct_global(const OctArgs& A, OctSh& sh, long long* s_key) {
  int* wsum = sh.wsum;
  lorb::I4* wsum4 = sh.wsum4;
  int& s_L = sh.L;
  int& s_mode = sh.mode;
  int& s_state = sh.state;
  int& s_cm = sh.cm;
  int& s_E = sh.E;
  const int l = blockIdx.x, t = threadIdx.x;
  const OctLevel V = A.lv[l];
  float* kx = A.kx + V.key_base;
  float* ky = A.ky + V.key_base;
  float* kr = A.kr + V.key_base;
  int* perm = A.perm + V.key_base;
  int* perm2 = A.perm2 + V.key_base;
  int* cls = A.cls + V.key_base;
  int* own = A.own + V.key_base;
  int* hd = A.hd + V.key_base;
  lorb::I4* ex = A.ex + V.key_base + l;
  OctNode* cur = A.na + V.node_base;
  OctNode* nxt = A.nb + V.node_base;
  int* act = A.act + V.node_base;
  int* rank = A.rank + V.node_base;
  int* ech = A.ech + V.node_base;
  int* tmp = A.tmp + V.node_base;
  int* surv = A.surv + V.node_base;
  lorb::I4* cnt = A.cnt + V.node_base;

  // 1. vToDistributeKeys: the level's cells in row-major order, FAST order inside (:827-872)
  int n = 0;
  for (int base = V.cell_begin; base < V.cell_end; base += kOctThreads) {
    const int c = base + t;
    const int v = c < V.cell_end ? A.cell_cnt[c] : 0;
    int tot;
    const int e0 = lorb::block_excl_scan<kOctThreads>(v, wsum, &tot);
    if (c < V.cell_end && n + e0 + v <= V.key_cap) {
      const int ob = A.cells[c].out_base;
      for (int q = 0; q < v; q++) {
        kx[n + e0 + q] = A.fx[ob + q]; ky[n + e0 + q] = A.fy[ob + q]; kr[n + e0 + q] = A.fr[ob + q];
      }
    }
    n += tot;
  }
  __syncthreads();  // the keys written above are read by other threads below
  if (n > V.key_cap) { if (t == 0) A.out_cnt[l] = -1; return; }
  if (n == 0) { if (t == 0) A.out_cnt[l] = 0; return; }
  const int per = (n + kOctThreads - 1) / kOctThreads;
  const int pb = min(n, t * per), pe = min(n, pb + per);

  // 2. initial nodes (:575-609): keys bucketed by x / hX, stable; empty nodes erased
  {
    lorb::I4 loc = {{0, 0, 0, 0}};
    for (int p = pb; p < pe; p++) {
      const int b = min((int)(kx[p] / V.hx), V.n_ini - 1);
      cls[p] = b;
      loc.v[b] += 1;
    }
    lorb::I4 tot;
    lorb::I4 run = lorb::block_excl_scan4<kOctThreads>(loc, wsum4, &tot);
    int start[4] = {0, tot.v[0], tot.v[0] + tot.v[1], tot.v[0] + tot.v[1] + tot.v[2]};
    for (int p = pb; p < pe; p++) {
      const int b = cls[p];
      perm[start[b] + run.v[b]++] = p;
    }
    if (t == 0) {
      int L = 0, beg = 0;
      for (int b = 0; b < V.n_ini; b++) {
        const int k = tot.v[b];
        if (k > 0) {
          OctNode nd;
          nd.x0 = (int)(V.hx * (float)b); nd.x1 = (int)(V.hx * (float)(b + 1)); nd.y0 = 0; nd.y1 = V.ht;
          nd.beg = beg; nd.end = beg + k; nd.cre = b; nd.pend = 0;
          cur[L++] = nd;
        }
        beg += k;
      }
      s_L = L; s_mode = 0; s_state = 0;
    }
    __syncthreads();
  }

  // 3. division passes (:619-772)
  for (int pass = 0;; pass++) {
    const int L = s_L, mode = s_mode;  // mode 0: main loop pass, 1: focused-loop iteration
    if (s_state != 0) break;
    if (pass >= kOctMaxPasses) { if (t == 0) A.out_cnt[l] = -1; return; }
    // A. dividing candidates; segment heads
    for (int i = t; i < L; i += kOctThreads) {
      const OctNode nd = cur[i];
      act[i] = mode == 0 ? (nd.end - nd.beg >= 2) : nd.pend;
    }
    for (int p = pb; p < pe; p++) hd[p] = -1;
    __syncthreads();
    for (int i = t; i < L; i += kOctThreads) hd[cur[i].beg] = i;
    __syncthreads();
    // B. owner of every position (last segment head at or before it), child class, class scans
    {
      int m = -1;
      for (int p = pb; p < pe; p++) m = hd[p] >= 0 ? p : m;
      int run = lorb::block_excl_max<kOctThreads>(m, -1, wsum);
      lorb::I4 loc = {{0, 0, 0, 0}};
      for (int p = pb; p < pe; p++) {
        run = hd[p] >= 0 ? p : run;
        const int o = hd[run];
        own[p] = o;
        int c = -1;
        if (act[o]) {
          const int k = perm[p];
          c = oct_class(kx[k], ky[k], cur[o]);
          loc.v[c] += 1;
        }
        cls[p] = c;
      }
      lorb::I4 tot;
      lorb::I4 r4 = lorb::block_excl_scan4<kOctThreads>(loc, wsum4, &tot);
      for (int p = pb; p < pe; p++) {
        ex[p] = r4;
        const int c = cls[p];
        if (c >= 0) r4.v[c] += 1;
      }
      if (t == kOctThreads - 1) ex[n] = tot;
    }
    __syncthreads();
    // C. children per dividing node; processing order
    for (int i = t; i < L; i += kOctThreads) {
      if (!act[i]) { ech[i] = 0; continue; }
      const OctNode nd = cur[i];
      const lorb::I4 a = ex[nd.beg], b = ex[nd.end];
      lorb::I4 k;
      int e = 0;
      for (int q = 0; q < 4; q++) { k.v[q] = b.v[q] - a.v[q]; e += k.v[q] > 0; }
      cnt[i] = k;
      ech[i] = e;
    }
    if (mode == 0) {
      for (int i = t; i < L; i += kOctThreads) tmp[i] = act[i];
      __syncthreads();
      oct_scan(tmp, L, wsum);
      for (int i = t; i < L; i += kOctThreads) rank[i] = tmp[i];
    } else {  // descending (size, creation): sort(vPrev...) then j from the back (:717-718)
      // pending nodes as (size << 32 | creation) keys, staged in LDS chunk by chunk
      for (int i = t; i < L; i += kOctThreads) rank[i] = 0;
      for (int c0 = 0; c0 < L; c0 += kOctKeyChunk) {
        const int cn = min(kOctKeyChunk, L - c0);
        __syncthreads();
        for (int j = t; j < cn; j += kOctThreads) {
          const OctNode nd = cur[c0 + j];
          s_key[j] = act[c0 + j] ? ((long long)(nd.end - nd.beg) << 32) | (unsigned)nd.cre : -1ll;
        }
        __syncthreads();
        for (int i = t; i < L; i += kOctThreads) {
          if (!act[i]) continue;
          const long long ki = ((long long)(cur[i].end - cur[i].beg) << 32) | (unsigned)cur[i].cre;
          int r = 0;
          for (int j = 0; j < cn; j++) r += s_key[j] > ki;
          rank[i] += r;
        }
      }
    }
    __syncthreads();
    // D. children counts in processing order; the focused loop's break (:763-764)
    for (int i = t; i < L; i += kOctThreads) if (act[i]) tmp[rank[i]] = ech[i];
    __syncthreads();
    int n_act = 0;
    {
      int s = 0;
      for (int i = t; i < L; i += kOctThreads) s += act[i];
      int tot;
      (void)lorb::block_excl_scan<kOctThreads>(s, wsum, &tot);
      n_act = tot;
    }
    // inclusive prefix of children in processing order -> surv (as scratch), then the break
    for (int r = t; r < n_act; r += kOctThreads) surv[r] = tmp[r];
    __syncthreads();
    (void)oct_scan(surv, n_act, wsum);  // surv[r] = exclusive prefix in processing order
    if (t == 0) s_cm = n_act;
    __syncthreads();
    if (mode == 1) {
      for (int r = t; r < n_act; r += kOctThreads) {
        const int live = L + (surv[r] + tmp[r]) - (r + 1);  // after processing r
        if (live >= V.N) atomicMin(&s_cm, r + 1);
      }
    }
    __syncthreads();
    if (t == 0) s_E = s_cm > 0 ? surv[s_cm - 1] + tmp[s_cm - 1] : 0;
    __syncthreads();
    const int cm = s_cm, E = s_E;
    // E. survivors (not divided this pass) keep their order after the new children
    for (int i = t; i < L; i += kOctThreads) {
      const bool div = act[i] && rank[i] < cm;
      act[i] = div;
      tmp[i] = div ? 0 : 1;
    }
    __syncthreads();
    const int n_surv = oct_scan(tmp, L, wsum);  // tmp[i] = survivor rank
    const int newL = E + n_surv;
    if (newL > V.node_cap) { if (t == 0) A.out_cnt[l] = -1; return; }
    // F. new permutation (stable partition of the divided segments) and the new node list
    for (int p = pb; p < pe; p++) {
      const int o = own[p];
      if (act[o]) {
        const OctNode nd = cur[o];
        const int c = cls[p];
        const lorb::I4 k = cnt[o];
        int off = 0;
        for (int q = 0; q < c; q++) off += k.v[q];
        perm2[nd.beg + off + (ex[p].v[c] - ex[nd.beg].v[c])] = perm[p];
      } else {
        perm2[p] = perm[p];
      }
    }
    int n_pend = 0;
    for (int i = t; i < L; i += kOctThreads) {
      const OctNode nd = cur[i];
      if (!act[i]) {
        OctNode s = nd;
        s.pend = 0;
        nxt[E + tmp[i]] = s;
        continue;
      }
      const int r = rank[i];
      const int incl = surv[r] + ech[i];
      int slot = E - incl;  // children of the last processed parent come first
      const lorb::I4 k = cnt[i];
      int beg = nd.beg + k.v[0] + k.v[1] + k.v[2] + k.v[3];
      for (int c = 3; c >= 0; c--) {  // push_front n1, n2, n3, n4 -> the list reads n4 n3 n2 n1
        const int kc = k.v[c];
        beg -= kc;
        if (kc == 0) continue;
        nxt[slot++] = oct_child(nd, c, beg, kc, 4 * r + c);
        n_pend += kc > 1;
      }
    }
    {
      int tot;
      (void)lorb::block_excl_scan<kOctThreads>(n_pend, wsum, &tot);
      n_pend = tot;
    }
    __syncthreads();
    // G. termination (:703-707, :767-768)
    if (t == 0) {
      if (A.trace && pass < 64) {
        int* tr = A.trace + (l * 64 + pass) * 72;
        tr[0] = L; tr[1] = mode; tr[2] = n_act; tr[3] = cm; tr[4] = E; tr[5] = n_surv; tr[6] = newL; tr[7] = n_pend;
        for (int q = 0; q < 16 && q < newL; q++) {
          tr[8 + 4 * q] = nxt[q].beg; tr[9 + 4 * q] = nxt[q].end; tr[10 + 4 * q] = nxt[q].x0; tr[11 + 4 * q] = nxt[q].y0;
        }
      }
      int state = 0, m = mode;
      if (newL >= V.N || newL == L) state = 1;
      else if (mode == 0 && newL + 3 * n_pend > V.N) m = 1;
      s_state = state; s_mode = m; s_L = newL;
    }
    {
      int* sw = perm; perm = perm2; perm2 = sw;
      OctNode* nw = cur; cur = nxt; nxt = nw;
    }
    __syncthreads();
  }
  // 4. the strongest key of each node (:776-794)
  const int L = s_L;
  for (int i = t; i < L; i += kOctThreads) {
    const OctNode nd = cur[i];
    int best = perm[nd.beg];
    float m = kr[best];
    for (int q = nd.beg + 1; q < nd.end; q++) {
      const int k = perm[q];
      if (kr[k] > m) { best = k; m = kr[k]; }
    }
    A.out_key[V.node_base + i] = best;
  }
  if (t == 0) A.out_cnt[l] = L;
}

// LDS layout of the octree fast path (oct_lds below).
constexpr int kOctNC = 1024, kOctCells = 2048;
constexpr int kQB = 8;  // sweep steps whose loads are issued together
struct OctLds {
  OctNode na[kOctNC], nb[kOctNC];  // nb first holds the cell offsets / output bases (gathering)
  int act[kOctNC], rank[kOctNC], ech[kOctNC], tmp[kOctNC], surv[kOctNC];
  lorb::I4 cnt[kOctNC], exb[kOctNC];
  int2 mid[kOctNC];  // DivideNode's split point of a dividing candidate (x = -1: not dividing)
};
static_assert(sizeof(OctNode) * kOctNC >= sizeof(int) * 2 * (kOctCells + 1), "cell arrays alias nb");

// register-resident four counters indexed by a runtime class (selects, no scratch indexing)
__device__ __forceinline__ int i4get(const lorb::I4& a, int c) {
  return c == 0 ? a.v[0] : c == 1 ? a.v[1] : c == 2 ? a.v[2] : a.v[3];
}
__device__ __forceinline__ lorb::I4 i4one(int c) {  // one-hot (c < 0: zeros)
  lorb::I4 r;
#pragma unroll
  for (int u = 0; u < 4; ++u) r.v[u] = c == u;
  return r;
}
__device__ __forceinline__ void i4add(lorb::I4& a, const lorb::I4& b) {
#pragma unroll
  for (int u = 0; u < 4; ++u) a.v[u] += b.v[u];
}
// inclusive scans across the 64 lanes of a wavefront on DPP (no LDS): within rows of 16 by
// row_shr 1, 2, 4, 8, then row_bcast:15 into rows 1 / 3 and row_bcast:31 into rows 2 / 3 (GFX9 DPP)
template <int CTRL, int RM>
__device__ __forceinline__ int dpp_i(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, RM, 0xf, false);
}
__device__ __forceinline__ int wave_iadd(int x) {
  x += dpp_i<0x111, 0xf>(0, x);
  x += dpp_i<0x112, 0xf>(0, x);
  x += dpp_i<0x114, 0xf>(0, x);
  x += dpp_i<0x118, 0xf>(0, x);
  x += dpp_i<0x142, 0xa>(0, x);
  x += dpp_i<0x143, 0xc>(0, x);
  return x;
}
__device__ __forceinline__ int wave_imax(int x, int /*lane*/) {
  constexpr int lo = (int)0x80000000;
  x = max(x, dpp_i<0x111, 0xf>(lo, x));
  x = max(x, dpp_i<0x112, 0xf>(lo, x));
  x = max(x, dpp_i<0x114, 0xf>(lo, x));
  x = max(x, dpp_i<0x118, 0xf>(lo, x));
  x = max(x, dpp_i<0x142, 0xa>(lo, x));
  x = max(x, dpp_i<0x143, 0xc>(lo, x));
  return x;
}
__device__ __forceinline__ int wave_prev(int x, int old) { return dpp_i<0x138, 0xf>(old, x); }  // wave_shr:1
__device__ __forceinline__ int lane63(int x) { return __builtin_amdgcn_readlane(x, 63); }

// Per-wave sweep state shared across the workgroup's 16 waves (exclusive carries between waves).
struct OctWaves {
  int last[kOctThreads / 64];        // last segment head (position << 11 | node) of each wave's chunk
  lorb::I4 cnt[kOctThreads / 64];    // class (or bucket) counts of each wave's chunk
};
// carry into wave wv: the last head before its chunk (or -1); the class counts before its chunk
__device__ __forceinline__ int oct_wave_last(const OctWaves& ww, int wv) {
  int c = -1;
  for (int w = 0; w < wv; ++w) c = max(c, ww.last[w]);
  return c;
}
__device__ __forceinline__ lorb::I4 oct_wave_base(const OctWaves& ww, int wv) {
  lorb::I4 b = {{0, 0, 0, 0}};
  for (int w = 0; w < wv; ++w) i4add(b, ww.cnt[w]);
  return b;
}

// The LDS path (a level whose node list fits kOctNC nodes and cells kOctCells): the passes of
// oct_global with the node list and every per-node array in LDS and the keys kept in position
// order (key index, x | y << 16), each wave sweeping a contiguous chunk of positions 64 at a time
// (coalesced loads and stores; segment owners and class ranks by wave scans with carries between
// chunks and waves).  Segment heads are pass-stamped (hd[p] = (pass + 1) << 16 | node): no
// clearing pass.  The keys are gathered from the cells one thread per key.
__device__ __forceinline__ void oct_lds(const OctArgs& A, OctSh& sh, OctLds& S, OctWaves& ww, long long* s_key) {
  // lorb_orb_debug_octree only: cycle stamps of the phases in the trace's spare words
  const unsigned long long oct_t0 = __builtin_amdgcn_s_memtime();
  int oct_ns = 0;
#define OCT_STAMP() do { if (A.trace && threadIdx.x == 0 && oct_ns < 60) \
    A.trace[A.n_levels * 64 * 72 + blockIdx.x * 16384 + oct_ns++] = (int)(__builtin_amdgcn_s_memtime() - oct_t0); } while (0)
  int* wsum = sh.wsum;
  const int l = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const OctLevel V = A.lv[l];
  float* kx = A.kx + V.key_base;
  float* ky = A.ky + V.key_base;
  float* kr = A.kr + V.key_base;
  int* hd = A.hd + V.key_base;
  // position-ordered keys (double-buffered): key index, and x | y << 16 (FAST keys sit on integer
  // pixel coordinates, k_orb_fast, below 2^16); per position the pass's owner | class | head word
  // and class prefix
  int* pk0 = A.perm + V.key_base;
  int* pk1 = A.perm2 + V.key_base;
  int* pxy0 = A.cls + V.key_base;
  int* pxy1 = A.own + V.key_base;
  int* meta = reinterpret_cast<int*>(A.ex + V.key_base + l);  // (key_cap + 1) I4 >= 2 key_cap ints
  int* rk = meta + V.key_cap;
  const int ncell = V.cell_end - V.cell_begin;

  // 1. vToDistributeKeys (:827-872): cell offsets, then one thread per key
  int* coff = reinterpret_cast<int*>(S.nb);
  int* cob = coff + kOctCells + 1;
  int n = 0;
  for (int base = 0; base < ncell; base += kOctThreads) {
    const int c = base + t;
    const int v = c < ncell ? A.cell_cnt[V.cell_begin + c] : 0;
    const int ob = c < ncell ? A.cells[V.cell_begin + c].out_base : 0;
    int tot;
    const int e0 = lorb::block_excl_scan<kOctThreads>(v, wsum, &tot);
    if (c < ncell) { coff[c] = n + e0; cob[c] = ob; }
    n += tot;
  }
  if (t == 0) coff[ncell] = n;
  __syncthreads();
  if (n > V.key_cap) { if (t == 0) A.out_cnt[l] = -1; return; }
  if (n == 0) { if (t == 0) A.out_cnt[l] = 0; return; }
  for (int k0 = t; k0 < n; k0 += 4 * kOctThreads) {  // four keys per thread in flight
    int src[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kOctThreads;
      int lo = 0, hi = ncell - 1;  // the last cell whose offset is <= k (a non-empty one)
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (coff[mid] <= k) lo = mid; else hi = mid - 1;
      }
      src[u] = k < n ? cob[lo] + (k - coff[lo]) : 0;
    }
    float fx[4], fy[4], fr[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { fx[u] = A.fx[src[u]]; fy[u] = A.fy[src[u]]; fr[u] = A.fr[src[u]]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * kOctThreads;
      if (k < n) { kx[k] = fx[u]; ky[k] = fy[u]; kr[k] = fr[u]; }
    }
  }
  __syncthreads();  // the keys written above are read by other threads below
  OCT_STAMP();
  // wave wv sweeps positions [c0, c1), 64 per step
  const int chunk = (n + kOctThreads - 1) / kOctThreads * 64;
  const int c0 = min(n, wv * chunk), c1 = min(n, c0 + chunk);

  // 2. initial nodes (:575-609): keys bucketed by x / hX, stable; empty nodes erased
  {
    lorb::I4 cnt = {{0, 0, 0, 0}};
    for (int p0 = c0 + lane; p0 < c1; p0 += 64 * kQB) {
      float xv[kQB];
#pragma unroll
      for (int q = 0; q < kQB; ++q) xv[q] = p0 + 64 * q < c1 ? kx[p0 + 64 * q] : 0.f;
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = p0 + 64 * q;
        if (p < c1) {
          i4add(cnt, i4one(min((int)(xv[q] / V.hx), V.n_ini - 1)));
          hd[p] = 0;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) cnt.v[u] = __reduce_add_sync(~0ull, cnt.v[u]);
    if (lane == 0) ww.cnt[wv] = cnt;
    __syncthreads();
    lorb::I4 tot = {{0, 0, 0, 0}}, run = oct_wave_base(ww, wv);
    for (int w = 0; w < kOctThreads / 64; ++w) i4add(tot, ww.cnt[w]);
    const int start[4] = {0, tot.v[0], tot.v[0] + tot.v[1], tot.v[0] + tot.v[1] + tot.v[2]};
    for (int pb0 = c0; pb0 < c1; pb0 += 64 * kQB) {
    float xv[kQB], yv[kQB];
#pragma unroll
    for (int q = 0; q < kQB; ++q) {
      const int p = pb0 + 64 * q + lane;
      xv[q] = p < c1 ? kx[p] : 0.f;
      yv[q] = p < c1 ? ky[p] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kQB; ++q) {
      const int p = pb0 + 64 * q + lane;
      const float x = xv[q], y = yv[q];
      const int b = p < c1 ? min((int)(x / V.hx), V.n_ini - 1) : -1;
      // the four bucket counters packed 8 bits each (a step counts at most 64)
      const int inc = wave_iadd(b >= 0 ? 1 << (8 * b) : 0);
      if (p < c1) {
        const int pos = (b == 0 ? 0 : b == 1 ? start[1] : b == 2 ? start[2] : start[3]) + i4get(run, b) +
                        ((inc >> (8 * b)) & 0xff) - 1;
        pk0[pos] = p; pxy0[pos] = (int)x | ((int)y << 16);
      }
      const int wt = lane63(inc);
#pragma unroll
      for (int u = 0; u < 4; ++u) run.v[u] += (wt >> (8 * u)) & 0xff;
    }
    }
    if (t == 0) {
      int L = 0, beg = 0;
      for (int b = 0; b < V.n_ini; b++) {
        const int k = tot.v[b];
        if (k > 0) {
          OctNode nd;
          nd.x0 = (int)(V.hx * (float)b); nd.x1 = (int)(V.hx * (float)(b + 1)); nd.y0 = 0; nd.y1 = V.ht;
          nd.beg = beg; nd.end = beg + k; nd.cre = b; nd.pend = 0;
          S.na[L++] = nd;
        }
        beg += k;
      }
      sh.L = L; sh.mode = 0; sh.state = 0;
    }
    __syncthreads();
  }
  OCT_STAMP();

  // the owner sweep shared by the passes and the final step: ww.last = each wave's last head
  auto wave_last_head = [&](int stamp) {
    int last = -1;
    for (int p0 = c0 + lane; p0 < c1; p0 += 64 * kQB) {
      int hv[kQB];
#pragma unroll
      for (int q = 0; q < kQB; ++q) hv[q] = p0 + 64 * q < c1 ? hd[p0 + 64 * q] : 0;
#pragma unroll
      for (int q = 0; q < kQB; ++q)
        if (p0 + 64 * q < c1 && (hv[q] >> 16) == stamp) last = max(last, ((p0 + 64 * q) << 11) | (hv[q] & 0x7ff));
    }
    last = __reduce_max_sync(~0ull, last);
    if (lane == 0) ww.last[wv] = last;
  };

  // 3. division passes (:619-772)
  OctNode* cur = S.na;
  OctNode* nxt = S.nb;
  for (int pass = 0;; pass++) {
    const int L = sh.L, mode = sh.mode;
    if (sh.state != 0) break;
    if (pass >= kOctMaxPasses) { if (t == 0) A.out_cnt[l] = -1; return; }
    const int stamp = pass + 1;
    // A. dividing candidates (split points); segment heads (stamped)
    for (int i = t; i < L; i += kOctThreads) {
      const OctNode nd = cur[i];
      const int a = mode == 0 ? (nd.end - nd.beg >= 2) : nd.pend;
      S.act[i] = a;
      S.mid[i] = a ? make_int2(nd.x0 + (int)ceilf((float)(nd.x1 - nd.x0) / 2), nd.y0 + (int)ceilf((float)(nd.y1 - nd.y0) / 2))
                   : make_int2(-1, 0);
      hd[nd.beg] = (stamp << 16) | i;
    }
    __syncthreads();
    // B. owners (segment heads + a max-scan), classes (DivideNode's quadrant, :527-541), class counts
    wave_last_head(stamp);
    __syncthreads();
    {
      int own = oct_wave_last(ww, wv);  // (position << 11 | node) of the head owning the next position
      lorb::I4 cnt = {{0, 0, 0, 0}};
      for (int pb0 = c0; pb0 < c1; pb0 += 64 * kQB) {
      int hv[kQB], xyv[kQB];
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = pb0 + 64 * q + lane;
        hv[q] = p < c1 ? hd[p] : 0;
        xyv[q] = p < c1 ? pxy0[p] : 0;
      }
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = pb0 + 64 * q + lane;
        const bool in = p < c1;
        const int h = hv[q], xy = xyv[q];
        const bool head = in && (h >> 16) == stamp;
        const int sc = wave_imax(head ? (p << 11) | (h & 0x7ff) : -1, lane);
        const int o = max(own, sc) & 0x7ff;
        int c = -1;
        if (in) {
          const int2 md = S.mid[o];  // oct_class on integer coordinates (exact)
          if (md.x >= 0) c = ((xy & 0xffff) < md.x ? 0 : 1) + ((xy >> 16) < md.y ? 0 : 2);
          meta[p] = o | ((c + 1) << 11) | ((int)head << 14);
        }
        i4add(cnt, i4one(c));
        own = max(own, lane63(sc));
      }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) cnt.v[u] = __reduce_add_sync(~0ull, cnt.v[u]);
      if (lane == 0) ww.cnt[wv] = cnt;
    }
    __syncthreads();
    // B'. class prefix per position (for the placement) and per node at its segment start (exb)
    //     and end (cnt, turned into counts in C)
    {
      lorb::I4 run = oct_wave_base(ww, wv);
      int prev = oct_wave_last(ww, wv);  // owner of the position before this wave's chunk
      prev = prev >= 0 ? (prev & 0x7ff) : -1;
      for (int pb0 = c0; pb0 < c1; pb0 += 64 * kQB) {
      int mv[kQB];
#pragma unroll
      for (int q = 0; q < kQB; ++q) mv[q] = pb0 + 64 * q + lane < c1 ? meta[pb0 + 64 * q + lane] : 0;
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = pb0 + 64 * q + lane;
        const bool in = p < c1;
        const int m = mv[q];
        const int o = m & 0x7ff, c = in ? ((m >> 11) & 7) - 1 : -1;
        const int inc = wave_iadd(c >= 0 ? 1 << (8 * c) : 0);  // class counters packed 8 bits each
        lorb::I4 pre = run;  // exclusive prefix at p
#pragma unroll
        for (int u = 0; u < 4; ++u) pre.v[u] += ((inc >> (8 * u)) & 0xff) - (c == u);
        const int po = wave_prev(o, prev);  // owner of p - 1 (lane 0: the carried owner)
        if (in) {
          if ((m >> 14) & 1) {
            S.exb[o] = pre;
            if (po >= 0) S.cnt[po] = pre;  // the previous segment ends here
          }
          if (c >= 0) rk[p] = i4get(pre, c);
          if (p == n - 1) {  // the last segment ends at n
            lorb::I4 e = pre;
            i4add(e, i4one(c));
            S.cnt[o] = e;
          }
        }
        prev = lane63(o);
        const int wt = lane63(inc);
#pragma unroll
        for (int u = 0; u < 4; ++u) run.v[u] += (wt >> (8 * u)) & 0xff;
      }
      }
    }
    __syncthreads();
    OCT_STAMP();
    // C. children per dividing node; processing order
    for (int i = t; i < L; i += kOctThreads) {
      if (!S.act[i]) { S.ech[i] = 0; continue; }
      const lorb::I4 a = S.exb[i], b = S.cnt[i];
      lorb::I4 k;
      int e = 0;
      for (int q = 0; q < 4; q++) { k.v[q] = b.v[q] - a.v[q]; e += k.v[q] > 0; }
      S.cnt[i] = k;
      S.ech[i] = e;
    }
    if (mode == 0) {
      for (int i = t; i < L; i += kOctThreads) S.tmp[i] = S.act[i];
      __syncthreads();
      oct_scan(S.tmp, L, wsum);
      for (int i = t; i < L; i += kOctThreads) S.rank[i] = S.tmp[i];
    } else {  // descending (size, creation): sort(vPrev...) then j from the back (:717-718)
      for (int i = t; i < L; i += kOctThreads) S.rank[i] = 0;
      for (int q0 = 0; q0 < L; q0 += kOctKeyChunk) {
        const int cn = min(kOctKeyChunk, L - q0);
        __syncthreads();
        for (int j = t; j < cn; j += kOctThreads) {
          const OctNode nd = cur[q0 + j];
          s_key[j] = S.act[q0 + j] ? ((long long)(nd.end - nd.beg) << 32) | (unsigned)nd.cre : -1ll;
        }
        __syncthreads();
        for (int i = t; i < L; i += kOctThreads) {
          if (!S.act[i]) continue;
          const long long ki = ((long long)(cur[i].end - cur[i].beg) << 32) | (unsigned)cur[i].cre;
          int r = 0;
          for (int j = 0; j < cn; j++) r += s_key[j] > ki;
          S.rank[i] += r;
        }
      }
    }
    __syncthreads();
    // D. children counts in processing order; the focused loop's break (:763-764)
    for (int i = t; i < L; i += kOctThreads) if (S.act[i]) S.tmp[S.rank[i]] = S.ech[i];
    __syncthreads();
    int n_act = 0;
    {
      int s2 = 0;
      for (int i = t; i < L; i += kOctThreads) s2 += S.act[i];
      int tt;
      (void)lorb::block_excl_scan<kOctThreads>(s2, wsum, &tt);
      n_act = tt;
    }
    for (int r = t; r < n_act; r += kOctThreads) S.surv[r] = S.tmp[r];
    __syncthreads();
    (void)oct_scan(S.surv, n_act, wsum);  // surv[r] = exclusive prefix in processing order
    if (t == 0) sh.cm = n_act;
    __syncthreads();
    if (mode == 1) {
      for (int r = t; r < n_act; r += kOctThreads) {
        const int live = L + (S.surv[r] + S.tmp[r]) - (r + 1);  // after processing r
        if (live >= V.N) atomicMin(&sh.cm, r + 1);
      }
    }
    __syncthreads();
    if (t == 0) sh.E = sh.cm > 0 ? S.surv[sh.cm - 1] + S.tmp[sh.cm - 1] : 0;
    __syncthreads();
    const int cm = sh.cm, E = sh.E;
    // E. survivors (not divided this pass) keep their order after the new children
    for (int i = t; i < L; i += kOctThreads) {
      const bool div = S.act[i] && S.rank[i] < cm;
      S.act[i] = div;
      S.tmp[i] = div ? 0 : 1;
    }
    __syncthreads();
    const int n_surv = oct_scan(S.tmp, L, wsum);  // tmp[i] = survivor rank
    const int newL = E + n_surv;
    OCT_STAMP();
    if (newL > V.node_cap || newL > kOctNC) { if (t == 0) A.out_cnt[l] = -1; return; }
    // F. the keys in their new positions (stable partition of the divided segments), the new list
    for (int p0 = c0 + lane; p0 < c1; p0 += 64 * kQB) {
      int mv[kQB], rv[kQB], kv[kQB], xv[kQB];
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = p0 + 64 * q;
        const bool in = p < c1;
        mv[q] = in ? meta[p] : 0;
        rv[q] = in ? rk[p] : 0;
        kv[q] = in ? pk0[p] : 0;
        xv[q] = in ? pxy0[p] : 0;
      }
#pragma unroll
      for (int q = 0; q < kQB; ++q) {
        const int p = p0 + 64 * q;
        if (p < c1) {
          const int m = mv[q], o = m & 0x7ff, c = ((m >> 11) & 7) - 1;
          int dst = p;
          if (S.act[o]) {
            const lorb::I4 k = S.cnt[o];
            const int off = (c > 0 ? k.v[0] : 0) + (c > 1 ? k.v[1] : 0) + (c > 2 ? k.v[2] : 0);
            dst = cur[o].beg + off + (rv[q] - i4get(S.exb[o], c));
          }
          pk1[dst] = kv[q]; pxy1[dst] = xv[q];
        }
      }
    }
    int n_pend = 0;
    for (int i = t; i < L; i += kOctThreads) {
      const OctNode nd = cur[i];
      if (!S.act[i]) {
        OctNode s2 = nd;
        s2.pend = 0;
        nxt[E + S.tmp[i]] = s2;
        continue;
      }
      const int r = S.rank[i];
      const int incl = S.surv[r] + S.ech[i];
      int slot = E - incl;  // children of the last processed parent come first
      const lorb::I4 k = S.cnt[i];
      int beg = nd.beg + k.v[0] + k.v[1] + k.v[2] + k.v[3];
      for (int c = 3; c >= 0; c--) {  // push_front n1, n2, n3, n4 -> the list reads n4 n3 n2 n1
        const int kc = k.v[c];
        beg -= kc;
        if (kc == 0) continue;
        nxt[slot++] = oct_child(nd, c, beg, kc, 4 * r + c);
        n_pend += kc > 1;
      }
    }
    {
      int tt;
      (void)lorb::block_excl_scan<kOctThreads>(n_pend, wsum, &tt);
      n_pend = tt;
    }
    __syncthreads();
    // G. termination (:703-707, :767-768)
    if (t == 0) {
      if (A.trace && pass < 64) {
        int* tr = A.trace + (l * 64 + pass) * 72;
        tr[0] = L; tr[1] = mode; tr[2] = n_act; tr[3] = cm; tr[4] = E; tr[5] = n_surv; tr[6] = newL; tr[7] = n_pend;
        for (int q = 0; q < 16 && q < newL; q++) {
          tr[8 + 4 * q] = nxt[q].beg; tr[9 + 4 * q] = nxt[q].end; tr[10 + 4 * q] = nxt[q].x0; tr[11 + 4 * q] = nxt[q].y0;
        }
      }
      int state = 0, m = mode;
      if (newL >= V.N || newL == L) state = 1;
      else if (mode == 0 && newL + 3 * n_pend > V.N) m = 1;
      sh.state = state; sh.mode = m; sh.L = newL;
    }
    {
      OctNode* nw = cur; cur = nxt; nxt = nw;
      int* w1 = pk0; pk0 = pk1; pk1 = w1;
      int* w2 = pxy0; pxy0 = pxy1; pxy1 = w2;
    }
    __syncthreads();
    OCT_STAMP();
  }
  // 4. the strongest key of each node (:776-794: strict >, so the first of the strongest in vKeys
  //    order): the final segment heads stamped once more, every key's owner as in a pass, and a
  //    per-node LDS max of (response as an ordered int) << 32 | ~position
  const int L = sh.L;
  {
    const int sf = kOctMaxPasses + 1;  // above every pass stamp
    for (int i = t; i < L; i += kOctThreads) {
      hd[cur[i].beg] = (sf << 16) | i;
      s_key[i] = 0;
    }
    __syncthreads();
    wave_last_head(sf);
    __syncthreads();
    int own = oct_wave_last(ww, wv);
    for (int pb0 = c0; pb0 < c1; pb0 += 64 * kQB) {
    int hv[kQB];
    float rv[kQB];
#pragma unroll
    for (int q = 0; q < kQB; ++q) {
      const int p = pb0 + 64 * q + lane;
      hv[q] = p < c1 ? hd[p] : 0;
      rv[q] = p < c1 ? kr[pk0[p]] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kQB; ++q) {
      const int p = pb0 + 64 * q + lane;
      const bool in = p < c1;
      const int h = hv[q];
      const bool head = in && (h >> 16) == sf;
      const int sc = wave_imax(head ? (p << 11) | (h & 0x7ff) : -1, lane);
      const int o = max(own, sc) & 0x7ff;
      if (in) {
        const unsigned b = __float_as_uint(rv[q]);
        const unsigned ord = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
        atomicMax(reinterpret_cast<unsigned long long*>(&s_key[o]),
                  ((unsigned long long)ord << 32) | (unsigned)(0xffffffffu - (unsigned)p));
      }
      own = max(own, lane63(sc));
    }
    }
    __syncthreads();
    for (int i = t; i < L; i += kOctThreads) {
      const unsigned pos = 0xffffffffu - (unsigned)(s_key[i] & 0xffffffffull);
      A.out_key[V.node_base + i] = pk0[pos];
    }
  }
  OCT_STAMP();
#undef OCT_STAMP
  if (t == 0) A.out_cnt[l] = L;
}

__global__ __launch_bounds__(kOctThreads) void k_orb_octree(OctArgs A) {
  __shared__ OctSh sh;
  __shared__ long long s_key[kOctKeyChunk];
  __shared__ OctLds S;
  __shared__ OctWaves ww;
  const OctLevel& V = A.lv[blockIdx.x];
  // the LDS path when the level's node list and cells fit
  if (V.node_cap <= kOctNC && V.cell_end - V.cell_begin <= kOctCells)
    oct_lds(A, sh, S, ww, s_key);
  else
    oct_global(A, sh, s_key);
}

// Gathers the per-level results in level order: level coordinates, octave, size, response and the
// level-0 (scaled) coordinates (:881-891, :1141-1147); level_off[n_levels + 1] and *n_total (-1
// when a level failed).
__global__ __launch_bounds__(256) void k_orb_gather(OctArgs A, int cap, float* __restrict__ lx, float* __restrict__ ly,
                                                    float* __restrict__ sx, float* __restrict__ sy,
                                                    int* __restrict__ oct, float* __restrict__ size,
                                                    float* __restrict__ resp, int* __restrict__ level_off,
                                                    int* __restrict__ n_total) {
  __shared__ int off[LORB_MAX_LEVELS + 1];
  __shared__ int bad;
  if (threadIdx.x == 0) {
    int s = 0, b = 0;
    for (int l = 0; l < A.n_levels; l++) {
      off[l] = s;
      const int c = A.out_cnt[l];
      b |= c < 0;
      s += c < 0 ? 0 : c;
    }
    off[A.n_levels] = s;
    bad = b || s > cap;
    if (blockIdx.x == 0) {
      for (int l = 0; l <= A.n_levels; l++) level_off[l] = off[l];
      *n_total = bad ? -1 : s;
    }
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (bad || i >= off[A.n_levels]) return;
  int l = 0;
  while (l + 1 < A.n_levels && i >= off[l + 1]) ++l;
  const OctLevel& V = A.lv[l];
  const int k = A.out_key[V.node_base + i - off[l]];
  const float x = A.kx[V.key_base + k] + (float)kBorder, y = A.ky[V.key_base + k] + (float)kBorder;
  lx[i] = x; ly[i] = y;
  sx[i] = l != 0 ? x * V.scale : x;
  sy[i] = l != 0 ? y * V.scale : y;
  oct[i] = l; size[i] = V.size; resp[i] = A.kr[V.key_base + k];
}

// Host plan of the keypoint stage: cells, capacities and the octree arguments (device pointers are
// filled by orb_alloc).
struct OrbPlan {
  std::vector<FastCell> cells;
  int fast_cap = 0, key_total = 0, node_total = 0, out_cap = 0;
  OctArgs A{};
};

int orb_plan(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired, const float* sf, OrbPlan* P) {
  P->cells.clear();
  P->fast_cap = P->key_total = P->node_total = P->out_cap = 0;
  std::memset(&P->A, 0, sizeof(P->A));
  P->A.n_levels = pyr->n_levels;
  std::vector<int> cells;
  for (int l = 0; l < pyr->n_levels; l++) {
    int nc, nr;
    const int ncl = orb_cells(pyr->rows[l], pyr->cols[l], cells, &nc, &nr);
    if (ncl < 0) return lorb::set_error(ctx, LORB_E_INVALID, "level %d (%d x %d) too small for one 30-pixel cell", l,
                                        pyr->rows[l], pyr->cols[l]);
    OctLevel& V = P->A.lv[l];
    V.cell_begin = (int)P->cells.size();
    int kcap = 0;
    for (int c = 0; c < ncl; c++) {
      const int* g = &cells[6 * (size_t)c];
      if (g[2] <= 0 || g[3] <= 0) continue;
      if (g[2] > kCellMax || g[3] > kCellMax)
        return lorb::set_error(ctx, LORB_E_INVALID, "level %d cell %d x %d exceeds the LDS tile", l, g[2], g[3]);
      const int cap = ((g[2] + 1) / 2) * ((g[3] + 1) / 2);  // 3x3 maxima are never 8-adjacent
      P->cells.push_back(FastCell{l, g[0], g[1], g[2], g[3], P->fast_cap, g[4], g[5]});
      P->fast_cap += cap;
      kcap += cap;
    }
    V.cell_end = (int)P->cells.size();
    const int minX = kBorder, maxX = pyr->cols[l] - kBorder, minY = kBorder, maxY = pyr->rows[l] - kBorder;
    V.wd = maxX - minX; V.ht = maxY - minY;
    V.n_ini = (int)std::round((float)(maxX - minX) / (float)(maxY - minY));  // :559
    if (V.n_ini < 1 || V.n_ini > 4)
      return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "level %d: %d initial quadtree nodes (1..4 supported)", l, V.n_ini);
    V.hx = (float)(maxX - minX) / (float)V.n_ini;
    V.N = std::max(0, (int)n_desired[l]);
    V.node_cap = 4 * std::max(V.N, 4) + 16;
    V.key_cap = std::max(kcap, 1);
    V.key_base = P->key_total;
    V.node_base = P->node_total;
    V.size = (float)(int)(31 * sf[l]);
    V.scale = sf[l];
    P->key_total += V.key_cap;
    P->node_total += V.node_cap;
  }
  P->out_cap = P->node_total;
  return LORB_OK;
}

// allocates the scratch of a plan (slots S_ORB + 20 ..) and fills the device pointers of P->A
int orb_alloc(lorb_ctx* ctx, OrbPlan* P, FastCell** d_cells, int** d_cnt) {
  OctArgs& A = P->A;
  const size_t K = (size_t)std::max(P->key_total, 1), NN = (size_t)std::max(P->node_total, 1);
  const size_t F = (size_t)std::max(P->fast_cap, 1);
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 20, P->cells.data(), P->cells.size(), d_cells));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 21, std::max<size_t>(P->cells.size(), 1), d_cnt));
  float *fx, *fy, *fr, *kx, *ky, *kr;
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 22, F, &fx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 23, F, &fy));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 24, F, &fr));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 25, K, &kx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 26, K, &ky));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 27, K, &kr));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 28, K, &A.perm));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 29, K, &A.perm2));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 30, K, &A.cls));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 31, K, &A.own));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 32, K, &A.hd));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 33, K + LORB_MAX_LEVELS, &A.ex));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 34, NN, &A.na));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 35, NN, &A.nb));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 36, NN, &A.act));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 37, NN, &A.rank));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 38, NN, &A.ech));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 39, NN, &A.tmp));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 40, NN, &A.surv));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 41, NN, &A.cnt));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 42, NN, &A.out_key));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 43, (size_t)LORB_MAX_LEVELS, &A.out_cnt));
  A.cells = *d_cells; A.cell_cnt = *d_cnt;
  A.fx = fx; A.fy = fy; A.fr = fr; A.kx = kx; A.ky = ky; A.kr = kr;
  return LORB_OK;
}

// FAST cells + DistributeOctTree of every level, enqueued on the ctx stream (device pyramid)
int enqueue_keypoints(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const uint8_t* d_data, OrbPlan* P, int ini_th,
                      int min_th) {
  FastCell* dcells;
  int* dcnt;
  LORB_TRY(orb_alloc(ctx, P, &dcells, &dcnt));
  OrbPyr Q{};
  for (int l = 0; l < pyr->n_levels; l++) { Q.offset[l] = pyr->offset[l]; Q.step[l] = pyr->step[l]; }
  if (!P->cells.empty())
    hipLaunchKernelGGL(k_orb_fast, dim3((unsigned)P->cells.size()), dim3(kFastThreads), 0, ctx->stream, d_data, Q,
                       dcells, ini_th, min_th, const_cast<float*>(P->A.fx), const_cast<float*>(P->A.fy),
                       const_cast<float*>(P->A.fr), dcnt);
  hipLaunchKernelGGL(k_orb_octree, dim3(pyr->n_levels), dim3(kOctThreads), 0, ctx->stream, P->A);
  LORB_CHECK_LAUNCH(ctx);
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
  return enqueue_orb(ctx, d_pyr, d_pyr->data, n, nullptr, d_x, d_y, d_level, d_pattern, d_angle, d_desc);
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
  LORB_TRY(enqueue_orb(ctx, pyr, dd, n, nullptr, dx, dy, dl, dp, dang, ddesc));
  if (n > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(angle, dang, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(desc, ddesc, (size_t)32 * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
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

namespace {

// dummy n_desired for the FAST-only entry point (DistributeOctTree is not run)
int plan_fast_only(lorb_ctx* ctx, const lorb_image_pyramid* pyr, OrbPlan* P) {
  std::vector<int32_t> nd(pyr->n_levels, 1);
  std::vector<float> sf(pyr->n_levels, 1.0f);
  return orb_plan(ctx, pyr, nd.data(), sf.data(), P);
}

}  // namespace

extern "C" {

int lorb_orb_fast_cells(lorb_ctx* ctx, const lorb_image_pyramid* pyr, int32_t ini_th, int32_t min_th,
                        int32_t max_keypoints, float* x, float* y, float* response, int32_t max_cells,
                        int32_t* cell_base, int32_t* cell_off, int32_t* n_keypoints) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, 0));
  if (!cell_base || !cell_off || !n_keypoints || max_keypoints < 0 || max_cells < 0 || (max_keypoints > 0 && (!x || !y || !response)))
    return lorb::set_error(ctx, LORB_E_INVALID, "null argument");
  OrbPlan P;
  LORB_TRY(plan_fast_only(ctx, pyr, &P));
  FastCell* dcells;
  int* dcnt;
  uint8_t* dd;
  LORB_TRY(orb_alloc(ctx, &P, &dcells, &dcnt));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 1, pyr->data, (size_t)pyr_extent(pyr), &dd));
  OrbPyr Q{};
  for (int l = 0; l < pyr->n_levels; l++) { Q.offset[l] = pyr->offset[l]; Q.step[l] = pyr->step[l]; }
  if (!P.cells.empty())
    hipLaunchKernelGGL(k_orb_fast, dim3((unsigned)P.cells.size()), dim3(kFastThreads), 0, ctx->stream, dd, Q, dcells,
                       ini_th, min_th, const_cast<float*>(P.A.fx), const_cast<float*>(P.A.fy),
                       const_cast<float*>(P.A.fr), dcnt);
  LORB_CHECK_LAUNCH(ctx);
  const size_t nc = P.cells.size(), F = (size_t)std::max(P.fast_cap, 1);
  std::vector<int> cnt(std::max<size_t>(nc, 1));
  std::vector<float> hx(F), hy(F), hr(F);
  if (nc) {
    LORB_HIP(ctx, hipMemcpyAsync(cnt.data(), dcnt, sizeof(int) * nc, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hx.data(), P.A.fx, sizeof(float) * F, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hy.data(), P.A.fy, sizeof(float) * F, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(hr.data(), P.A.fr, sizeof(float) * F, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // the whole grid of every level (skipped cells hold no keypoint), level coordinates
  int nk = 0, ng = 0;
  size_t k = 0;
  std::vector<int> cells;
  for (int l = 0; l < pyr->n_levels; l++) {
    int ncol, nrow;
    const int ncl = orb_cells(pyr->rows[l], pyr->cols[l], cells, &ncol, &nrow);
    if (ng + ncl > max_cells) return lorb::set_error(ctx, LORB_E_INVALID, "more than max_cells = %d cells", max_cells);
    cell_base[l] = ng;
    for (int c = 0; c < ncl; c++) {
      cell_off[ng + c + l] = nk;
      const int* g = &cells[6 * (size_t)c];
      if (g[2] <= 0 || g[3] <= 0) continue;
      const FastCell& fc = P.cells[k];
      for (int q = 0; q < cnt[k]; q++, nk++)
        if (nk < max_keypoints) {
          x[nk] = hx[fc.out_base + q] + (float)kBorder; y[nk] = hy[fc.out_base + q] + (float)kBorder;
          response[nk] = hr[fc.out_base + q];
        }
      k++;
    }
    ng += ncl;
    cell_off[ng + l] = nk;
  }
  cell_base[pyr->n_levels] = ng;
  *n_keypoints = nk;
  if (nk > max_keypoints)
    return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints exceed max_keypoints = %d", nk, max_keypoints);
  return LORB_OK;
}

int lorb_orb_detect(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired,
                    const float* scale_factors, int32_t ini_th, int32_t min_th, int32_t max_keypoints, float* x,
                    float* y, int32_t* octave, float* size, float* response, int32_t* level_off,
                    int32_t* n_keypoints) {
  if (!ctx) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, 0));
  if (!n_desired || !scale_factors || !level_off || !n_keypoints || max_keypoints < 0)
    return lorb::set_error(ctx, LORB_E_INVALID, "null argument");
  OrbPlan P;
  LORB_TRY(orb_plan(ctx, pyr, n_desired, scale_factors, &P));
  uint8_t* dd;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 1, pyr->data, (size_t)pyr_extent(pyr), &dd));
  LORB_TRY(enqueue_keypoints(ctx, pyr, dd, &P, ini_th, min_th));
  const size_t cap = (size_t)std::max(P.out_cap, 1);
  float *lx, *ly, *sx, *sy, *sz, *rs;
  int *oc, *lo, *nt;
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 44, cap, &lx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 45, cap, &ly));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 46, cap, &sx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 47, cap, &sy));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 6, cap, &sz));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 7, cap, &rs));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 3, cap, &oc));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 4, (size_t)LORB_MAX_LEVELS + 1, &lo));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 5, (size_t)1, &nt));
  hipLaunchKernelGGL(k_orb_gather, dim3(lorb::ceil_div(cap, 256)), dim3(256), 0, ctx->stream, P.A, (int)cap, lx, ly, sx,
                     sy, oc, sz, rs, lo, nt);
  LORB_CHECK_LAUNCH(ctx);
  int n = 0;
  LORB_HIP(ctx, hipMemcpyAsync(&n, nt, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(level_off, lo, sizeof(int) * (pyr->n_levels + 1), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (n < 0) return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "DistributeOctTree exceeded its node capacity");
  *n_keypoints = n;
  if (n > max_keypoints)
    return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints exceed max_keypoints = %d", n, max_keypoints);
  if (n > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(x, lx, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(y, ly, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(octave, oc, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(size, sz, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(response, rs, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

// diagnostics: lorb_orb_detect with the per-pass trace of the device quadtree (8 ints per pass:
// L, mode, dividing nodes, divided, new children, survivors, new L, pending children; 64 passes
// per level; trace holds n_levels * 512 ints)
int lorb_orb_debug_octree(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired,
                          const float* scale_factors, int32_t ini_th, int32_t min_th, int32_t* trace) {
  if (!ctx || !trace) return LORB_E_INVALID;
  LORB_TRY(check_orb(ctx, pyr, 0));
  OrbPlan P;
  LORB_TRY(orb_plan(ctx, pyr, n_desired, scale_factors, &P));
  uint8_t* dd;
  int* dtr;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 1, pyr->data, (size_t)pyr_extent(pyr), &dd));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 50, (size_t)pyr->n_levels * (64 * 72 + 16384), &dtr));
  LORB_HIP(ctx, hipMemsetAsync(dtr, 0, sizeof(int) * pyr->n_levels * (64 * 72 + 16384), ctx->stream));
  P.A.trace = dtr;
  LORB_TRY(enqueue_keypoints(ctx, pyr, dd, &P, ini_th, min_th));
  LORB_HIP(ctx, hipMemcpyAsync(trace, dtr, sizeof(int) * pyr->n_levels * (64 * 72 + 16384), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_orb_extract_capacity(int32_t rows, int32_t cols, int32_t n_levels, const float* scale_factors,
                              const int32_t* n_desired, int32_t* max_keypoints, int64_t* pyramid_bytes) {
  if (!scale_factors || !n_desired || !max_keypoints || rows < 1 || cols < 1 || n_levels < 1 || n_levels > LORB_MAX_LEVELS)
    return LORB_E_INVALID;
  lorb_image_pyramid L;
  const int64_t need = pyramid_layout(rows, cols, n_levels, scale_factors, &L);
  int cap = 0;
  for (int l = 0; l < n_levels; l++) cap += 4 * std::max(std::max(0, (int)n_desired[l]), 4) + 16;
  *max_keypoints = cap;
  if (pyramid_bytes) *pyramid_bytes = need;
  return LORB_OK;
}

// ORBextractor::operator() (src/ORBextractor.cpp:1087-1151) on the device.  d_image, d_pattern and
// every output are device arrays; d_n (1 int) and d_level_off (n_levels + 1 ints) too.  The call
// returns once the pyramid is built (its resize tables are host-staged); the rest runs async.
int lorb_orb_extract_dev(lorb_ctx* ctx, const uint8_t* d_image, int32_t rows, int32_t cols, int32_t step,
                         int32_t n_levels, const float* scale_factors, const int32_t* n_desired, int32_t ini_th,
                         int32_t min_th, const int32_t* d_pattern, int32_t max_keypoints, uint8_t* d_pyramid,
                         int64_t pyramid_bytes, float* d_x, float* d_y, int32_t* d_octave, float* d_size,
                         float* d_angle, float* d_response, uint8_t* d_desc, int32_t* d_level_off, int32_t* d_n) {
  if (!ctx) return LORB_E_INVALID;
  if (!d_image || !scale_factors || !n_desired || !d_pattern || !d_pyramid || !d_x || !d_y || !d_octave || !d_size ||
      !d_angle || !d_response || !d_desc || !d_level_off || !d_n || rows < 1 || cols < 1 || step < cols ||
      n_levels < 1 || n_levels > LORB_MAX_LEVELS)
    return lorb::set_error(ctx, LORB_E_INVALID, "bad image / level / output arguments");
  lorb_image_pyramid pyr;
  const int64_t need = pyramid_layout(rows, cols, n_levels, scale_factors, &pyr);
  if (pyramid_bytes < need)
    return lorb::set_error(ctx, LORB_E_INVALID, "pyramid buffer holds %lld bytes, %lld needed", (long long)pyramid_bytes,
                           (long long)need);
  OrbPlan P;
  LORB_TRY(orb_plan(ctx, &pyr, n_desired, scale_factors, &P));
  if (max_keypoints < P.out_cap)
    return lorb::set_error(ctx, LORB_E_INVALID, "max_keypoints %d below the extractor's bound %d (lorb_orb_extract_capacity)",
                           max_keypoints, P.out_cap);
  FastCell* dcells;
  int* dcnt;
  LORB_TRY(orb_alloc(ctx, &P, &dcells, &dcnt));  // uploads the cells; the pyramid's sync covers them
  LORB_TRY(enqueue_pyramid(ctx, d_image, rows, cols, step, pyr, d_pyramid));
  pyr.data = d_pyramid;
  OrbPyr Q{};
  for (int l = 0; l < n_levels; l++) { Q.offset[l] = pyr.offset[l]; Q.step[l] = pyr.step[l]; }
  if (!P.cells.empty())
    hipLaunchKernelGGL(k_orb_fast, dim3((unsigned)P.cells.size()), dim3(kFastThreads), 0, ctx->stream, d_pyramid, Q,
                       dcells, ini_th, min_th, const_cast<float*>(P.A.fx), const_cast<float*>(P.A.fy),
                       const_cast<float*>(P.A.fr), dcnt);
  hipLaunchKernelGGL(k_orb_octree, dim3(n_levels), dim3(kOctThreads), 0, ctx->stream, P.A);
  const size_t cap = (size_t)P.out_cap;
  float *lx, *ly;
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 44, cap, &lx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 45, cap, &ly));
  hipLaunchKernelGGL(k_orb_gather, dim3(lorb::ceil_div(cap, 256)), dim3(256), 0, ctx->stream, P.A, (int)cap, lx, ly, d_x,
                     d_y, d_octave, d_size, d_response, d_level_off, d_n);
  LORB_CHECK_LAUNCH(ctx);
  return enqueue_orb(ctx, &pyr, d_pyramid, (int)cap, d_n, lx, ly, d_octave, d_pattern, d_angle, d_desc);
}

int lorb_orb_extract(lorb_ctx* ctx, const uint8_t* image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                     const float* scale_factors, const int32_t* n_desired, int32_t ini_th, int32_t min_th,
                     const int32_t* pattern, int32_t max_keypoints, float* x, float* y, int32_t* octave, float* size,
                     float* angle, float* response, uint8_t* desc, int32_t* level_off, int32_t* n_keypoints) {
  if (!ctx) return LORB_E_INVALID;
  if (!image || !scale_factors || !n_desired || !pattern || !level_off || !n_keypoints || rows < 1 || cols < 1 ||
      step < cols || n_levels < 1 || n_levels > LORB_MAX_LEVELS || max_keypoints < 0)
    return lorb::set_error(ctx, LORB_E_INVALID, "bad image / level arguments");
  int32_t cap = 0;
  int64_t pb = 0;
  LORB_TRY(lorb_orb_extract_capacity(rows, cols, n_levels, scale_factors, n_desired, &cap, &pb));
  uint8_t *dimg, *dpyr, *ddesc;
  int32_t *dpat, *doct, *dlo, *dn;
  float *dx, *dy, *dsz, *dang, *drs;
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 16, image, (size_t)(rows - 1) * step + cols, &dimg));
  LORB_TRY(lorb::upload_t(ctx, S_ORB + 19, pattern, (size_t)1024, &dpat));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 17, (size_t)pb, &dpyr));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 48, (size_t)cap, &dx));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 49, (size_t)cap, &dy));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 2, (size_t)cap, &doct));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 6, (size_t)cap, &dsz));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 7, (size_t)cap, &dang));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 3, (size_t)cap, &drs));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 18, (size_t)cap * 32, &ddesc));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 4, (size_t)LORB_MAX_LEVELS + 1, &dlo));
  LORB_TRY(lorb::scratch_t(ctx, S_ORB + 5, (size_t)1, &dn));
  LORB_TRY(lorb_orb_extract_dev(ctx, dimg, rows, cols, step, n_levels, scale_factors, n_desired, ini_th, min_th, dpat, cap,
                                dpyr, pb, dx, dy, doct, dsz, dang, drs, ddesc, dlo, dn));
  int n = 0;
  LORB_HIP(ctx, hipMemcpyAsync(&n, dn, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipMemcpyAsync(level_off, dlo, sizeof(int) * (n_levels + 1), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (n < 0) return lorb::set_error(ctx, LORB_E_UNSUPPORTED, "DistributeOctTree exceeded its node capacity");
  *n_keypoints = n;
  if (n > max_keypoints)
    return lorb::set_error(ctx, LORB_E_INVALID, "%d keypoints exceed max_keypoints = %d", n, max_keypoints);
  if (n > 0) {
    LORB_HIP(ctx, hipMemcpyAsync(x, dx, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(y, dy, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(octave, doct, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(size, dsz, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(angle, dang, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(response, drs, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream));
    LORB_HIP(ctx, hipMemcpyAsync(desc, ddesc, (size_t)32 * n, hipMemcpyDeviceToHost, ctx->stream));
  }
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

}  // extern "C"
