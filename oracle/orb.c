/*
 * orb.c -- TEST INFRASTRUCTURE ONLY (see lorb_oracle.h).  CPU restatement of the descriptor stage
 * of ORBextractor::operator() (src/ORBextractor.cpp:1087-1154), SURVEY §8f row 3:
 *   - the IC_Angle orientation of every keypoint on its pyramid level (:79-107, :487-493), with
 *     OpenCV 3.1's cv::fastAtan2 restated (core/src/mathfuncs.cpp: degree polynomial of order 7);
 *   - GaussianBlur(level, 7x7, sigma 2, BORDER_REFLECT_101) (:1131-1132) restated from OpenCV 3.1:
 *     getGaussianKernel(7, 2, CV_32F), and for 8U -> 8U smoothing kernels
 *     createSeparableLinearFilter's fixed-point path (kernel * 256 rounded to int, integer row and
 *     column passes, (s + 2^15) >> 16 with saturation);
 *   - computeOrbDescriptor with the caller's 256-pair pattern (:110-150).
 * OpenCV is absent from this image, so the OpenCV parts are restated from its published source
 * (version pinned by the reference: find_package(OpenCV 3.1), CMakeLists.txt:10) and are
 * "parity unpinned"; tests/ cross-check them against independent numpy/scipy computations.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lorb_oracle.h"

#define HALF_PATCH_SIZE 15
#define OR_CV_PI 3.1415926535897932384626433832795  /* CV_PI */

/* ORBextractor::ORBextractor, src/ORBextractor.cpp:469-483: row half-widths of the circular patch */
void or_orb_umax(int* umax /* HALF_PATCH_SIZE + 1 */) {
  int v, v0;
  const int vmax = (int)floor(HALF_PATCH_SIZE * sqrt(2.f) / 2 + 1);
  const int vmin = (int)ceil(HALF_PATCH_SIZE * sqrt(2.f) / 2);
  const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
  for (v = 0; v <= vmax; ++v) umax[v] = (int)lrint(sqrt(hp2 - v * v));
  for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
}

/* cv::fastAtan2 (OpenCV 3.1), degrees in [0, 360) */
float or_fast_atan2(float y, float x) {
  const float p1 = 0.9997878412794807f * (float)(180 / OR_CV_PI);
  const float p3 = -0.3258083974640975f * (float)(180 / OR_CV_PI);
  const float p5 = 0.1555786518463281f * (float)(180 / OR_CV_PI);
  const float p7 = -0.04432655554792128f * (float)(180 / OR_CV_PI);
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

/* cv::getGaussianKernel(7, 2, CV_32F) then convertTo(CV_32S, 256) (float arithmetic, cvRound) */
void or_orb_gauss_kernel(int32_t* k7) {
  float cf[7];
  double sum = 0;
  const double sigmaX = 2.0, scale2X = -0.5 / (sigmaX * sigmaX);
  for (int i = 0; i < 7; i++) {
    const double x = i - (7 - 1) * 0.5;
    cf[i] = (float)exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  for (int i = 0; i < 7; i++) cf[i] = (float)(cf[i] * sum);
  for (int i = 0; i < 7; i++) k7[i] = (int32_t)lrintf(cf[i] * 256.f);
}

static int reflect101(int p, int n) {  /* BORDER_REFLECT_101: gfedcb|abcdefgh|gfedcba */
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

/* GaussianBlur(src, dst, Size(7,7), 2, 2, BORDER_REFLECT_101) on one 8U image (rows x cols) */
void or_orb_blur(const uint8_t* src, int rows, int cols, int sstep, uint8_t* dst, int dstep) {
  int32_t k[7];
  or_orb_gauss_kernel(k);
  int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * (size_t)(rows > 0 ? rows : 1) * (size_t)(cols > 0 ? cols : 1));
  for (int y = 0; y < rows; y++)
    for (int x = 0; x < cols; x++) {
      int32_t s = 0;
      for (int d = -3; d <= 3; d++) s += k[d + 3] * src[(size_t)y * sstep + reflect101(x + d, cols)];
      tmp[(size_t)y * cols + x] = s;
    }
  for (int y = 0; y < rows; y++)
    for (int x = 0; x < cols; x++) {
      int64_t s = 0;
      for (int d = -3; d <= 3; d++) s += (int64_t)k[d + 3] * tmp[(size_t)reflect101(y + d, rows) * cols + x];
      int64_t v = (s + (1 << 15)) >> 16;
      dst[(size_t)y * dstep + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
  free(tmp);
}

/* IC_Angle, src/ORBextractor.cpp:79-107 (pt in level coordinates) */
float or_orb_ic_angle(const uint8_t* img, int step, float px, float py, const int* umax) {
  int m_01 = 0, m_10 = 0;
  const uint8_t* center = img + (ptrdiff_t)lrintf(py) * step + lrintf(px);
  for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
  for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
    int v_sum = 0;
    const int d = umax[v];
    for (int u = -d; u <= d; ++u) {
      const int val_plus = center[u + v * step], val_minus = center[u - v * step];
      v_sum += (val_plus - val_minus);
      m_10 += u * (val_plus + val_minus);
    }
    m_01 += v * v_sum;
  }
  return or_fast_atan2((float)m_01, (float)m_10);
}

/* computeOrbDescriptor, src/ORBextractor.cpp:110-150 */
void or_orb_descriptor(const uint8_t* img, int step, float px, float py, float angle_deg, const int32_t* pattern,
                       uint8_t* desc) {
  const float factorPI = (float)(OR_CV_PI / 180.f);
  const float angle = angle_deg * factorPI;
  /* `cos(angle)` with a float argument under `using namespace std` (:69) is std::cos(float), i.e.
   * libm's cosf / sinf -- not the double cos rounded to float (they differ on ~0.1 % of angles) */
  const float a = cosf(angle), b = sinf(angle);
  const uint8_t* center = img + (ptrdiff_t)lrintf(py) * step + lrintf(px);
  for (int i = 0; i < 32; ++i) {
    int val = 0;
    for (int k = 0; k < 8; ++k) {
      const int32_t* p0 = pattern + 4 * (8 * i + k);  /* points 2 (8i+k) and 2 (8i+k) + 1 */
      const int t0 = center[lrintf(p0[0] * b + p0[1] * a) * step + lrintf(p0[0] * a - p0[1] * b)];
      const int t1 = center[lrintf(p0[2] * b + p0[3] * a) * step + lrintf(p0[2] * a - p0[3] * b)];
      val |= (t0 < t1) << k;
    }
    desc[i] = (uint8_t)val;
  }
}

/* The descriptor stage over a pyramid: angle (computeOrientation on the raw level), then the
 * descriptor on the blurred level.  Keypoint coordinates are level coordinates. */
void or_orb_describe(const lorb_image_pyramid* P, int n, const float* x, const float* y, const int32_t* level,
                     const int32_t* pattern, float* angle, uint8_t* desc) {
  int umax[HALF_PATCH_SIZE + 1];
  or_orb_umax(umax);
  uint8_t* blurred[LORB_MAX_LEVELS] = {0};
  for (int l = 0; l < P->n_levels; l++) {
    blurred[l] = (uint8_t*)malloc((size_t)(P->rows[l] > 0 ? P->rows[l] : 1) * (size_t)(P->cols[l] > 0 ? P->cols[l] : 1));
    or_orb_blur(P->data + P->offset[l], P->rows[l], P->cols[l], P->step[l], blurred[l], P->cols[l]);
  }
  for (int i = 0; i < n; i++) {
    const int l = level[i];
    angle[i] = or_orb_ic_angle(P->data + P->offset[l], P->step[l], x[i], y[i], umax);
    or_orb_descriptor(blurred[l], P->cols[l], x[i], y[i], angle[i], pattern, desc + 32 * (size_t)i);
  }
  for (int l = 0; l < P->n_levels; l++) free(blurred[l]);
}

/* ---- ORBextractor::ComputePyramid (src/ORBextractor.cpp:1157-1184) ------------------------
 * Level 0 is the image; level l is cv::resize(level l-1, Size(cvRound(cols * inv_l),
 * cvRound(rows * inv_l)), INTER_LINEAR) with inv_l = 1.0f / scale_l.  OpenCV 3.1's 8U linear
 * resize is restated from imgwarp.cpp: fixed-point taps (cvRound(c * 2048) as short), exact
 * integer horizontal pass, and the vertical pass of VResizeLinearVec_32s8u (SSE2) for the first
 * columns -- (S >> 4) as int16, _mm_mulhi_epi16 with the taps, saturating add, (+2) >> 2, packus --
 * followed by the scalar FixedPtCast ((s + 2^21) >> 22) for the remaining ones.  The borders
 * copyMakeBorder adds are never read downstream (keypoints keep EDGE_THRESHOLD) and are not
 * produced.  IPP builds of OpenCV may resize differently; that cannot be checked here. */
static int16_t sat16(int v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
static uint8_t satu8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

int or_resize_simd_cols(int width) {  /* columns [0, x) take the SSE2 path */
  int x = 0;
  while (x <= width - 16) x += 16;
  while (x < width - 4) x += 4;
  return x;
}

void or_resize_tabs(int ssize, int dsize, int* ofs, int16_t* a /* 2 per entry */, int* xmax_out) {
  const double inv_scale = (double)dsize / ssize, scale = 1. / inv_scale;
  int xmax = dsize;
  for (int dx = 0; dx < dsize; dx++) {
    float f = (float)((dx + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= s;
    if (s < 0) { f = 0; s = 0; }  /* sx < ksize2 - 1 = 0 */
    if (s + 1 >= ssize) {
      xmax = xmax < dx ? xmax : dx;
      if (s >= ssize - 1) { f = 0; s = ssize - 1; }
    }
    ofs[dx] = s;
    const float c0 = 1.f - f, c1 = f;
    a[2 * dx] = sat16((int)lrintf(c0 * 2048));
    a[2 * dx + 1] = sat16((int)lrintf(c1 * 2048));
  }
  if (xmax_out) *xmax_out = xmax;
}

void or_resize_linear_8u(const uint8_t* src, int sh, int sw, int sstep, uint8_t* dst, int dh, int dw, int dstep) {
  int* xofs = (int*)malloc(sizeof(int) * dw);
  int* yofs = (int*)malloc(sizeof(int) * dh);
  int16_t* ia = (int16_t*)malloc(sizeof(int16_t) * 2 * dw);
  int16_t* ib = (int16_t*)malloc(sizeof(int16_t) * 2 * dh);
  int xmax;
  or_resize_tabs(sw, dw, xofs, ia, &xmax);
  /* rows: fy = (float)((dy+0.5)*scale_y - 0.5), sy = floor, no clamp of fy here (imgwarp.cpp) */
  {
    const double scale_y = 1. / ((double)dh / sh);
    for (int dy = 0; dy < dh; dy++) {
      float f = (float)((dy + 0.5) * scale_y - 0.5);
      const int s = (int)floorf(f);
      f -= s;
      yofs[dy] = s;
      ib[2 * dy] = sat16((int)lrintf((1.f - f) * 2048));
      ib[2 * dy + 1] = sat16((int)lrintf(f * 2048));
    }
  }
  const int xs = or_resize_simd_cols(dw);
  int* r0 = (int*)malloc(sizeof(int) * dw);
  int* r1 = (int*)malloc(sizeof(int) * dw);
  for (int dy = 0; dy < dh; dy++) {
    int* rr[2] = {r0, r1};
    for (int k = 0; k < 2; k++) {
      int sy = yofs[dy] + k;
      sy = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);  /* clip(sy0 - ksize2 + 1 + k, 0, height) */
      const uint8_t* S = src + (size_t)sy * sstep;
      for (int dx = 0; dx < dw; dx++) {
        const int sx = xofs[dx];
        rr[k][dx] = dx < xmax ? S[sx] * ia[2 * dx] + S[sx + 1] * ia[2 * dx + 1] : S[sx] * 2048;
      }
    }
    const int b0 = ib[2 * dy], b1 = ib[2 * dy + 1];
    uint8_t* D = dst + (size_t)dy * dstep;
    for (int x = 0; x < dw; x++) {
      if (x < xs) {
        const int16_t x0 = sat16(r0[x] >> 4), y0 = sat16(r1[x] >> 4);
        const int16_t m0 = (int16_t)(((int)x0 * b0) >> 16), m1 = (int16_t)(((int)y0 * b1) >> 16);
        const int16_t s = sat16((int)m0 + (int)m1);
        const int16_t t = (int16_t)(sat16((int)s + 2) >> 2);
        D[x] = satu8(t);
      } else {
        D[x] = satu8((r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22);
      }
    }
  }
  free(xofs); free(yofs); free(ia); free(ib); free(r0); free(r1);
}

/* the pyramid of one image: level l is rows_l x cols_l with cvRound((float)size * (1.0f / scale_l)),
 * packed row-major in `out` at the offsets it returns in P (data = out) */
void or_orb_pyramid(const uint8_t* img, int rows, int cols, int step, int n_levels, const float* scale_factors,
                    uint8_t* out, lorb_image_pyramid* P) {
  int64_t off = 0;
  memset(P, 0, sizeof(*P));
  P->n_levels = n_levels;
  for (int l = 0; l < n_levels; l++) {
    const float inv = 1.0f / scale_factors[l];
    const int w = (int)lrintf((float)cols * inv), h = (int)lrintf((float)rows * inv);
    P->offset[l] = off; P->rows[l] = h; P->cols[l] = w; P->step[l] = w;
    uint8_t* D = out + off;
    if (l == 0) {
      for (int r = 0; r < h; r++) memcpy(D + (size_t)r * w, img + (size_t)r * step, (size_t)w);
    } else {
      or_resize_linear_8u(out + P->offset[l - 1], P->rows[l - 1], P->cols[l - 1], P->step[l - 1], D, h, w, w);
    }
    off += (int64_t)w * h;
  }
  P->data = out;
}

/* ORBextractor::operator() (src/ORBextractor.cpp:1087-1151) on one image: ComputePyramid,
 * ComputeKeyPointsOctTree (keypoints + IC_Angle orientation, :895-896), then per level the Gaussian
 * blur and the descriptors, and the keypoint coordinates scaled to level 0 (pt *= mvScaleFactor[l]
 * for l != 0, :1141-1147).  Outputs in the reference's order (level, then DistributeOctTree's list
 * order): x, y, octave, size, angle, response, desc (32 bytes each); level_off[n_levels + 1].
 * Returns the keypoint count or -1. */
int or_orb_extract(const uint8_t* img, int rows, int cols, int step, int n_levels, const float* scale_factors,
                   const int32_t* n_desired, int ini_th, int min_th, const int32_t* pattern, int max_kp, float* ox,
                   float* oy, int32_t* ooct, float* osize, float* oangle, float* oresp, uint8_t* odesc,
                   int32_t* level_off) {
  size_t total = 0;
  for (int l = 0; l < n_levels; l++) {
    const float inv = 1.0f / scale_factors[l];
    total += (size_t)lrintf((float)rows * inv) * (size_t)lrintf((float)cols * inv);
  }
  uint8_t* pyr = (uint8_t*)malloc(total + 16);
  lorb_image_pyramid P;
  memset(&P, 0, sizeof(P));
  or_orb_pyramid(img, rows, cols, step, n_levels, scale_factors, pyr, &P);
  P.data = pyr;
  const int n = or_orb_detect(&P, n_desired, scale_factors, ini_th, min_th, max_kp, ox, oy, ooct, osize, oresp,
                              level_off);
  if (n < 0) { free(pyr); return -1; }
  or_orb_describe(&P, n, ox, oy, ooct, pattern, oangle, odesc);
  for (int i = 0; i < n; i++)
    if (ooct[i] != 0) { ox[i] = ox[i] * scale_factors[ooct[i]]; oy[i] = oy[i] * scale_factors[ooct[i]]; }
  free(pyr);
  return n;
}
