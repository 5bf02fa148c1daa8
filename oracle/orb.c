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
  const float a = (float)cos(angle), b = (float)sin(angle);
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
