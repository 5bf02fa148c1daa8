// lorb_sincosf.h -- libm's single-precision cosf / sinf as the reference calls them
// (src/ORBextractor.cpp:114-115: `cos(angle)` on a float under `using namespace std` is
// std::cos(float) = cosf), restated for the device so that rBRIEF's sample offsets round exactly
// as on the reference's Linux host.
//
// The algorithm is the published one of glibc >= 2.28 (from ARM's optimized-routines, sincosf.h /
// sincosf_data.c): for |x| < pi/4 a double-precision polynomial; for |x| < 120 a reduction
// x - n pi/2 in double (n rounded from x * 2/pi * 2^24 by integer arithmetic) and the sine or cosine
// polynomial of the quadrant with the table's sign / negated-cosine variant.  Every step is one
// IEEE double operation (compiled with -ffp-contract=off), so host and device produce the same
// bits.  tests/test_sincosf.py checks this restatement against the libm of the machine running
// the tests for every float angle the descriptor forms ((float)deg * factorPI, deg in [0, 360)).
// Arguments with |x| >= 120 (never formed by the extractor: angles are in [0, 2 pi)) are outside the
// restated range and evaluate through the generic double path.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#ifdef __HIP_DEVICE_COMPILE__
#define LORB_SC_FN __host__ __device__ __forceinline__
#elif defined(__HIPCC__)
#define LORB_SC_FN __host__ __device__ inline
#else
#define LORB_SC_FN inline
#endif

namespace lorb_sc {

struct Tab {
  double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

// sincosf_data.c: [0] the plain polynomials, [1] with the cosine polynomial negated (quadrants 2, 3)
#define LORB_SC_TAB(neg)                                                                          \
  {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, (neg) * 0x1p0,             \
   (neg) * -0x1.ffffffd0c621cp-2, (neg) * 0x1.55553e1068f19p-5, (neg) * -0x1.6c087e89a359dp-10,   \
   (neg) * 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}

LORB_SC_FN uint32_t top12(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return (u >> 20) & 0x7ff;
}

// sinf_poly: n even -> sine polynomial of x, n odd -> cosine polynomial
LORB_SC_FN float poly(double x, double x2, const Tab& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = p.s2 + x2 * p.s3;
    const double x7 = x3 * x2;
    const double s = x + x3 * p.s1;
    return (float)(s + x7 * s1);
  }
  const double x4 = x2 * x2;
  const double c2 = p.c3 + x2 * p.c4;
  const double c1 = p.c0 + x2 * p.c1;
  const double x6 = x4 * x2;
  const double c = c1 + x4 * p.c2;
  return (float)(c + x6 * c2);
}

// reduce_fast without TOINT_INTRINSICS (x86_64): n = round(x * 2/pi) by integer arithmetic
LORB_SC_FN double reduce(double x, const Tab& p, int* np) {
  const double r = x * p.hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return x - n * p.hpi;
}

// is_cos = 0: sinf, 1: cosf
LORB_SC_FN float eval(float y, int is_cos) {
  const Tab t0 = LORB_SC_TAB(1.0), t1 = LORB_SC_TAB(-1.0);
  double x = y;
  if (top12(y) < top12(0x1.921FB6p-1f)) {  // |y| < pi/4
    const double x2 = x * x;
    if (top12(y) < top12(0x1p-12f)) return is_cos ? 1.0f : y;
    return poly(x, x2, t0, is_cos);
  }
  if (top12(y) < top12(120.0f)) {
    int n;
    x = reduce(x, t0, &n);
    const double s = t0.sign[n & 3];
    return poly(x * s, x * x, (n & 2) ? t1 : t0, is_cos ? (n ^ 1) : n);
  }
  return (float)(is_cos ? cos((double)y) : sin((double)y));
}

}  // namespace lorb_sc

LORB_SC_FN float lorb_cosf(float x) { return lorb_sc::eval(x, 1); }
LORB_SC_FN float lorb_sinf(float x) { return lorb_sc::eval(x, 0); }
