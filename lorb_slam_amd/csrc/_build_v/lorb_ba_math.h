// lorb_ba_math.h -- device math for the reprojection residuals of src/bundle_adjust.cpp.
//
// Residual values follow the reference functors exactly (T = double instantiation):
//   Xc = AngleAxisRotatePoint(aa, X) + t ;  u = Xc.x / Xc.z * fx + cx ;  r = (u - obs.u, ...)
// (PoseCost src/bundle_adjust.cpp:22-64 uses fx for v -> caller passes fyv = fx;
//  MPCost :68-113 and PoseMPCost :116-151 use fy).
// Jacobians are the analytic chain rule with forward-mode duals over the angle-axis only
// (Ceres AutoDiff differentiates the same expression; they agree to rounding).
#pragma once
#include <hip/hip_runtime.h>

namespace lorb {

struct Dual3 {  // value + d/d(aa0,aa1,aa2)
  double a, v0, v1, v2;
};
__device__ __forceinline__ Dual3 dconst(double a) { return {a, 0.0, 0.0, 0.0}; }
__device__ __forceinline__ Dual3 operator+(Dual3 f, Dual3 g) { return {f.a + g.a, f.v0 + g.v0, f.v1 + g.v1, f.v2 + g.v2}; }
__device__ __forceinline__ Dual3 operator-(Dual3 f, Dual3 g) { return {f.a - g.a, f.v0 - g.v0, f.v1 - g.v1, f.v2 - g.v2}; }
__device__ __forceinline__ Dual3 operator*(Dual3 f, Dual3 g) {
  return {f.a * g.a, f.a * g.v0 + f.v0 * g.a, f.a * g.v1 + f.v1 * g.a, f.a * g.v2 + f.v2 * g.a};
}
__device__ __forceinline__ Dual3 operator*(Dual3 f, double s) { return {f.a * s, f.v0 * s, f.v1 * s, f.v2 * s}; }

// ceres::AngleAxisRotatePoint is split into a per-rotation part (theta, cos, sin, unit axis --
// the transcendentals) and a per-point part, so that kernels evaluating many points under one
// camera compute the former once per camera.  The per-point operation sequence is unchanged,
// so split and fused evaluation give bit-identical results.
constexpr double kAarpEps = 2.220446049250313e-16;  // std::numeric_limits<double>::epsilon()

struct RotVal {  // value-only rotation state
  double cs, sn, w0, w1, w2, aa0, aa1, aa2;
  int big;  // theta^2 > eps (else first-order branch)
};
__device__ __forceinline__ RotVal rot_val(const double aa[3]) {
  RotVal R;
  R.aa0 = aa[0]; R.aa1 = aa[1]; R.aa2 = aa[2];
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  R.big = theta2 > kAarpEps;
  // evaluated on both branches and selected by value: stores through &R.sn / &R.cs on one branch
  // and plain zero stores on the other were merged into one store through a selected address,
  // which put R in scratch (24 B per lane in k_ba_bs2 / k_ba_chol_2s)
  const double th = sqrt(theta2);
  double sn, cs;
  sincos(th, &sn, &cs);
  const double ti = 1.0 / th;
  R.sn = R.big ? sn : 0.0; R.cs = R.big ? cs : 0.0;
  R.w0 = R.big ? aa[0] * ti : 0.0; R.w1 = R.big ? aa[1] * ti : 0.0; R.w2 = R.big ? aa[2] * ti : 0.0;
  return R;
}
__device__ __forceinline__ void aarp_s(const RotVal& R, const double pt[3], double out[3]) {
  if (R.big) {
    const double w0 = R.w0, w1 = R.w1, w2 = R.w2, cs = R.cs, sn = R.sn;
    const double x0 = w1 * pt[2] - w2 * pt[1], x1 = w2 * pt[0] - w0 * pt[2], x2 = w0 * pt[1] - w1 * pt[0];
    const double tmp = (w0 * pt[0] + w1 * pt[1] + w2 * pt[2]) * (1.0 - cs);
    out[0] = pt[0] * cs + x0 * sn + w0 * tmp;
    out[1] = pt[1] * cs + x1 * sn + w1 * tmp;
    out[2] = pt[2] * cs + x2 * sn + w2 * tmp;
  } else {
    out[0] = pt[0] + (R.aa1 * pt[2] - R.aa2 * pt[1]);
    out[1] = pt[1] + (R.aa2 * pt[0] - R.aa0 * pt[2]);
    out[2] = pt[2] + (R.aa0 * pt[1] - R.aa1 * pt[0]);
  }
}

struct RotJet {  // rotation state with d/d(aa) (forward-mode duals)
  Dual3 c, s, w0, w1, w2;
  double aa0, aa1, aa2;
  int big;
};
__device__ __forceinline__ RotJet rot_jet(const double aa[3]) {
  RotJet R;
  R.aa0 = aa[0]; R.aa1 = aa[1]; R.aa2 = aa[2];
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  R.big = theta2 > kAarpEps;
  if (R.big) {
    const Dual3 A0 = {aa[0], 1.0, 0.0, 0.0}, A1 = {aa[1], 0.0, 1.0, 0.0}, A2 = {aa[2], 0.0, 0.0, 1.0};
    const Dual3 t2 = A0 * A0 + A1 * A1 + A2 * A2;
    const double th = sqrt(t2.a);
    const double hinv = 0.5 / th;
    const Dual3 theta = {th, t2.v0 * hinv, t2.v1 * hinv, t2.v2 * hinv};
    double sn, cs;
    sincos(th, &sn, &cs);
    R.c = {cs, -sn * theta.v0, -sn * theta.v1, -sn * theta.v2};
    R.s = {sn, cs * theta.v0, cs * theta.v1, cs * theta.v2};
    const double ti = 1.0 / th;
    const double dti = -ti * ti;
    const Dual3 tinv = {ti, dti * theta.v0, dti * theta.v1, dti * theta.v2};
    R.w0 = A0 * tinv; R.w1 = A1 * tinv; R.w2 = A2 * tinv;
  } else {
    R.c = R.s = R.w0 = R.w1 = R.w2 = dconst(0.0);
  }
  return R;
}
// value + d(out)/d(aa) (3x3, row = output coord) + d(out)/d(pt) (3x3)
__device__ __forceinline__ void aarp_jac_s(const RotJet& R, const double pt[3], double out[3],
                                           double dO_daa[9], double dO_dpt[9]) {
  if (R.big) {
    const Dual3 c = R.c, s = R.s, w0 = R.w0, w1 = R.w1, w2 = R.w2;
    const Dual3 p0 = dconst(pt[0]), p1 = dconst(pt[1]), p2 = dconst(pt[2]);
    const Dual3 x0 = w1 * p2 - w2 * p1, x1 = w2 * p0 - w0 * p2, x2 = w0 * p1 - w1 * p0;
    const Dual3 omc = dconst(1.0) - c;
    const Dual3 tmp = (w0 * p0 + w1 * p1 + w2 * p2) * omc;
    const Dual3 o0 = p0 * c + x0 * s + w0 * tmp;
    const Dual3 o1 = p1 * c + x1 * s + w1 * tmp;
    const Dual3 o2 = p2 * c + x2 * s + w2 * tmp;
    out[0] = o0.a; out[1] = o1.a; out[2] = o2.a;
    dO_daa[0] = o0.v0; dO_daa[1] = o0.v1; dO_daa[2] = o0.v2;
    dO_daa[3] = o1.v0; dO_daa[4] = o1.v1; dO_daa[5] = o1.v2;
    dO_daa[6] = o2.v0; dO_daa[7] = o2.v1; dO_daa[8] = o2.v2;
    // R = c I + s [w]x + (1-c) w w^T
    const double cs = c.a, sn = s.a;
    const double W0 = w0.a, W1 = w1.a, W2 = w2.a, oc = omc.a;
    dO_dpt[0] = cs + oc * W0 * W0;      dO_dpt[1] = -sn * W2 + oc * W0 * W1; dO_dpt[2] = sn * W1 + oc * W0 * W2;
    dO_dpt[3] = sn * W2 + oc * W1 * W0; dO_dpt[4] = cs + oc * W1 * W1;       dO_dpt[5] = -sn * W0 + oc * W1 * W2;
    dO_dpt[6] = -sn * W1 + oc * W2 * W0; dO_dpt[7] = sn * W0 + oc * W2 * W1; dO_dpt[8] = cs + oc * W2 * W2;
  } else {
    const double aa[3] = {R.aa0, R.aa1, R.aa2};
    // first-order branch: out = pt + aa x pt
    out[0] = pt[0] + (aa[1] * pt[2] - aa[2] * pt[1]);
    out[1] = pt[1] + (aa[2] * pt[0] - aa[0] * pt[2]);
    out[2] = pt[2] + (aa[0] * pt[1] - aa[1] * pt[0]);
    // d(aa x pt)/d aa = -[pt]x
    dO_daa[0] = 0.0;    dO_daa[1] = pt[2];  dO_daa[2] = -pt[1];
    dO_daa[3] = -pt[2]; dO_daa[4] = 0.0;    dO_daa[5] = pt[0];
    dO_daa[6] = pt[1];  dO_daa[7] = -pt[0]; dO_daa[8] = 0.0;
    // I + [aa]x
    dO_dpt[0] = 1.0;    dO_dpt[1] = -aa[2]; dO_dpt[2] = aa[1];
    dO_dpt[3] = aa[2];  dO_dpt[4] = 1.0;    dO_dpt[5] = -aa[0];
    dO_dpt[6] = -aa[1]; dO_dpt[7] = aa[0];  dO_dpt[8] = 1.0;
  }
}

__device__ __forceinline__ void aarp_jac(const double aa[3], const double pt[3], double out[3],
                                         double dO_daa[9], double dO_dpt[9]) {
  aarp_jac_s(rot_jet(aa), pt, out, dO_daa, dO_dpt);
}

// plain double ceres::AngleAxisRotatePoint
__device__ __forceinline__ void aarp(const double aa[3], const double pt[3], double out[3]) {
  aarp_s(rot_val(aa), pt, out);
}

__device__ __forceinline__ void residual(const double pose[6], const double X[3], double fx,
                                         double fyv, double cx, double cy, double u, double v,
                                         double r[2]) {
  double p[3];
  aarp(pose, X, p);
  p[0] += pose[3]; p[1] += pose[4]; p[2] += pose[5];
  r[0] = p[0] / p[2] * fx + cx - u;
  r[1] = p[1] / p[2] * fyv + cy - v;
}

// residual + Jp (2x3, d/dX) + Jc (2x6, d/d(aa,t))
__device__ __forceinline__ void residual_jac_s(const RotJet& R, const double t[3], const double X[3],
                                               double fx, double fyv, double cx, double cy, double u,
                                               double v, double r[2], double Jp[6], double Jc[12]) {
  double p[3], daa[9], dpt[9];
  aarp_jac_s(R, X, p, daa, dpt);
  p[0] += t[0]; p[1] += t[1]; p[2] += t[2];
  const double iz = 1.0 / p[2];
  r[0] = p[0] / p[2] * fx + cx - u;
  r[1] = p[1] / p[2] * fyv + cy - v;
  // d(u,v)/d(p): [fx*iz, 0, -fx*p0*iz^2 ; 0, fyv*iz, -fyv*p1*iz^2]
  const double a0 = fx * iz, a2 = -fx * p[0] * iz * iz;
  const double b1 = fyv * iz, b2 = -fyv * p[1] * iz * iz;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    Jp[k] = a0 * dpt[k] + a2 * dpt[6 + k];
    Jp[3 + k] = b1 * dpt[3 + k] + b2 * dpt[6 + k];
    Jc[k] = a0 * daa[k] + a2 * daa[6 + k];
    Jc[6 + k] = b1 * daa[3 + k] + b2 * daa[6 + k];
  }
  Jc[3] = a0; Jc[4] = 0.0; Jc[5] = a2;
  Jc[9] = 0.0; Jc[10] = b1; Jc[11] = b2;
}

__device__ __forceinline__ void residual_jac(const double pose[6], const double X[3], double fx,
                                             double fyv, double cx, double cy, double u, double v,
                                             double r[2], double Jp[6], double Jc[12]) {
  residual_jac_s(rot_jet(pose), pose + 3, X, fx, fyv, cx, cy, u, v, r, Jp, Jc);
}

// residual with a precomputed rotation state (t = pose[3..5])
__device__ __forceinline__ void residual_s(const RotVal& R, const double t[3], const double X[3],
                                           double fx, double fyv, double cx, double cy, double u,
                                           double v, double r[2]) {
  double p[3];
  aarp_s(R, X, p);
  p[0] += t[0]; p[1] += t[1]; p[2] += t[2];
  r[0] = p[0] / p[2] * fx + cx - u;
  r[1] = p[1] / p[2] * fyv + cy - v;
}

}  // namespace lorb
