/*
 * ba.c -- TEST INFRASTRUCTURE ONLY (parity unpinned vs the real reference; see lorb_oracle.h).
 *
 * CPU restatement of BA::ProjectPoseOptimization (src/bundle_adjust.cpp:158-202) and
 * BA::LocalPoseOptimization (src/bundle_adjust.cpp:207-330) together with the third-party
 * algorithm they call: ceres::Solve with default options + DENSE_SCHUR,
 * ceres::AutoDiffCostFunction Jets and ceres::AngleAxisRotatePoint.  Ceres is not vendored by
 * the reference and its version is unpinned (CMakeLists.txt:19); its published algorithm
 * (trust_region_minimizer / levenberg_marquardt_strategy / schur_eliminator, Ceres 1.x-2.x)
 * is restated here.
 */
#include "lorb_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define JN 9
typedef struct { double a; double v[JN]; } jet;

static jet jc(double a) { jet r; r.a = a; memset(r.v, 0, sizeof(r.v)); return r; }
static jet jvar(double a, int k) { jet r = jc(a); r.v[k] = 1.0; return r; }
static jet jadd(jet f, jet g) { jet r; r.a = f.a + g.a; for (int i = 0; i < JN; i++) r.v[i] = f.v[i] + g.v[i]; return r; }
static jet jsub(jet f, jet g) { jet r; r.a = f.a - g.a; for (int i = 0; i < JN; i++) r.v[i] = f.v[i] - g.v[i]; return r; }
static jet jmul(jet f, jet g) {
  jet r; r.a = f.a * g.a;
  for (int i = 0; i < JN; i++) r.v[i] = f.a * g.v[i] + f.v[i] * g.a;
  return r;
}
static jet jdiv(jet f, jet g) {  /* ceres/jet.h operator/(Jet, Jet) */
  const double gi = 1.0 / g.a;
  const double fg = f.a * gi;
  jet r; r.a = fg;
  for (int i = 0; i < JN; i++) r.v[i] = (f.v[i] - fg * g.v[i]) * gi;
  return r;
}
static jet jsqrt(jet f) {
  const double t = sqrt(f.a);
  const double two_a_inv = 1.0 / (2.0 * t);
  jet r; r.a = t;
  for (int i = 0; i < JN; i++) r.v[i] = f.v[i] * two_a_inv;
  return r;
}
static jet jcos(jet f) { jet r; r.a = cos(f.a); const double s = -sin(f.a); for (int i = 0; i < JN; i++) r.v[i] = s * f.v[i]; return r; }
static jet jsin(jet f) { jet r; r.a = sin(f.a); const double c = cos(f.a); for (int i = 0; i < JN; i++) r.v[i] = c * f.v[i]; return r; }

/* ceres::AngleAxisRotatePoint (ceres/rotation.h), templated on Jet */
static void jet_aarp(const jet aa[3], const jet pt[3], jet out[3]) {
  const jet theta2 = jadd(jadd(jmul(aa[0], aa[0]), jmul(aa[1], aa[1])), jmul(aa[2], aa[2]));
  if (theta2.a > DBL_EPSILON) {
    const jet theta = jsqrt(theta2);
    const jet c = jcos(theta);
    const jet s = jsin(theta);
    const jet ti = jdiv(jc(1.0), theta);
    const jet w[3] = {jmul(aa[0], ti), jmul(aa[1], ti), jmul(aa[2], ti)};
    const jet wx[3] = {jsub(jmul(w[1], pt[2]), jmul(w[2], pt[1])),
                       jsub(jmul(w[2], pt[0]), jmul(w[0], pt[2])),
                       jsub(jmul(w[0], pt[1]), jmul(w[1], pt[0]))};
    const jet tmp = jmul(jadd(jadd(jmul(w[0], pt[0]), jmul(w[1], pt[1])), jmul(w[2], pt[2])),
                         jsub(jc(1.0), c));
    for (int i = 0; i < 3; i++) out[i] = jadd(jadd(jmul(pt[i], c), jmul(wx[i], s)), jmul(w[i], tmp));
  } else {
    const jet wx[3] = {jsub(jmul(aa[1], pt[2]), jmul(aa[2], pt[1])),
                       jsub(jmul(aa[2], pt[0]), jmul(aa[0], pt[2])),
                       jsub(jmul(aa[0], pt[1]), jmul(aa[1], pt[0]))};
    for (int i = 0; i < 3; i++) out[i] = jadd(pt[i], wx[i]);
  }
}

/* plain double AngleAxisRotatePoint */
void or_angle_axis_rotate_point(const double aa[3], const double pt[3], double out[3]) {
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > DBL_EPSILON) {
    const double theta = sqrt(theta2);
    const double c = cos(theta), s = sin(theta), ti = 1.0 / theta;
    const double w[3] = {aa[0] * ti, aa[1] * ti, aa[2] * ti};
    const double wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
    const double tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (1.0 - c);
    for (int i = 0; i < 3; i++) out[i] = pt[i] * c + wx[i] * s + w[i] * tmp;
  } else {
    const double wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
    for (int i = 0; i < 3; i++) out[i] = pt[i] + wx[i];
  }
}

/* Residual functors, src/bundle_adjust.cpp:22-151.  kind 0 PoseCost(R,T) with v*fy_eff,
 * 1 MPCost(X) with a constant float pose, 2 PoseMPCost(X, pose). */
void or_residual_jet(int kind, const double* X, const double* pose, double fx, double fy,
                     double cx, double cy, double u, double v, double* res, double* jac) {
  jet aa[3], t[3], p[3], rp[3];
  int np;
  if (kind == 0) {        /* PoseCost: params (tempR[3], tempT[3]) */
    for (int i = 0; i < 3; i++) { aa[i] = jvar(pose[i], i); t[i] = jvar(pose[3 + i], 3 + i); p[i] = jc(X[i]); }
    np = 6;
  } else if (kind == 1) { /* MPCost: params (tempMP[3]) */
    for (int i = 0; i < 3; i++) { aa[i] = jc(pose[i]); t[i] = jc(pose[3 + i]); p[i] = jvar(X[i], i); }
    np = 3;
  } else {                /* PoseMPCost: params (tempMP[3], tempPose[6]) */
    for (int i = 0; i < 3; i++) { p[i] = jvar(X[i], i); aa[i] = jvar(pose[i], 3 + i); t[i] = jvar(pose[3 + i], 6 + i); }
    np = 9;
  }
  jet_aarp(aa, p, rp);
  for (int i = 0; i < 3; i++) rp[i] = jadd(rp[i], t[i]);
  const jet uu = jadd(jmul(jdiv(rp[0], rp[2]), jc(fx)), jc(cx));
  const jet vv = jadd(jmul(jdiv(rp[1], rp[2]), jc(fy)), jc(cy));
  const jet r0 = jsub(uu, jc(u));
  const jet r1 = jsub(vv, jc(v));
  res[0] = r0.a; res[1] = r1.a;
  if (jac) for (int k = 0; k < np; k++) { jac[k] = r0.v[k]; jac[np + k] = r1.v[k]; }
}

/* T = double instantiation of the same functors (residual-only evaluation) */
static void residual_plain(int kind, const double* X, const double* pose, double fx, double fy,
                           double cx, double cy, double u, double v, double* res) {
  double rp[3];
  (void)kind;
  or_angle_axis_rotate_point(pose, X, rp);
  for (int i = 0; i < 3; i++) rp[i] += pose[3 + i];
  res[0] = rp[0] / rp[2] * fx + cx - u;
  res[1] = rp[1] / rp[2] * fy + cy - v;
}

/* ---------------------------------------------------------------------------------------- */
typedef struct {
  int kind, point, pose;   /* point / pose block index or -1 */
  double X[3];             /* PoseCost constant point */
  double fpose[6];         /* MPCost constant pose */
  double fx, fy, cx, cy, u, v;
} or_res;

typedef struct {
  int n_pose, n_point, n_res;
  or_res* res;
} or_prob;

void or_lm_options_default(lorb_lm_options* o) {
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
}

/* x layout: [n_pose*6 | n_point*3] */
static const double* res_pose(const or_prob* P, const or_res* r, const double* x) {
  return r->pose >= 0 ? x + 6 * r->pose : r->fpose;
}
static const double* res_point(const or_prob* P, const or_res* r, const double* x) {
  return r->point >= 0 ? x + 6 * P->n_pose + 3 * r->point : r->X;
}

static double eval_cost(const or_prob* P, const double* x) {
  double cost = 0.0;
  for (int k = 0; k < P->n_res; k++) {
    const or_res* r = &P->res[k];
    double rr[2];
    residual_plain(r->kind, res_point(P, r, x), res_pose(P, r, x), r->fx, r->fy, r->cx, r->cy, r->u, r->v, rr);
    cost += 0.5 * (rr[0] * rr[0] + rr[1] * rr[1]);
  }
  return cost;
}

/* residuals + block Jacobians: Jp (2x3 row-major) and Jc (2x6 row-major), unscaled */
static double eval_jac(const or_prob* P, const double* x, double* r, double* Jp, double* Jc) {
  double cost = 0.0;
  for (int k = 0; k < P->n_res; k++) {
    const or_res* q = &P->res[k];
    double jac[18];
    or_residual_jet(q->kind, res_point(P, q, x), res_pose(P, q, x), q->fx, q->fy, q->cx, q->cy, q->u, q->v, r + 2 * k, jac);
    memset(Jp + 6 * k, 0, 6 * sizeof(double));
    memset(Jc + 12 * k, 0, 12 * sizeof(double));
    if (q->kind == 0) {
      for (int i = 0; i < 2; i++) for (int j = 0; j < 6; j++) Jc[12 * k + 6 * i + j] = jac[6 * i + j];
    } else if (q->kind == 1) {
      for (int i = 0; i < 2; i++) for (int j = 0; j < 3; j++) Jp[6 * k + 3 * i + j] = jac[3 * i + j];
    } else {
      for (int i = 0; i < 2; i++) {
        for (int j = 0; j < 3; j++) Jp[6 * k + 3 * i + j] = jac[9 * i + j];
        for (int j = 0; j < 6; j++) Jc[12 * k + 6 * i + j] = jac[9 * i + 3 + j];
      }
    }
    cost += 0.5 * (r[2 * k] * r[2 * k] + r[2 * k + 1] * r[2 * k + 1]);
  }
  return cost;
}

/* in-place lower Cholesky of an n x n row-major SPD matrix; returns 0 on failure */
static int chol(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double d = A[j * n + j];
    for (int k = 0; k < j; k++) d -= A[j * n + k] * A[j * n + k];
    if (!(d > 0.0)) return 0;
    const double l = sqrt(d);
    A[j * n + j] = l;
    for (int i = j + 1; i < n; i++) {
      double s = A[i * n + j];
      for (int k = 0; k < j; k++) s -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = s / l;
    }
  }
  return 1;
}
static void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; i++) { double s = b[i]; for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k]; b[i] = s / L[i * n + i]; }
  for (int i = n - 1; i >= 0; i--) { double s = b[i]; for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k]; b[i] = s / L[i * n + i]; }
}
static int inv3_spd(const double* A, double* inv) {
  double L[9];
  memcpy(L, A, sizeof(L));
  if (!chol(L, 3)) return 0;
  for (int c = 0; c < 3; c++) {
    double e[3] = {0, 0, 0};
    e[c] = 1.0;
    chol_solve(L, 3, e);
    for (int r = 0; r < 3; r++) inv[3 * r + c] = e[r];
  }
  return 1;
}

/* Point-partitioned solve (the multi-GPU design): every rank holds all poses and
 * its own points.  R == NULL: single process.  Otherwise every quantity that sums over
 * residuals is all-reduced through R->fn, exactly where the GPU path exchanges. */
typedef struct {
  or_allreduce_fn fn;
  void* user;
  int rank;
} or_reducer;
static int ar(const or_reducer* R, double* buf, int64_t n, int op) { return R ? R->fn(R->user, buf, n, op) : 0; }
static double ar1(const or_reducer* R, double v, int op) { if (R) R->fn(R->user, &v, 1, op); return v; }

typedef struct {
  double *r, *Jp, *Jc;           /* current residuals and SCALED jacobians */
  int* pt_res_off; int* pt_res;  /* residuals of each point (CSR) */
} lin_state;

/* Solve (Js^T Js + D^2) y = Js^T r by Schur elimination of the point blocks
 * (ceres SchurEliminator + DenseSchurComplementSolver).  Returns 0 on failure. */
static int schur_solve(const or_prob* P, const lin_state* L, const double* D, double* y, const or_reducer* R) {
  const int nc = 6 * P->n_pose;
  double* S = (double*)calloc((size_t)nc * nc + 1, sizeof(double));
  double* rhs = (double*)calloc((size_t)nc + 1, sizeof(double));
  int ok = 1;
  /* camera (F) blocks: F^T F + D_f^2, F^T b */
  for (int k = 0; k < P->n_res; k++) {
    const or_res* q = &P->res[k];
    if (q->pose < 0) continue;
    const double* J = L->Jc + 12 * k;
    const int c0 = 6 * q->pose;
    for (int a = 0; a < 6; a++) {
      rhs[c0 + a] += J[a] * L->r[2 * k] + J[6 + a] * L->r[2 * k + 1];
      for (int b = 0; b < 6; b++) S[(c0 + a) * nc + c0 + b] += J[a] * J[b] + J[6 + a] * J[6 + b];
    }
  }
  if (!R || R->rank == 0)
    for (int i = 0; i < nc; i++) S[i * nc + i] += D[i] * D[i];
  /* eliminate every point block */
  double* ete_inv = (double*)malloc(sizeof(double) * 9 * (size_t)(P->n_point > 0 ? P->n_point : 1));
  double* etb = (double*)malloc(sizeof(double) * 3 * (size_t)(P->n_point > 0 ? P->n_point : 1));
  for (int p = 0; p < P->n_point && ok; p++) {
    double ete[9] = {0}, b[3] = {0};
    for (int e = L->pt_res_off[p]; e < L->pt_res_off[p + 1]; e++) {
      const int k = L->pt_res[e];
      const double* J = L->Jp + 6 * k;
      for (int a = 0; a < 3; a++) {
        b[a] += J[a] * L->r[2 * k] + J[3 + a] * L->r[2 * k + 1];
        for (int c = 0; c < 3; c++) ete[3 * a + c] += J[a] * J[c] + J[3 + a] * J[3 + c];
      }
    }
    const double* Dp = D + nc + 3 * p;
    for (int a = 0; a < 3; a++) ete[4 * a] += Dp[a] * Dp[a];
    if (!inv3_spd(ete, ete_inv + 9 * p)) { ok = 0; if (!R) break; continue; }
    memcpy(etb + 3 * p, b, sizeof(b));
    const double* Ei = ete_inv + 9 * p;
    /* W_a = Jc_a^T Jp_a (6x3); Y_a = W_a Ei */
    for (int ea = L->pt_res_off[p]; ea < L->pt_res_off[p + 1]; ea++) {
      const int ka = L->pt_res[ea];
      const or_res* qa = &P->res[ka];
      if (qa->pose < 0) continue;
      double W[18], Y[18];
      const double* Jca = L->Jc + 12 * ka; const double* Jpa = L->Jp + 6 * ka;
      for (int i = 0; i < 6; i++) for (int j = 0; j < 3; j++) W[3 * i + j] = Jca[i] * Jpa[j] + Jca[6 + i] * Jpa[3 + j];
      for (int i = 0; i < 6; i++) for (int j = 0; j < 3; j++) Y[3 * i + j] = W[3 * i] * Ei[j] + W[3 * i + 1] * Ei[3 + j] + W[3 * i + 2] * Ei[6 + j];
      const int ca = 6 * qa->pose;
      for (int i = 0; i < 6; i++) rhs[ca + i] -= Y[3 * i] * b[0] + Y[3 * i + 1] * b[1] + Y[3 * i + 2] * b[2];
      for (int eb = L->pt_res_off[p]; eb < L->pt_res_off[p + 1]; eb++) {
        const int kb = L->pt_res[eb];
        const or_res* qb = &P->res[kb];
        if (qb->pose < 0) continue;
        double Wb[18];
        const double* Jcb = L->Jc + 12 * kb; const double* Jpb = L->Jp + 6 * kb;
        for (int i = 0; i < 6; i++) for (int j = 0; j < 3; j++) Wb[3 * i + j] = Jcb[i] * Jpb[j] + Jcb[6 + i] * Jpb[3 + j];
        const int cb = 6 * qb->pose;
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 6; j++)
            S[(ca + i) * nc + cb + j] -= Y[3 * i] * Wb[3 * j] + Y[3 * i + 1] * Wb[3 * j + 1] + Y[3 * i + 2] * Wb[3 * j + 2];
      }
    }
  }
  if (R) {  /* exchange 2: S, rhs and the point-block failure flag */
    ok = ar1(R, ok ? 0.0 : 1.0, LORB_OP_MAX) == 0.0;
    ar(R, S, (int64_t)nc * nc, LORB_OP_SUM);
    ar(R, rhs, nc, LORB_OP_SUM);
  }
  if (ok && nc > 0) {
    ok = chol(S, nc);
    if (ok) chol_solve(S, nc, rhs);
  }
  if (ok) {
    memcpy(y, rhs, sizeof(double) * (size_t)nc);
    for (int p = 0; p < P->n_point; p++) {
      double b[3] = {etb[3 * p], etb[3 * p + 1], etb[3 * p + 2]};
      for (int e = L->pt_res_off[p]; e < L->pt_res_off[p + 1]; e++) {
        const int k = L->pt_res[e];
        const or_res* q = &P->res[k];
        if (q->pose < 0) continue;
        const double* Jc = L->Jc + 12 * k; const double* Jp = L->Jp + 6 * k;
        const double* yc = y + 6 * q->pose;
        for (int j = 0; j < 3; j++) {
          double w = 0.0;
          for (int i = 0; i < 6; i++) w += (Jc[i] * Jp[j] + Jc[6 + i] * Jp[3 + j]) * yc[i];
          b[j] -= w;
        }
      }
      const double* Ei = ete_inv + 9 * p;
      for (int j = 0; j < 3; j++) y[nc + 3 * p + j] = Ei[3 * j] * b[0] + Ei[3 * j + 1] * b[1] + Ei[3 * j + 2] * b[2];
    }
    const int np = nc + 3 * P->n_point;
    for (int i = 0; i < np; i++) if (!isfinite(y[i])) { ok = 0; break; }
    if (R) ok = ar1(R, ok ? 0.0 : 1.0, LORB_OP_MAX) == 0.0;
  }
  free(S); free(rhs); free(ete_inv); free(etb);
  return ok;
}

/* Per-iteration records (lorb_lm_iteration) of the last lm_solve, when a sink is set: the iteration
 * summary Ceres' TrustRegionMinimizer keeps (cost, model cost change, candidate cost, radius, |step|). */
static lorb_lm_iteration* g_trace = NULL;
static int g_trace_cap = 0, g_trace_n = 0;
void or_lm_trace(lorb_lm_iteration* buf, int cap) { g_trace = buf; g_trace_cap = buf ? cap : 0; g_trace_n = 0; }
int or_lm_trace_count(void) { return g_trace_n; }
static void trace_put(int iter, int outcome, double cost, double mcc, double new_cost, double radius, double step_norm) {
  if (!g_trace || iter < 1 || iter > g_trace_cap) return;
  lorb_lm_iteration* r = &g_trace[iter - 1];
  r->iteration = iter; r->outcome = outcome; r->cost = cost; r->model_cost_change = mcc;
  r->new_cost = new_cost; r->radius = radius; r->step_norm = step_norm;
  if (iter > g_trace_n) g_trace_n = iter;
}

/* The Ceres TrustRegionMinimizer + LevenbergMarquardtStrategy loop (Appendix B). */
static int lm_solve(const or_prob* P, const lorb_lm_options* o, double* x, lorb_ba_summary* sum,
                    const or_reducer* R) {
  const int nc = 6 * P->n_pose;
  const int np = nc + 3 * P->n_point;
  const int nr = P->n_res;
  lin_state L;
  L.r = (double*)malloc(sizeof(double) * 2 * (size_t)(nr + 1));
  L.Jp = (double*)malloc(sizeof(double) * 6 * (size_t)(nr + 1));
  L.Jc = (double*)malloc(sizeof(double) * 12 * (size_t)(nr + 1));
  L.pt_res_off = (int*)calloc((size_t)P->n_point + 1, sizeof(int));
  L.pt_res = (int*)malloc(sizeof(int) * (size_t)(nr + 1));
  for (int k = 0; k < nr; k++) if (P->res[k].point >= 0) L.pt_res_off[P->res[k].point + 1]++;
  for (int p = 0; p < P->n_point; p++) L.pt_res_off[p + 1] += L.pt_res_off[p];
  {
    int* fill = (int*)calloc((size_t)P->n_point + 1, sizeof(int));
    for (int k = 0; k < nr; k++) { const int p = P->res[k].point; if (p >= 0) L.pt_res[L.pt_res_off[p] + fill[p]++] = k; }
    free(fill);
  }
  g_trace_n = 0;
  uint8_t* active = (uint8_t*)calloc((size_t)np + 1, 1);
  for (int k = 0; k < nr; k++) {
    if (P->res[k].pose >= 0) memset(active + 6 * P->res[k].pose, 1, 6);
    if (P->res[k].point >= 0) memset(active + nc + 3 * P->res[k].point, 1, 3);
  }
  if (R && nc > 0) {  /* a pose is active if any rank observes it */
    double* a = (double*)malloc(sizeof(double) * (size_t)nc);
    for (int i = 0; i < nc; i++) a[i] = active[i];
    ar(R, a, nc, LORB_OP_MAX);
    for (int i = 0; i < nc; i++) active[i] = a[i] > 0.0;
    free(a);
  }
  double* scale = (double*)malloc(sizeof(double) * (size_t)(np + 1));
  double* diag = (double*)malloc(sizeof(double) * (size_t)(np + 1));
  double* D = (double*)malloc(sizeof(double) * (size_t)(np + 1));
  double* y = (double*)malloc(sizeof(double) * (size_t)(np + 1));
  double* xn = (double*)malloc(sizeof(double) * (size_t)(np + 1));
  double* g = (double*)malloc(sizeof(double) * (size_t)(np + 1));

  /* gradient (unscaled J^T r) and column norms from the current L (unscaled) */
#define COLS_AND_GRAD(colsq, grad)                                                        \
  do {                                                                                    \
    memset(colsq, 0, sizeof(double) * (size_t)np);                                        \
    memset(grad, 0, sizeof(double) * (size_t)np);                                         \
    for (int k = 0; k < nr; k++) {                                                        \
      const or_res* q = &P->res[k];                                                       \
      if (q->pose >= 0)                                                                   \
        for (int j = 0; j < 6; j++) {                                                     \
          const double a = L.Jc[12 * k + j], b = L.Jc[12 * k + 6 + j];                    \
          colsq[6 * q->pose + j] += a * a + b * b;                                        \
          grad[6 * q->pose + j] += a * L.r[2 * k] + b * L.r[2 * k + 1];                   \
        }                                                                                 \
      if (q->point >= 0)                                                                  \
        for (int j = 0; j < 3; j++) {                                                     \
          const double a = L.Jp[6 * k + j], b = L.Jp[6 * k + 3 + j];                      \
          colsq[nc + 3 * q->point + j] += a * a + b * b;                                  \
          grad[nc + 3 * q->point + j] += a * L.r[2 * k] + b * L.r[2 * k + 1];             \
        }                                                                                 \
    }                                                                                     \
  } while (0)

  /* exchange 1 (per linearisation): cost, pose column norms and gradient (sum), gradient max */
#define LIN_EXCHANGE()                                                                    \
  do {                                                                                    \
    if (R) { cost = ar1(R, cost, LORB_OP_SUM); ar(R, diag, nc, LORB_OP_SUM); ar(R, g, nc, LORB_OP_SUM); } \
  } while (0)
#define GMAX()                                                                            \
  do {                                                                                    \
    gmax = 0.0;                                                                           \
    for (int i = 0; i < np; i++) if (active[i]) { const double d = fabs(x[i] - (x[i] + -g[i])); if (d > gmax) gmax = d; } \
    gmax = ar1(R, gmax, LORB_OP_MAX);                                                     \
  } while (0)
  double cost = eval_jac(P, x, L.r, L.Jp, L.Jc);
  COLS_AND_GRAD(diag, g);
  LIN_EXCHANGE();
  sum->initial_cost = cost;
  for (int i = 0; i < np; i++) scale[i] = o->jacobi_scaling ? 1.0 / (1.0 + sqrt(diag[i])) : 1.0;
  double gmax = 0.0;
  GMAX();
#define SCALE_J()                                                                         \
  do {                                                                                    \
    for (int k = 0; k < nr; k++) {                                                        \
      const or_res* q = &P->res[k];                                                       \
      if (q->pose >= 0)                                                                   \
        for (int j = 0; j < 6; j++) { L.Jc[12 * k + j] *= scale[6 * q->pose + j]; L.Jc[12 * k + 6 + j] *= scale[6 * q->pose + j]; } \
      if (q->point >= 0)                                                                  \
        for (int j = 0; j < 3; j++) { L.Jp[6 * k + j] *= scale[nc + 3 * q->point + j]; L.Jp[6 * k + 3 + j] *= scale[nc + 3 * q->point + j]; } \
    }                                                                                     \
  } while (0)
  SCALE_J();
  /* |x|: poses are replicated, points are rank-local */
#define XNORM()                                                                           \
  do {                                                                                    \
    double xp = 0.0, xq = 0.0;                                                            \
    for (int i = 0; i < nc; i++) if (active[i]) xp += x[i] * x[i];                        \
    for (int i = nc; i < np; i++) if (active[i]) xq += x[i] * x[i];                       \
    x_norm = sqrt(xp + ar1(R, xq, LORB_OP_SUM));                                          \
  } while (0)
  double x_norm = 0.0;
  XNORM();

  double radius = o->initial_trust_region_radius, decrease_factor = 2.0;
  int reuse_diagonal = 0, n_invalid = 0, iter = 0, n_success = 0;
  int term = LORB_TERM_NO_CONVERGENCE;
  int last_successful = 1;  /* IterationZero counts as a successful step */

  for (;;) {
    /* FinalizeIterationAndCheckIfMinimizerCanContinue */
    if (iter >= o->max_num_iterations) { term = LORB_TERM_NO_CONVERGENCE; break; }
    if (last_successful && gmax <= o->gradient_tolerance) { term = LORB_TERM_GRADIENT_TOL; break; }
    if (radius <= o->min_trust_region_radius) { term = LORB_TERM_MIN_RADIUS; break; }
    iter++;
    /* LevenbergMarquardtStrategy::ComputeStep */
    if (!reuse_diagonal) {
      double* colsq = diag;
      memset(colsq, 0, sizeof(double) * (size_t)np);
      for (int k = 0; k < nr; k++) {
        const or_res* q = &P->res[k];
        if (q->pose >= 0) for (int j = 0; j < 6; j++) { const double a = L.Jc[12 * k + j], b = L.Jc[12 * k + 6 + j]; colsq[6 * q->pose + j] += a * a + b * b; }
        if (q->point >= 0) for (int j = 0; j < 3; j++) { const double a = L.Jp[6 * k + j], b = L.Jp[6 * k + 3 + j]; colsq[nc + 3 * q->point + j] += a * a + b * b; }
      }
      ar(R, diag, nc, LORB_OP_SUM);
      for (int i = 0; i < np; i++) diag[i] = fmin(fmax(diag[i], o->min_lm_diagonal), o->max_lm_diagonal);
    }
    for (int i = 0; i < np; i++) D[i] = sqrt(diag[i] / radius);
    int solved = schur_solve(P, &L, D, y, R);
    reuse_diagonal = 1;
    double model_cost_change = 0.0;
    int valid = 0;
    if (solved) {
      for (int i = 0; i < np; i++) y[i] = -y[i];  /* step */
      double mcc = 0.0;
      for (int k = 0; k < nr; k++) {
        const or_res* q = &P->res[k];
        double m0 = 0.0, m1 = 0.0;
        if (q->point >= 0) for (int j = 0; j < 3; j++) { const double s = y[nc + 3 * q->point + j]; m0 += L.Jp[6 * k + j] * s; m1 += L.Jp[6 * k + 3 + j] * s; }
        if (q->pose >= 0) for (int j = 0; j < 6; j++) { const double s = y[6 * q->pose + j]; m0 += L.Jc[12 * k + j] * s; m1 += L.Jc[12 * k + 6 + j] * s; }
        mcc += m0 * (L.r[2 * k] + m0 / 2.0) + m1 * (L.r[2 * k + 1] + m1 / 2.0);
      }
      model_cost_change = -ar1(R, mcc, LORB_OP_SUM);  /* exchange 3 */
      valid = model_cost_change > 0.0;
    }
    if (!valid) {
      /* HandleInvalidStep -> StepIsInvalid == StepRejected(0) */
      trace_put(iter, LORB_LM_STEP_INVALID, cost, model_cost_change, 0.0, radius, 0.0);
      if (++n_invalid >= o->max_num_consecutive_invalid_steps) { term = LORB_TERM_FAILURE; break; }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = 1;
      last_successful = 0;
      continue;
    }
    n_invalid = 0;
    for (int i = 0; i < np; i++) xn[i] = x[i] + y[i] * scale[i];
    const double new_cost = ar1(R, eval_cost(P, xn), LORB_OP_SUM);
    double sp = 0.0, sq = 0.0;
    for (int i = 0; i < nc; i++) if (active[i]) { const double d = x[i] - xn[i]; sp += d * d; }
    for (int i = nc; i < np; i++) if (active[i]) { const double d = x[i] - xn[i]; sq += d * d; }
    const double step_norm = sqrt(sp + ar1(R, sq, LORB_OP_SUM));
    if (step_norm <= o->parameter_tolerance * (x_norm + o->parameter_tolerance)) {
      trace_put(iter, LORB_LM_STEP_PARAM_TOL, cost, model_cost_change, new_cost, radius, step_norm);
      term = LORB_TERM_PARAMETER_TOL; break;
    }
    const double cost_change = cost - new_cost;
    if (fabs(cost_change) <= o->function_tolerance * cost) {
      trace_put(iter, LORB_LM_STEP_FUNC_TOL, cost, model_cost_change, new_cost, radius, step_norm);
      term = LORB_TERM_FUNCTION_TOL; break;
    }
    const double relative_decrease = cost_change / model_cost_change;
    trace_put(iter, relative_decrease > o->min_relative_decrease ? LORB_LM_STEP_ACCEPTED : LORB_LM_STEP_REJECTED,
              cost, model_cost_change, new_cost, radius, step_norm);
    if (relative_decrease > o->min_relative_decrease) {
      /* HandleSuccessfulStep */
      memcpy(x, xn, sizeof(double) * (size_t)np);
      XNORM();
      cost = eval_jac(P, x, L.r, L.Jp, L.Jc);
      COLS_AND_GRAD(D, g);   /* D used as scratch for the (unused) unscaled column norms */
      if (R) { cost = ar1(R, cost, LORB_OP_SUM); ar(R, g, nc, LORB_OP_SUM); }
      GMAX();
      SCALE_J();
      n_success++;
      last_successful = 1;
      /* StepAccepted */
      const double t = 2.0 * relative_decrease - 1.0;
      radius = radius / fmax(1.0 / 3.0, 1.0 - t * t * t);
      radius = fmin(o->max_trust_region_radius, radius);
      decrease_factor = 2.0;
      reuse_diagonal = 0;
    } else {
      last_successful = 0;
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diagonal = 1;
    }
  }
  sum->iterations = iter;
  sum->successful_steps = n_success;
  sum->termination = term;
  sum->final_cost = cost;
  free(L.r); free(L.Jp); free(L.Jc); free(L.pt_res_off); free(L.pt_res);
  free(active); free(scale); free(diag); free(D); free(y); free(xn); free(g);
  return LORB_OK;
#undef COLS_AND_GRAD
#undef SCALE_J
#undef LIN_EXCHANGE
#undef GMAX
#undef XNORM
}

/* (a12) BA::ProjectPoseOptimization, src/bundle_adjust.cpp:158-202 */
int or_ba_pose_only(const lorb_pose_problem_batch* prob, const lorb_lm_options* opt,
                    double* pose_out, float* Tcw_out, lorb_ba_summary* summaries) {
  for (int f = 0; f < prob->n_frames; f++) {
    const int r0 = prob->res_off[f], r1 = prob->res_off[f + 1];
    or_prob P;
    P.n_pose = 1; P.n_point = 0; P.n_res = r1 - r0;
    P.res = (or_res*)calloc((size_t)(P.n_res > 0 ? P.n_res : 1), sizeof(or_res));
    const float* in = prob->intr + 4 * f;
    for (int k = 0; k < P.n_res; k++) {
      or_res* q = &P.res[k];
      q->kind = 0; q->point = -1; q->pose = 0;
      for (int i = 0; i < 3; i++) q->X[i] = prob->pts3d[3 * (size_t)(r0 + k) + i];
      q->fx = in[0]; q->fy = in[1]; q->cx = in[2]; q->cy = in[3];
      q->u = prob->obs2d[2 * (size_t)(r0 + k)]; q->v = prob->obs2d[2 * (size_t)(r0 + k) + 1];
    }
    double x[6];
    for (int i = 0; i < 6; i++) x[i] = prob->pose_init[6 * f + i];
    lorb_ba_summary s;
    memset(&s, 0, sizeof(s));
    if (P.n_res > 0) lm_solve(&P, opt, x, &s, NULL);  /* an empty ceres::Problem leaves the pose untouched */
    for (int i = 0; i < 6; i++) pose_out[6 * f + i] = x[i];
    if (Tcw_out) {
      const float R[3] = {(float)x[0], (float)x[1], (float)x[2]};
      const float T[3] = {(float)x[3], (float)x[4], (float)x[5]};
      or_pose_to_Tcw(R, T, Tcw_out + 16 * f);
    }
    if (summaries) summaries[f] = s;
    free(P.res);
  }
  return LORB_OK;
}

/* (a13) BA::LocalPoseOptimization, src/bundle_adjust.cpp:207-330 */
int or_ba_local(int n_windows, const lorb_ba_window* W, const lorb_lm_options* opt,
                double* const* pose_out, double* const* point_out, lorb_ba_summary* summaries) {
  for (int w = 0; w < n_windows; w++) {
    const lorb_ba_window* win = &W[w];
    or_prob P;
    P.n_pose = win->n_poses; P.n_point = win->n_points; P.n_res = win->n_obs;
    P.res = (or_res*)calloc((size_t)(P.n_res > 0 ? P.n_res : 1), sizeof(or_res));
    for (int k = 0; k < P.n_res; k++) {
      or_res* q = &P.res[k];
      q->point = win->obs_point[k];
      const int f = win->obs_frame[k];
      if (f >= 0) { q->kind = 2; q->pose = f; }
      else { q->kind = 1; q->pose = -1; for (int i = 0; i < 6; i++) q->fpose[i] = win->fixed_pose[6 * (size_t)(-1 - f) + i]; }
      q->fx = win->fx; q->fy = win->fy; q->cx = win->cx; q->cy = win->cy;
      q->u = win->obs_uv[2 * (size_t)k]; q->v = win->obs_uv[2 * (size_t)k + 1];
    }
    const int np = 6 * P.n_pose + 3 * P.n_point;
    double* x = (double*)malloc(sizeof(double) * (size_t)(np + 1));
    for (int i = 0; i < 6 * P.n_pose; i++) x[i] = win->pose_init[i];
    for (int i = 0; i < 3 * P.n_point; i++) x[6 * P.n_pose + i] = win->point_init[i];
    lorb_ba_summary s;
    memset(&s, 0, sizeof(s));
    if (P.n_res > 0) lm_solve(&P, opt, x, &s, NULL);
    memcpy(pose_out[w], x, sizeof(double) * 6 * (size_t)P.n_pose);
    memcpy(point_out[w], x + 6 * P.n_pose, sizeof(double) * 3 * (size_t)P.n_point);
    if (summaries) summaries[w] = s;
    free(x); free(P.res);
  }
  return LORB_OK;
}

/* Point-partitioned variant of or_ba_local: `shards` holds this rank's points and
 * all of their observations; poses, fixed poses and intrinsics are identical on every rank. */
int or_ba_local_sharded(int n_windows, const lorb_ba_window* W, const lorb_lm_options* opt, int rank,
                        or_allreduce_fn fn, void* user, double* const* pose_out, double* const* point_out,
                        lorb_ba_summary* summaries) {
  const or_reducer R = {fn, user, rank};
  for (int w = 0; w < n_windows; w++) {
    const lorb_ba_window* win = &W[w];
    or_prob P;
    P.n_pose = win->n_poses; P.n_point = win->n_points; P.n_res = win->n_obs;
    P.res = (or_res*)calloc((size_t)(P.n_res > 0 ? P.n_res : 1), sizeof(or_res));
    for (int k = 0; k < P.n_res; k++) {
      or_res* q = &P.res[k];
      q->point = win->obs_point[k];
      const int f = win->obs_frame[k];
      if (f >= 0) { q->kind = 2; q->pose = f; }
      else { q->kind = 1; q->pose = -1; for (int i = 0; i < 6; i++) q->fpose[i] = win->fixed_pose[6 * (size_t)(-1 - f) + i]; }
      q->fx = win->fx; q->fy = win->fy; q->cx = win->cx; q->cy = win->cy;
      q->u = win->obs_uv[2 * (size_t)k]; q->v = win->obs_uv[2 * (size_t)k + 1];
    }
    const int np = 6 * P.n_pose + 3 * P.n_point;
    double* x = (double*)malloc(sizeof(double) * (size_t)(np + 1));
    for (int i = 0; i < 6 * P.n_pose; i++) x[i] = win->pose_init[i];
    for (int i = 0; i < 3 * P.n_point; i++) x[6 * P.n_pose + i] = win->point_init[i];
    lorb_ba_summary s;
    memset(&s, 0, sizeof(s));
    if (ar1(&R, (double)P.n_res, LORB_OP_SUM) > 0.0) lm_solve(&P, opt, x, &s, &R);
    memcpy(pose_out[w], x, sizeof(double) * 6 * (size_t)P.n_pose);
    memcpy(point_out[w], x + 6 * P.n_pose, sizeof(double) * 3 * (size_t)P.n_point);
    if (summaries) summaries[w] = s;
    free(x); free(P.res);
  }
  return LORB_OK;
}
