// lorb_ba_solver.hip -- BA::LocalPoseOptimization for callers that build a new window per call
// (the drop-in src/bundle_adjust.cpp:207-330, called from src/local_mapping.cpp:32; VERDICT r02
// item 1).
//
// The reference builds its Ceres problem on every call.  lorb_ba_local mirrors that with a host-built
// plan (allocations, sorting, pair lists, graph capture, frees: ~7.5 ms at C4 against a 1.2 ms
// solve).  The solver instead keeps device-built plans (lorb_ba_plan_create_dev) resident across
// calls, one per camera count (the plan's camera dimension is fixed; a small LRU holds the counts a
// caller alternates between), with point / observation / fixed-pose capacities that only grow.  A
// call is then:
//   1. the window packed into pinned staging (validated on the way) and ONE host-to-device copy;
//   2. the device plan build from those arrays (lorb_ba_plan_update_dev: one small readback);
//   3. the LM solve (the plan's captured hipGraph, replayed: no capture per call);
//   4. the solution in double, caller order, plus the summary: one kernel, ONE device-to-host copy.
// Fixed poses are padded to the plan's capacity with rows no observation references, which the
// device build ignores.  Windows the device plans do not take (no cameras / points / observations,
// a point with kGB or more observations) run through lorb_ba_local (the host-built plan on the
// same GPU kernels): there is no CPU path.
#include <algorithm>

#include "lorb_internal.h"

namespace {

constexpr int kSlots = 4;

struct Slot {
  int C = -1, F_cap = 0, P_cap = 0, K_cap = 0;
  lorb_ba_plan* plan = nullptr;
  unsigned char* d_in = nullptr;  // packed window (counts | pose | fixed | point | obs_point | obs_frame | uv)
  size_t in_bytes = 0;
  double* d_out = nullptr;        // 6C + 3 P_cap + 5
  unsigned long long last_use = 0;
};

inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

// byte offsets of the packed window for C cameras, F fixed rows, P points and K observations
struct Layout {
  size_t pose, fixed, point, opt, ofr, uv, end;
  Layout(int C, int F, int P, int K) {
    pose = 16;
    fixed = al16(pose + sizeof(float) * 6 * (size_t)C);
    point = al16(fixed + sizeof(float) * 6 * (size_t)F);
    opt = al16(point + sizeof(float) * 3 * (size_t)P);
    ofr = al16(opt + sizeof(int) * (size_t)K);
    uv = al16(ofr + sizeof(int) * (size_t)K);
    end = al16(uv + sizeof(float) * 2 * (size_t)K);
  }
};

}  // namespace

struct lorb_ba_solver {
  lorb_ctx* ctx = nullptr;
  Slot slot[kSlots];
  unsigned long long clock = 0;
  unsigned char* h_in = nullptr; size_t h_in_sz = 0;    // pinned staging
  double* h_out = nullptr; size_t h_out_n = 0;
  int creations = 0, last_fallback = 0, last_slot = -1;
  bool sorted = false;  // the current window's observations are sorted by point
  ~lorb_ba_solver() {
    if (ctx) (void)hipStreamSynchronize(ctx->stream);
    for (Slot& s : slot) {
      if (s.plan) (void)lorb_ba_plan_destroy(s.plan);
      if (s.d_in) (void)hipFree(s.d_in);
      if (s.d_out) (void)hipFree(s.d_out);
    }
    if (h_in) (void)hipHostFree(h_in);
    if (h_out) (void)hipHostFree(h_out);
  }
};

namespace {

void release(Slot& s) {
  if (s.plan) (void)lorb_ba_plan_destroy(s.plan);
  if (s.d_in) (void)hipFree(s.d_in);
  if (s.d_out) (void)hipFree(s.d_out);
  s = Slot{};
}

int pinned_grow(lorb_ba_solver* S, size_t in_bytes, size_t out_n) {
  lorb_ctx* ctx = S->ctx;
  if (S->h_in_sz < in_bytes) {
    if (S->h_in) (void)hipHostFree(S->h_in);
    S->h_in = nullptr; S->h_in_sz = 0;
    const size_t n = in_bytes + in_bytes / 4;
    LORB_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&S->h_in), n));
    S->h_in_sz = n;
  }
  if (S->h_out_n < out_n) {
    if (S->h_out) (void)hipHostFree(S->h_out);
    S->h_out = nullptr; S->h_out_n = 0;
    const size_t n = out_n + out_n / 4;
    LORB_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&S->h_out), sizeof(double) * n));
    S->h_out_n = n;
  }
  return LORB_OK;
}

// the slot for C cameras with room for F fixed rows, P points, K observations (fresh = no plan yet)
int pick_slot(lorb_ba_solver* S, int C, int F, int P, int K, Slot** out) {
  lorb_ctx* ctx = S->ctx;
  Slot* hit = nullptr;
  for (Slot& s : S->slot)
    if (s.C == C) hit = &s;
  if (hit && (hit->F_cap < F || hit->P_cap < P || hit->K_cap < K)) {  // outgrown: rebuild larger
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const int f = std::max(hit->F_cap, F), p = std::max(hit->P_cap, P), k = std::max(hit->K_cap, K);
    release(*hit);
    hit->F_cap = f + f / 2; hit->P_cap = p + p / 2; hit->K_cap = k + k / 2;
  }
  if (!hit) {
    Slot* lru = &S->slot[0];
    for (Slot& s : S->slot) {
      if (s.C < 0) { lru = &s; break; }
      if (s.last_use < lru->last_use) lru = &s;
    }
    if (lru->C >= 0) {
      LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
      release(*lru);
    }
    hit = lru;
    hit->F_cap = std::max(F + F / 2, 8); hit->P_cap = std::max(P + P / 4, 64); hit->K_cap = std::max(K + K / 4, 256);
  }
  if (!hit->d_in) {
    hit->C = C;
    hit->in_bytes = Layout(C, hit->F_cap, hit->P_cap, hit->K_cap).end;
    LORB_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&hit->d_in), hit->in_bytes));
    LORB_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&hit->d_out), sizeof(double) * (6 * (size_t)C + 3 * (size_t)hit->P_cap + 5)));
  }
  hit->last_use = ++S->clock;
  *out = hit;
  return LORB_OK;
}

int solve_fallback(lorb_ba_solver* S, const lorb_ba_window* w, const lorb_lm_options* opt, double* pose_out,
                   double* point_out, lorb_ba_summary* summary) {
  S->last_fallback = 1;
  double* const po[1] = {pose_out};
  double* const pt[1] = {point_out};
  lorb_ba_summary s{};
  LORB_TRY(lorb_ba_local(S->ctx, 1, w, opt, po, pt, &s));
  if (summary) *summary = s;
  return LORB_OK;
}

}  // namespace

extern "C" {

int lorb_ba_solver_create(lorb_ctx* ctx, lorb_ba_solver** out) {
  if (!ctx || !out) return LORB_E_INVALID;
  *out = nullptr;
  lorb_ba_solver* S = new (std::nothrow) lorb_ba_solver();
  if (!S) return LORB_E_NOMEM;
  S->ctx = ctx;
  *out = S;
  return LORB_OK;
}

int lorb_ba_solver_solve(lorb_ba_solver* S, const lorb_ba_window* w, const lorb_lm_options* opt, double* pose_out,
                         double* point_out, lorb_ba_summary* summary) {
  if (!S || !w || !opt) return LORB_E_INVALID;
  lorb_ctx* ctx = S->ctx;
  const int C = w->n_poses, F = w->n_fixed, P = w->n_points, K = w->n_obs;
  if (C < 0 || F < 0 || P < 0 || K < 0) return lorb::set_error(ctx, LORB_E_INVALID, "window: negative sizes");
  if ((C > 0 && (!w->pose_init || !pose_out)) || (F > 0 && !w->fixed_pose) || (P > 0 && (!w->point_init || !point_out)) ||
      (K > 0 && (!w->obs_point || !w->obs_frame || !w->obs_uv)))
    return lorb::set_error(ctx, LORB_E_INVALID, "window: missing arrays");
  S->last_fallback = 0;
  if (C == 0 || P == 0 || K == 0) return solve_fallback(S, w, opt, pose_out, point_out, summary);
  Slot* sl = nullptr;
  LORB_TRY(pick_slot(S, C, F, P, K, &sl));
  S->last_slot = (int)(sl - S->slot);
  const Layout L(C, sl->F_cap, P, K);
  const size_t out_n = 6 * (size_t)C + 3 * (size_t)P + 5;
  LORB_TRY(pinned_grow(S, L.end, out_n));
  // 1. pack (the pinned staging is free: the previous call ended with a synchronisation)
  unsigned char* h = S->h_in;
  const int32_t counts[4] = {P, K, 0, 0};
  memcpy(h, counts, sizeof(counts));
  memcpy(h + L.pose, w->pose_init, sizeof(float) * 6 * (size_t)C);
  float* fx = reinterpret_cast<float*>(h + L.fixed);
  if (F > 0) memcpy(fx, w->fixed_pose, sizeof(float) * 6 * (size_t)F);
  std::fill(fx + 6 * (size_t)F, fx + 6 * (size_t)sl->F_cap, 0.0f);
  memcpy(h + L.point, w->point_init, sizeof(float) * 3 * (size_t)P);
  {  // index validation as min / max reductions (vectorisable); the offending slot only on failure
    int pmn = 0, pmx = 0, fmn = 0, fmx = 0, unsorted = 0;
    if (K > 0) { pmn = pmx = w->obs_point[0]; fmn = fmx = w->obs_frame[0]; }
    for (int k = 0; k < K; ++k) {
      pmn = std::min(pmn, w->obs_point[k]); pmx = std::max(pmx, w->obs_point[k]);
      fmn = std::min(fmn, w->obs_frame[k]); fmx = std::max(fmx, w->obs_frame[k]);
      unsorted |= k > 0 && w->obs_point[k - 1] > w->obs_point[k];
    }
    // the drop-in gathers a window point by point: its slots are sorted and the device build needs
    // no counting sort
    S->sorted = !unsorted;
    if (pmn < 0 || pmx >= P || fmn < -F || fmx >= C)
      for (int k = 0; k < K; ++k) {
        const int p = w->obs_point[k], f = w->obs_frame[k];
        if (p < 0 || p >= P) return lorb::set_error(ctx, LORB_E_INVALID, "window 0 obs %d: bad point %d", k, p);
        if (f >= C || f < -F) return lorb::set_error(ctx, LORB_E_INVALID, "window 0 obs %d: bad frame %d", k, f);
      }
  }
  memcpy(h + L.opt, w->obs_point, sizeof(int32_t) * (size_t)K);
  memcpy(h + L.ofr, w->obs_frame, sizeof(int32_t) * (size_t)K);
  memcpy(h + L.uv, w->obs_uv, sizeof(float) * 2 * (size_t)K);
  LORB_HIP(ctx, hipMemcpyAsync(sl->d_in, h, L.end, hipMemcpyHostToDevice, ctx->stream));
  lorb_ba_window_dev wd{};
  wd.n_poses = C; wd.n_fixed = sl->F_cap; wd.max_points = sl->P_cap; wd.max_obs = sl->K_cap;
  wd.d_n_points = reinterpret_cast<const int32_t*>(sl->d_in); wd.d_n_obs = wd.d_n_points + 1;
  wd.fx = w->fx; wd.fy = w->fy; wd.cx = w->cx; wd.cy = w->cy;
  wd.d_pose_init = reinterpret_cast<const float*>(sl->d_in + L.pose);
  wd.d_fixed_pose = reinterpret_cast<const float*>(sl->d_in + L.fixed);
  wd.d_point_init = reinterpret_cast<const float*>(sl->d_in + L.point);
  wd.d_obs_point = reinterpret_cast<const int32_t*>(sl->d_in + L.opt);
  wd.d_obs_frame = reinterpret_cast<const int32_t*>(sl->d_in + L.ofr);
  wd.d_obs_uv = reinterpret_cast<const float*>(sl->d_in + L.uv);
  // 2. the device plan build (one readback)
  int rc;
  if (!sl->plan) {
    rc = lorb_ba_plan_create_dev(ctx, &wd, &sl->plan);
    if (rc == LORB_OK) S->creations++;
  } else {
    lorb::ba_plan_sorted_hint(sl->plan, S->sorted);
    rc = lorb_ba_plan_update_dev(sl->plan, &wd);
  }
  if (rc == LORB_E_UNSUPPORTED) {
    // a point with more observations than a device plan's point group holds: the host-built plan
    // takes it (a point observed twice by one camera is an error in both builders)
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (!sl->plan) release(*sl);
    return solve_fallback(S, w, opt, pose_out, point_out, summary);
  }
  if (rc != LORB_OK && !sl->plan) release(*sl);
  LORB_TRY(rc);
  // 3. LM (captured graph)  4. result + summary, one copy
  LORB_TRY(lorb_ba_plan_solve(sl->plan, opt));
  LORB_TRY(lorb::ba_plan_result64_dev(sl->plan, sl->d_out));
  LORB_HIP(ctx, hipMemcpyAsync(S->h_out, sl->d_out, sizeof(double) * out_n, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, lorb::spin_sync(ctx));
  memcpy(pose_out, S->h_out, sizeof(double) * 6 * (size_t)C);
  memcpy(point_out, S->h_out + 6 * (size_t)C, sizeof(double) * 3 * (size_t)P);
  if (summary) {
    const double* s = S->h_out + 6 * (size_t)C + 3 * (size_t)P;
    lorb_ba_summary r{};
    r.iterations = (int32_t)s[0]; r.successful_steps = (int32_t)s[1]; r.termination = (int32_t)s[2];
    r.initial_cost = s[3]; r.final_cost = s[4];
    *summary = r;
  }
  return LORB_OK;
}

int lorb_ba_solver_info(lorb_ba_solver* S, int32_t* info, int32_t n) {
  if (!S || !info || n < 0) return LORB_E_INVALID;
  int resident = 0;
  for (const Slot& s : S->slot) resident += s.plan != nullptr;
  int32_t pinfo[8] = {0, -1, 0, 0, 0, 0, 0, 0};
  if (!S->last_fallback && S->last_slot >= 0 && S->slot[S->last_slot].plan)
    LORB_TRY(lorb_ba_plan_info(S->slot[S->last_slot].plan, pinfo, 8));
  const int32_t v[6] = {resident, S->creations, S->last_fallback, pinfo[0], pinfo[1], pinfo[7]};
  for (int i = 0; i < n && i < 6; ++i) info[i] = v[i];
  return LORB_OK;
}

int lorb_ba_solver_trace(lorb_ba_solver* S, lorb_lm_iteration* out, int32_t cap, int32_t* n_out) {
  if (!S || !n_out) return LORB_E_INVALID;
  *n_out = 0;
  if (S->last_fallback || S->last_slot < 0 || !S->slot[S->last_slot].plan) return LORB_OK;
  return lorb_ba_plan_trace(S->slot[S->last_slot].plan, 0, out, cap, n_out);
}

int lorb_ba_solver_destroy(lorb_ba_solver* S) {
  delete S;
  return LORB_OK;
}

int lorb_ctx_ba_solver(lorb_ctx* ctx, lorb_ba_solver** out) {
  if (!ctx || !out) return LORB_E_INVALID;
  if (!ctx->solver) {
    const int rc = lorb_ba_solver_create(ctx, &ctx->solver);
    if (rc != LORB_OK) return rc;
  }
  *out = ctx->solver;
  return LORB_OK;
}

}  // extern "C"
