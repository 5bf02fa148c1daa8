/* tests/cpp/abi_loopback.c -- TEST DOUBLE, linked only into the sanitizer builds of
 * tests/cpp/test_adapters.cpp (tests/test_sanitizers.py).  It implements the C-ABI entry points
 * that the host layer (include/lorb/adapters.hpp, local_mapping.hpp) calls by forwarding to the
 * oracle, so that the host-side gather / apply / queue code runs under ASan+UBSan and TSan on a
 * machine without a GPU.  It is never part of liblorb.so: the product path has no CPU fallback. */
#include <stdlib.h>
#include <string.h>

#include "../../oracle/lorb_oracle.h"

struct lorb_ba_solver;
struct lorb_ctx {
  int device;
  struct lorb_ba_solver* solver; /* lorb_ctx_ba_solver's, freed with the ctx */
};

int lorb_create(int device, lorb_ctx** out) {
  if (!out) return LORB_E_INVALID;
  *out = (lorb_ctx*)calloc(1, sizeof(lorb_ctx));
  if (!*out) return LORB_E_NOMEM;
  (*out)->device = device;
  return LORB_OK;
}

int lorb_destroy(lorb_ctx* ctx) {
  if (ctx) free(ctx->solver);
  free(ctx);
  return LORB_OK;
}

const char* lorb_last_error(const lorb_ctx* ctx) {
  (void)ctx;
  return "loopback";
}

void lorb_lm_options_default(lorb_lm_options* opt) { or_lm_options_default(opt); }

void lorb_pose_to_Tcw(const float rvec[3], const float tvec[3], float Tcw[16]) { or_pose_to_Tcw(rvec, tvec, Tcw); }

int lorb_bf_match(lorb_ctx* ctx, int32_t n_problems, const uint8_t* q_desc, const int32_t* q_off,
                  const uint8_t* t_desc, const int32_t* t_off, int32_t* cc_train, int32_t* cc_dist,
                  int32_t* match_train, int32_t* n_matches) {
  if (!ctx) return LORB_E_INVALID;
  for (int p = 0; p < n_problems; p++)
    n_matches[p] = or_bf_match(q_desc + 32 * (size_t)q_off[p], q_off[p + 1] - q_off[p], t_desc + 32 * (size_t)t_off[p],
                               t_off[p + 1] - t_off[p], cc_train + q_off[p], cc_dist + q_off[p], match_train + q_off[p]);
  return LORB_OK;
}

int lorb_search_by_projection_frame(lorb_ctx* ctx, const lorb_frame_params* cur, const float cur_Tcw[16],
                                    const lorb_keypoints* cur_kps, const uint8_t* cur_slot_state,
                                    const lorb_last_frame* last, float th, int32_t* assign, int32_t* nmatches) {
  if (!ctx) return LORB_E_INVALID;
  return or_search_by_projection_frame(cur, cur_Tcw, cur_kps, cur_slot_state, last, th, assign, nmatches);
}

int lorb_search_by_projection_local(lorb_ctx* ctx, const lorb_frame_params* frame, const lorb_keypoints* kps,
                                    const uint8_t* slot_state, const lorb_local_points* pts, float th,
                                    int32_t* assign, int32_t* nmatches) {
  if (!ctx) return LORB_E_INVALID;
  return or_search_by_projection_local(frame, kps, slot_state, pts, th, assign, nmatches);
}

int lorb_ba_pose_only(lorb_ctx* ctx, const lorb_pose_problem_batch* prob, const lorb_lm_options* opt,
                      double* pose_out, float* Tcw_out, lorb_ba_summary* summaries) {
  if (!ctx) return LORB_E_INVALID;
  return or_ba_pose_only(prob, opt, pose_out, Tcw_out, summaries);
}

int lorb_ba_local(lorb_ctx* ctx, int32_t n_windows, const lorb_ba_window* windows, const lorb_lm_options* opt,
                  double* const* pose_out, double* const* point_out, lorb_ba_summary* summaries) {
  if (!ctx) return LORB_E_INVALID;
  return or_ba_local(n_windows, windows, opt, pose_out, point_out, summaries);
}

struct lorb_ba_solver {
  lorb_ctx* ctx;
};

int lorb_ba_solver_create(lorb_ctx* ctx, lorb_ba_solver** out) {
  if (!ctx || !out) return LORB_E_INVALID;
  *out = (lorb_ba_solver*)calloc(1, sizeof(lorb_ba_solver));
  if (!*out) return LORB_E_NOMEM;
  (*out)->ctx = ctx;
  return LORB_OK;
}

int lorb_ba_solver_solve(lorb_ba_solver* s, const lorb_ba_window* w, const lorb_lm_options* opt, double* pose_out,
                         double* point_out, lorb_ba_summary* summary) {
  if (!s || !w || !opt) return LORB_E_INVALID;
  double* const po[1] = {pose_out};
  double* const pt[1] = {point_out};
  return or_ba_local(1, w, opt, po, pt, summary);
}

int lorb_ba_solver_destroy(lorb_ba_solver* s) {
  free(s);
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

int lorb_compute_stereo_matches(lorb_ctx* ctx, const lorb_frame_params* frame, const lorb_stereo_keys* left,
                                const lorb_stereo_keys* right, const lorb_image_pyramid* left_pyr,
                                const lorb_image_pyramid* right_pyr, float* u_right, float* depth) {
  if (!ctx) return LORB_E_INVALID;
  (void)or_compute_stereo_matches(frame, left, right, left_pyr, right_pyr, u_right, depth);
  return LORB_OK;
}

int lorb_compute_descriptor(lorb_ctx* ctx, int32_t n_points, const int32_t* d_off, const uint8_t* desc,
                            int32_t* best, uint8_t* out_desc) {
  if (!ctx) return LORB_E_INVALID;
  or_compute_descriptor(n_points, d_off, desc, best);
  for (int p = 0; out_desc && p < n_points; p++) {
    if (best[p] >= 0) memcpy(out_desc + 32 * (size_t)p, desc + 32 * (size_t)(d_off[p] + best[p]), 32);
    else memset(out_desc + 32 * (size_t)p, 0, 32);
  }
  return LORB_OK;
}

/* VisualOdometry::EstimatePoseLocal's local-map loop restated by the oracle, as
 * oracle.py:track_local_map does (src/visual_odometry.cpp:173-201). */
int lorb_track_local_map(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16], const lorb_keypoints* kps,
                         const uint8_t* slot_state, const lorb_map_points_dev* pts, float viewing_cos_limit, float th,
                         uint8_t* in_view, float* track, int32_t* level, int32_t* assign, int32_t* nmatches) {
  if (!ctx) return LORB_E_INVALID;
  const int n = pts->n;
  lorb_frustum_points fp = {n, pts->pos, pts->normal, pts->max_dist, pts->min_dist};
  or_is_in_frustum(frame, Tcw, &fp, viewing_cos_limit, in_view, track, track + n, track + 2 * n, level, track + 3 * n);
  int any = 0;
  for (int i = 0; i < n; i++) {
    if ((pts->in_frame && pts->in_frame[i]) || (pts->is_bad && pts->is_bad[i])) in_view[i] = 0;
    any |= in_view[i];
  }
  for (int j = 0; j < kps->n; j++) assign[j] = LORB_ASSIGN_UNCHANGED;
  *nmatches = 0;
  if (!any) return LORB_OK;
  lorb_local_points lp = {n, in_view, pts->is_bad, pts->locked, track, track + n, track + 2 * n, level, track + 3 * n,
                          pts->desc};
  return or_search_by_projection_local(frame, kps, slot_state, &lp, th, assign, nmatches);
}

int lorb_ba_solver_info(lorb_ba_solver* s, int32_t* info, int32_t n) {
  (void)s; (void)info; (void)n;
  return LORB_E_UNSUPPORTED;  /* no resident plans in the loopback */
}
