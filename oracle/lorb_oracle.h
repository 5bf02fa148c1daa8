/*
 * lorb_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the LORB_SLAM hot path.
 *
 * Parity status: "parity unpinned" against the real reference.  The reference
 * (abstract-liu/LORB_SLAM @ v0) cannot be compiled in this image (it needs OpenCV 3.1, Ceres,
 * Eigen3 and Pangolin; g++ stops at include/common.h:6) and ships no tests, golden vectors or
 * fixtures.  This restatement follows the reference source line by line
 * (file:line cited on every function) and restates the third-party behaviour it calls
 * (OpenCV 3.x BFMatcher crossCheck / cv::gemm / cv::Rodrigues / cv::Mat::inv, Ceres LM +
 * DENSE_SCHUR + AutoDiff Jets) from their published algorithms.  It is cross-checked against
 * independent computations (numpy bitwise_count for Hamming, exhaustive integer identities,
 * scipy.optimize.least_squares for the BA optimum) in tests/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this code.
 * The product path (liblorb.so) never links or calls it.
 */
#ifndef LORB_ORACLE_H
#define LORB_ORACLE_H

#include "../include/lorb_c.h"

#ifdef __cplusplus
extern "C" {
#endif

/* src/matcher.cpp:369-385 */
int or_descriptor_distance(const uint8_t* a, const uint8_t* b);
/* src/matcher.cpp:430-436 */
float or_radius_by_viewing_cos(float view_cos);
/* src/matcher.cpp:387-428 ; hist_sizes[L] */
void or_compute_three_maxima(const int* hist_sizes, int L, int* ind1, int* ind2, int* ind3);

/* OpenCV 3.x BFMatcher(NORM_HAMMING, crossCheck=true).match + src/matcher.cpp:42-56 filter.
 * Single problem.  Returns the number of accepted matches. */
int or_bf_match(const uint8_t* q, int nq, const uint8_t* t, int nt,
                int32_t* cc_train, int32_t* cc_dist, int32_t* match_train);
/* a5 with an unbounded window (train order = candidate order) */
void or_bf_top2(const uint8_t* q, int nq, const uint8_t* t, int nt, const int32_t* t_level,
                int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                int32_t* second_dist, int32_t* second_level, uint8_t* accepted);
/* multithreaded variant used only by bench.py's cpu_baseline leg (rows split over threads) */
void or_bf_top2_mt(const uint8_t* q, int nq, const uint8_t* t, int nt, const int32_t* t_level,
                   int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                   int32_t* second_dist, int32_t* second_level, uint8_t* accepted, int threads);

/* MapPoint::ComputeDescriptor, src/map_point.cpp:69-129, batched (CSR d_off); best -1 if empty */
void or_compute_descriptor(int n_points, const int32_t* d_off, const uint8_t* desc, int32_t* best);

/* Frame grid: src/frame.cpp:87-115 (AssignFeaturesToGrid / PosInGrid) and
 * GetFeaturesInArea src/frame.cpp:370-423.  Grid stored as CSR over cells, cell = ix*ROWS+iy. */
typedef struct or_grid {
  int32_t cell_off[LORB_GRID_COLS * LORB_GRID_ROWS + 1];
  int32_t* idx;  /* n entries max */
} or_grid;
void or_grid_build(const lorb_frame_params* fp, const lorb_keypoints* kps, or_grid* g);
void or_grid_free(or_grid* g);
/* returns count written into out (capacity n) */
int or_features_in_area(const lorb_frame_params* fp, const lorb_keypoints* kps, const or_grid* g,
                        float x, float y, float r, int min_level, int max_level, int32_t* out);

/* (a4) src/matcher.cpp:64-218 */
int or_search_by_projection_frame(const lorb_frame_params* cur, const float cur_Tcw[16],
                                  const lorb_keypoints* cur_kps, const uint8_t* cur_slot_state,
                                  const lorb_last_frame* last, float th,
                                  int32_t* assign, int32_t* nmatches);
/* (a5) src/matcher.cpp:220-316 */
int or_search_by_projection_local(const lorb_frame_params* frame, const lorb_keypoints* kps,
                                  const uint8_t* slot_state, const lorb_local_points* pts,
                                  float th, int32_t* assign, int32_t* nmatches);
/* (a8) src/frame.cpp:425-494 + src/map_point.cpp:267-284 */
void or_is_in_frustum(const lorb_frame_params* frame, const float Tcw[16],
                      const lorb_frustum_points* pts, float viewing_cos_limit,
                      uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                      int32_t* pred_level, float* view_cos);
/* (a20) src/frame.cpp:335-356 */
void or_unproject_stereo(const lorb_frame_params* frame, const float Tcw[16], int n,
                         const float* x, const float* y, const float* depth, float* out_xyz);
/* cv::Mat::inv() of a 4x4 CV_32F (DECOMP_LU, hal::LU32f) ; returns 0 if singular */
int or_inv4_f32(const float A[16], float out[16]);
/* cv::Rodrigues (vector -> matrix), then Frame::UpdatePoseMat (src/frame.cpp:577-594) */
void or_pose_to_Tcw(const float rvec[3], const float tvec[3], float Tcw[16]);

/* ---- bundle adjustment (src/bundle_adjust.cpp) with Ceres LM + DENSE_SCHUR restated ---- */
void or_lm_options_default(lorb_lm_options* opt);
int or_ba_pose_only(const lorb_pose_problem_batch* prob, const lorb_lm_options* opt,
                    double* pose_out, float* Tcw_out, lorb_ba_summary* summaries);
int or_ba_local(int n_windows, const lorb_ba_window* windows, const lorb_lm_options* opt,
                double* const* pose_out, double* const* point_out, lorb_ba_summary* summaries);
/* Sink for the per-iteration records of the next LM solves (each solve restarts at record 0, so
 * after a multi-window call it holds the last window's); NULL switches it off. */
void or_lm_trace(lorb_lm_iteration* buf, int cap);
int or_lm_trace_count(void);
/* Point-partitioned local BA (the multi-GPU exchange pattern of SURVEY §8e, restated on the
 * CPU): each rank passes its shard; fn all-reduces `count` doubles in place (op LORB_OP_*). */
typedef int (*or_allreduce_fn)(void* user, double* buf, int64_t count, int32_t op);
int or_ba_local_sharded(int n_windows, const lorb_ba_window* shards, const lorb_lm_options* opt, int rank,
                        or_allreduce_fn fn, void* user, double* const* pose_out, double* const* point_out,
                        lorb_ba_summary* summaries);
/* Residual + Jacobian of one observation by Ceres-style Jets (AutoDiffCostFunction).
 * kind 0 = PoseCost (params aa,t ; v uses fy_eff), 1 = MPCost (params X), 2 = PoseMPCost
 * (params X, pose).  jac: 2 x nparams row-major (nparams 6 / 3 / 9). */
void or_residual_jet(int kind, const double* X, const double* pose, double fx, double fy,
                     double cx, double cy, double u, double v, double* res, double* jac);
/* AngleAxisRotatePoint (ceres/rotation.h) in double */
void or_angle_axis_rotate_point(const double aa[3], const double pt[3], double out[3]);

/* src/frame.cpp:125-333 (stereo.c).  Returns the number of pairs before the median rejection. */
int or_compute_stereo_matches(const lorb_frame_params* fp, const lorb_stereo_keys* L, const lorb_stereo_keys* R,
                              const lorb_image_pyramid* PL, const lorb_image_pyramid* PR, float* u_right,
                              float* depth);

/* orb.c: the descriptor stage of ORBextractor::operator() (src/ORBextractor.cpp:79-150, 469-493,
 * 1131-1132) with OpenCV 3.1's fastAtan2 / getGaussianKernel / fixed-point 8U smoothing restated */
void or_orb_umax(int* umax);
float or_fast_atan2(float y, float x);
void or_orb_gauss_kernel(int32_t* k7);
void or_orb_blur(const uint8_t* src, int rows, int cols, int sstep, uint8_t* dst, int dstep);
float or_orb_ic_angle(const uint8_t* img, int step, float px, float py, const int* umax);
void or_orb_descriptor(const uint8_t* img, int step, float px, float py, float angle_deg, const int32_t* pattern,
                       uint8_t* desc);
void or_orb_describe(const lorb_image_pyramid* P, int n, const float* x, const float* y, const int32_t* level,
                     const int32_t* pattern, float* angle, uint8_t* desc);

/* fast.c: cv::FAST (OpenCV 3.1 FAST_t<16> + cornerScore<16>) and ORBextractor::
 * ComputeKeyPointsOctTree + DistributeOctTree (src/ORBextractor.cpp:554-897) */
int or_fast_score(const uint8_t* ptr, const int* pixel, int threshold);
int or_fast(const uint8_t* img, int w, int h, int step, int threshold, int max_out, float* ox, float* oy,
            float* oresp);
int or_orb_cells(int rows, int cols, int* cells, int max_cells, int* ncols, int* nrows);
int or_orb_fast_cells(const lorb_image_pyramid* P, int ini_th, int min_th, int max_kp, float* x, float* y,
                      float* resp, int max_cells, int32_t* cell_base, int32_t* cell_off);
int or_distribute_octree(const float* kx, const float* ky, const float* resp, int n, int minX, int maxX, int minY,
                         int maxY, int N, int32_t* out);
int or_orb_detect(const lorb_image_pyramid* P, const int32_t* n_desired, const float* scale_factors, int ini_th,
                  int min_th, int max_kp, float* ox, float* oy, int32_t* ooct, float* osize, float* oresp,
                  int32_t* level_off);
/* orb.c: the whole ORBextractor::operator() (src/ORBextractor.cpp:1087-1151) */
int or_orb_extract(const uint8_t* img, int rows, int cols, int step, int n_levels, const float* scale_factors,
                   const int32_t* n_desired, int ini_th, int min_th, const int32_t* pattern, int max_kp, float* ox,
                   float* oy, int32_t* ooct, float* osize, float* oangle, float* oresp, uint8_t* odesc,
                   int32_t* level_off);

/* orb.c: ORBextractor::ComputePyramid with OpenCV 3.1's 8U INTER_LINEAR resize restated */
int or_resize_simd_cols(int width);
void or_resize_linear_8u(const uint8_t* src, int sh, int sw, int sstep, uint8_t* dst, int dh, int dw, int dstep);
void or_orb_pyramid(const uint8_t* img, int rows, int cols, int step, int n_levels, const float* scale_factors,
                    uint8_t* out, lorb_image_pyramid* P);

#ifdef __cplusplus
}
#endif
#endif
