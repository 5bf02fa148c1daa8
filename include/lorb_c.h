/*
 * lorb_c.h -- C-ABI drop-in boundary of the MI355X-native LORB_SLAM hot path.
 *
 * Everything here is `extern "C"`, POD structs and plain pointers + sizes.  No torch, no
 * OpenCV, no Ceres types cross this boundary.  Each entry point names the reference
 * interface it replaces (paths relative to the reference repo abstract-liu/LORB_SLAM @ v0).
 *
 * Conventions
 *   - Every function returns int: LORB_OK (0) or a negative LORB_E_* code.  The message of
 *     the last error on a context is available from lorb_last_error(ctx).  No C++ exception
 *     ever crosses the ABI.
 *   - Functions without a `_dev` suffix take HOST pointers; they stage through device
 *     buffers owned by the context and are synchronous.  `_dev` variants take DEVICE
 *     pointers (allocated with lorb_malloc) and are asynchronous on the context's stream.
 *   - The library never takes ownership of caller memory.
 *   - One lorb_ctx per calling thread (it owns one hipStream_t).  A ctx is not thread-safe.
 *   - Keypoint / map-point identity: the C-ABI never sees MapPoint*.  Results are returned as
 *     per-slot "assign" codes that the C++ adapter applies to Frame::mvpMapPoints.
 */
#ifndef LORB_C_H
#define LORB_C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LORB_ABI_VERSION 1

#define LORB_OK 0
#define LORB_E_INVALID (-1)   /* bad argument / shape */
#define LORB_E_DEVICE  (-2)   /* HIP runtime error (no device, launch failure, OOM) */
#define LORB_E_NOMEM   (-3)   /* host allocation failure */
#define LORB_E_UNSUPPORTED (-4)
#define LORB_E_COMM    (-5)   /* RCCL error */

/* Matcher constants, src/matcher.cpp:6-8 */
#define LORB_TH_HIGH 100
#define LORB_TH_LOW 50
#define LORB_HISTO_LENGTH 30
/* Frame grid, include/frame.h:13-14 */
#define LORB_GRID_ROWS 48
#define LORB_GRID_COLS 64
#define LORB_DESC_BYTES 32
#define LORB_MAX_LEVELS 16

/* assign codes written per current-frame keypoint slot by the windowed matchers */
#define LORB_ASSIGN_UNCHANGED (-1)  /* slot keeps whatever MapPoint* it held */
#define LORB_ASSIGN_NULL      (-2)  /* slot set to NULL (rotation-consistency null-out) */

/* slot state of a current-frame keypoint before a windowed match
 * (reference test: `if(F->mvpMapPoints[i] && F->mvpMapPoints[i]->mnObs>0) continue;`,
 *  src/matcher.cpp:149-151, 273-275) */
#define LORB_SLOT_EMPTY   0  /* mvpMapPoints[i] == NULL            */
#define LORB_SLOT_FREE    1  /* MapPoint present with mnObs == 0   */
#define LORB_SLOT_LOCKED  2  /* MapPoint present with mnObs  > 0   */

typedef struct lorb_ctx lorb_ctx;

/* ----------------------------------------------------------------------------------------
 * Context / runtime
 * -------------------------------------------------------------------------------------- */
int lorb_abi_version(void);
int lorb_device_count(int* count);
int lorb_create(int device, lorb_ctx** out);
int lorb_destroy(lorb_ctx* ctx);
const char* lorb_last_error(const lorb_ctx* ctx);
int lorb_sync(lorb_ctx* ctx);                       /* hipStreamSynchronize(ctx stream) */
int lorb_malloc(lorb_ctx* ctx, void** dptr, size_t bytes);
int lorb_free(lorb_ctx* ctx, void* dptr);
int lorb_memcpy_h2d(lorb_ctx* ctx, void* dst, const void* src, size_t bytes);  /* sync */
int lorb_memcpy_d2h(lorb_ctx* ctx, void* dst, const void* src, size_t bytes);  /* sync */
int lorb_memset_dev(lorb_ctx* ctx, void* dst, int value, size_t bytes);        /* async */
/* hipEvent timer on the ctx stream: marks, then elapsed ms between two marks */
int lorb_timer_mark(lorb_ctx* ctx, int slot);        /* slot in [0,64) */
int lorb_timer_elapsed_ms(lorb_ctx* ctx, int slot_begin, int slot_end, float* ms);
/* Per-kernel device timing (HIP events recorded around every launch of the named kernel
 * family on the ctx stream).  Used by bench.py for roofline.achieved.  Kernel ids: */
#define LORB_K_BF_SCAN_TOP2 0
#define LORB_K_BF_SCAN_TOP1 1
#define LORB_K_BA_SCHUR     2
#define LORB_K_BA_LINEARIZE 3
#define LORB_K_BA_CHOLESKY  4
#define LORB_K_WINDOW_CAND  5
#define LORB_K_STEREO       6
#define LORB_K_ALLREDUCE    7   /* the sharded plans' ncclAllReduce exchanges (eager, timed runs) */
#define LORB_K_COUNT        8
int lorb_kernel_timing_enable(lorb_ctx* ctx, int enable);
/* sums (and resets) the recorded launches of kernel id k: total ms and launch count */
int lorb_kernel_timing_read(lorb_ctx* ctx, int k, double* total_ms, int* launches);

/* ----------------------------------------------------------------------------------------
 * Frame description shared by the matchers (all fields are the reference Frame's, float)
 * -------------------------------------------------------------------------------------- */
typedef struct lorb_frame_params {
  float fx, fy, cx, cy;               /* Frame::fx,fy,cx,cy        include/frame.h:96 */
  float bf, b;                        /* Frame::mbf, Frame::mb     include/frame.h:96 */
  float min_x, max_x, min_y, max_y;   /* Frame::mnMinX..mnMaxY     include/frame.h:98-101 */
  float grid_w_inv, grid_h_inv;       /* mfGridElementWidthInv/HeightInv, src/frame.cpp:83-84 */
  int32_t n_levels;                   /* mnScaleLevels */
  float log_scale_factor;             /* mfLogScaleFactor */
  float scale_factors[LORB_MAX_LEVELS]; /* mvScaleFactors */
} lorb_frame_params;

/* SoA view of a frame's undistorted keypoints (Frame::mvKeysUn) + stereo + descriptors */
typedef struct lorb_keypoints {
  int32_t n;                 /* Frame::mnMapPoints */
  const float* x;            /* mvKeysUn[i].pt.x */
  const float* y;            /* mvKeysUn[i].pt.y */
  const int32_t* octave;     /* mvKeysUn[i].octave */
  const float* angle;        /* mvKeysUn[i].angle */
  const float* u_right;      /* mvuRight[i] (NULL => all -1) */
  const uint8_t* desc;       /* mDescriptors, n x 32 bytes row-major */
} lorb_keypoints;

/* ----------------------------------------------------------------------------------------
 * (a2/a3) brute-force Hamming + OpenCV-3.x crossCheck + the reference's outlier filter.
 * Replaces cv::BFMatcher(NORM_HAMMING,true).match at src/matcher.cpp:36-39 and :342-345 and
 * the minDist filter at src/matcher.cpp:42-56 / :348-362.
 *
 * Batched over n_problems independent (query set, train set) pairs, concatenated:
 *   problem p owns queries [q_off[p], q_off[p+1]) and trains [t_off[p], t_off[p+1]).
 *   q_off / t_off are HOST arrays of n_problems+1 entries (also for the _dev variant).
 * Outputs per query (global query index):
 *   cc_train[q]  : OpenCV crossCheck train index (problem-local) or -1 (no DMatch emitted)
 *   cc_dist[q]   : its Hamming distance (undefined when cc_train == -1)
 *   match_train[q]: cc_train[q] if cc_dist <= max(2*minDist, 30) else -1   (src/matcher.cpp:52)
 * n_matches[p] : number of accepted matches of problem p (the reference's return value).
 * -------------------------------------------------------------------------------------- */
int lorb_bf_match(lorb_ctx* ctx, int32_t n_problems,
                  const uint8_t* q_desc, const int32_t* q_off,
                  const uint8_t* t_desc, const int32_t* t_off,
                  int32_t* cc_train, int32_t* cc_dist, int32_t* match_train,
                  int32_t* n_matches);
int lorb_bf_match_dev(lorb_ctx* ctx, int32_t n_problems,
                      const uint8_t* d_q_desc, const int32_t* q_off,
                      const uint8_t* d_t_desc, const int32_t* t_off,
                      int32_t* d_cc_train, int32_t* d_cc_dist, int32_t* d_match_train,
                      int32_t* d_n_matches);

/* ----------------------------------------------------------------------------------------
 * (a5 with an unbounded window; BASELINE config "2000x2000 random 256-bit, ratio test")
 * Brute-force best/second-best with the reference's exact tie semantics
 * (src/matcher.cpp:289-301: strict '<', first candidate in train order wins) and the
 * level-gated ratio test + TH_HIGH acceptance (src/matcher.cpp:305-311).
 * t_level: per-train octave (NULL => all 0, i.e. ratio test always active).
 * Outputs per query: best_idx (-1 if none), best_dist (256 if none), best_level (-1),
 *   second_dist (256), second_level (-1), accepted (0/1).
 * -------------------------------------------------------------------------------------- */
int lorb_bf_top2(lorb_ctx* ctx, int32_t n_problems,
                 const uint8_t* q_desc, const int32_t* q_off,
                 const uint8_t* t_desc, const int32_t* t_off, const int32_t* t_level,
                 int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                 int32_t* second_dist, int32_t* second_level, uint8_t* accepted);
int lorb_bf_top2_dev(lorb_ctx* ctx, int32_t n_problems,
                     const uint8_t* d_q_desc, const int32_t* q_off,
                     const uint8_t* d_t_desc, const int32_t* t_off, const int32_t* d_t_level,
                     int32_t* d_best_idx, int32_t* d_best_dist, int32_t* d_best_level,
                     int32_t* d_second_dist, int32_t* d_second_level, uint8_t* d_accepted);

/* ----------------------------------------------------------------------------------------
 * (a4) Matcher::SearchByProjection(Frame* CurrentFrame, Frame* LastFrame, const float th)
 *      src/matcher.cpp:64-218, incl. Frame::GetFeaturesInArea (src/frame.cpp:370-423),
 *      the grid (src/frame.cpp:87-115) and the rotation histogram / ComputeThreeMaxima.
 * -------------------------------------------------------------------------------------- */
typedef struct lorb_last_frame {
  int32_t n;                 /* LastFrame->mnMapPoints */
  const float* Tcw;          /* LastFrame->mTcw, 4x4 row-major */
  const uint8_t* has_mp;     /* mvpMapPoints[i] != NULL */
  const uint8_t* outlier;    /* mvbOutlier[i] (NULL => all false) */
  const uint8_t* mp_locked;  /* mvpMapPoints[i]->mnObs > 0 */
  const float* mp_pos;       /* mvpMapPoints[i]->GetPos(), n x 3 */
  const uint8_t* mp_desc;    /* mvpMapPoints[i]->GetDescriptor(), n x 32 */
  const int32_t* octave;     /* LastFrame->mvKeys[i].octave */
  const float* angle;        /* LastFrame->mvKeysUn[i].angle */
} lorb_last_frame;

/* assign[j] for current keypoint j: LORB_ASSIGN_UNCHANGED, LORB_ASSIGN_NULL, or i >= 0 meaning
 * CurrentFrame->mvpMapPoints[j] = LastFrame->mvpMapPoints[i].  *nmatches = return value. */
int lorb_search_by_projection_frame(lorb_ctx* ctx,
                                    const lorb_frame_params* cur, const float cur_Tcw[16],
                                    const lorb_keypoints* cur_kps, const uint8_t* cur_slot_state,
                                    const lorb_last_frame* last, float th,
                                    int32_t* assign, int32_t* nmatches);

/* ----------------------------------------------------------------------------------------
 * (a5) Matcher::SearchByProjection(Frame* F, const std::set<MapPoint*>&, const float th)
 *      src/matcher.cpp:220-316.  Points are given flattened in std::set iteration order.
 * -------------------------------------------------------------------------------------- */
typedef struct lorb_local_points {
  int32_t n;
  const uint8_t* track_in_view;   /* mbTrackInView */
  const uint8_t* is_bad;          /* IsBad() (NULL => none) */
  const uint8_t* locked;          /* mnObs > 0 */
  const float* proj_x;            /* mTrackProjX */
  const float* proj_y;            /* mTrackProjY */
  const float* proj_xr;           /* mTrackProjXR */
  const int32_t* pred_level;      /* mnTrackScaleLevel */
  const float* view_cos;          /* mTrackViewCos */
  const uint8_t* desc;            /* GetDescriptor(), n x 32 */
} lorb_local_points;

/* assign[j]: LORB_ASSIGN_UNCHANGED or local point index k (F->mvpMapPoints[j] = point k). */
int lorb_search_by_projection_local(lorb_ctx* ctx,
                                    const lorb_frame_params* frame, const lorb_keypoints* kps,
                                    const uint8_t* slot_state,
                                    const lorb_local_points* pts, float th,
                                    int32_t* assign, int32_t* nmatches);

/* ----------------------------------------------------------------------------------------
 * (a8) Frame::IsInFrustum (src/frame.cpp:425-494) + MapPoint::PredictScale
 *      (src/map_point.cpp:267-284), batched over points.  Writes the tracking fields.
 * -------------------------------------------------------------------------------------- */
typedef struct lorb_frustum_points {
  int32_t n;
  const float* pos;        /* GetPos(), n x 3 */
  const float* normal;     /* mNormalVector, n x 3 */
  const float* max_dist;   /* mfMaxDistance  (GetMaxDistanceInvariance = 1.2f*mfMaxDistance) */
  const float* min_dist;   /* mfMinDistance  (GetMinDistanceInvariance = 0.8f*mfMinDistance) */
} lorb_frustum_points;
int lorb_is_in_frustum(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                       const lorb_frustum_points* pts, float viewing_cos_limit,
                       uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                       int32_t* pred_level, float* view_cos);

/* device-resident local-map tracking -- VisualOdometry::EstimatePoseLocal's
 * sequence (src/visual_odometry.cpp:173-201): IsInFrustum(MP, viewing_cos_limit) for every local
 * map point that is neither already matched in the frame (mnLastFrameSeen == frame id) nor bad,
 * then SearchByProjection(F, localMPs, th), with frame and map data resident on the device.
 * All pointers below are DEVICE pointers (a lorb_keypoints whose arrays live on the device);
 * frame / Tcw are host values.  Outputs: d_in_view (mbTrackInView), d_track (n x 4 as four
 * planes: mTrackProjX, mTrackProjY, mTrackProjXR, mTrackViewCos), d_level (mnTrackScaleLevel),
 * d_assign / d_nmatches as lorb_search_by_projection_local.  Asynchronous on the ctx stream while
 * n_points * n_keypoints <= 8M; larger calls read the candidate count back once. */
typedef struct lorb_map_points_dev {
  int32_t n;
  const float* pos;          /* GetPos(), n x 3 */
  const float* normal;       /* mNormalVector, n x 3 */
  const float* max_dist;     /* mfMaxDistance */
  const float* min_dist;     /* mfMinDistance */
  const uint8_t* desc;       /* GetDescriptor(), n x 32 */
  const uint8_t* locked;     /* mnObs > 0 */
  const uint8_t* is_bad;     /* IsBad() (NULL => none) */
  const uint8_t* in_frame;   /* mnLastFrameSeen == frame id (NULL => none) */
} lorb_map_points_dev;
int lorb_track_local_map_dev(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                             const lorb_keypoints* d_kps, const uint8_t* d_slot_state,
                             const lorb_map_points_dev* pts, float viewing_cos_limit, float th,
                             uint8_t* d_in_view, float* d_track, int32_t* d_level,
                             int32_t* d_assign, int32_t* d_nmatches);
/* host-pointer variant (synchronous): the same structs with host arrays; d_track -> track (4 x n) */
int lorb_track_local_map(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                         const lorb_keypoints* kps, const uint8_t* slot_state,
                         const lorb_map_points_dev* pts, float viewing_cos_limit, float th,
                         uint8_t* in_view, float* track, int32_t* level,
                         int32_t* assign, int32_t* nmatches);

/* (a20) Frame::UnprojectStereo, src/frame.cpp:335-356, batched over keypoints. */
int lorb_unproject_stereo(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                          int32_t n, const float* x, const float* y, const float* depth,
                          float* out_xyz);
/* device-pointer variant (async on the ctx stream); frame / Tcw are host values */
int lorb_unproject_stereo_dev(lorb_ctx* ctx, const lorb_frame_params* frame, const float Tcw[16],
                              int32_t n, const float* d_x, const float* d_y, const float* d_depth,
                              float* d_out_xyz);

/* Frame::ComputeStereoMatches, src/frame.cpp:125-333 -- per left keypoint the
 * best right keypoint in its row band (Hamming < (TH_HIGH+TH_LOW)/2, octave within +-1, disparity in
 * [0, bf/b]), 11x11 SAD refinement over +-5 columns on the keypoint's pyramid level, parabola
 * sub-pixel fit, and the 2.1 x median SAD outlier rejection.  One image pyramid per camera
 * (ORBextractor::mvImagePyramid): level l is rows[l] x cols[l] u8 pixels at data + offset[l],
 * step[l] bytes per row. */
typedef struct lorb_image_pyramid {
  int32_t n_levels;
  const uint8_t* data;
  int64_t offset[LORB_MAX_LEVELS];
  int32_t rows[LORB_MAX_LEVELS], cols[LORB_MAX_LEVELS], step[LORB_MAX_LEVELS];
} lorb_image_pyramid;
/* SoA view of one camera's distorted keypoints (Frame::mvKeys / mvKeysRight) + descriptors */
typedef struct lorb_stereo_keys {
  int32_t n;
  const float* x;            /* kp.pt.x */
  const float* y;            /* kp.pt.y */
  const int32_t* octave;     /* kp.octave */
  const uint8_t* desc;       /* mDescriptors / mDescriptorsRight, n x 32 */
} lorb_stereo_keys;
/* Outputs mvuRight / mvDepth (n_left floats each, -1 where no depth).  Host pointers. */
int lorb_compute_stereo_matches(lorb_ctx* ctx, const lorb_frame_params* frame,
                                const lorb_stereo_keys* left, const lorb_stereo_keys* right,
                                const lorb_image_pyramid* left_pyr, const lorb_image_pyramid* right_pyr,
                                float* u_right, float* depth);
/* device-pointer variant: every array (keys, pyramid data, outputs) lives on the device; the structs
 * themselves and frame are host values.  Async on the ctx stream. */
int lorb_compute_stereo_matches_dev(lorb_ctx* ctx, const lorb_frame_params* frame,
                                    const lorb_stereo_keys* d_left, const lorb_stereo_keys* d_right,
                                    const lorb_image_pyramid* d_left_pyr, const lorb_image_pyramid* d_right_pyr,
                                    float* d_u_right, float* d_depth);

/* SURVEY §8f row 3 (descriptor stage of ORBextractor::operator(), src/ORBextractor.cpp:1087-1154):
 * for every keypoint (level coordinates, i.e. before the `pt *= scale` of :1144-1149) the IC_Angle
 * orientation on its raw pyramid level (computeOrientation, :79-107, :487-493; cv::fastAtan2) and
 * the 32-byte rBRIEF descriptor on the level blurred by GaussianBlur(7x7, sigma 2,
 * BORDER_REFLECT_101) (:1131-1132, :110-150).  pattern: the 512 test points as 1024 ints
 * (x0, y0, x1, y1, ...), the reference's bit_pattern_31_ (:152).  Outputs: angle[n] (KeyPoint::angle,
 * degrees) and desc (n x 32).  Defined for keypoints at least 19 px (EDGE_THRESHOLD, :76) inside
 * their level, as the extractor produces them; the host entry point rejects others. */
int lorb_orb_describe(lorb_ctx* ctx, const lorb_image_pyramid* pyr, int32_t n, const float* x, const float* y,
                      const int32_t* level, const int32_t* pattern, float* angle, uint8_t* desc);
int lorb_orb_describe_dev(lorb_ctx* ctx, const lorb_image_pyramid* d_pyr, int32_t n, const float* d_x,
                          const float* d_y, const int32_t* d_level, const int32_t* d_pattern, float* d_angle,
                          uint8_t* d_desc);

/* SURVEY §8f row 3, FAST stage of ORBextractor::ComputeKeyPointsOctTree (src/ORBextractor.cpp:
 * 803-872): per level the grid of 30-pixel cells with a 6-pixel overlap inside the
 * EDGE_THRESHOLD - 3 = 16-pixel border, and per cell cv::FAST(cell, ini_th, nonmax = true), re-run
 * with min_th when the cell found NO corner (:855-859).  Keypoints come out in level coordinates,
 * grouped by level, then cell (row-major), then FAST's scan order -- the order of vToDistributeKeys
 * -- with response = FAST score.  Cell c of level l spans [cell_off[cell_base[l] + l + c],
 * cell_off[cell_base[l] + l + c + 1]); cell_base has n_levels + 1 entries.  Host pointers; sync. */
int lorb_orb_fast_cells(lorb_ctx* ctx, const lorb_image_pyramid* pyr, int32_t ini_th, int32_t min_th,
                        int32_t max_keypoints, float* x, float* y, float* response, int32_t max_cells,
                        int32_t* cell_base, int32_t* cell_off, int32_t* n_keypoints);

/* SURVEY §8f row 3, ORBextractor::ComputePyramid (src/ORBextractor.cpp:1157-1184): level 0 is
 * the image, level l = cv::resize(level l-1, cvRound(size / scale_factors[l]), INTER_LINEAR)
 * (OpenCV 3.1's 8U fixed-point resize incl. its SSE2 vertical pass, see oracle/orb.c).  Levels are
 * packed row-major into `out` (out_bytes capacity); `layout` receives the lorb_image_pyramid view
 * (data = out).  The reference's copyMakeBorder margins are never read downstream and are not
 * produced.  _dev: device image and out (returns after the levels are written). */
int lorb_orb_pyramid(lorb_ctx* ctx, const uint8_t* image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                     const float* scale_factors, uint8_t* out, int64_t out_bytes, lorb_image_pyramid* layout);
int lorb_orb_pyramid_dev(lorb_ctx* ctx, const uint8_t* d_image, int32_t rows, int32_t cols, int32_t step,
                         int32_t n_levels, const float* scale_factors, uint8_t* d_out, int64_t out_bytes,
                         lorb_image_pyramid* layout);

/* SURVEY §8f row 3, ORBextractor::ComputeKeyPointsOctTree without the orientation
 * (src/ORBextractor.cpp:799-892): lorb_orb_fast_cells, then DistributeOctTree per level
 * (:554-797; N = n_desired[l] = mnFeaturesPerLevel[l]) -- the quadtree that keeps the strongest
 * keypoint of every node -- then the border offset, octave and size (PATCH_SIZE * scale_factors[l]
 * truncated to int, :881).  Per keypoint: x, y (level coordinates), octave, size, response, in the
 * reference's order (level, then the final std::list order of the quadtree nodes);
 * level_off[n_levels + 1].  Nodes holding equal key counts are ranked by creation order where the
 * reference compares std::list node addresses (:717).  Host pointers; synchronous. */
int lorb_orb_detect(lorb_ctx* ctx, const lorb_image_pyramid* pyr, const int32_t* n_desired,
                    const float* scale_factors, int32_t ini_th, int32_t min_th, int32_t max_keypoints, float* x,
                    float* y, int32_t* octave, float* size, float* response, int32_t* level_off,
                    int32_t* n_keypoints);

/* SURVEY §8f row 3, the whole ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (src/ORBextractor.cpp:1087-1151): ComputePyramid, ComputeKeyPointsOctTree (+ IC_Angle
 * orientation), GaussianBlur + rBRIEF per level with the caller's 256-pair pattern
 * (bit_pattern_31_, :152), and the coordinates of level > 0 keypoints scaled to level 0 (:1141-1147).
 * Outputs in the reference's keypoint order: x, y, octave, size, angle (degrees), response and the
 * 32-byte descriptors; level_off[n_levels + 1]; *n_keypoints.  max_keypoints must be at least
 * lorb_orb_extract_capacity()'s bound for the _dev variant.  Host pointers; synchronous. */
int lorb_orb_extract(lorb_ctx* ctx, const uint8_t* image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                     const float* scale_factors, const int32_t* n_desired, int32_t ini_th, int32_t min_th,
                     const int32_t* pattern, int32_t max_keypoints, float* x, float* y, int32_t* octave, float* size,
                     float* angle, float* response, uint8_t* desc, int32_t* level_off, int32_t* n_keypoints);
/* device variant: image, pattern (1024 ints), the pyramid buffer (pyramid_bytes) and every output
 * are device arrays, d_level_off (n_levels + 1) and d_n (1) too.  Returns once the pyramid is
 * built (its resize tables are host-staged); detection and description run asynchronously on the
 * ctx stream.  *d_n = -1 when a quadtree exceeded its node capacity. */
int lorb_orb_extract_dev(lorb_ctx* ctx, const uint8_t* d_image, int32_t rows, int32_t cols, int32_t step,
                         int32_t n_levels, const float* scale_factors, const int32_t* n_desired, int32_t ini_th,
                         int32_t min_th, const int32_t* d_pattern, int32_t max_keypoints, uint8_t* d_pyramid,
                         int64_t pyramid_bytes, float* d_x, float* d_y, int32_t* d_octave, float* d_size,
                         float* d_angle, float* d_response, uint8_t* d_desc, int32_t* d_level_off, int32_t* d_n);
/* output capacity (keypoints) and pyramid bytes lorb_orb_extract_dev needs for an image size */
int lorb_orb_extract_capacity(int32_t rows, int32_t cols, int32_t n_levels, const float* scale_factors,
                              const int32_t* n_desired, int32_t* max_keypoints, int64_t* pyramid_bytes);

/* ----------------------------------------------------------------------------------------
 * Bundle adjustment: Ceres-default Levenberg-Marquardt + DENSE_SCHUR restated
 * (src/bundle_adjust.cpp:158-202 and :207-330; solver defaults in SURVEY Appendix B).
 * -------------------------------------------------------------------------------------- */
#define LORB_TERM_NO_CONVERGENCE 0   /* max_num_iterations reached */
#define LORB_TERM_FUNCTION_TOL   1
#define LORB_TERM_GRADIENT_TOL   2
#define LORB_TERM_PARAMETER_TOL  3
#define LORB_TERM_MIN_RADIUS     4
#define LORB_TERM_FAILURE        5   /* too many consecutive invalid steps */

typedef struct lorb_lm_options {       /* defaults == ceres::Solver::Options defaults */
  int32_t max_num_iterations;          /* 50 */
  double function_tolerance;           /* 1e-6 */
  double gradient_tolerance;           /* 1e-10 */
  double parameter_tolerance;          /* 1e-8 */
  double initial_trust_region_radius;  /* 1e4 */
  double max_trust_region_radius;      /* 1e16 */
  double min_trust_region_radius;      /* 1e-32 */
  double min_relative_decrease;        /* 1e-3 */
  double min_lm_diagonal;              /* 1e-6 */
  double max_lm_diagonal;              /* 1e32 */
  int32_t max_num_consecutive_invalid_steps; /* 5 */
  int32_t jacobi_scaling;              /* 1 */
} lorb_lm_options;
void lorb_lm_options_default(lorb_lm_options* opt);

typedef struct lorb_ba_summary {
  int32_t iterations;          /* LM iterations performed (successful + unsuccessful) */
  int32_t successful_steps;
  int32_t termination;         /* LORB_TERM_* */
  int32_t pad_;
  double initial_cost;         /* 0.5 * sum r^2 */
  double final_cost;
} lorb_ba_summary;

/* Per-iteration record of a local-BA solve (diagnostics / parity): one record per
 * LM iteration that computed a step, as Ceres' IterationSummary holds it (trust_region_minimizer.cc:
 * cost, model cost change, the candidate's cost, the radius the step was computed with, |step|).
 * The first LORB_LM_TRACE_CAP iterations of every window are recorded. */
#define LORB_LM_STEP_INVALID   0   /* linear solve failed / non-positive model decrease */
#define LORB_LM_STEP_ACCEPTED  1
#define LORB_LM_STEP_REJECTED  2   /* relative decrease <= min_relative_decrease */
#define LORB_LM_STEP_PARAM_TOL 3   /* solve ends: |step| <= parameter_tolerance * (|x| + ptol) */
#define LORB_LM_STEP_FUNC_TOL  4   /* solve ends: |cost change| <= function_tolerance * cost */
#define LORB_LM_TRACE_CAP 64
typedef struct lorb_lm_iteration {
  int32_t iteration;           /* 1-based */
  int32_t outcome;             /* LORB_LM_STEP_* */
  double cost;                 /* cost at the current point */
  double model_cost_change;    /* -(J step)^T (r + J step / 2), the linear model's decrease */
  double new_cost;             /* cost at the candidate x + step (valid steps) */
  double radius;               /* trust-region radius the step was computed with */
  double step_norm;            /* |x_candidate - x| (valid steps) */
} lorb_lm_iteration;

/* (a12) BA::ProjectPoseOptimization: pose-only, one PoseCost per matched map point.
 * The PoseCost quirk (v projected with fx, src/bundle_adjust.cpp:51) is reproduced by passing
 * fy_eff = fx; pass the real fy to get the "fixed" projection.  Batched over frames:
 * frame f owns residuals [res_off[f], res_off[f+1]) (HOST array).
 * pose_init: n_frames x 6 floats = (mRvec | mTvec)  (src/bundle_adjust.cpp:163-168)
 * pose_out:  n_frames x 6 doubles (the Ceres parameter blocks after Solve)
 * Tcw_out (optional): n_frames x 16 floats, Frame::SetPose(T,R) write-back via Rodrigues
 *   (src/bundle_adjust.cpp:198-201 -> src/frame.cpp:577-594). */
typedef struct lorb_pose_problem_batch {
  int32_t n_frames;
  const int32_t* res_off;      /* n_frames+1 */
  const float* intr;           /* n_frames x 4: fx, fy_eff, cx, cy */
  const float* pose_init;      /* n_frames x 6 */
  const float* pts3d;          /* n_res x 3 (MapPoint::GetPos) */
  const float* obs2d;          /* n_res x 2 (Frame::GetKp2d) */
} lorb_pose_problem_batch;
int lorb_ba_pose_only(lorb_ctx* ctx, const lorb_pose_problem_batch* prob,
                      const lorb_lm_options* opt, double* pose_out, float* Tcw_out,
                      lorb_ba_summary* summaries);

/* (a13) BA::LocalPoseOptimization: poses + points, MPCost for out-of-window (fixed) frames,
 * PoseMPCost for window frames.  One window per problem; batched over windows.
 * obs_frame[k] >= 0 : optimised pose index (PoseMPCost, src/bundle_adjust.cpp:293-301)
 * obs_frame[k] <  0 : fixed frame index (-1 - obs_frame[k]) (MPCost, :283-290) */
typedef struct lorb_ba_window {
  int32_t n_poses, n_fixed, n_points, n_obs;
  float fx, fy, cx, cy;
  const float* pose_init;      /* n_poses x 6 (mRvec|mTvec) */
  const float* fixed_pose;     /* n_fixed x 6 */
  const float* point_init;     /* n_points x 3 */
  const int32_t* obs_point;    /* n_obs */
  const int32_t* obs_frame;    /* n_obs */
  const float* obs_uv;         /* n_obs x 2 */
} lorb_ba_window;

/* (a13) BA::LocalPoseOptimization (src/bundle_adjust.cpp:207-330) over independent windows.  Any
 * number of cameras; LORB_E_UNSUPPORTED for a point observed by more than 256 cameras, or by two
 * cameras more than 127 apart in the plan's camera order (the point-major Schur's point groups,
 * DESIGN.md §7). */
int lorb_ba_local(lorb_ctx* ctx, int32_t n_windows, const lorb_ba_window* windows,
                  const lorb_lm_options* opt, double* const* pose_out,
                  double* const* point_out, lorb_ba_summary* summaries);

/* Device-resident plan for repeated solves of the same window batch (benchmarks, LM in
 * a captured HIP graph).  create: uploads + builds the Schur structure; solve: runs the LM
 * from the uploaded initial values entirely on the device (async); read: copies results. */
typedef struct lorb_ba_plan lorb_ba_plan;
int lorb_ba_plan_create(lorb_ctx* ctx, int32_t n_windows, const lorb_ba_window* windows,
                        lorb_ba_plan** out);
int lorb_ba_plan_solve(lorb_ba_plan* plan, const lorb_lm_options* opt);
int lorb_ba_plan_read(lorb_ba_plan* plan, double* const* pose_out, double* const* point_out,
                      lorb_ba_summary* summaries);
int lorb_ba_plan_destroy(lorb_ba_plan* plan);
/* Device-resident plan of ONE window whose arrays already live in HBM (the LocalMapping step
 * appends the new keyframe's observations on the device).  Sizes that change from call to call are
 * device ints; the capacities bound them.  Observation slots k < *d_n_obs with
 * d_obs_frame[k] < -n_fixed are unused (skipped) -- how a keyframe leaves the window without a
 * compaction.  Observations of one point come out in slot order, as lorb_ba_window's do.  A point
 * may be observed at most once per camera (the reference keys observations by Frame*,
 * include/map_point.h:83).  create: capacity allocations + the first build; update: rebuild from
 * the arrays' current contents (one small readback of counts and the camera covisibility, then
 * sorting and point groups on the device).  solve / read / info / destroy as
 * lorb_ba_plan_*; result_dev writes the solution as float in the caller's pose order (device
 * pointers, either may be NULL; async). */
typedef struct lorb_ba_window_dev {
  int32_t n_poses, n_fixed;          /* host values */
  int32_t max_points, max_obs;       /* capacities of the arrays below */
  const int32_t* d_n_points;         /* device: points in use (<= max_points) */
  const int32_t* d_n_obs;            /* device: observation slots in use (<= max_obs) */
  float fx, fy, cx, cy;
  const float* d_pose_init;          /* n_poses x 6 (mRvec | mTvec) */
  const float* d_fixed_pose;         /* n_fixed x 6 */
  const float* d_point_init;         /* max_points x 3 */
  const int32_t* d_obs_point;        /* max_obs */
  const int32_t* d_obs_frame;        /* max_obs: >= 0 optimised pose, -1-j fixed pose j, < -n_fixed unused */
  const float* d_obs_uv;             /* max_obs x 2 */
} lorb_ba_window_dev;
/* n_poses <= 128 (the camera tables travel as kernel arguments; LORB_E_UNSUPPORTED above) */
int lorb_ba_plan_create_dev(lorb_ctx* ctx, const lorb_ba_window_dev* win, lorb_ba_plan** out);
int lorb_ba_plan_update_dev(lorb_ba_plan* plan, const lorb_ba_window_dev* win);
int lorb_ba_plan_result_dev(lorb_ba_plan* plan, float* d_pose_out, float* d_point_out);
/* (a13) BA::LocalPoseOptimization for a caller that gathers a NEW window on every call -- the drop-in
 * (src/bundle_adjust.cpp:207-330; the call site src/local_mapping.cpp:32).  Same inputs, outputs and
 * errors as lorb_ba_local with one window, but the solver keeps device-built plans
 * (lorb_ba_plan_create_dev) resident across calls, one per camera count (a small LRU), with capacities
 * that grow, so a call costs one host-to-device copy of the window, the device plan build (one small
 * readback), the captured LM graph and one device-to-host copy of the solution -- no per-call plan
 * construction, allocation or graph capture.  Windows the device plans do not take (no cameras /
 * points / observations, more than 128 cameras, a point with 256 or more observations) run through lorb_ba_local's
 * host-built plan on the same GPU kernels.  A point observed twice by one camera is an error (both
 * plan builders; the reference keys observations by Frame*).  One solver per ctx / thread.
 * pose_out: n_poses x 6 doubles (caller order), point_out: n_points x 3 doubles.  Synchronous. */
typedef struct lorb_ba_solver lorb_ba_solver;
int lorb_ba_solver_create(lorb_ctx* ctx, lorb_ba_solver** out);
int lorb_ba_solver_solve(lorb_ba_solver* solver, const lorb_ba_window* window, const lorb_lm_options* opt,
                         double* pose_out, double* point_out, lorb_ba_summary* summary);
/* first n of: [0] resident plans, [1] plan creations so far, [2] 1 if the last call ran on the host-built
 * plan, [3] its S half band, [4] its Cholesky kernel, [5] 1 if its cameras were reordered (RCM) */
int lorb_ba_solver_info(lorb_ba_solver* solver, int32_t* info, int32_t n);
/* the last call's per-iteration records (lorb_ba_plan_trace of the resident plan it ran on; none after a
 * call that took the host-built plan) */
int lorb_ba_solver_trace(lorb_ba_solver* solver, lorb_lm_iteration* out, int32_t cap, int32_t* n_out);
int lorb_ba_solver_destroy(lorb_ba_solver* solver);
/* The ctx's own solver: created on the first call, destroyed by lorb_destroy(ctx) (so it never
 * outlives its ctx, and a new ctx never inherits it).  Not to be passed to lorb_ba_solver_destroy.
 * The adapters' LocalPoseOptimization uses it (include/lorb/adapters.hpp). */
int lorb_ctx_ba_solver(lorb_ctx* ctx, lorb_ba_solver** out);
/* plan structure, first n of: [0] S half band (max over windows, scalar rows), [1] Cholesky kernel of
 * the last solve (0 k_ba_chol, 1 k_ba_chol_w, 2 k_ba_chol_2s, -1 none yet), [2] (camera, camera)
 * blocks, [3] point groups, [4] observations, [5] points, [6] cameras, [7] 1 if some window's
 * cameras were reordered (reverse Cuthill-McKee on the covisibility graph; outputs keep the
 * caller's order), [8] 1: the point-major Schur path (the only one since round 6; point groups span
 * <= 128 cameras), [9] its partial-reduction width (threads per block: 256, 512 or 1024), [10] partial
 * runs of the last build (0: one partial per point group; else the runs of several groups that
 * k_ba_ls_sup folds into one partial each -- windows of more than 512 point groups) */
int lorb_ba_plan_info(lorb_ba_plan* plan, int32_t* info, int32_t n);
/* the last solve's per-iteration records of window w (at most min(cap, LORB_LM_TRACE_CAP)); *n_out =
 * records written.  Synchronises. */
int lorb_ba_plan_trace(lorb_ba_plan* plan, int32_t window, lorb_lm_iteration* out, int32_t cap, int32_t* n_out);
/* diagnostics: Cholesky phase stamps of window 0 (non-zero only in LORB_CHOL_STAMPS builds) */
int lorb_ba_plan_debug_stamps(lorb_ba_plan* plan, unsigned long long* out8);
/* Plan group: the LM solves of several plans on ONE ctx launched as one set of kernels (one launch per
 * kernel for all members, one captured graph), as a plan of several windows is -- for independent
 * windows whose plans are built separately (the device-built plans of several lorb_map windows:
 * lorb_map_group_*).  No reference counterpart (the reference solves one window per call,
 * src/bundle_adjust.cpp:308-314).  Each member's results (poses, points, summary, trace) are
 * bit-identical to lorb_ba_plan_solve of that plan.  Up to 4 members run fused when every member is
 * an unsharded plan on the two-sided Cholesky (lorb_ba_plan_info [1] == 2 after a solve; C3 / C4
 * windows); otherwise the members are solved one after another.  The group does not own its plans:
 * they must outlive it, and may be rebuilt (lorb_ba_plan_update_dev) between solves.  solve is
 * asynchronous (read the members with lorb_ba_plan_read). */
typedef struct lorb_ba_group lorb_ba_group;
int lorb_ba_group_create(lorb_ctx* ctx, int32_t n_plans, lorb_ba_plan* const* plans, lorb_ba_group** out);
int lorb_ba_group_solve(lorb_ba_group* group, const lorb_lm_options* opt);
/* first n of: [0] member plans, [1] solves that ran as one set of launches, [2] graph captures */
int lorb_ba_group_info(lorb_ba_group* group, int32_t* info, int32_t n);
int lorb_ba_group_destroy(lorb_ba_group* group);

/* ----------------------------------------------------------------------------------------
 * SURVEY §8 a17, the LocalMapping "full step" (SURVEY §7 item 8): a local map resident in HBM and
 * the chained step over it.  Replaces LocalMapping::ProcessNewFrames' disabled steps 1-3 followed by
 * BA::LocalPoseOptimization (src/local_mapping.cpp:24-33, 55-76; src/bundle_adjust.cpp:207-330).
 *
 * The map holds keyframes by id: the window [t0, t0 + W) is optimised, the F keyframes before it
 * are fixed (MPCost), older ones are gone.  create: keyframes [0, W) optimised, [-F, 0) fixed.
 * Per step the new keyframe gets id t0 + W and:
 *   1. its descriptors are matched against the map's points (Matcher::SearchLocalPoints,
 *      src/matcher.cpp:319-366 -- crossCheck + minDist filter, trains in map order);
 *   2. a matched keypoint adds an observation (point, keyframe, keypoint uv) to its point
 *      (MapPoint::AddObservation, src/local_mapping.cpp:57-70); an unmatched keypoint with
 *      depth > 0 becomes a new map point at Frame::UnprojectStereo (src/frame.cpp:335-356) with the
 *      keypoint's descriptor, observed by the keyframe.  Appended in keypoint order;
 *   3. the window slides by one keyframe: points that no window keyframe observes leave the map,
 *      observations by keyframes older than the F fixed ones are dropped; order is kept (stable);
 *   4. BA::LocalPoseOptimization of the window (device-built plan, LM with `opt`), then the float
 *      write-back of the window's poses and all points (src/bundle_adjust.cpp:317-329).
 * step_dev is asynchronous except for one small readback (the plan's counts and covisibility).
 * Errors: a step whose new points / observations would exceed the capacities returns LORB_E_NOMEM
 * and leaves the map as it was.  A step that fails later (the plan build of step 4, e.g. a point
 * with 256 or more observations) returns that error with steps 1-3 applied: the map stays usable
 * (its host counts are re-read from the device) and the next step rebuilds the plan.  If even that
 * re-read fails, the map is marked broken and every later step returns LORB_E_DEVICE.
 * ---------------------------------------------------------------------------------------- */
typedef struct lorb_map lorb_map;
typedef struct lorb_map_init {
  int32_t n_window, n_fixed;          /* W <= 128 optimised keyframes (ids 0..W-1), F fixed (ids -1..-F) */
  int32_t max_points, max_obs, max_keypoints;   /* capacities */
  float fx, fy, cx, cy;
  const float* pose;                  /* W x 6 (mRvec | mTvec), row j = keyframe j */
  const float* fixed_pose;            /* F x 6, row j = keyframe -1-j */
  int32_t n_points, n_obs;
  const float* point;                 /* n_points x 3 (MapPoint::GetPos) */
  const uint8_t* point_desc;          /* n_points x 32 (MapPoint::GetDescriptor) */
  const int32_t* obs_point;           /* n_obs */
  const int32_t* obs_kf;              /* n_obs: keyframe id in [-F, W); a point at most once per keyframe */
  const float* obs_uv;                /* n_obs x 2 */
} lorb_map_init;
/* host buffers for lorb_map_read (any may be NULL): sizes from lorb_map_counts */
typedef struct lorb_map_state {
  float* point;                       /* n_points x 3 */
  uint8_t* point_desc;                /* n_points x 32 */
  int32_t* obs_point;                 /* n_obs */
  int32_t* obs_kf;                    /* n_obs: keyframe ids */
  float* obs_uv;                      /* n_obs x 2 */
  int32_t* obs_frame;                 /* n_obs: the BA slot (lorb_ba_window convention) */
  float* pose;                        /* W x 6: keyframes t0 .. t0 + W - 1 */
  float* fixed_pose;                  /* F x 6: keyframes t0 - 1 .. t0 - F */
  int32_t* match_train;               /* last step's keypoints: matched map point (pre-step index) or -1 */
  lorb_ba_summary* summary;           /* last BA solve */
} lorb_map_state;
int lorb_map_create(lorb_ctx* ctx, const lorb_map_init* init, lorb_map** out);
/* frame / pose (the tracked mRvec | mTvec) / Tcw (its 4x4) are host values; descriptors, x, y
 * (Frame::mvKeysUn) and depth (Frame::mvDepth) are device arrays of n keypoints */
int lorb_map_step_dev(lorb_map* map, const lorb_frame_params* frame, const float pose[6], const float Tcw[16],
                      int32_t n, const uint8_t* d_desc, const float* d_x, const float* d_y, const float* d_depth,
                      const lorb_lm_options* opt);
/* Overlap of consecutive steps (default off): with enable = 1, step t+1's match and append run on a
 * stream the map owns, concurrently with step t's BA solve, ordered only after step t's plan build
 * (they touch the map's descriptors, new slots and counts and the map's own key buffers -- nothing
 * the solve or its write-back reads or writes).  Results are bit-identical to enable = 0.
 * REQUIREMENT while enabled: the keyframe arrays handed to lorb_map_step_dev (d_desc, d_x, d_y,
 * d_depth) must be complete when the call is made -- uploaded or produced by work the caller has
 * already synchronised.  The map's stream is not ordered after work still queued on the ctx stream
 * or any other stream, so inputs produced asynchronously need enable = 0 (then every kernel of a
 * step runs on the ctx stream, in order).  The reference's LocalMapping::Run consumes keyframes the
 * tracking thread has finished (src/local_mapping.cpp:19-40), which is the enabled case.  Per-kernel
 * timing (lorb_kernel_timing_enable) runs the steps serially either way. */
int lorb_map_set_overlap(lorb_map* map, int32_t enable);
/* first n of: [0] points, [1] observations, [2] t0, [3] last step's keypoints, [4] its new points,
 * [5] its new observations (matches + new points), [6] its matches, [7] W, [8] steps whose match and
 * append ran overlapped (lorb_map_set_overlap).  Synchronises. */
int lorb_map_counts(lorb_map* map, int32_t* out, int32_t n);
int lorb_map_read(lorb_map* map, const lorb_map_state* state);
int lorb_map_plan(lorb_map* map, lorb_ba_plan** out);   /* the map's BA plan (owned by the map) */
int lorb_map_destroy(lorb_map* map);
/* Several maps stepped together (independent LocalMapping windows on one GPU, north_star's sharding
 * unit): every map on the same ctx.  A group step gives each map its keyframe (kfs[i] for maps[i]) and
 * runs steps 1-3 and the plan build of every map, then ONE BA solve over all of their plans
 * (lorb_ba_group, fused for up to 4 maps per group of launches), then the write-backs.  Each map's
 * state after the step is bit-identical to lorb_map_step_dev of that map alone.  Errors: a map whose
 * steps 1-3 or plan build fail is left as lorb_map_step_dev leaves it after that error; when a map's
 * steps 1-3 fail, the maps after it in the group are not stepped; every other map completes its step
 * (solve and write-back).  The first error is returned.  The group does not own its maps: they must
 * outlive it. */
typedef struct lorb_map_group lorb_map_group;
typedef struct lorb_map_keyframe {
  const lorb_frame_params* frame;
  const float* pose;                  /* 6 (host) */
  const float* Tcw;                   /* 16 (host) */
  int32_t n;
  const uint8_t* d_desc;              /* device arrays of n keypoints, as lorb_map_step_dev */
  const float* d_x;
  const float* d_y;
  const float* d_depth;
} lorb_map_keyframe;
int lorb_map_group_create(int32_t n_maps, lorb_map* const* maps, lorb_map_group** out);
int lorb_map_group_step_dev(lorb_map_group* group, const lorb_map_keyframe* kfs, const lorb_lm_options* opt);
/* first n of: [0] maps, [1] plan groups, [2] steps whose solves all ran as one set of launches per plan
 * group, [3] graph captures over the plan groups */
int lorb_map_group_info(lorb_map_group* group, int32_t* info, int32_t n);
int lorb_map_group_destroy(lorb_map_group* group);

/* ----------------------------------------------------------------------------------------
 * Multi-GPU: point-partitioned ("sharded") local BA.  No reference counterpart:
 * the reference is single-process (its Ceres solve is src/bundle_adjust.cpp:308-314).
 *
 * One process (or thread) per GPU, each with its own lorb_ctx.  Every rank passes the SAME
 * window poses / fixed poses / intrinsics and only ITS points with all of their observations
 * (every observation of a point on the rank that owns the point).  Per LM iteration the ranks
 * all-reduce (i) the camera normal blocks, cost and gradient norms of the linearisation,
 * (ii) the reduced camera system S and its right-hand side, (iii) the model/candidate cost
 * and step norms.  The Cholesky of S and every LM decision are replicated, so all ranks hold
 * identical poses; each rank holds its own points.
 *
 * Communicators: RCCL (ncclAllReduce on the ctx stream, capturable in the LM hipGraph) or a
 * host callback (any host transport, e.g. gloo in tests; the plan then runs eagerly).
 * -------------------------------------------------------------------------------------- */
#define LORB_OP_SUM 0
#define LORB_OP_MAX 1
#define LORB_OP_MIN 2
#define LORB_UNIQUE_ID_BYTES 128
typedef struct lorb_comm lorb_comm;
/* host all-reduce over all ranks, in place on `buf` (count doubles); returns 0 on success */
typedef int (*lorb_host_allreduce_fn)(void* user, double* buf, int64_t count, int32_t op);

int lorb_comm_unique_id(void* id_out /* LORB_UNIQUE_ID_BYTES */);        /* rank 0 only */
int lorb_comm_init_rccl(lorb_ctx* ctx, int32_t nranks, int32_t rank, const void* unique_id,
                        lorb_comm** out);
int lorb_comm_init_host(lorb_ctx* ctx, int32_t nranks, int32_t rank, lorb_host_allreduce_fn fn,
                        void* user, lorb_comm** out);
int lorb_comm_destroy(lorb_comm* comm);
/* ranks in the communicator (ncclCommCount / ncclCommUserRank for RCCL); rank may be NULL */
int lorb_comm_size(lorb_comm* comm, int32_t* nranks, int32_t* rank);
/* all-reduce of device doubles on the ctx stream (send == recv allowed) */
int lorb_comm_allreduce_f64(lorb_comm* comm, const double* d_send, double* d_recv, int64_t count,
                            int32_t op);

/* plan over this rank's shard of each window; solve / read / destroy as lorb_ba_plan_*.
 * read returns the (replicated) poses and this rank's points. */
int lorb_ba_plan_create_sharded(lorb_ctx* ctx, lorb_comm* comm, int32_t n_windows,
                                const lorb_ba_window* shards, lorb_ba_plan** out);

/* the device-built plan (lorb_ba_plan_create_dev) over this rank's shard of ONE window: the shard's
 * points with all of their observations in device arrays (lorb_ba_window_dev; point indices local to
 * the shard), the same n_poses / n_fixed / poses on every rank.  Each build all-reduces the camera
 * covisibility and counts (camera order, band and activity are global; the block pair lists are this
 * rank's), so lorb_ba_plan_update_dev is collective: every rank calls it, and an error on any rank
 * is returned on all of them.  solve / read / result_dev as for lorb_ba_plan_create_sharded. */
int lorb_ba_plan_create_sharded_dev(lorb_ctx* ctx, lorb_comm* comm, const lorb_ba_window_dev* shard,
                                    lorb_ba_plan** out);

/* (a2/a3) with query rows split over ranks.  This rank holds queries
 * [q_base[p], q_base[p] + q_off[p+1] - q_off[p]) of problem p (global numbering) and ALL of its
 * trains.  Outputs as lorb_bf_match_dev for the local queries (global train indices);
 * n_matches[p] is the count over all ranks.  q_off / t_off / q_base are HOST arrays. */
int lorb_bf_match_sharded_dev(lorb_ctx* ctx, lorb_comm* comm, int32_t n_problems,
                              const uint8_t* d_q_desc, const int32_t* q_off, const int32_t* q_base,
                              const uint8_t* d_t_desc, const int32_t* t_off,
                              int32_t* d_cc_train, int32_t* d_cc_dist, int32_t* d_match_train,
                              int32_t* d_n_matches);

/* MapPoint::ComputeDescriptor (src/map_point.cpp:69-129; called at src/visual_odometry.cpp:94,392),
 * batched over map points.  Point p's candidate descriptors -- its observations in
 * std::map<Frame*, size_t> order, bad frames skipped (:74-81) -- are rows [d_off[p], d_off[p+1]) of
 * desc (32 bytes each).  best[p] = index within the point's list of the descriptor whose median
 * Hamming distance to the list (self included; element floor((n-1)/2) of the sorted row) is
 * smallest, first index on ties; -1 for an empty list (the reference indexes an empty vector
 * there).  out_desc (optional, n_points x 32) receives the chosen descriptor (zeros when -1).
 * d_off is a HOST array for lorb_compute_descriptor and a DEVICE array for the _dev variant. */
int lorb_compute_descriptor(lorb_ctx* ctx, int32_t n_points, const int32_t* d_off,
                            const uint8_t* desc, int32_t* best, uint8_t* out_desc);
int lorb_compute_descriptor_dev(lorb_ctx* ctx, int32_t n_points, const int32_t* d_off,
                                const uint8_t* d_desc, int32_t* d_best, uint8_t* d_out_desc);

/* Rodrigues vector -> Tcw (float), cv::Rodrigues semantics (double internally). */
void lorb_pose_to_Tcw(const float rvec[3], const float tvec[3], float Tcw[16]);

#ifdef __cplusplus
}
#endif
#endif /* LORB_C_H */
