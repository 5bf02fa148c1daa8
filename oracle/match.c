/*
 * match.c -- TEST INFRASTRUCTURE ONLY (see lorb_oracle.h header: parity unpinned vs the real
 * reference, which is unbuildable here).  CPU restatement of the reference matcher path.
 * Compiled with -O2 -ffp-contract=off so every float expression rounds like the reference's
 * un-contracted x86-64 build.
 */
#include "lorb_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* Matcher::DescriptorDistance, src/matcher.cpp:369-385: 8 int32 words, SWAR popcount. */
int or_descriptor_distance(const uint8_t* a, const uint8_t* b) {
  int dist = 0;
  for (int i = 0; i < 8; i++) {
    int32_t pa, pb;
    memcpy(&pa, a + 4 * i, 4);
    memcpy(&pb, b + 4 * i, 4);
    unsigned int v = (unsigned int)(pa ^ pb);
    v = v - ((v >> 1) & 0x55555555u);
    v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
    dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
  }
  return dist;
}

/* Matcher::RadiusByViewingCos, src/matcher.cpp:430-436 (float promoted to double compare) */
float or_radius_by_viewing_cos(float view_cos) {
  if ((double)view_cos > 0.998) return 2.5f;
  return 4.0f;
}

/* Matcher::ComputeThreeMaxima, src/matcher.cpp:387-428 */
void or_compute_three_maxima(const int* hist, int L, int* ind1, int* ind2, int* ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = hist[i];
    if (s > max1) {
      max3 = max2; max2 = max1; max1 = s;
      *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
    } else if (s > max2) {
      max3 = max2; max2 = s;
      *ind3 = *ind2; *ind2 = i;
    } else if (s > max3) {
      max3 = s; *ind3 = i;
    }
  }
  if ((float)max2 < 0.1f * (float)max1) {
    *ind2 = -1; *ind3 = -1;
  } else if ((float)max3 < 0.1f * (float)max1) {
    *ind3 = -1;
  }
}

/* OpenCV 3.x batchDistance(crossCheck=true, K=1) semantics, called at
 * src/matcher.cpp:36-39, followed by the reference's minDist filter src/matcher.cpp:42-56. */
int or_bf_match(const uint8_t* q, int nq, const uint8_t* t, int nt,
                int32_t* cc_train, int32_t* cc_dist, int32_t* match_train) {
  for (int i = 0; i < nq; i++) { cc_train[i] = -1; cc_dist[i] = 0; match_train[i] = -1; }
  if (nq == 0 || nt == 0) return 0;  /* BFMatcher::knnMatchImpl: empty set -> no matches */
  int* tidx = (int*)malloc(sizeof(int) * (size_t)nt);
  int* tdist = (int*)malloc(sizeof(int) * (size_t)nt);
  int* dist = (int*)malloc(sizeof(int) * (size_t)nq);
  /* reverse pass: for each train row, nearest query (first index on ties, strict <) */
  for (int j = 0; j < nt; j++) {
    int best = INT_MAX, bi = -1;
    for (int i = 0; i < nq; i++) {
      int d = or_descriptor_distance(q + 32 * (size_t)i, t + 32 * (size_t)j);
      if (d < best) { best = d; bi = i; }
    }
    tidx[j] = bi; tdist[j] = best;
  }
  for (int i = 0; i < nq; i++) dist[i] = INT_MAX;
  for (int j = 0; j < nt; j++) {
    int i = tidx[j];
    if (tdist[j] < dist[i]) { dist[i] = tdist[j]; cc_train[i] = j; }
  }
  double minDist = DBL_MAX;
  for (int i = 0; i < nq; i++)
    if (cc_train[i] >= 0) { cc_dist[i] = dist[i]; if ((double)dist[i] < minDist) minDist = dist[i]; }
  int n = 0;
  for (int i = 0; i < nq; i++) {
    if (cc_train[i] < 0) continue;
    double thr = 2 * minDist > 30.0 ? 2 * minDist : 30.0;
    if ((double)(float)cc_dist[i] > thr) continue;
    match_train[i] = cc_train[i];
    n++;
  }
  free(tidx); free(tdist); free(dist);
  return n;
}

/* best / second-best scan of src/matcher.cpp:289-311 over all trains in order */
static void top2_rows(const uint8_t* q, int i0, int i1, const uint8_t* t, int nt,
                      const int32_t* t_level, int32_t* best_idx, int32_t* best_dist,
                      int32_t* best_level, int32_t* second_dist, int32_t* second_level,
                      uint8_t* accepted) {
  for (int i = i0; i < i1; i++) {
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    const uint8_t* qd = q + 32 * (size_t)i;
    for (int j = 0; j < nt; j++) {
      const int dist = or_descriptor_distance(qd, t + 32 * (size_t)j);
      const int lev = t_level ? t_level[j] : 0;
      if (dist < bestDist) {
        bestDist2 = bestDist; bestDist = dist;
        bestLevel2 = bestLevel; bestLevel = lev; bestIdx = j;
      } else if (dist < bestDist2) {
        bestLevel2 = lev; bestDist2 = dist;
      }
    }
    int acc = 0;
    if (bestDist <= LORB_TH_HIGH) {
      acc = 1;
      if (bestLevel == bestLevel2 && (double)bestDist > 0.8 * (double)bestDist2) acc = 0;
    }
    best_idx[i] = bestIdx; best_dist[i] = bestDist; best_level[i] = bestLevel;
    second_dist[i] = bestDist2; second_level[i] = bestLevel2; accepted[i] = (uint8_t)acc;
  }
}

void or_bf_top2(const uint8_t* q, int nq, const uint8_t* t, int nt, const int32_t* t_level,
                int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                int32_t* second_dist, int32_t* second_level, uint8_t* accepted) {
  top2_rows(q, 0, nq, t, nt, t_level, best_idx, best_dist, best_level, second_dist,
            second_level, accepted);
}

typedef struct {
  const uint8_t *q, *t; int i0, i1, nt; const int32_t* t_level;
  int32_t *bi, *bd, *bl, *sd, *sl; uint8_t* acc;
} top2_job;
static void* top2_thread(void* p) {
  top2_job* j = (top2_job*)p;
  top2_rows(j->q, j->i0, j->i1, j->t, j->nt, j->t_level, j->bi, j->bd, j->bl, j->sd, j->sl,
            j->acc);
  return NULL;
}
void or_bf_top2_mt(const uint8_t* q, int nq, const uint8_t* t, int nt, const int32_t* t_level,
                   int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                   int32_t* second_dist, int32_t* second_level, uint8_t* accepted, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  top2_job jobs[256];
  for (int k = 0; k < threads; k++) {
    top2_job* j = &jobs[k];
    j->q = q; j->t = t; j->nt = nt; j->t_level = t_level;
    j->i0 = (int)((long)nq * k / threads); j->i1 = (int)((long)nq * (k + 1) / threads);
    j->bi = best_idx; j->bd = best_dist; j->bl = best_level; j->sd = second_dist;
    j->sl = second_level; j->acc = accepted;
    pthread_create(&th[k], NULL, top2_thread, j);
  }
  for (int k = 0; k < threads; k++) pthread_join(th[k], NULL);
}

/* ---------------------------------------------------------------------------------------- */
/* Frame grid: AssignFeaturesToGrid / PosInGrid, src/frame.cpp:87-115 */
static int pos_in_grid(const lorb_frame_params* fp, float x, float y, int* px, int* py) {
  *px = (int)roundf((x - fp->min_x) * fp->grid_w_inv);
  *py = (int)roundf((y - fp->min_y) * fp->grid_h_inv);
  if (*px < 0 || *px >= LORB_GRID_COLS || *py < 0 || *py >= LORB_GRID_ROWS) return 0;
  return 1;
}

void or_grid_build(const lorb_frame_params* fp, const lorb_keypoints* kps, or_grid* g) {
  const int NC = LORB_GRID_COLS * LORB_GRID_ROWS;
  int* cnt = (int*)calloc((size_t)NC, sizeof(int));
  int* cell = (int*)malloc(sizeof(int) * (size_t)(kps->n > 0 ? kps->n : 1));
  for (int i = 0; i < kps->n; i++) {
    int px, py;
    if (pos_in_grid(fp, kps->x[i], kps->y[i], &px, &py)) {
      cell[i] = px * LORB_GRID_ROWS + py;
      cnt[cell[i]]++;
    } else {
      cell[i] = -1;
    }
  }
  g->cell_off[0] = 0;
  for (int c = 0; c < NC; c++) g->cell_off[c + 1] = g->cell_off[c] + cnt[c];
  g->idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)(kps->n > 0 ? kps->n : 1));
  memset(cnt, 0, sizeof(int) * (size_t)NC);
  for (int i = 0; i < kps->n; i++)  /* insertion order = keypoint order (push_back) */
    if (cell[i] >= 0) g->idx[g->cell_off[cell[i]] + cnt[cell[i]]++] = i;
  free(cnt); free(cell);
}

void or_grid_free(or_grid* g) { free(g->idx); g->idx = NULL; }

/* Frame::GetFeaturesInArea, src/frame.cpp:370-423 */
int or_features_in_area(const lorb_frame_params* fp, const lorb_keypoints* kps, const or_grid* g,
                        float x, float y, float r, int minLevel, int maxLevel, int32_t* out) {
  int n = 0;
  const int nMinCellX0 = (int)floorf((x - fp->min_x - r) * fp->grid_w_inv);
  const int nMinCellX = nMinCellX0 > 0 ? nMinCellX0 : 0;
  if (nMinCellX >= LORB_GRID_COLS) return 0;
  const int nMaxCellX0 = (int)ceilf((x - fp->min_x + r) * fp->grid_w_inv);
  const int nMaxCellX = nMaxCellX0 < LORB_GRID_COLS - 1 ? nMaxCellX0 : LORB_GRID_COLS - 1;
  if (nMaxCellX < 0) return 0;
  const int nMinCellY0 = (int)floorf((y - fp->min_y - r) * fp->grid_h_inv);
  const int nMinCellY = nMinCellY0 > 0 ? nMinCellY0 : 0;
  if (nMinCellY >= LORB_GRID_ROWS) return 0;
  const int nMaxCellY0 = (int)ceilf((y - fp->min_y + r) * fp->grid_h_inv);
  const int nMaxCellY = nMaxCellY0 < LORB_GRID_ROWS - 1 ? nMaxCellY0 : LORB_GRID_ROWS - 1;
  if (nMaxCellY < 0) return 0;
  const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
  for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
    for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
      const int c = ix * LORB_GRID_ROWS + iy;
      for (int k = g->cell_off[c]; k < g->cell_off[c + 1]; k++) {
        const int j = g->idx[k];
        if (bCheckLevels) {
          if (kps->octave[j] < minLevel) continue;
          if (maxLevel >= 0)
            if (kps->octave[j] > maxLevel) continue;
        }
        const float distx = kps->x[j] - x;
        const float disty = kps->y[j] - y;
        if (fabsf(distx) < r && fabsf(disty) < r) out[n++] = j;
      }
    }
  }
  return n;
}

/* cv::Mat float (3x3)*(3x1) [+ c] through cv::gemm: float operands, double accumulation,
 * one cast to float (OpenCV GEMMSingleMul<float,double>; exact agreement with a given
 * OpenCV build is unpinned). */
static float gemv3_row(const float* R, const float* x, float c) {
  double s = (double)R[0] * (double)x[0] + (double)R[1] * (double)x[1] + (double)R[2] * (double)x[2];
  return (float)(s + (double)c);
}

/* (a4) Matcher::SearchByProjection(Frame*, Frame*, const float th), src/matcher.cpp:64-218 */
int or_search_by_projection_frame(const lorb_frame_params* cur, const float Tcw[16],
                                  const lorb_keypoints* ck, const uint8_t* slot_state_in,
                                  const lorb_last_frame* last, float th,
                                  int32_t* assign, int32_t* nmatches_out) {
  const int nc = ck->n;
  int nmatches = 0;
  const float factor = LORB_HISTO_LENGTH / 360.0f;
  int* hist_cnt = (int*)calloc(LORB_HISTO_LENGTH, sizeof(int));
  int* hist_bin = (int*)malloc(sizeof(int) * (size_t)(last->n > 0 ? last->n : 1));   /* per accept */
  int* hist_slot = (int*)malloc(sizeof(int) * (size_t)(last->n > 0 ? last->n : 1));
  int n_acc = 0;
  uint8_t* state = (uint8_t*)malloc((size_t)(nc > 0 ? nc : 1));
  for (int j = 0; j < nc; j++) { assign[j] = LORB_ASSIGN_UNCHANGED; state[j] = slot_state_in ? slot_state_in[j] : 0; }
  or_grid g;
  or_grid_build(cur, ck, &g);
  int32_t* cand = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nc > 0 ? nc : 1));

  /* src/matcher.cpp:74-87 */
  const float Rcw[9] = {Tcw[0], Tcw[1], Tcw[2], Tcw[4], Tcw[5], Tcw[6], Tcw[8], Tcw[9], Tcw[10]};
  const float tcw[3] = {Tcw[3], Tcw[7], Tcw[11]};
  float twc[3];
  for (int i = 0; i < 3; i++) {  /* -Rcw.t()*tcw */
    double s = (double)Rcw[i] * tcw[0] + (double)Rcw[3 + i] * tcw[1] + (double)Rcw[6 + i] * tcw[2];
    twc[i] = (float)(-s);
  }
  const float* L = last->Tcw;
  const float Rlw[9] = {L[0], L[1], L[2], L[4], L[5], L[6], L[8], L[9], L[10]};
  const float tlw[3] = {L[3], L[7], L[11]};
  const float tlc2 = gemv3_row(Rlw + 6, twc, tlw[2]);
  const int bForward = tlc2 > cur->b;
  const int bBackward = -tlc2 > cur->b;

  for (int i = 0; i < last->n; i++) {
    if (!last->has_mp[i]) continue;
    if (last->outlier && last->outlier[i]) continue;
    const float* X = last->mp_pos + 3 * (size_t)i;
    const float xc = gemv3_row(Rcw + 0, X, tcw[0]);
    const float yc = gemv3_row(Rcw + 3, X, tcw[1]);
    const float zc = gemv3_row(Rcw + 6, X, tcw[2]);
    const float invzc = (float)(1.0 / (double)zc);
    if (invzc < 0) continue;
    const float u = cur->fx * xc * invzc + cur->cx;
    const float v = cur->fy * yc * invzc + cur->cy;
    if (u < cur->min_x || u > cur->max_x) continue;
    if (v < cur->min_y || v > cur->max_y) continue;
    const int nLastOctave = last->octave[i];
    const float radius = th * cur->scale_factors[nLastOctave];
    int nc_found;
    if (bForward)
      nc_found = or_features_in_area(cur, ck, &g, u, v, radius, nLastOctave, -1, cand);
    else if (bBackward)
      nc_found = or_features_in_area(cur, ck, &g, u, v, radius, 0, nLastOctave, cand);
    else
      nc_found = or_features_in_area(cur, ck, &g, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand);
    if (nc_found == 0) continue;
    const uint8_t* dMP = last->mp_desc + 32 * (size_t)i;
    int bestDist = 256, bestIdx2 = -1;
    for (int k = 0; k < nc_found; k++) {
      const int i2 = cand[k];
      if (state[i2] == LORB_SLOT_LOCKED) continue;
      if (ck->u_right && ck->u_right[i2] > 0) {
        const float ur = u - cur->bf * invzc;
        const float er = fabsf(ur - ck->u_right[i2]);
        if (er > radius) continue;
      }
      const int dist = or_descriptor_distance(dMP, ck->desc + 32 * (size_t)i2);
      if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
    }
    if (bestDist <= LORB_TH_HIGH) {
      assign[bestIdx2] = i;
      state[bestIdx2] = last->mp_locked[i] ? LORB_SLOT_LOCKED : LORB_SLOT_FREE;
      nmatches++;
      float rot = last->angle[i] - ck->angle[bestIdx2];
      if (rot < 0.0) rot += 360.0f;
      int bin = (int)roundf(rot * factor);
      if (bin == LORB_HISTO_LENGTH) bin = 0;
      hist_cnt[bin]++;
      hist_bin[n_acc] = bin; hist_slot[n_acc] = bestIdx2; n_acc++;
    }
  }
  /* rotation consistency, src/matcher.cpp:196-215 */
  int ind1 = -1, ind2 = -1, ind3 = -1;
  or_compute_three_maxima(hist_cnt, LORB_HISTO_LENGTH, &ind1, &ind2, &ind3);
  for (int a = 0; a < n_acc; a++) {
    const int b = hist_bin[a];
    if (b != ind1 && b != ind2 && b != ind3) { assign[hist_slot[a]] = LORB_ASSIGN_NULL; nmatches--; }
  }
  *nmatches_out = nmatches;
  or_grid_free(&g);
  free(cand); free(state); free(hist_cnt); free(hist_bin); free(hist_slot);
  return LORB_OK;
}

/* (a5) Matcher::SearchByProjection(Frame*, const std::set<MapPoint*>&, const float th),
 * src/matcher.cpp:220-316 */
int or_search_by_projection_local(const lorb_frame_params* fp, const lorb_keypoints* kps,
                                  const uint8_t* slot_state_in, const lorb_local_points* pts,
                                  float th, int32_t* assign, int32_t* nmatches_out) {
  const int nk = kps->n;
  int nmatches = 0;
  const int bFactor = th != 1.0f;
  uint8_t* state = (uint8_t*)malloc((size_t)(nk > 0 ? nk : 1));
  for (int j = 0; j < nk; j++) { assign[j] = LORB_ASSIGN_UNCHANGED; state[j] = slot_state_in ? slot_state_in[j] : 0; }
  or_grid g;
  or_grid_build(fp, kps, &g);
  int32_t* cand = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nk > 0 ? nk : 1));
  for (int m = 0; m < pts->n; m++) {
    if (!pts->track_in_view[m]) continue;
    if (pts->is_bad && pts->is_bad[m]) continue;
    const int nPredictedLevel = pts->pred_level[m];
    float r = or_radius_by_viewing_cos(pts->view_cos[m]);
    if (bFactor) r *= th;
    const float rs = r * fp->scale_factors[nPredictedLevel];
    const int nc = or_features_in_area(fp, kps, &g, pts->proj_x[m], pts->proj_y[m], rs,
                                       nPredictedLevel - 1, nPredictedLevel, cand);
    if (nc == 0) continue;
    const uint8_t* MPd = pts->desc + 32 * (size_t)m;
    int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
    for (int k = 0; k < nc; k++) {
      const int idx = cand[k];
      if (state[idx] == LORB_SLOT_LOCKED) continue;
      if (kps->u_right && kps->u_right[idx] > 0) {
        const float er = fabsf(pts->proj_xr[m] - kps->u_right[idx]);
        if (er > r * fp->scale_factors[nPredictedLevel]) continue;
      }
      const int dist = or_descriptor_distance(MPd, kps->desc + 32 * (size_t)idx);
      if (dist < bestDist) {
        bestDist2 = bestDist; bestDist = dist;
        bestLevel2 = bestLevel; bestLevel = kps->octave[idx]; bestIdx = idx;
      } else if (dist < bestDist2) {
        bestLevel2 = kps->octave[idx]; bestDist2 = dist;
      }
    }
    if (bestDist <= LORB_TH_HIGH) {
      if (bestLevel == bestLevel2 && (double)bestDist > 0.8 * (double)bestDist2) continue;
      assign[bestIdx] = m;
      state[bestIdx] = pts->locked[m] ? LORB_SLOT_LOCKED : LORB_SLOT_FREE;
      nmatches++;
    }
  }
  *nmatches_out = nmatches;
  or_grid_free(&g);
  free(cand); free(state);
  return LORB_OK;
}

/* ---------------------------------------------------------------------------------------- */
/* cv::invert(DECOMP_LU) for 4x4 CV_32F -> hal::LU32f (Gaussian elimination with partial
 * pivoting in float, eps = 10*FLT_EPSILON) applied to the identity. */
int or_inv4_f32(const float Ain[16], float out[16]) {
  float A[16], b[16];
  memcpy(A, Ain, sizeof(A));
  for (int i = 0; i < 16; i++) b[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  const int m = 4, n = 4;
  const float eps = FLT_EPSILON * 10;
  for (int i = 0; i < m; i++) {
    int k = i;
    for (int j = i + 1; j < m; j++)
      if (fabsf(A[j * 4 + i]) > fabsf(A[k * 4 + i])) k = j;
    if (fabsf(A[k * 4 + i]) < eps) { memset(out, 0, 16 * sizeof(float)); return 0; }
    if (k != i) {
      for (int j = i; j < m; j++) { float t = A[i * 4 + j]; A[i * 4 + j] = A[k * 4 + j]; A[k * 4 + j] = t; }
      for (int j = 0; j < n; j++) { float t = b[i * 4 + j]; b[i * 4 + j] = b[k * 4 + j]; b[k * 4 + j] = t; }
    }
    const float d = -1 / A[i * 4 + i];
    for (int j = i + 1; j < m; j++) {
      const float alpha = A[j * 4 + i] * d;
      for (int kk = i + 1; kk < m; kk++) A[j * 4 + kk] += alpha * A[i * 4 + kk];
      for (int kk = 0; kk < n; kk++) b[j * 4 + kk] += alpha * b[i * 4 + kk];
    }
  }
  for (int i = m - 1; i >= 0; i--)
    for (int j = 0; j < n; j++) {
      float s = b[i * 4 + j];
      for (int k = i + 1; k < m; k++) s -= A[i * 4 + k] * b[k * 4 + j];
      b[i * 4 + j] = s / A[i * 4 + i];
    }
  memcpy(out, b, sizeof(b));
  return 1;
}

/* 4x4 float * 4x1 float through cv::gemm (double accumulation) */
static void gemv4(const float M[16], const float x[4], float out[4]) {
  for (int r = 0; r < 4; r++) {
    double s = (double)M[4 * r] * x[0] + (double)M[4 * r + 1] * x[1] + (double)M[4 * r + 2] * x[2] +
               (double)M[4 * r + 3] * x[3];
    out[r] = (float)s;
  }
}

/* (a8) Frame::IsInFrustum, src/frame.cpp:425-494 ; MapPoint::PredictScale,
 * src/map_point.cpp:267-284 ; Get{Min,Max}DistanceInvariance src/map_point.cpp:209-217 */
void or_is_in_frustum(const lorb_frame_params* fp, const float Tcw[16],
                      const lorb_frustum_points* pts, float viewingCosLimit,
                      uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                      int32_t* pred_level, float* view_cos) {
  float Twc[16];
  or_inv4_f32(Tcw, Twc);
  const float Ow[3] = {Twc[3], Twc[7], Twc[11]};
  for (int m = 0; m < pts->n; m++) {
    in_view[m] = 0;
    const float* P = pts->pos + 3 * (size_t)m;
    const float PM[4] = {P[0], P[1], P[2], 1.0f};
    float Pc[4];
    gemv4(Tcw, PM, Pc);
    if (Pc[2] < 0.0f) continue;
    const float invz = 1.0f / Pc[2];
    const float u = fp->fx * Pc[0] * invz + fp->cx;
    const float v = fp->fy * Pc[1] * invz + fp->cy;
    if (u < fp->min_x || u > fp->max_x) continue;
    if (v < fp->min_y || v > fp->max_y) continue;
    const float maxDistance = 1.2f * pts->max_dist[m];
    const float minDistance = 0.8f * pts->min_dist[m];
    const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
    const float dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
    if (dist < minDistance || dist > maxDistance) continue;
    const float* Pn = pts->normal + 3 * (size_t)m;
    const float dot = PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2];
    const float viewCos = dot / dist;
    if (viewCos < viewingCosLimit) continue;
    /* PredictScale */
    const float ratio = pts->max_dist[m] / dist;
    int nScale = (int)ceilf(logf(ratio) / fp->log_scale_factor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= fp->n_levels) nScale = fp->n_levels - 1;
    in_view[m] = 1;
    proj_x[m] = u;
    proj_xr[m] = u - fp->bf * invz;
    proj_y[m] = v;
    pred_level[m] = nScale;
    view_cos[m] = viewCos;
  }
}

/* (a20) Frame::UnprojectStereo, src/frame.cpp:335-356 */
void or_unproject_stereo(const lorb_frame_params* fp, const float Tcw[16], int n,
                         const float* x, const float* y, const float* depth, float* out) {
  float Twc[16];
  or_inv4_f32(Tcw, Twc);
  for (int i = 0; i < n; i++) {
    const float z = depth[i];
    if (z > 0) {
      const float xx = (x[i] - fp->cx) * z / fp->fx;
      const float yy = (y[i] - fp->cy) * z / fp->fy;
      const float X[4] = {xx, yy, z, 1.0f};
      float W[4];
      gemv4(Twc, X, W);
      out[3 * i] = W[0]; out[3 * i + 1] = W[1]; out[3 * i + 2] = W[2];
    } else {
      out[3 * i] = 0.0f; out[3 * i + 1] = 0.0f; out[3 * i + 2] = 0.0f;
    }
  }
}

/* cv::Rodrigues(vector->matrix) (double internally, OpenCV 3.x cvRodrigues2) then
 * Frame::UpdatePoseMat, src/frame.cpp:577-594 (mTcw initialised as eye(4)). */
void or_pose_to_Tcw(const float rvec[3], const float tvec[3], float T[16]) {
  double rx = rvec[0], ry = rvec[1], rz = rvec[2];
  double theta = sqrt(rx * rx + ry * ry + rz * rz);
  double R[9];
  if (theta < DBL_EPSILON) {
    for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
  } else {
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double c = cos(theta), s = sin(theta), c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta; ry *= itheta; rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rx_[k];
  }
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[3 * r + c];
    T[4 * r + 3] = tvec[r];
  }
  T[12] = 0.0f; T[13] = 0.0f; T[14] = 0.0f; T[15] = 1.0f;
}

/* MapPoint::ComputeDescriptor, src/map_point.cpp:69-129: all-pairs distance matrix (:84-109),
 * per row a sorted copy and its element 0.5*(n-1) truncated (:113-118), strict '<' on the
 * median (:119).  Batched over points (CSR d_off); best = -1 for an empty list. */
static int or_cmp_int(const void* a, const void* b) { return (*(const int*)a > *(const int*)b) - (*(const int*)a < *(const int*)b); }
void or_compute_descriptor(int n_points, const int32_t* d_off, const uint8_t* desc, int32_t* best) {
  for (int p = 0; p < n_points; p++) {
    const int o0 = d_off[p], n = d_off[p + 1] - o0;
    if (n <= 0) { best[p] = -1; continue; }
    int* dist = (int*)malloc(sizeof(int) * (size_t)n * (size_t)n);
    int* row = (int*)malloc(sizeof(int) * (size_t)n);
    for (int i = 0; i < n; i++) {
      dist[i * n + i] = 0;
      for (int j = i + 1; j < n; j++) {
        const int d = or_descriptor_distance(desc + 32 * (size_t)(o0 + i), desc + 32 * (size_t)(o0 + j));
        dist[i * n + j] = d;
        dist[j * n + i] = d;
      }
    }
    int bestIdx = 0, bestMedian = 0x7fffffff;
    for (int i = 0; i < n; i++) {
      memcpy(row, dist + (size_t)i * n, sizeof(int) * (size_t)n);
      qsort(row, (size_t)n, sizeof(int), or_cmp_int);
      const int median = row[(size_t)(0.5 * (n - 1))];
      if (median < bestMedian) { bestMedian = median; bestIdx = i; }
    }
    best[p] = bestIdx;
    free(dist); free(row);
  }
}
