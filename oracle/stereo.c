/*
 * stereo.c -- TEST INFRASTRUCTURE ONLY (see lorb_oracle.h).  CPU restatement of
 * Frame::ComputeStereoMatches, src/frame.cpp:125-333.
 *
 * Behaviour the reference leaves undefined, defined here and in the HIP path alike:
 *  - right keypoint bands reaching outside [0, nRows) are clipped (the reference indexes
 *    vRowIndices out of range, src/frame.cpp:159-160);
 *  - a left keypoint whose row (size_t)vL is outside [0, nRows) has no candidates (:184);
 *  - an 11x11 window (IL or any IR of the +-5 sweep) reaching outside its pyramid level is a
 *    "no depth" (the reference's cv::Mat::rowRange/colRange assert and throw, :242,261);
 *  - no accepted pair: the median rejection is skipped (the reference reads vDistIdx[0] of an
 *    empty vector, :320).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lorb_oracle.h"

typedef struct { int dist, idx; } or_dist_idx;

static int cmp_dist_idx(const void* a, const void* b) {
  const or_dist_idx* x = (const or_dist_idx*)a;
  const or_dist_idx* y = (const or_dist_idx*)b;
  if (x->dist != y->dist) return x->dist < y->dist ? -1 : 1;
  return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* 11x11 window with top-left (r0, c0) on level `lv` of pyramid P lies inside the level */
static int win_inside(const lorb_image_pyramid* P, int lv, int r0, int c0) {
  return r0 >= 0 && c0 >= 0 && r0 + 11 <= P->rows[lv] && c0 + 11 <= P->cols[lv];
}

static int px(const lorb_image_pyramid* P, int lv, int r, int c) {
  return P->data[P->offset[lv] + (int64_t)r * P->step[lv] + c];
}

/* src/frame.cpp:125-333 */
int or_compute_stereo_matches(const lorb_frame_params* fp, const lorb_stereo_keys* L, const lorb_stereo_keys* R,
                              const lorb_image_pyramid* PL, const lorb_image_pyramid* PR, float* u_right,
                              float* depth) {
  const int nL = L->n, nR = R->n;
  for (int i = 0; i < nL; i++) { u_right[i] = -1.0f; depth[i] = -1.0f; }        /* :127-128 */
  const int thOrbDist = (LORB_TH_HIGH + LORB_TH_LOW) / 2;                         /* :130 */
  const int nRows = PL->rows[0];                                                  /* :132 */
  /* row table (:140-161), CSR in iR order */
  int* cnt = (int*)calloc((size_t)nRows + 1, sizeof(int));
  for (int iR = 0; iR < nR; iR++) {
    const float kpY = R->y[iR];
    const float r = 2.0f * fp->scale_factors[R->octave[iR]];
    const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
    for (int yi = minr < 0 ? 0 : minr; yi <= maxr && yi < nRows; yi++) cnt[yi + 1]++;
  }
  for (int i = 0; i < nRows; i++) cnt[i + 1] += cnt[i];
  int* rows = (int*)malloc(sizeof(int) * (size_t)(cnt[nRows] + 1));
  int* fill = (int*)calloc((size_t)nRows, sizeof(int));
  for (int iR = 0; iR < nR; iR++) {
    const float kpY = R->y[iR];
    const float r = 2.0f * fp->scale_factors[R->octave[iR]];
    const int maxr = (int)ceilf(kpY + r), minr = (int)floorf(kpY - r);
    for (int yi = minr < 0 ? 0 : minr; yi <= maxr && yi < nRows; yi++) rows[cnt[yi] + fill[yi]++] = iR;
  }
  const float minZ = fp->b;                                                       /* :164-166 */
  const float minD = 0;
  const float maxD = fp->bf / minZ;
  or_dist_idx* vDistIdx = (or_dist_idx*)malloc(sizeof(or_dist_idx) * (size_t)(nL + 1));
  int nDI = 0;
  for (int iL = 0; iL < nL; iL++) {                                               /* :176 */
    const int levelL = L->octave[iL];
    const float vL = L->y[iL], uL = L->x[iL];
    if (!(vL >= 0.0f) || vL >= (float)nRows) continue;
    const int row = (int)vL;                                                      /* :184 */
    if (cnt[row + 1] == cnt[row]) continue;
    const float minU = uL - maxD, maxU = uL - minD;                               /* :189-193 */
    if (maxU < 0) continue;
    int bestDist = LORB_TH_HIGH, bestIdxR = 0;                                    /* :195-225 */
    const uint8_t* dL = L->desc + (size_t)iL * 32;
    for (int c = cnt[row]; c < cnt[row + 1]; c++) {
      const int iR = rows[c];
      if (R->octave[iR] < levelL - 1 || R->octave[iR] > levelL + 1) continue;
      const float uR = R->x[iR];
      if (uR >= minU && uR <= maxU) {
        const int dist = or_descriptor_distance(dL, R->desc + (size_t)iR * 32);
        if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
      }
    }
    if (bestDist >= thOrbDist) continue;                                          /* :230 */
    const float uR0 = R->x[bestIdxR];                                             /* :234-238 */
    const float scaleFactor = 1.0f / fp->scale_factors[levelL];
    const float scaleduL = roundf(uL * scaleFactor);
    const float scaledvL = roundf(vL * scaleFactor);
    const float scaleduR0 = roundf(uR0 * scaleFactor);
    const int w = 5, Lw = 5;                                                      /* :241,248 */
    const int cu = (int)scaleduL, cv = (int)scaledvL, cr = (int)scaleduR0;
    const float iniu = scaleduR0 + Lw - w, endu = scaleduR0 + Lw + w + 1;         /* :253-256 */
    if (!win_inside(PL, levelL, cv - w, cu - w)) continue;
    if (iniu < 0 || endu >= PR->cols[levelL]) continue;
    if (!win_inside(PR, levelL, cv - w, cr - Lw - w)) continue;
    const int cL = px(PL, levelL, cv, cu);                                       /* :243-244 */
    int bestSad = INT32_MAX, bestincR = 0;
    float vDists[11];
    for (int incR = -Lw; incR <= Lw; incR++) {                                    /* :258-273 */
      const int cRc = px(PR, levelL, cv, cr + incR);
      int sad = 0;
      for (int dy = -w; dy <= w; dy++)
        for (int dx = -w; dx <= w; dx++) {
          const int a = px(PL, levelL, cv + dy, cu + dx) - cL;
          const int b = px(PR, levelL, cv + dy, cr + incR + dx) - cRc;
          sad += abs(a - b);
        }
      const float dist = (float)sad;
      if (dist < (float)bestSad) { bestSad = (int)dist; bestincR = incR; }
      vDists[Lw + incR] = dist;
    }
    if (bestincR == -Lw || bestincR == Lw) continue;                              /* :275-276 */
    const float dist1 = vDists[Lw + bestincR - 1];                                /* :282-290 */
    const float dist2 = vDists[Lw + bestincR];
    const float dist3 = vDists[Lw + bestincR + 1];
    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
    if (deltaR < -1 || deltaR > 1) continue;
    float bestuR = fp->scale_factors[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);  /* :296 */
    float disparity = (uL - bestuR);                                              /* :299-313 */
    if (disparity >= minD && disparity < maxD) {
      if (disparity <= 0) {
        disparity = (float)0.01;
        bestuR = (float)((double)uL - 0.01);
      }
      depth[iL] = fp->bf / disparity;
      u_right[iL] = bestuR;
      vDistIdx[nDI].dist = bestSad; vDistIdx[nDI].idx = iL; nDI++;
    }
  }
  if (nDI > 0) {                                                                  /* :319-332 */
    qsort(vDistIdx, (size_t)nDI, sizeof(or_dist_idx), cmp_dist_idx);
    const float median = (float)vDistIdx[nDI / 2].dist;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = nDI - 1; i >= 0; i--) {
      if ((float)vDistIdx[i].dist < thDist) break;
      u_right[vDistIdx[i].idx] = -1;
      depth[vDistIdx[i].idx] = -1;
    }
  }
  const int nacc = nDI;
  free(cnt); free(rows); free(fill); free(vDistIdx);
  return nacc;
}
