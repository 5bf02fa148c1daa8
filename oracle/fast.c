/*
 * fast.c -- TEST INFRASTRUCTURE ONLY (see lorb_oracle.h).  CPU restatement of the detection stage
 * of ORBextractor::ComputeKeyPointsOctTree (src/ORBextractor.cpp:898-1000), SURVEY §8f row 3:
 * the per-level cell grid (:903-990) and, per cell, cv::FAST(cell, iniThFAST, true) re-run with
 * minThFAST when it finds at most 3 corners (:990-996).  cv::FAST is OpenCV 3.1's FAST_t<16>
 * (9 contiguous of the 16-pixel circle of radius 3, threshold_tab prefilter) with cornerScore<16>
 * and 3x3 non-maximum suppression, restated from its published source (features2d/src/fast.cpp,
 * fast_score.cpp); OpenCV is absent here, so this is "parity unpinned" (tests/ cross-check it
 * against an independent numpy restatement).  The retention that follows (KeyPointsFilter::
 * retainBest, :1000-1067) is restated at the end of this file together with the libstdc++
 * algorithms it runs on.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lorb_oracle.h"

/* makeOffsets(pixel, step, 16): the circle, then its first 9 entries again (N = 25) */
static const int kOff16[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1}, {2, -2}, {1, -3},
                                  {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

static void make_offsets(int* pixel, int step) {
  for (int k = 0; k < 16; k++) pixel[k] = kOff16[k][0] + kOff16[k][1] * step;
  for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
}

/* cornerScore<16> */
int or_fast_score(const uint8_t* ptr, const int* pixel, int threshold) {
  const int K = 8, N = K * 3 + 1;
  int k, v = ptr[0];
  short d[25];
  for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
  int a0 = threshold;
  for (k = 0; k < 16; k += 2) {
    int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
    a = a < d[k + 3] ? a : d[k + 3];
    if (a <= a0) continue;
    for (int m = 4; m <= 8; m++) a = a < d[k + m] ? a : d[k + m];
    const int e0 = a < d[k] ? a : d[k], e9 = a < d[k + 9] ? a : d[k + 9];
    a0 = a0 > e0 ? a0 : e0;
    a0 = a0 > e9 ? a0 : e9;
  }
  int b0 = -a0;
  for (k = 0; k < 16; k += 2) {
    int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
    for (int m = 3; m <= 5; m++) b = b > d[k + m] ? b : d[k + m];
    if (b >= b0) continue;
    for (int m = 6; m <= 8; m++) b = b > d[k + m] ? b : d[k + m];
    const int e0 = b > d[k] ? b : d[k], e9 = b > d[k + 9] ? b : d[k + 9];
    b0 = b0 < e0 ? b0 : e0;
    b0 = b0 < e9 ? b0 : e9;
  }
  return -b0 - 1;
}

/* FAST_t<16>(img (w x h view, row stride step), threshold, nonmax_suppression = true).  Writes up
 * to max_out keypoints (x, y in view coordinates, response) in the order cv::FAST emits them;
 * returns the number found. */
int or_fast(const uint8_t* img, int w, int h, int step, int threshold, int max_out, float* ox, float* oy,
            float* oresp) {
  int pixel[25];
  make_offsets(pixel, step);
  threshold = threshold < 0 ? 0 : (threshold > 255 ? 255 : threshold);
  uint8_t tab[512];
  for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);
  uint8_t* score = (uint8_t*)calloc((size_t)(w > 0 ? w : 1) * (size_t)(h > 0 ? h : 1), 1);
  uint8_t* corner = (uint8_t*)calloc((size_t)(w > 0 ? w : 1) * (size_t)(h > 0 ? h : 1), 1);
  for (int i = 3; i < h - 3; i++)
    for (int j = 3; j < w - 3; j++) {
      const uint8_t* ptr = img + (size_t)i * step + j;
      const int v = ptr[0];
      const uint8_t* t = tab - v + 255;
      int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
      if (d == 0) continue;
      d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
      d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
      d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
      if (d == 0) continue;
      d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
      d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
      d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
      d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
      int is = 0;
      if (d & 1) {
        const int vt = v - threshold;
        int count = 0;
        for (int k = 0; k < 25; k++) {
          if (ptr[pixel[k]] < vt) { if (++count > 8) { is = 1; break; } }
          else count = 0;
        }
      }
      if (!is && (d & 2)) {
        const int vt = v + threshold;
        int count = 0;
        for (int k = 0; k < 25; k++) {
          if (ptr[pixel[k]] > vt) { if (++count > 8) { is = 1; break; } }
          else count = 0;
        }
      }
      if (is) {
        corner[(size_t)i * w + j] = 1;
        score[(size_t)i * w + j] = (uint8_t)or_fast_score(ptr, pixel, threshold);
      }
    }
  int n = 0;
  for (int i = 3; i < h - 3; i++)
    for (int j = 3; j < w - 3; j++) {
      if (!corner[(size_t)i * w + j]) continue;
      const int s = score[(size_t)i * w + j];
      int keep = 1;
      for (int di = -1; di <= 1 && keep; di++)
        for (int dj = -1; dj <= 1; dj++)
          if ((di || dj) && !(s > score[(size_t)(i + di) * w + j + dj])) { keep = 0; break; }
      if (!keep) continue;
      if (n < max_out) { ox[n] = (float)j; oy[n] = (float)i; oresp[n] = (float)s; }
      n++;
    }
  free(score);
  free(corner);
  return n;
}

/* The cell grid of one level, src/ORBextractor.cpp:903-990.  cells[4 c + 0..3] = iniX, iniY, hX,
 * hY of cell c = i * levelCols + j (hX = hY = 0: the reference skips it).  Returns the number of
 * cells (levelRows * levelCols), or -1 when the grid is degenerate (levelCols or levelRows < 1:
 * the reference divides by zero). */
int or_orb_cells(int rows, int cols, int n_desired, float image_ratio, int* cells, int max_cells) {
  const int EDGE = 19;
  const int levelCols = (int)sqrtf((float)n_desired / (5 * image_ratio));
  const int levelRows = (int)(image_ratio * levelCols);
  if (levelCols < 1 || levelRows < 1) return -1;
  const int minBorderX = EDGE, minBorderY = EDGE, maxBorderX = cols - EDGE, maxBorderY = rows - EDGE;
  const int W = maxBorderX - minBorderX, H = maxBorderY - minBorderY;
  const int cellW = (int)ceilf((float)W / levelCols), cellH = (int)ceilf((float)H / levelRows);
  const int nCells = levelRows * levelCols;
  if (nCells > max_cells) return -1;
  float hY = (float)(cellH + 6);
  for (int i = 0; i < levelRows; i++) {
    const float iniY = (float)(minBorderY + i * cellH - 3);
    int skip_row = 0;
    if (i == levelRows - 1) {
      hY = maxBorderY + 3 - iniY;
      if (hY <= 0) skip_row = 1;
    }
    float hX = (float)(cellW + 6);
    for (int j = 0; j < levelCols; j++) {
      const float iniX = (float)(minBorderX + j * cellW - 3);
      int* c = cells + 4 * (i * levelCols + j);
      c[0] = (int)iniX; c[1] = (int)iniY; c[2] = 0; c[3] = 0;
      if (skip_row) continue;
      if (j == levelCols - 1) {
        hX = maxBorderX + 3 - iniX;
        if (hX <= 0) continue;
      }
      c[2] = (int)hX; c[3] = (int)hY;
    }
  }
  return nCells;
}

/* Detection over every cell of every level: FAST(ini_th), re-run with min_th when <= 3 corners.
 * Keypoints in level coordinates (cell offset added), grouped by level then cell (row-major),
 * FAST's order within a cell.  cell_off[] gets, per level, levelRows*levelCols + 1 offsets
 * (concatenated over levels; level l starts at cell_base[l]).  Returns the keypoint count or -1. */
int or_orb_fast_cells(const lorb_image_pyramid* P, const int32_t* n_desired, int ini_th, int min_th, int max_kp,
                      float* x, float* y, float* resp, int max_cells, int32_t* cell_base, int32_t* cell_off) {
  const float ratio = (float)P->cols[0] / P->rows[0];
  int nk = 0, nc = 0;
  int* cells = (int*)malloc(sizeof(int) * 4 * (size_t)max_cells);
  for (int l = 0; l < P->n_levels; l++) {
    const int ncl = or_orb_cells(P->rows[l], P->cols[l], n_desired[l], ratio, cells, max_cells - nc);
    if (ncl < 0) { free(cells); return -1; }
    cell_base[l] = nc;
    for (int c = 0; c < ncl; c++) {
      cell_off[nc + c + l] = nk;
      const int* g = cells + 4 * c;
      if (g[2] <= 0 || g[3] <= 0) continue;
      const uint8_t* img = P->data + P->offset[l] + (int64_t)g[1] * P->step[l] + g[0];
      const int cap = max_kp - nk;
      int n = or_fast(img, g[2], g[3], P->step[l], ini_th, cap, x + nk, y + nk, resp + nk);
      if (n <= 3) n = or_fast(img, g[2], g[3], P->step[l], min_th, cap, x + nk, y + nk, resp + nk);
      if (n > cap) { free(cells); return -1; }
      for (int k = 0; k < n; k++) { x[nk + k] += (float)g[0]; y[nk + k] += (float)g[1]; }
      nk += n;
    }
    cell_off[nc + ncl + l] = nk;
    nc += ncl;
  }
  cell_base[P->n_levels] = nc;
  free(cells);
  return nk;
}

/* ---- retention (src/ORBextractor.cpp:984-1067) -------------------------------------------
 * KeyPointsFilter::retainBest (OpenCV 3.1) is std::nth_element + std::partition; the order they
 * leave equal responses in decides which keypoints the following resize() keeps, so libstdc++'s
 * algorithms (bits/stl_algo.h, stl_heap.h: introselect with median-of-3 pivots, heap_select past
 * the depth limit, insertion sort; the bidirectional partition) are restated here step for step. */
typedef struct { float x, y, size, resp; int octave; } or_kp;

static int kp_greater(const or_kp* a, const or_kp* b) { return a->resp > b->resp; }  /* KeypointResponseGreater */
static void kp_swap(or_kp* a, or_kp* b) { or_kp t = *a; *a = *b; *b = t; }

static void adjust_heap(or_kp* f, long hole, long len, or_kp value) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (kp_greater(&f[second], &f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  /* __push_heap */
  long parent = (hole - 1) / 2;
  while (hole > top && kp_greater(&f[parent], &value)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = value;
}
static void make_heap(or_kp* f, long len) {
  if (len < 2) return;
  long parent = (len - 2) / 2;
  while (1) {
    or_kp v = f[parent];
    adjust_heap(f, parent, len, v);
    if (parent == 0) return;
    parent--;
  }
}
static void heap_select(or_kp* f, long mid, long last) {
  make_heap(f, mid);
  for (long i = mid; i < last; ++i)
    if (kp_greater(&f[i], &f[0])) {  /* __pop_heap(first, middle, i) */
      or_kp v = f[i];
      f[i] = f[0];
      adjust_heap(f, 0, mid, v);
    }
}
static void move_median_to_first(or_kp* f, long r, long a, long b, long c) {
  if (kp_greater(&f[a], &f[b])) {
    if (kp_greater(&f[b], &f[c])) kp_swap(&f[r], &f[b]);
    else if (kp_greater(&f[a], &f[c])) kp_swap(&f[r], &f[c]);
    else kp_swap(&f[r], &f[a]);
  } else if (kp_greater(&f[a], &f[c])) kp_swap(&f[r], &f[a]);
  else if (kp_greater(&f[b], &f[c])) kp_swap(&f[r], &f[c]);
  else kp_swap(&f[r], &f[b]);
}
static long unguarded_partition(or_kp* f, long first, long last, long pivot) {
  while (1) {
    while (kp_greater(&f[first], &f[pivot])) ++first;
    --last;
    while (kp_greater(&f[pivot], &f[last])) --last;
    if (!(first < last)) return first;
    kp_swap(&f[first], &f[last]);
    ++first;
  }
}
static void insertion_sort(or_kp* f, long first, long last) {
  if (first == last) return;
  for (long i = first + 1; i != last; ++i) {
    if (kp_greater(&f[i], &f[first])) {
      or_kp v = f[i];
      memmove(&f[first + 1], &f[first], sizeof(or_kp) * (size_t)(i - first));
      f[first] = v;
    } else {
      or_kp v = f[i];
      long l = i, nx = i - 1;
      while (kp_greater(&v, &f[nx])) { f[l] = f[nx]; l = nx; --nx; }
      f[l] = v;
    }
  }
}
static int lg(long n) { int k = 0; while (n > 1) { n >>= 1; k++; } return k; }
static void nth_element(or_kp* f, long nth, long n) {
  if (n == 0 || nth == n) return;
  long first = 0, last = n;
  int depth = 2 * lg(n);
  while (last - first > 3) {
    if (depth == 0) {
      heap_select(f + first, nth + 1 - first, last - first);
      kp_swap(&f[first], &f[nth]);
      return;
    }
    --depth;
    const long mid = first + (last - first) / 2;
    move_median_to_first(f, first, first + 1, mid, last - 1);
    const long cut = unguarded_partition(f, first + 1, last, first);
    if (cut <= nth) first = cut; else last = cut;
  }
  insertion_sort(f, first, last);
}
/* std::partition (bidirectional) with pred = response >= value; returns the new end */
static long partition_ge(or_kp* f, long first, long last, float value) {
  while (1) {
    while (1) {
      if (first == last) return first;
      if (f[first].resp >= value) ++first; else break;
    }
    --last;
    while (1) {
      if (first == last) return first;
      if (!(f[last].resp >= value)) --last; else break;
    }
    kp_swap(&f[first], &f[last]);
    ++first;
  }
}
/* KeyPointsFilter::retainBest; returns the new size */
static long retain_best(or_kp* f, long n, long n_points) {
  if (n_points >= 0 && n > n_points) {
    if (n_points == 0) return 0;
    nth_element(f, n_points, n);
    const float amb = f[n_points - 1].resp;
    return partition_ge(f, n_points, n, amb);
  }
  return n;
}

/* Detection + retention of every level (src/ORBextractor.cpp:898-1067): FAST per cell (above),
 * the nToRetain distribution, retainBest + resize per cell, cell offsets added, octave and size,
 * and the level-wide retainBest when more than n_desired survive.  Outputs per keypoint x, y (level
 * coordinates), octave, size, response; level_off[n_levels + 1].  Returns the count or -1. */
int or_orb_detect(const lorb_image_pyramid* P, const int32_t* n_desired, const float* scale_factors, int ini_th,
                  int min_th, int max_kp, float* ox, float* oy, int32_t* ooct, float* osize, float* oresp,
                  int32_t* level_off) {
  const int max_cells = 1 << 16;
  int32_t* base = (int32_t*)malloc(sizeof(int32_t) * (P->n_levels + 1));
  int32_t* coff = (int32_t*)malloc(sizeof(int32_t) * (max_cells + P->n_levels + 1));
  const int cap = 1 << 22;
  float* fx = (float*)malloc(sizeof(float) * cap);
  float* fy = (float*)malloc(sizeof(float) * cap);
  float* fr = (float*)malloc(sizeof(float) * cap);
  int nk = or_orb_fast_cells(P, n_desired, ini_th, min_th, cap, fx, fy, fr, max_cells, base, coff);
  int out = 0, ok = nk >= 0;
  const float ratio = (float)P->cols[0] / P->rows[0];
  int* cells = (int*)malloc(sizeof(int) * 4 * (size_t)max_cells);
  for (int l = 0; ok && l < P->n_levels; l++) {
    level_off[l] = out;
    const int nd = n_desired[l];
    const int levelCols = (int)sqrtf((float)nd / (5 * ratio));
    const int levelRows = (int)(ratio * levelCols);
    const int nCells = levelRows * levelCols;
    or_orb_cells(P->rows[l], P->cols[l], nd, ratio, cells, max_cells);
    const int nfeaturesCell = (int)ceilf((float)nd / nCells);
    int* nToRetain = (int*)calloc((size_t)nCells, sizeof(int));
    int* nTotal = (int*)calloc((size_t)nCells, sizeof(int));
    char* bNoMore = (char*)calloc((size_t)nCells, 1);
    int nNoMore = 0, nToDistribute = 0;
    const int32_t* co = coff + base[l] + l;
    for (int c = 0; c < nCells; c++) {
      if (cells[4 * c + 2] <= 0 || cells[4 * c + 3] <= 0) continue;  /* skipped cell (:940, :960) */
      const int nKeys = co[c + 1] - co[c];
      nTotal[c] = nKeys;
      if (nKeys > nfeaturesCell) { nToRetain[c] = nfeaturesCell; bNoMore[c] = 0; }
      else { nToRetain[c] = nKeys; nToDistribute += nfeaturesCell - nKeys; bNoMore[c] = 1; nNoMore++; }
    }
    while (nToDistribute > 0 && nNoMore < nCells) {
      const int nNew = (int)(nfeaturesCell + ceilf((float)nToDistribute / (nCells - nNoMore)));
      nToDistribute = 0;
      for (int c = 0; c < nCells; c++)
        if (!bNoMore[c]) {
          if (nTotal[c] > nNew) { nToRetain[c] = nNew; bNoMore[c] = 0; }
          else { nToRetain[c] = nTotal[c]; nToDistribute += nNew - nTotal[c]; bNoMore[c] = 1; nNoMore++; }
        }
    }
    const int scaledPatchSize = (int)(31 * scale_factors[l]);
    or_kp* lv = (or_kp*)malloc(sizeof(or_kp) * (size_t)(co[nCells] - co[0] + 1));
    long nl = 0;
    for (int c = 0; c < nCells; c++) {
      or_kp* cell = lv + nl;
      long n = 0;
      for (int k = co[c]; k < co[c + 1]; k++) {  /* FAST order, cell coordinates restored below */
        cell[n].x = fx[k] - (float)cells[4 * c]; cell[n].y = fy[k] - (float)cells[4 * c + 1];
        cell[n].resp = fr[k]; cell[n].size = 7.f; cell[n].octave = 0; n++;
      }
      n = retain_best(cell, n, nToRetain[c]);
      if (n > nToRetain[c]) n = nToRetain[c];
      for (long k = 0; k < n; k++) {
        cell[k].x += (float)cells[4 * c]; cell[k].y += (float)cells[4 * c + 1];
        cell[k].octave = l; cell[k].size = (float)scaledPatchSize;
      }
      nl += n;
    }
    if (nl > nd) { nl = retain_best(lv, nl, nd); nl = nd < nl ? nd : nl; }
    for (long k = 0; k < nl && ok; k++) {
      if (out >= max_kp) { ok = 0; break; }
      ox[out] = lv[k].x; oy[out] = lv[k].y; ooct[out] = lv[k].octave; osize[out] = lv[k].size; oresp[out] = lv[k].resp;
      out++;
    }
    free(lv); free(nToRetain); free(nTotal); free(bNoMore);
  }
  level_off[P->n_levels] = out;
  free(cells); free(base); free(coff); free(fx); free(fy); free(fr);
  return ok ? out : -1;
}
