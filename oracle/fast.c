/*
 * fast.c -- TEST INFRASTRUCTURE ONLY (see lorb_oracle.h).  CPU restatement of the keypoint stage
 * of ORBextractor::operator() (src/ORBextractor.cpp:1087-1103), SURVEY §8f row 3:
 * ComputeKeyPointsOctTree (:799-897) -- per level, 30-pixel cells with a 6-pixel overlap inside
 * the EDGE_THRESHOLD-3 border, cv::FAST(cell, iniThFAST, true) re-run with minThFAST only when a
 * cell finds NO corner (:849-859) -- and DistributeOctTree (:554-797), the quadtree that keeps the
 * strongest keypoint of each node.  (The reference also holds ComputeKeyPointsOld, :899-1076; it is
 * dead code -- operator() calls ComputeKeyPointsOctTree, the Old call is commented out at :1103 --
 * and is not restated.)  cv::FAST is OpenCV 3.1's FAST_t<16> (9 contiguous of the 16-pixel circle
 * of radius 3, threshold_tab prefilter) with cornerScore<16> and 3x3 non-maximum suppression,
 * restated from its published source (features2d/src/fast.cpp, fast_score.cpp); OpenCV is absent
 * here, so FAST is cross-checked against an independent numpy restatement in tests/.
 *
 * Pointer-order model.  DistributeOctTree sorts vector<pair<int, ExtractorNode*>> (:717), so nodes
 * with equal key counts are ordered by the ADDRESS of their std::list element, which depends on the
 * allocator.  This restatement (and the device kernel) orders them by creation order (the n-th
 * node pushed into lNodes compares below every later one), i.e. the address order of a heap that
 * hands out increasing addresses; it is the same kind of convention as the std::set<MapPoint*>
 * iteration order the adapters take from the caller.
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


/* The cell grid of one level, src/ORBextractor.cpp:803-847.  cells[4 c + 0..3] = iniX, iniY, width,
 * height of cell c = i * nCols + j in level pixels (width = height = 0: the reference skips it,
 * :833-834, :843-844).  *ncols / *nrows = the grid; returns nRows * nCols, or -1 when the level is
 * too small for one 30-pixel cell (the reference divides by zero there). */
int or_orb_cells(int rows, int cols, int* cells, int max_cells, int* ncols, int* nrows) {
  const float W = 30;
  const int minBorderX = 19 - 3, minBorderY = minBorderX;  /* EDGE_THRESHOLD - 3 */
  const int maxBorderX = cols - 19 + 3, maxBorderY = rows - 19 + 3;
  const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
  const int nCols = (int)(width / W), nRows = (int)(height / W);
  if (nCols < 1 || nRows < 1 || nCols * nRows > max_cells) return -1;
  const int wCell = (int)ceilf(width / (float)nCols), hCell = (int)ceilf(height / (float)nRows);
  for (int i = 0; i < nRows; i++) {
    const float iniY = (float)(minBorderY + i * hCell);
    float maxY = iniY + (float)hCell + 6;
    const int skip_row = iniY >= (float)(maxBorderY - 3);
    if (maxY > (float)maxBorderY) maxY = (float)maxBorderY;
    for (int j = 0; j < nCols; j++) {
      const float iniX = (float)(minBorderX + j * wCell);
      float maxX = iniX + (float)wCell + 6;
      int* c = cells + 4 * (i * nCols + j);
      c[0] = (int)iniX; c[1] = (int)iniY; c[2] = 0; c[3] = 0;
      if (skip_row || iniX >= (float)(maxBorderX - 6)) continue;
      if (maxX > (float)maxBorderX) maxX = (float)maxBorderX;
      c[2] = (int)maxX - (int)iniX; c[3] = (int)maxY - (int)iniY;  /* rowRange / colRange */
    }
  }
  if (ncols) *ncols = nCols;
  if (nrows) *nrows = nRows;
  return nRows * nCols;
}

/* FAST over every cell of every level: FAST(ini_th), re-run with min_th when the cell found none.
 * Keypoints in level coordinates (cell offset added), grouped by level then cell (row-major),
 * FAST's order within a cell -- the order of vToDistributeKeys.  cell_off[] gets, per level,
 * nRows*nCols + 1 offsets (concatenated over levels; level l starts at cell_base[l] + l).
 * Returns the keypoint count, or -1 (degenerate level, capacity). */
int or_orb_fast_cells(const lorb_image_pyramid* P, int ini_th, int min_th, int max_kp, float* x, float* y,
                      float* resp, int max_cells, int32_t* cell_base, int32_t* cell_off) {
  int nk = 0, nc = 0;
  int* cells = (int*)malloc(sizeof(int) * 4 * (size_t)(max_cells > 0 ? max_cells : 1));
  for (int l = 0; l < P->n_levels; l++) {
    const int ncl = or_orb_cells(P->rows[l], P->cols[l], cells, max_cells - nc, NULL, NULL);
    if (ncl < 0) { free(cells); return -1; }
    cell_base[l] = nc;
    for (int c = 0; c < ncl; c++) {
      cell_off[nc + c + l] = nk;
      const int* g = cells + 4 * c;
      if (g[2] <= 0 || g[3] <= 0) continue;
      const uint8_t* img = P->data + P->offset[l] + (int64_t)g[1] * P->step[l] + g[0];
      const int cap = max_kp - nk;
      int n = or_fast(img, g[2], g[3], P->step[l], ini_th, cap, x + nk, y + nk, resp + nk);
      if (n == 0) n = or_fast(img, g[2], g[3], P->step[l], min_th, cap, x + nk, y + nk, resp + nk);
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

/* ---- DistributeOctTree, src/ORBextractor.cpp:496-797 ---------------------------------------
 * The list lNodes is a doubly linked list of node records; vKeys holds key indices in the order
 * the reference's vectors hold the keypoints.  UL / UR / BL / BR are always an axis-aligned box, so
 * a node keeps (x0, y0) = UL and (x1, y1) = BR. */
typedef struct oct_node {
  int x0, y0, x1, y1;
  int* keys;
  int n;
  int no_more;            /* bNoMore */
  long creation;          /* pointer-order model, see the file header */
  struct oct_node *prev, *next;
} oct_node;

typedef struct {
  oct_node *head, *tail;
  long size, created;
} oct_list;

static oct_node* oct_new(oct_list* L, int x0, int y0, int x1, int y1, int cap) {
  oct_node* n = (oct_node*)calloc(1, sizeof(oct_node));
  n->x0 = x0; n->y0 = y0; n->x1 = x1; n->y1 = y1;
  n->keys = (int*)malloc(sizeof(int) * (size_t)(cap > 0 ? cap : 1));
  n->creation = L->created++;
  return n;
}
static void oct_push_back(oct_list* L, oct_node* n) {
  n->prev = L->tail; n->next = NULL;
  if (L->tail) L->tail->next = n; else L->head = n;
  L->tail = n; L->size++;
}
static void oct_push_front(oct_list* L, oct_node* n) {
  n->next = L->head; n->prev = NULL;
  if (L->head) L->head->prev = n; else L->tail = n;
  L->head = n; L->size++;
}
static oct_node* oct_erase(oct_list* L, oct_node* n) {  /* returns the next element */
  oct_node* nx = n->next;
  if (n->prev) n->prev->next = n->next; else L->head = n->next;
  if (n->next) n->next->prev = n->prev; else L->tail = n->prev;
  L->size--;
  free(n->keys);
  free(n);
  return nx;
}

/* ExtractorNode::DivideNode (:496-552): the four children n1..n4 (returned in c[0..3], never
 * NULL), each key of the parent appended to the child whose box holds it, in parent order. */
static void oct_divide(oct_list* L, const oct_node* p, const float* kx, const float* ky, oct_node* c[4]) {
  const int halfX = (int)ceilf((float)(p->x1 - p->x0) / 2);
  const int halfY = (int)ceilf((float)(p->y1 - p->y0) / 2);
  const int mx = p->x0 + halfX, my = p->y0 + halfY;
  c[0] = oct_new(L, p->x0, p->y0, mx, my, p->n);
  c[1] = oct_new(L, mx, p->y0, p->x1, my, p->n);
  c[2] = oct_new(L, p->x0, my, mx, p->y1, p->n);
  c[3] = oct_new(L, mx, my, p->x1, p->y1, p->n);
  for (int i = 0; i < p->n; i++) {
    const int k = p->keys[i];
    oct_node* d;
    if (kx[k] < (float)mx) d = ky[k] < (float)my ? c[0] : c[2];
    else d = ky[k] < (float)my ? c[1] : c[3];
    d->keys[d->n++] = k;
  }
  for (int q = 0; q < 4; q++) c[q]->no_more = c[q]->n == 1;
}

typedef struct { int size; long creation; oct_node* node; } oct_pair;
static int oct_pair_cmp(const void* a, const void* b) {  /* std::pair operator<, pointers as creation */
  const oct_pair* p = (const oct_pair*)a;
  const oct_pair* q = (const oct_pair*)b;
  if (p->size != q->size) return p->size < q->size ? -1 : 1;
  return (p->creation > q->creation) - (p->creation < q->creation);
}

/* push the non-empty children to the front (n1 first, so the list reads n4 n3 n2 n1 ...), record
 * the ones holding more than one key in (pairs, *np); returns how many were recorded */
static int oct_push_children(oct_list* L, oct_node* c[4], oct_pair* pairs, long* np) {
  int rec = 0;
  for (int q = 0; q < 4; q++) {
    if (c[q]->n > 0) {
      oct_push_front(L, c[q]);
      if (c[q]->n > 1) {
        pairs[(*np)++] = (oct_pair){c[q]->n, c[q]->creation, c[q]};
        rec++;
      }
    } else {
      free(c[q]->keys);
      free(c[q]);
    }
  }
  return rec;
}

/* kx, ky: key coordinates relative to (minX, minY); resp: responses; n keys in vToDistributeKeys
 * order.  Writes the kept key indices in lNodes order to out (capacity >= n) and returns their
 * count, or -1 when the level is degenerate (nIni < 1). */
int or_distribute_octree(const float* kx, const float* ky, const float* resp, int n, int minX, int maxX, int minY,
                         int maxY, int N, int32_t* out) {
  const int nIni = (int)roundf((float)(maxX - minX) / (float)(maxY - minY));
  if (nIni < 1) return -1;
  const float hX = (float)(maxX - minX) / (float)nIni;
  oct_list L = {NULL, NULL, 0, 0};
  oct_node** ini = (oct_node**)malloc(sizeof(oct_node*) * (size_t)nIni);
  for (int i = 0; i < nIni; i++) {  /* :575-586 */
    const int ulx = (int)(hX * (float)i), urx = (int)(hX * (float)(i + 1));
    ini[i] = oct_new(&L, ulx, 0, urx, maxY - minY, n);
    oct_push_back(&L, ini[i]);
  }
  for (int i = 0; i < n; i++) {  /* :590-594 */
    oct_node* d = ini[(size_t)(kx[i] / hX)];
    d->keys[d->n++] = i;
  }
  free(ini);
  for (oct_node* it = L.head; it;) {  /* :596-609 */
    if (it->n == 1) { it->no_more = 1; it = it->next; }
    else if (it->n == 0) it = oct_erase(&L, it);
    else it = it->next;
  }
  long cap_pairs = 4 * (long)(n + 4), npairs = 0, nprev = 0;
  oct_pair* pairs = (oct_pair*)malloc(sizeof(oct_pair) * (size_t)cap_pairs);
  oct_pair* prevp = (oct_pair*)malloc(sizeof(oct_pair) * (size_t)cap_pairs);
  int finish = 0;
  while (!finish) {  /* :619-772 */
    long prevSize = L.size;
    int nToExpand = 0;
    npairs = 0;
    for (oct_node* it = L.head; it;) {
      if (it->no_more) { it = it->next; continue; }
      oct_node* c[4];
      oct_divide(&L, it, kx, ky, c);
      nToExpand += oct_push_children(&L, c, pairs, &npairs);
      it = oct_erase(&L, it);
    }
    if (L.size >= N || L.size == prevSize) {
      finish = 1;
    } else if (L.size + nToExpand * 3 > N) {
      while (!finish) {  /* :709-770 */
        prevSize = L.size;
        memcpy(prevp, pairs, sizeof(oct_pair) * (size_t)npairs);
        nprev = npairs;
        npairs = 0;
        qsort(prevp, (size_t)nprev, sizeof(oct_pair), oct_pair_cmp);
        for (long j = nprev - 1; j >= 0; j--) {
          oct_node* c[4];
          oct_divide(&L, prevp[j].node, kx, ky, c);
          oct_push_children(&L, c, pairs, &npairs);
          oct_erase(&L, prevp[j].node);
          if (L.size >= N) break;
        }
        if (L.size >= N || L.size == prevSize) finish = 1;
      }
    }
  }
  int m = 0;
  for (oct_node* it = L.head; it; it = it->next) {  /* :776-794 */
    int best = it->keys[0];
    float maxResponse = resp[best];
    for (int k = 1; k < it->n; k++)
      if (resp[it->keys[k]] > maxResponse) { best = it->keys[k]; maxResponse = resp[best]; }
    out[m++] = best;
  }
  while (L.head) oct_erase(&L, L.head);
  free(pairs);
  free(prevp);
  return m;
}

/* ComputeKeyPointsOctTree without the orientation (:799-892): FAST cells, DistributeOctTree per
 * level with mnFeaturesPerLevel[l] = n_desired[l], then the border offset, octave and size
 * (PATCH_SIZE * mvScaleFactor[l], truncated to int, :881).  Per keypoint x, y (level coordinates),
 * octave, size, response; level_off[n_levels + 1].  Returns the count or -1. */
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
  int32_t* kept = (int32_t*)malloc(sizeof(int32_t) * cap);
  const int nk = or_orb_fast_cells(P, ini_th, min_th, cap, fx, fy, fr, max_cells, base, coff);
  int out = 0, ok = nk >= 0;
  for (int l = 0; ok && l < P->n_levels; l++) {
    level_off[l] = out;
    const int minBorderX = 16, minBorderY = 16, maxBorderX = P->cols[l] - 16, maxBorderY = P->rows[l] - 16;
    const int k0 = coff[base[l] + l], k1 = coff[base[l + 1] + l];
    for (int k = k0; k < k1; k++) { fx[k] -= (float)minBorderX; fy[k] -= (float)minBorderY; }
    const int m = or_distribute_octree(fx + k0, fy + k0, fr + k0, k1 - k0, minBorderX, maxBorderX, minBorderY,
                                       maxBorderY, n_desired[l], kept);
    if (m < 0) { ok = 0; break; }
    const int scaledPatchSize = (int)(31 * scale_factors[l]);
    for (int q = 0; q < m; q++) {
      if (out >= max_kp) { ok = 0; break; }
      const int k = k0 + kept[q];
      ox[out] = fx[k] + (float)minBorderX; oy[out] = fy[k] + (float)minBorderY;
      ooct[out] = l; osize[out] = (float)scaledPatchSize; oresp[out] = fr[k];
      out++;
    }
  }
  level_off[P->n_levels] = out;
  free(base); free(coff); free(fx); free(fy); free(fr); free(kept);
  return ok ? out : -1;
}
