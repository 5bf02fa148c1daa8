/* tests/cpp/sanitize_oracle.c -- TEST INFRASTRUCTURE: drives the oracle entry points that the
 * host-layer test (test_adapters.cpp) does not reach, on small synthetic inputs, so that the
 * ASan+UBSan build (tests/test_sanitizers.py) covers all of oracle/*.c.  Exit 0 = clean run. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/lorb_oracle.h"

static unsigned long long s = 0x243F6A8885A308D3ull;
static unsigned rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (unsigned)(s >> 17); }
static float urand(float a, float b) { return a + (b - a) * (float)(rnd() & 0xffffff) / 16777216.0f; }

static int sum_ar(void* user, double* buf, int64_t n, int32_t op) {
  (void)user; (void)buf; (void)n; (void)op;  /* one rank: the all-reduce is the identity */
  return 0;
}

int main(void) {
  /* bf top-2 (+ threaded variant) */
  enum { NQ = 300, NT = 400 };
  uint8_t* q = malloc(NQ * 32), *t = malloc(NT * 32);
  int32_t lev[NT], bi[NQ], bd[NQ], bl[NQ], sd[NQ], sl[NQ], bi2[NQ], bd2[NQ], bl2[NQ], sd2[NQ], sl2[NQ];
  uint8_t acc[NQ], acc2[NQ];
  for (int i = 0; i < NQ * 32; i++) q[i] = (uint8_t)rnd();
  for (int i = 0; i < NT * 32; i++) t[i] = (uint8_t)rnd();
  for (int i = 0; i < NT; i++) lev[i] = (int32_t)(rnd() % 8);
  or_bf_top2(q, NQ, t, NT, lev, bi, bd, bl, sd, sl, acc);
  or_bf_top2_mt(q, NQ, t, NT, lev, bi2, bd2, bl2, sd2, sl2, acc2, 3);
  if (memcmp(bi, bi2, sizeof bi) || memcmp(acc, acc2, sizeof acc)) { puts("bf_top2_mt differs"); return 1; }

  /* unprojection */
  lorb_frame_params fp;
  memset(&fp, 0, sizeof fp);
  fp.fx = fp.fy = 435.2f; fp.cx = 367.5f; fp.cy = 252.2f; fp.bf = 47.9f;
  const float r[3] = {0.01f, -0.02f, 0.005f}, tt[3] = {0.1f, -0.05f, 0.2f};
  float T[16], X[3 * 64], xs[64], ys[64], ds[64];
  or_pose_to_Tcw(r, tt, T);
  for (int i = 0; i < 64; i++) { xs[i] = urand(0, 752); ys[i] = urand(0, 480); ds[i] = i % 5 ? urand(1, 20) : -1.0f; }
  or_unproject_stereo(&fp, T, 64, xs, ys, ds, X);

  /* point-partitioned local BA with one rank */
  enum { NK = 4, NP = 60 };
  float pose[6 * NK], fixed[6], pts[3 * NP], uv[2 * NP * (NK + 1)];
  int32_t op[NP * (NK + 1)], of[NP * (NK + 1)];
  int no = 0;
  memset(fixed, 0, sizeof fixed);
  for (int k = 0; k < NK; k++)
    for (int c = 0; c < 6; c++) pose[6 * k + c] = c == 3 ? 0.1f * (float)k : urand(-1e-3f, 1e-3f);
  for (int p = 0; p < NP; p++) {
    pts[3 * p] = urand(-3, 3); pts[3 * p + 1] = urand(-2, 2); pts[3 * p + 2] = urand(4, 12);
    for (int k = -1; k < NK; k++) {
      op[no] = p; of[no] = k;
      uv[2 * no] = fp.fx * pts[3 * p] / pts[3 * p + 2] + fp.cx + urand(-1, 1);
      uv[2 * no + 1] = fp.fy * pts[3 * p + 1] / pts[3 * p + 2] + fp.cy + urand(-1, 1);
      no++;
    }
  }
  lorb_ba_window w = {NK, 1, NP, no, fp.fx, fp.fy, fp.cx, fp.cy, pose, fixed, pts, op, of, uv};
  lorb_lm_options opt;
  or_lm_options_default(&opt);
  double po[6 * NK], pp[3 * NP], po2[6 * NK], pp2[3 * NP];
  double* a = po, *b = pp, *a2 = po2, *b2 = pp2;
  lorb_ba_summary sm, sm2;
  or_ba_local(1, &w, &opt, &a, &b, &sm);
  or_ba_local_sharded(1, &w, &opt, 0, sum_ar, NULL, &a2, &b2, &sm2);
  if (fabs(sm.final_cost - sm2.final_cost) > 1e-9 * fabs(sm.final_cost)) { puts("sharded BA differs"); return 1; }

  /* ORB descriptor stage: pyramid, blur, orientation, rBRIEF, FAST */
  enum { H = 120, W = 160 };
  uint8_t* img = malloc(H * W);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) img[y * W + x] = (uint8_t)(127 + 60 * sinf(x * 0.31f + y * 0.07f) + (float)(rnd() % 97) - 48);
  const float sf[4] = {1.0f, 1.2f, 1.44f, 1.728f};
  uint8_t* pyr = malloc(4 * H * W);
  lorb_image_pyramid P;
  memset(&P, 0, sizeof P);
  or_orb_pyramid(img, H, W, W, 4, sf, pyr, &P);
  P.data = pyr;
  int32_t pattern[1024];
  for (int i = 0; i < 1024; i++) pattern[i] = (int32_t)(rnd() % 26) - 13;
  float kx[40], ky[40], ang[40];
  int32_t kl[40];
  uint8_t desc[40 * 32];
  for (int i = 0; i < 40; i++) {
    kl[i] = i % 4;
    kx[i] = urand(20, (float)P.cols[kl[i]] - 21); ky[i] = urand(20, (float)P.rows[kl[i]] - 21);
  }
  or_orb_describe(&P, 40, kx, ky, kl, pattern, ang, desc);
  float fx_[4096], fy_[4096], fr_[4096];
  const int nf = or_fast(img, W, H, W, 20, 4096, fx_, fy_, fr_);
  if (nf < 0) { puts("fast failed"); return 1; }
  printf("sanitize_oracle ok (%d FAST corners)\n", nf);
  free(q); free(t); free(img); free(pyr);
  return 0;
}
