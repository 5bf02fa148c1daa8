// tests/cpp/test_adapters.cpp -- the C++ host layer (include/lorb/adapters.hpp,
// local_mapping.hpp) driven exactly like the reference's VisualOdometry drives Matcher / BA /
// LocalMapping, with plain test frames standing in for Simple_ORB_SLAM::Frame/MapPoint.  Every
// GPU result is checked against the oracle (test infrastructure, linked only here).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <thread>
#include <vector>

#include "../../include/lorb/adapters.hpp"
#include "../../include/lorb/local_mapping.hpp"
#include "../../oracle/lorb_oracle.h"

struct MiniFrame;
struct MiniPoint {
  float pos[3];
  uint8_t desc[32];
  size_t nobs = 0;
  bool bad = false;
  bool in_view = false;
  float proj[4] = {0, 0, 0, 0};  // x, y, xr, viewcos
  int level = 0;
  std::map<MiniFrame*, size_t> obs;
  size_t first_id = 0;
  float normal[3] = {0, 0, 1};
  float maxd = 0, mind = 0;
  size_t last_seen = 0;
  int visible = 0;
};
struct MiniFrame {
  size_t id = 0;
  std::vector<float> x, y, angle, uR;
  // stereo side: raw left keypoints = (x, y, octave); right keypoints + pyramids
  std::vector<float> rx, ry, depth;
  std::vector<int> roct;
  std::vector<uint8_t> rdesc;
  std::vector<std::vector<uint8_t>> pyr[2];
  std::vector<int> prows, pcols;
  std::vector<int> octave;
  std::vector<uint8_t> desc;
  std::vector<MiniPoint*> mps;
  std::vector<bool> outlier;
  float Tcw[16];
  float rvec[3] = {0, 0, 0}, tvec[3] = {0, 0, 0};
  lorb_frame_params fp;
  std::vector<MiniFrame*> covis;
  bool bad = false;
};
struct MiniMap {
  std::vector<MiniFrame*> frames;
};

namespace lorb {
template <> struct FrameTraits<MiniFrame> {
  using point_type = MiniPoint;
  static size_t num_keypoints(MiniFrame* f) { return f->x.size(); }
  static void keypoint(MiniFrame* f, size_t i, float* x, float* y, int* o, float* a) {
    *x = f->x[i]; *y = f->y[i]; *o = f->octave[i]; *a = f->angle[i];
  }
  static void descriptor(MiniFrame* f, size_t i, uint8_t* d) { memcpy(d, &f->desc[32 * i], 32); }
  static bool has_right(MiniFrame* f) { return !f->uR.empty(); }
  static float u_right(MiniFrame* f, size_t i) { return f->uR[i]; }
  static MiniPoint* map_point(MiniFrame* f, size_t i) { return f->mps[i]; }
  static void set_map_point(MiniFrame* f, size_t i, MiniPoint* p) { f->mps[i] = p; }
  static bool outlier(MiniFrame* f, size_t i) { return f->outlier[i]; }
  static void params(MiniFrame* f, lorb_frame_params* fp) { *fp = f->fp; }
  static void Tcw(MiniFrame* f, float* T) { memcpy(T, f->Tcw, sizeof(f->Tcw)); }
  static void pose_vectors(MiniFrame* f, float* r, float* t) { memcpy(r, f->rvec, 12); memcpy(t, f->tvec, 12); }
  static void set_pose(MiniFrame* f, const float* t, const float* r) {
    memcpy(f->rvec, r, 12); memcpy(f->tvec, t, 12);
    lorb_pose_to_Tcw(r, t, f->Tcw);
  }
  static std::vector<MiniFrame*> covisible_frames(MiniFrame* f) { return f->covis; }
  static bool is_bad(MiniFrame* f) { return f->bad; }
  static size_t id(MiniFrame* f) { return f->id; }
  static void update_connections(MiniFrame*) {}
  static void map_add_frame(MiniMap* m, MiniFrame* f) { m->frames.push_back(f); }
  static void raw_keypoint(MiniFrame* f, size_t i, float* x, float* y, int* o) { *x = f->x[i]; *y = f->y[i]; *o = f->octave[i]; }
  static size_t num_right_keypoints(MiniFrame* f) { return f->rx.size(); }
  static void right_keypoint(MiniFrame* f, size_t i, float* x, float* y, int* o) { *x = f->rx[i]; *y = f->ry[i]; *o = f->roct[i]; }
  static void right_descriptor(MiniFrame* f, size_t i, uint8_t* d) { memcpy(d, &f->rdesc[32 * i], 32); }
  static int num_levels(MiniFrame* f) { return (int)f->prows.size(); }
  static void pyramid_level(MiniFrame* f, int side, int l, const uint8_t** d, int* rows, int* cols, int* step) {
    *d = f->pyr[side][l].data(); *rows = f->prows[l]; *cols = f->pcols[l]; *step = f->pcols[l];
  }
  static void set_stereo(MiniFrame* f, const float* uR, const float* depth, size_t n) {
    f->uR.assign(uR, uR + n); f->depth.assign(depth, depth + n);
  }
};
template <> struct PointTraits<MiniPoint> {
  static size_t num_obs(MiniPoint* p) { return p->nobs; }
  static void descriptor(MiniPoint* p, uint8_t* d) { memcpy(d, p->desc, 32); }
  static void pos(MiniPoint* p, float* X) { memcpy(X, p->pos, 12); }
  static void set_pos(MiniPoint* p, const float* X) { memcpy(p->pos, X, 12); }
  static bool is_bad(MiniPoint* p) { return p->bad; }
  static bool track_in_view(MiniPoint* p) { return p->in_view; }
  static void tracking(MiniPoint* p, float* t, int* l) { memcpy(t, p->proj, 16); *l = p->level; }
  static std::map<MiniFrame*, size_t> observations(MiniPoint* p) { return p->obs; }
  static bool is_in_frame(MiniPoint* p, MiniFrame* f) { return p->obs.count(f) > 0; }
  static void add_observation(MiniPoint* p, MiniFrame* f, size_t i) {
    if (p->obs.count(f)) return;
    p->obs[f] = i; p->nobs++;
  }
  static float found_ratio(MiniPoint*) { return 1.0f; }
  static void set_descriptor(MiniPoint* p, const uint8_t* d) { memcpy(p->desc, d, 32); }
  static void normal(MiniPoint* p, float* n) { memcpy(n, p->normal, 12); }
  static void distances(MiniPoint* p, float* mx, float* mn) { *mx = p->maxd; *mn = p->mind; }
  static size_t last_frame_seen(MiniPoint* p) { return p->last_seen; }
  static void set_tracking(MiniPoint* p, bool in_view, const float* t, int level) {
    p->in_view = in_view;
    if (in_view) { memcpy(p->proj, t, 16); p->level = level; }
  }
  static void increase_visible(MiniPoint* p) { p->visible++; }
  static void set_bad(MiniPoint* p) { p->bad = true; }
  static size_t first_frame_id(MiniPoint* p) { return p->first_id; }
};
}  // namespace lorb

static uint64_t s_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() { s_rng ^= s_rng << 13; s_rng ^= s_rng >> 7; s_rng ^= s_rng << 17; return (uint32_t)(s_rng >> 11); }
static float urand(float a, float b) { return a + (b - a) * (float)(rnd() & 0xffffff) / 16777216.0f; }

static lorb_frame_params make_fp() {
  lorb_frame_params fp;
  memset(&fp, 0, sizeof(fp));
  fp.fx = fp.fy = 435.2f; fp.cx = 367.5f; fp.cy = 252.2f; fp.bf = 47.9f; fp.b = fp.bf / fp.fx;
  fp.min_x = 0; fp.max_x = 752; fp.min_y = 0; fp.max_y = 480;
  fp.grid_w_inv = 64.0f / 752.0f; fp.grid_h_inv = 48.0f / 480.0f;
  fp.n_levels = 8; fp.log_scale_factor = logf(1.2f);
  float s = 1.0f;
  for (int i = 0; i < 8; i++) { fp.scale_factors[i] = s; s *= 1.2f; }
  return fp;
}

static void project(const float* T, const float* X, const lorb_frame_params& fp, float* u, float* v) {
  float Xc[3];
  for (int r = 0; r < 3; r++) Xc[r] = T[4 * r] * X[0] + T[4 * r + 1] * X[1] + T[4 * r + 2] * X[2] + T[4 * r + 3];
  *u = fp.fx * Xc[0] / Xc[2] + fp.cx;
  *v = fp.fy * Xc[1] / Xc[2] + fp.cy;
}

static MiniFrame* make_frame(size_t id, int n, const float r[3], const float t[3]) {
  MiniFrame* f = new MiniFrame();
  f->id = id;
  f->fp = make_fp();
  memcpy(f->rvec, r, 12); memcpy(f->tvec, t, 12);
  lorb_pose_to_Tcw(r, t, f->Tcw);
  for (int i = 0; i < n; i++) {
    f->x.push_back(urand(0, 752)); f->y.push_back(urand(0, 480));
    f->angle.push_back(urand(0, 360)); f->octave.push_back((int)(rnd() % 8) < 4 ? 0 : (int)(rnd() % 8));
    f->uR.push_back(rnd() % 3 == 0 ? f->x.back() - urand(3, 20) : -1.0f);
    for (int b = 0; b < 32; b++) f->desc.push_back((uint8_t)rnd());
  }
  f->mps.assign(n, nullptr);
  f->outlier.assign(n, false);
  return f;
}

static int g_fail = 0;
#define EXPECT(c, ...) do { if (!(c)) { printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); g_fail++; } } while (0)

int main() {
  lorb_ctx* ctx = lorb::thread_ctx(0);
  const int N = 800;
  const float r0[3] = {0, 0, 0}, t0[3] = {0, 0, 0};
  const float r1[3] = {0.01f, -0.005f, 0.002f}, t1[3] = {0.05f, 0.0f, 0.02f};
  MiniFrame* last = make_frame(1, N, r0, t0);
  // map points in the last frame, re-observed in the current one
  std::vector<MiniPoint*> pts;
  for (int i = 0; i < N; i++) {
    if (rnd() % 2) continue;
    MiniPoint* p = new MiniPoint();
    p->pos[0] = urand(-5, 5); p->pos[1] = urand(-3, 3); p->pos[2] = urand(2, 10);
    memcpy(p->desc, &last->desc[32 * i], 32);
    p->nobs = rnd() % 2;
    p->obs[last] = (size_t)i;
    last->mps[i] = p;
    float u, v;
    project(last->Tcw, p->pos, last->fp, &u, &v);
    last->x[i] = u; last->y[i] = v;
    pts.push_back(p);
  }
  MiniFrame* cur = make_frame(2, N, r1, t1);
  int k = 0;
  for (MiniPoint* p : pts) {
    float u, v;
    project(cur->Tcw, p->pos, cur->fp, &u, &v);
    if (u < 0 || u >= 752 || v < 0 || v >= 480 || k >= N) continue;
    cur->x[k] = u + urand(-0.5f, 0.5f); cur->y[k] = v + urand(-0.5f, 0.5f);
    memcpy(&cur->desc[32 * k], p->desc, 32);
    cur->desc[32 * k + (rnd() % 32)] ^= (uint8_t)(1u << (rnd() % 8));
    k++;
  }

  // ---- Matcher::SearchByProjection(curr, last, 15): adapter (GPU) vs oracle -------------
  {
    lorb::KeypointsSoA ks = lorb::gather_keypoints(cur);
    lorb_keypoints kv = ks.view();
    std::vector<uint8_t> st = lorb::gather_slot_state(cur);
    const size_t nl = last->x.size();
    std::vector<uint8_t> has(nl), out(nl, 0), lk(nl), ld(32 * nl);
    std::vector<float> pos(3 * nl), ang(last->angle);
    std::vector<int32_t> oct(last->octave.begin(), last->octave.end());
    for (size_t i = 0; i < nl; i++) {
      MiniPoint* p = last->mps[i];
      has[i] = p != nullptr;
      if (!p) continue;
      lk[i] = p->nobs > 0;
      memcpy(&pos[3 * i], p->pos, 12);
      memcpy(&ld[32 * i], p->desc, 32);
    }
    lorb_last_frame L{(int32_t)nl, last->Tcw, has.data(), out.data(), lk.data(), pos.data(), ld.data(), oct.data(), ang.data()};
    std::vector<int32_t> assign(N);
    int32_t nm_o = 0;
    or_search_by_projection_frame(&cur->fp, cur->Tcw, &kv, st.data(), &L, 15.0f, assign.data(), &nm_o);
    const size_t nm_g = lorb::SearchByProjectionFrame(ctx, cur, last, 15.0f);
    EXPECT((int)nm_g == nm_o, "frame match count gpu %zu oracle %d", nm_g, nm_o);
    int mism = 0;
    for (int j = 0; j < N; j++) {
      MiniPoint* want = assign[j] >= 0 ? last->mps[assign[j]] : nullptr;
      if (cur->mps[j] != want) mism++;
    }
    EXPECT(mism == 0, "frame match: %d slot mismatches", mism);
    printf("SearchByProjection(frame): %zu matches\n", nm_g);
  }

  // ---- BA::ProjectPoseOptimization(curr) -------------------------------------------------
  {
    std::vector<float> P3, P2;
    for (int j = 0; j < N; j++)
      if (cur->mps[j]) { P3.insert(P3.end(), cur->mps[j]->pos, cur->mps[j]->pos + 3); P2.push_back(cur->x[j]); P2.push_back(cur->y[j]); }
    float pinit[6] = {0, 0, 0, 0, 0, 0};  // the caller's initial pose (prev pose * motion model)
    memcpy(cur->rvec, pinit, 12); memcpy(cur->tvec, pinit + 3, 12);
    const float intr[4] = {cur->fp.fx, cur->fp.fx, cur->fp.cx, cur->fp.cy};
    const int32_t ro[2] = {0, (int32_t)(P2.size() / 2)};
    lorb_pose_problem_batch b{1, ro, intr, pinit, P3.data(), P2.data()};
    lorb_lm_options opt;
    lorb_lm_options_default(&opt);
    double po[6];
    float To[16];
    or_ba_pose_only(&b, &opt, po, To, nullptr);
    lorb::ProjectPoseOptimization(ctx, cur);
    double md = 0;
    for (int i = 0; i < 3; i++) {
      md = std::max(md, (double)fabsf(cur->rvec[i] - (float)po[i]) / std::max(1.0, fabs(po[i])));
      md = std::max(md, (double)fabsf(cur->tvec[i] - (float)po[3 + i]) / std::max(1.0, fabs(po[3 + i])));
    }
    EXPECT(md <= 1e-5, "pose-only BA rel diff %g", md);
    printf("ProjectPoseOptimization: t = %.5f %.5f %.5f (max rel diff %.2e)\n", cur->tvec[0], cur->tvec[1], cur->tvec[2], md);
  }

  // ---- LocalMapping: queue processed by the mapper thread, reference wiring --------------
  {
    MiniMap map;
    lorb::LocalMapping<MiniFrame, MiniMap> lm(&map);
    std::thread th([&] { lm.Run(); });
    lm.InsertKeyFrame(last);
    lm.InsertKeyFrame(cur);
    for (int i = 0; i < 2000 && lm.processed() < 2; i++) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    lm.RequestFinish();
    th.join();
    EXPECT(map.frames.size() == 2 && map.frames[0] == last && map.frames[1] == cur, "LocalMapping queue order");
    printf("LocalMapping: processed %zu keyframes\n", lm.processed());
  }

  // ---- BA::LocalPoseOptimization(curr) through the covisibility window --------------------
  {
    // every point observed by both frames; last is fixed (not covisible => MPCost)
    for (int j = 0; j < N; j++) {
      MiniPoint* p = cur->mps[j];
      if (p && !p->obs.count(cur)) { p->obs[cur] = (size_t)j; p->nobs++; }
    }
    cur->covis.clear();
    // oracle: gather the same window by hand
    std::vector<MiniPoint*> wp;
    std::set<MiniPoint*> seen;
    for (int j = 0; j < N; j++)
      if (cur->mps[j] && seen.insert(cur->mps[j]).second) wp.push_back(cur->mps[j]);
    std::vector<float> pi(cur->rvec, cur->rvec + 3), fx(last->rvec, last->rvec + 3), X, uv;
    pi.insert(pi.end(), cur->tvec, cur->tvec + 3);
    fx.insert(fx.end(), last->tvec, last->tvec + 3);
    std::vector<int32_t> op, of;
    for (size_t q = 0; q < wp.size(); q++) {
      X.insert(X.end(), wp[q]->pos, wp[q]->pos + 3);
      for (auto& ob : wp[q]->obs) {
        op.push_back((int32_t)q);
        of.push_back(ob.first == cur ? 0 : -1);
        uv.push_back(ob.first->x[ob.second]); uv.push_back(ob.first->y[ob.second]);
      }
    }
    lorb_ba_window w{1, 1, (int32_t)wp.size(), (int32_t)op.size(), cur->fp.fx, cur->fp.fy, cur->fp.cx, cur->fp.cy,
                     pi.data(), fx.data(), X.data(), op.data(), of.data(), uv.data()};
    lorb_lm_options opt;
    lorb_lm_options_default(&opt);
    std::vector<double> po(6), ppt(3 * wp.size());
    double* a = po.data();
    double* bpt = ppt.data();
    or_ba_local(1, &w, &opt, &a, &bpt, nullptr);
    lorb::LocalPoseOptimization(ctx, cur);
    double md = 0;
    for (size_t q = 0; q < wp.size(); q++)
      for (int i = 0; i < 3; i++)
        md = std::max(md, fabs((double)wp[q]->pos[i] - (double)(float)ppt[3 * q + i]) / std::max(1.0, fabs(ppt[3 * q + i])));
    EXPECT(md <= 1e-5, "local BA point rel diff %g", md);
    printf("LocalPoseOptimization: %zu points, %zu obs (max rel diff %.2e)\n", wp.size(), op.size(), md);
  }

  // ---- BA::LocalPoseOptimization at C4 size, twice ---------------------
  // 50 window keyframes (cur + 49 covisible, in the reference's ascending-weight order,
  // src/bundle_adjust.cpp:210-220 / src/frame.cpp:754-774) + 5 older fixed keyframes, 10,000
  // points on 7-8 consecutive keyframes.  The adapter runs on the thread's resident solver; the
  // second call (the window after the first call's float write-back) reuses the plan.
  {
#ifdef LORB_LOOPBACK  // sanitizer builds (the oracle behind the ABI): the same gather at a smaller size
    const int NW = 12, NFX = 3, NP = 1500;
#else
    const int NW = 50, NFX = 5, NP = 10000;
#endif
    std::vector<MiniFrame*> kf(NFX + NW);
    std::vector<float> tr(6 * (NFX + NW));
    for (int i = 0; i < NFX + NW; i++) {
      const float r[3] = {0.0f, 0.01f * i, 0.0f}, t[3] = {-0.1f * i, 0.0f, 0.0f};
      memcpy(&tr[6 * i], r, 12); memcpy(&tr[6 * i + 3], t, 12);
      kf[i] = new MiniFrame();
      kf[i]->id = 100 + i;
      kf[i]->fp = make_fp();
      memcpy(kf[i]->rvec, r, 12); memcpy(kf[i]->tvec, t, 12);
      lorb_pose_to_Tcw(r, t, kf[i]->Tcw);
    }
    auto observe = [&](MiniPoint* p, MiniFrame* f, const float* Xtrue) {
      float u, v;
      project(f->Tcw, Xtrue, f->fp, &u, &v);
      p->obs[f] = f->x.size();
      f->x.push_back(u + urand(-0.8f, 0.8f)); f->y.push_back(v + urand(-0.8f, 0.8f));
      f->octave.push_back(0); f->angle.push_back(0.0f);
      f->mps.push_back(p); f->outlier.push_back(false);
      p->nobs++;
    };
    std::vector<MiniPoint*> cpts;
    for (int q = 0; q < NP; q++) {
      MiniPoint* p = new MiniPoint();
      const int len = 7 + (int)(rnd() % 2), s = (int)(rnd() % (NW - len + 1));
      // in front of the keyframe in the middle of its range, inside its image (X = R^T (pc - t))
      float X[3];
      {
        const MiniFrame* fm = kf[NFX + s + len / 2];
        const float z = urand(4, 20), u = urand(60, 692), v = urand(60, 420);
        const float pc[3] = {(u - fm->fp.cx) / fm->fp.fx * z - fm->Tcw[3], (v - fm->fp.cy) / fm->fp.fy * z - fm->Tcw[7],
                             z - fm->Tcw[11]};
        for (int c = 0; c < 3; c++) X[c] = fm->Tcw[c] * pc[0] + fm->Tcw[4 + c] * pc[1] + fm->Tcw[8 + c] * pc[2];
      }
      for (int j = s; j < s + len; j++) observe(p, kf[NFX + j], X);
      if (s < 6) {  // the older points are also seen by two of the fixed keyframes (MPCost): the gauge
        const int a = (int)(rnd() % NFX), b = (a + 1 + (int)(rnd() % (NFX - 1))) % NFX;
        observe(p, kf[std::min(a, b)], X);
        observe(p, kf[std::max(a, b)], X);
      }
      for (int c = 0; c < 3; c++) p->pos[c] = X[c] + urand(-0.05f, 0.05f);
      cpts.push_back(p);
    }
    for (int i = NFX; i < NFX + NW; i++) {  // perturbed window poses
      for (int c = 0; c < 3; c++) { kf[i]->rvec[c] += urand(-2e-3f, 2e-3f); kf[i]->tvec[c] += urand(-2e-2f, 2e-2f); }
      lorb_pose_to_Tcw(kf[i]->rvec, kf[i]->tvec, kf[i]->Tcw);
    }
    MiniFrame* c4 = kf[NFX + NW - 1];
    {  // GetCovisibleFrames: the other window keyframes by ascending shared-point weight
      std::map<MiniFrame*, int> wgt;
      for (MiniPoint* p : cpts)
        if (p->obs.count(c4))
          for (auto& ob : p->obs)
            if (ob.first != c4) wgt[ob.first]++;
      std::vector<std::pair<int, MiniFrame*>> v;
      for (int i = NFX; i < NFX + NW - 1; i++) v.push_back({wgt.count(kf[i]) ? wgt[kf[i]] : 0, kf[i]});
      std::stable_sort(v.begin(), v.end(), [](const std::pair<int, MiniFrame*>& a, const std::pair<int, MiniFrame*>& b) { return a.first < b.first; });
      for (auto& e : v) c4->covis.push_back(e.second);
    }
    lorb_lm_options opt;
    lorb_lm_options_default(&opt);
    for (int call = 0; call < 2; call++) {
      // the window as src/bundle_adjust.cpp:207-330 gathers it: [cur] + covisible, points in
      // first-seen order, each point's observations in std::map<Frame*, size_t> order
      std::vector<MiniFrame*> fr{c4};
      for (MiniFrame* f : c4->covis) fr.push_back(f);
      std::map<MiniFrame*, int> fidx, xidx;
      for (size_t i = 0; i < fr.size(); i++) fidx[fr[i]] = (int)i;
      std::vector<MiniPoint*> wp;
      std::set<MiniPoint*> seen;
      for (MiniFrame* f : fr)
        for (MiniPoint* p : f->mps)
          if (p && seen.insert(p).second) wp.push_back(p);
      std::vector<float> pi, fx, X, uv;
      for (MiniFrame* f : fr) { pi.insert(pi.end(), f->rvec, f->rvec + 3); pi.insert(pi.end(), f->tvec, f->tvec + 3); }
      std::vector<int32_t> op, of;
      for (size_t q = 0; q < wp.size(); q++) {
        X.insert(X.end(), wp[q]->pos, wp[q]->pos + 3);
        for (auto& ob : wp[q]->obs) {
          int code;
          if (fidx.count(ob.first)) {
            code = fidx[ob.first];
          } else {
            if (!xidx.count(ob.first)) {
              const int j = (int)xidx.size();
              xidx[ob.first] = j;
              fx.insert(fx.end(), ob.first->rvec, ob.first->rvec + 3); fx.insert(fx.end(), ob.first->tvec, ob.first->tvec + 3);
            }
            code = -1 - xidx[ob.first];
          }
          op.push_back((int32_t)q); of.push_back(code);
          uv.push_back(ob.first->x[ob.second]); uv.push_back(ob.first->y[ob.second]);
        }
      }
      lorb_ba_window w{(int32_t)fr.size(), (int32_t)xidx.size(), (int32_t)wp.size(), (int32_t)op.size(), c4->fp.fx,
                       c4->fp.fy, c4->fp.cx, c4->fp.cy, pi.data(), fx.data(), X.data(), op.data(), of.data(), uv.data()};
      std::vector<double> po(6 * fr.size()), ppt(3 * wp.size());
      double* a = po.data();
      double* bpt = ppt.data();
      lorb_ba_summary so;
      or_ba_local(1, &w, &opt, &a, &bpt, &so);
      lorb::LocalPoseOptimization(ctx, c4);
      double md = 0;
      for (size_t q = 0; q < wp.size(); q++)
        for (int i = 0; i < 3; i++)
          md = std::max(md, fabs((double)wp[q]->pos[i] - (double)(float)ppt[3 * q + i]) / std::max(1.0, fabs(ppt[3 * q + i])));
      for (size_t f = 0; f < fr.size(); f++)
        for (int i = 0; i < 3; i++) {
          md = std::max(md, fabs((double)fr[f]->rvec[i] - (double)(float)po[6 * f + i]) / std::max(1.0, fabs(po[6 * f + i])));
          md = std::max(md, fabs((double)fr[f]->tvec[i] - (double)(float)po[6 * f + 3 + i]) / std::max(1.0, fabs(po[6 * f + 3 + i])));
        }
      EXPECT(md <= 1e-5, "C4 local BA call %d rel diff %g", call, md);
      printf("LocalPoseOptimization C4 call %d: %zu frames + %zu fixed, %zu points, %zu obs, oracle %d its (max rel diff %.2e)\n",
             call, fr.size(), xidx.size(), wp.size(), op.size(), so.iterations, md);
    }
    int32_t si[6];
    if (lorb_ba_solver_info(lorb::thread_ba_solver(ctx), si, 6) == LORB_OK)
      EXPECT(si[1] <= 2 && si[2] == 0 && si[3] <= 47, "solver: %d plan creations, fallback %d, band %d", si[1], si[2], si[3]);
  }

  // ---- Matcher::SearchLocalPoints(curr, set) ------------------------------------------------
  {
    std::set<MiniPoint*> s(pts.begin(), pts.end());
    std::vector<uint8_t> tdesc;
    for (MiniPoint* p : s) tdesc.insert(tdesc.end(), p->desc, p->desc + 32);
    lorb::KeypointsSoA ks = lorb::gather_keypoints(cur);
    std::vector<int32_t> a(N), b(N), c(N);
    const int no = or_bf_match(ks.desc.data(), N, tdesc.data(), (int)s.size(), a.data(), b.data(), c.data());
    for (auto& mp : cur->mps) mp = nullptr;
    const size_t ng = lorb::SearchLocalPoints(ctx, cur, s);
    EXPECT((int)ng == no, "SearchLocalPoints gpu %zu oracle %d", ng, no);
    printf("SearchLocalPoints: %zu matches\n", ng);
  }

  // ---- EstimatePoseLocal's local-map loop (§8f row 1): frustum + SearchByProjection ----------
  {
    MiniFrame* tf = make_frame(30, 1200, r1, t1);
    std::set<MiniPoint*> local;
    float Ow[3];
    {  // camera centre of tf: Ow = -R^T t
      const float* T = tf->Tcw;
      for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    }
    std::vector<MiniPoint*> own;
    for (int i = 0; i < 1500; i++) {
      MiniPoint* p = new MiniPoint();
      own.push_back(p);
      p->pos[0] = urand(-4, 4); p->pos[1] = urand(-3, 3); p->pos[2] = urand(1, 12);
      float d[3], dn = 0;
      for (int c = 0; c < 3; c++) { d[c] = p->pos[c] - Ow[c]; dn += d[c] * d[c]; }
      dn = sqrtf(dn);
      for (int c = 0; c < 3; c++) p->normal[c] = d[c] / dn;
      p->maxd = dn * urand(1.0f, 1.19f); p->mind = p->maxd / 3.5832f;  // predicted level 0 or 1
      for (int b = 0; b < 32; b++) p->desc[b] = (uint8_t)rnd();
      p->nobs = rnd() % 3;
      p->bad = rnd() % 50 == 0;
      p->last_seen = rnd() % 20 == 0 ? tf->id : 0;
      if (i < 900) {  // a keypoint near the projection with a close descriptor
        float u, v;
        project(tf->Tcw, p->pos, tf->fp, &u, &v);
        if (u > 5 && u < 747 && v > 5 && v < 475) {
          const size_t j = rnd() % tf->x.size();
          tf->x[j] = u + urand(-0.5f, 0.5f); tf->y[j] = v + urand(-0.5f, 0.5f); tf->octave[j] = 0;
          for (int b = 0; b < 32; b++) tf->desc[32 * j + b] = p->desc[b] ^ (uint8_t)(rnd() % 8 == 0);
        }
      }
      local.insert(p);
    }
    // oracle chain on the same gathered inputs (std::set order), before the adapter mutates them
    std::vector<MiniPoint*> mp(local.begin(), local.end());
    const size_t n = mp.size();
    std::vector<float> pos(3 * n), nrm(3 * n), mx(n), mn(n);
    std::vector<uint8_t> dsc(32 * n), lk(n), bd(n);
    for (size_t i = 0; i < n; i++) {
      memcpy(&pos[3 * i], mp[i]->pos, 12); memcpy(&nrm[3 * i], mp[i]->normal, 12);
      mx[i] = mp[i]->maxd; mn[i] = mp[i]->mind; memcpy(&dsc[32 * i], mp[i]->desc, 32);
      lk[i] = mp[i]->nobs > 0; bd[i] = mp[i]->bad;
    }
    lorb_frustum_points FPn{(int32_t)n, pos.data(), nrm.data(), mx.data(), mn.data()};
    std::vector<uint8_t> oiv(n);
    std::vector<float> ox(n), oy(n), oxr(n), ocos(n);
    std::vector<int32_t> olev(n);
    or_is_in_frustum(&tf->fp, tf->Tcw, &FPn, 0.5f, oiv.data(), ox.data(), oy.data(), oxr.data(), olev.data(), ocos.data());
    for (size_t i = 0; i < n; i++)
      if (mp[i]->last_seen == tf->id || mp[i]->bad) oiv[i] = 0;
    lorb::KeypointsSoA ks = lorb::gather_keypoints(tf);
    std::vector<uint8_t> st = lorb::gather_slot_state(tf);
    lorb_local_points LP{(int32_t)n, oiv.data(), bd.data(), lk.data(), ox.data(), oy.data(), oxr.data(), olev.data(),
                         ocos.data(), dsc.data()};
    lorb_keypoints kv = ks.view();
    std::vector<int32_t> oas(kv.n + 1);
    int32_t onm = 0;
    or_search_by_projection_local(&tf->fp, &kv, st.data(), &LP, 1.0f, oas.data(), &onm);
    const size_t ng = lorb::TrackLocalMap(ctx, tf, local, 1.0f);
    int diff = 0, inview = 0;
    for (size_t i = 0; i < n; i++) {
      if (mp[i]->last_seen == tf->id || mp[i]->bad) continue;
      diff += (mp[i]->in_view != (oiv[i] != 0));
      if (oiv[i]) {
        inview++;
        diff += memcmp(&mp[i]->proj[0], &ox[i], 4) != 0 || memcmp(&mp[i]->proj[1], &oy[i], 4) != 0 ||
                memcmp(&mp[i]->proj[2], &oxr[i], 4) != 0 || memcmp(&mp[i]->proj[3], &ocos[i], 4) != 0 ||
                mp[i]->level != olev[i] || mp[i]->visible != 1;
      }
    }
    for (int32_t j = 0; j < kv.n; j++)
      if (oas[j] >= 0) diff += tf->mps[j] != mp[oas[j]];
    EXPECT(diff == 0 && (int)ng == onm && onm > 100, "TrackLocalMap: %d diffs, gpu %zu oracle %d", diff, ng, onm);
    printf("TrackLocalMap: %d points in view, %zu matches, bit-exact\n", inview, ng);
  }

  // ---- Frame::ComputeStereoMatches (§8f row 2) ----------------------------------------------
  {
    MiniFrame* sf = make_frame(9, 1500, r0, t0);
    const float disp = 24.37f;
    float sc = 1.0f;
    for (int l = 0; l < 8; l++, sc *= 1.2f) {  // textured level images, right = left shifted by disp/scale
      const int rows = (int)lrintf(480 / sc), cols = (int)lrintf(752 / sc);
      sf->prows.push_back(rows); sf->pcols.push_back(cols);
      std::vector<uint8_t> L(rows * cols), R(rows * cols);
      for (int y = 0; y < rows; y++)
        for (int x = 0; x < cols; x++) {
          const float fx = x * sc, fy = y * sc;
          L[y * cols + x] = (uint8_t)(127 + 60 * sinf(fx * 0.31f + fy * 0.07f) + 50 * cosf(fy * 0.23f - fx * 0.11f) +
                                      (float)(rnd() % 9) - 4.0f);
          const float gx = fx + disp;
          R[y * cols + x] = (uint8_t)(127 + 60 * sinf(gx * 0.31f + fy * 0.07f) + 50 * cosf(fy * 0.23f - gx * 0.11f) +
                                      (float)(rnd() % 9) - 4.0f);
        }
      sf->pyr[0].push_back(L); sf->pyr[1].push_back(R);
    }
    for (size_t i = 0; i < sf->x.size(); i++) {  // keypoints away from the borders, a right twin for most
      const float b = 24.0f * sf->fp.scale_factors[sf->octave[i]];
      sf->x[i] = urand(b + 30, 752 - b); sf->y[i] = urand(b, 480 - b);
      if (rnd() % 4) {
        sf->rx.push_back(sf->x[i] - disp + urand(-0.4f, 0.4f)); sf->ry.push_back(sf->y[i] + urand(-0.5f, 0.5f));
        sf->roct.push_back(sf->octave[i]);
        for (int k = 0; k < 32; k++) sf->rdesc.push_back(sf->desc[32 * i + k] ^ (uint8_t)((rnd() % 16) == 0 ? 1 << (rnd() % 8) : 0));
      }
    }
    lorb::ComputeStereoMatches(ctx, sf);
    // oracle on the same inputs
    const size_t nl = sf->x.size(), nr = sf->rx.size();
    std::vector<int32_t> lo(sf->octave.begin(), sf->octave.end()), ro(sf->roct.begin(), sf->roct.end());
    lorb_stereo_keys L{(int32_t)nl, sf->x.data(), sf->y.data(), lo.data(), sf->desc.data()};
    lorb_stereo_keys R{(int32_t)nr, sf->rx.data(), sf->ry.data(), ro.data(), sf->rdesc.data()};
    lorb::PyramidPack pl = lorb::pack_pyramid(sf, 0), pr = lorb::pack_pyramid(sf, 1);
    std::vector<float> ouR(nl), odp(nl);
    const int npair = or_compute_stereo_matches(&sf->fp, &L, &R, &pl.view, &pr.view, ouR.data(), odp.data());
    int diff = 0, ndepth = 0;
    for (size_t i = 0; i < nl; i++) {
      diff += memcmp(&ouR[i], &sf->uR[i], 4) != 0 || memcmp(&odp[i], &sf->depth[i], 4) != 0;
      ndepth += sf->depth[i] > 0;
    }
    EXPECT(diff == 0 && npair > 300, "ComputeStereoMatches: %d differing slots, %d pairs", diff, npair);
    printf("ComputeStereoMatches: %d depths (%d pairs before the median cut), bit-exact\n", ndepth, npair);
  }

  // ---- MapPoint::ComputeDescriptor, batched (§8f row 4) ---------------------------------------
  {
    // more observers: three extra frames, each point seen in 0-3 of them at random slots
    MiniFrame* ex[3];
    for (int k = 0; k < 3; k++) ex[k] = make_frame(20 + k, 400, r0, t0);
    ex[1]->bad = true;  // a bad observer is skipped (src/map_point.cpp:75-77)
    for (MiniPoint* p : pts)
      for (int k = 0; k < 3; k++)
        if (rnd() % 2) p->obs[ex[k]] = rnd() % 400;
    std::vector<MiniPoint*> mps;
    std::vector<int32_t> off(1, 0);
    std::vector<uint8_t> cand;
    for (MiniPoint* p : pts) {
      mps.push_back(p);
      for (const auto& kv : p->obs)
        if (!kv.first->bad) cand.insert(cand.end(), &kv.first->desc[32 * kv.second], &kv.first->desc[32 * kv.second] + 32);
      off.push_back((int32_t)(cand.size() / 32));
    }
    std::vector<int32_t> best(mps.size() + 1);
    if (cand.empty()) cand.resize(32);
    or_compute_descriptor((int)mps.size(), off.data(), cand.data(), best.data());
    std::vector<uint8_t> before(32 * mps.size());
    for (size_t i = 0; i < mps.size(); i++) memcpy(&before[32 * i], mps[i]->desc, 32);
    lorb::ComputeDescriptors(ctx, mps);
    int diff = 0, changed = 0;
    for (size_t i = 0; i < mps.size(); i++) {
      const uint8_t* want = best[i] >= 0 ? &cand[32 * (size_t)(off[i] + best[i])] : &before[32 * i];
      diff += memcmp(mps[i]->desc, want, 32) != 0;
      changed += memcmp(mps[i]->desc, &before[32 * i], 32) != 0;
    }
    EXPECT(diff == 0, "ComputeDescriptors: %d points differ", diff);
    printf("ComputeDescriptors: %zu points, %d descriptors changed, bit-exact\n", mps.size(), changed);
  }

  printf(g_fail ? "RESULT FAIL (%d)\n" : "RESULT PASS\n", g_fail);
  return g_fail ? 1 : 0;
}
