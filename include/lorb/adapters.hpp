// lorb/adapters.hpp -- C++ host layer between the reference's class interfaces
// (Simple_ORB_SLAM::Matcher / BA / LocalMapping) and the C-ABI of lorb_c.h.
//
// The functions here are templates over the caller's Frame / MapPoint types and reach their
// fields only through FrameTraits<> / PointTraits<> specialisations.  The drop-in build
// (integration/Simple_ORB_SLAM/) specialises them for the reference's OpenCV-based Frame and
// MapPoint; tests/cpp specialises them for plain test frames.  Every function gathers the
// fields the reference reads into SoA arrays, calls liblorb.so (HIP kernels on the MI355X),
// and applies the results back exactly as the reference writes them (file:line per function).
//
// Error behaviour: the reference never fails (it returns counts / void).  A C-ABI error is
// raised as lorb::Error (std::runtime_error) -- there is deliberately no CPU fallback.
#pragma once

#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../lorb_c.h"

namespace lorb {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Specialise for the caller's types.  Required members are listed in integration/.
template <class FrameT> struct FrameTraits;
template <class PointT> struct PointTraits;

// One lorb_ctx (one HIP stream) per calling thread (SURVEY §8b "Threading").
inline lorb_ctx* thread_ctx(int device = 0) {
  struct Holder {
    lorb_ctx* ctx = nullptr;
    ~Holder() { if (ctx) lorb_destroy(ctx); }
  };
  thread_local Holder h;
  if (!h.ctx && lorb_create(device, &h.ctx) != LORB_OK)
    throw Error("lorb_create failed: no usable MI355X (liblorb.so has no CPU fallback)");
  return h.ctx;
}

// The ctx's BA solver (device-built plans resident across LocalPoseOptimization calls).  The ctx
// owns it (lorb_ctx_ba_solver): it is destroyed by lorb_destroy, so it never outlives the ctx
// whatever ctx the caller passes.
inline lorb_ba_solver* thread_ba_solver(lorb_ctx* ctx) {
  lorb_ba_solver* s = nullptr;
  if (lorb_ctx_ba_solver(ctx, &s) != LORB_OK) throw Error("lorb_ctx_ba_solver failed");
  return s;
}

inline void check(lorb_ctx* ctx, int rc, const char* what) {
  if (rc != LORB_OK) throw Error(std::string(what) + " failed: " + lorb_last_error(ctx));
}

// SoA gather of a frame's keypoints (Frame::mvKeysUn, mvuRight, mDescriptors)
struct KeypointsSoA {
  std::vector<float> x, y, angle, uR;
  std::vector<int32_t> octave;
  std::vector<uint8_t> desc;
  lorb_keypoints view() const {
    lorb_keypoints k;
    k.n = (int32_t)x.size(); k.x = x.data(); k.y = y.data(); k.octave = octave.data(); k.angle = angle.data();
    k.u_right = uR.empty() ? nullptr : uR.data(); k.desc = desc.data();
    return k;
  }
};

template <class FrameT>
KeypointsSoA gather_keypoints(FrameT* F) {
  using FT = FrameTraits<FrameT>;
  KeypointsSoA s;
  const size_t n = FT::num_keypoints(F);
  s.x.resize(n); s.y.resize(n); s.angle.resize(n); s.octave.resize(n); s.desc.resize(32 * n);
  for (size_t i = 0; i < n; ++i) {
    FT::keypoint(F, i, &s.x[i], &s.y[i], &s.octave[i], &s.angle[i]);
    FT::descriptor(F, i, &s.desc[32 * i]);
  }
  if (FT::has_right(F)) {
    s.uR.resize(n);
    for (size_t i = 0; i < n; ++i) s.uR[i] = FT::u_right(F, i);
  }
  return s;
}

// slot state of F->mvpMapPoints (src/matcher.cpp:149-151 occupancy test)
template <class FrameT>
std::vector<uint8_t> gather_slot_state(FrameT* F) {
  using FT = FrameTraits<FrameT>;
  using PT = PointTraits<typename FT::point_type>;
  const size_t n = FT::num_keypoints(F);
  std::vector<uint8_t> st(n, LORB_SLOT_EMPTY);
  for (size_t i = 0; i < n; ++i) {
    auto* p = FT::map_point(F, i);
    if (p) st[i] = PT::num_obs(p) > 0 ? LORB_SLOT_LOCKED : LORB_SLOT_FREE;
  }
  return st;
}

// ---- Matcher::SearchByProjection(Frame* curr, Frame* prev), src/matcher.cpp:13-62 ----------
template <class FrameT>
size_t SearchByProjectionBF(lorb_ctx* ctx, FrameT* curr, FrameT* prev) {
  using FT = FrameTraits<FrameT>;
  using P = typename FT::point_type;
  using PT = PointTraits<P>;
  std::vector<P*> prevMPs;
  std::vector<uint8_t> tdesc;
  for (size_t i = 0; i < FT::num_keypoints(prev); ++i) {
    P* p = FT::map_point(prev, i);
    if (!p) continue;
    prevMPs.push_back(p);
    tdesc.resize(tdesc.size() + 32);
    PT::descriptor(p, &tdesc[tdesc.size() - 32]);
  }
  KeypointsSoA k = gather_keypoints(curr);
  const int32_t nq = (int32_t)FT::num_keypoints(curr), nt = (int32_t)prevMPs.size();
  const int32_t q_off[2] = {0, nq}, t_off[2] = {0, nt};
  std::vector<int32_t> cc_t(nq + 1), cc_d(nq + 1), mt(nq + 1);
  int32_t nm = 0;
  check(ctx, lorb_bf_match(ctx, 1, k.desc.data(), q_off, tdesc.data(), t_off, cc_t.data(), cc_d.data(), mt.data(), &nm),
        "lorb_bf_match");
  for (int32_t q = 0; q < nq; ++q)
    if (mt[q] >= 0) FT::set_map_point(curr, q, prevMPs[mt[q]]);
  return (size_t)nm;
}

// ---- Matcher::SearchLocalPoints(Frame* curr, std::set<MapPoint*>), src/matcher.cpp:319-366 -
template <class FrameT, class PointT>
size_t SearchLocalPoints(lorb_ctx* ctx, FrameT* curr, const std::set<PointT*>& vpMPs) {
  using FT = FrameTraits<FrameT>;
  using PT = PointTraits<PointT>;
  std::vector<PointT*> mps;
  std::vector<uint8_t> tdesc;
  for (PointT* p : vpMPs) {  // std::set iteration order (pointer order), src/matcher.cpp:327
    if (!p) continue;
    mps.push_back(p);
    tdesc.resize(tdesc.size() + 32);
    PT::descriptor(p, &tdesc[tdesc.size() - 32]);
  }
  KeypointsSoA k = gather_keypoints(curr);
  const int32_t nq = (int32_t)FT::num_keypoints(curr), nt = (int32_t)mps.size();
  const int32_t q_off[2] = {0, nq}, t_off[2] = {0, nt};
  std::vector<int32_t> cc_t(nq + 1), cc_d(nq + 1), mt(nq + 1);
  int32_t nm = 0;
  check(ctx, lorb_bf_match(ctx, 1, k.desc.data(), q_off, tdesc.data(), t_off, cc_t.data(), cc_d.data(), mt.data(), &nm),
        "lorb_bf_match");
  for (int32_t q = 0; q < nq; ++q)
    if (mt[q] >= 0) FT::set_map_point(curr, q, mps[mt[q]]);
  return (size_t)nm;
}

template <class FrameT>
lorb_frame_params frame_params(FrameT* F) {
  using FT = FrameTraits<FrameT>;
  lorb_frame_params fp;
  std::memset(&fp, 0, sizeof(fp));
  FT::params(F, &fp);
  return fp;
}

// ---- Matcher::SearchByProjection(Frame* Cur, Frame* Last, const float th), src/matcher.cpp:64-218
template <class FrameT>
size_t SearchByProjectionFrame(lorb_ctx* ctx, FrameT* cur, FrameT* last, float th) {
  using FT = FrameTraits<FrameT>;
  using P = typename FT::point_type;
  using PT = PointTraits<P>;
  lorb_frame_params fp = frame_params(cur);
  float Tcur[16], Tlast[16];
  FT::Tcw(cur, Tcur);
  FT::Tcw(last, Tlast);
  KeypointsSoA k = gather_keypoints(cur);
  std::vector<uint8_t> st = gather_slot_state(cur);
  const size_t nl = FT::num_keypoints(last);
  std::vector<uint8_t> has(nl, 0), out(nl, 0), lk(nl, 0), ldesc(32 * nl, 0);
  std::vector<float> pos(3 * nl, 0.f), ang(nl, 0.f);
  std::vector<int32_t> oct(nl, 0);
  std::vector<P*> mps(nl, nullptr);
  for (size_t i = 0; i < nl; ++i) {
    P* p = FT::map_point(last, i);
    float kx, ky;
    FT::keypoint(last, i, &kx, &ky, &oct[i], &ang[i]);  // mvKeys == mvKeysUn (src/frame.cpp:358-362)
    if (!p) continue;
    mps[i] = p; has[i] = 1; out[i] = FT::outlier(last, i) ? 1 : 0;
    lk[i] = PT::num_obs(p) > 0 ? 1 : 0;
    PT::pos(p, &pos[3 * i]);
    PT::descriptor(p, &ldesc[32 * i]);
  }
  lorb_last_frame L;
  L.n = (int32_t)nl; L.Tcw = Tlast; L.has_mp = has.data(); L.outlier = out.data(); L.mp_locked = lk.data();
  L.mp_pos = pos.data(); L.mp_desc = ldesc.data(); L.octave = oct.data(); L.angle = ang.data();
  lorb_keypoints kv = k.view();
  std::vector<int32_t> assign(kv.n + 1);
  int32_t nm = 0;
  check(ctx, lorb_search_by_projection_frame(ctx, &fp, Tcur, &kv, st.data(), &L, th, assign.data(), &nm),
        "lorb_search_by_projection_frame");
  for (int32_t j = 0; j < kv.n; ++j) {
    if (assign[j] == LORB_ASSIGN_NULL) FT::set_map_point(cur, j, (P*)nullptr);
    else if (assign[j] >= 0) FT::set_map_point(cur, j, mps[assign[j]]);
  }
  return (size_t)nm;
}

// ---- Matcher::SearchByProjection(Frame* F, const set<MapPoint*>&, th), src/matcher.cpp:220-316
template <class FrameT, class PointT>
size_t SearchByProjectionLocal(lorb_ctx* ctx, FrameT* F, const std::set<PointT*>& vpMapPoints, float th) {
  using FT = FrameTraits<FrameT>;
  using PT = PointTraits<PointT>;
  lorb_frame_params fp = frame_params(F);
  KeypointsSoA k = gather_keypoints(F);
  std::vector<uint8_t> st = gather_slot_state(F);
  const size_t n = vpMapPoints.size();
  std::vector<PointT*> mps;
  mps.reserve(n);
  std::vector<uint8_t> iv, bad, lk, desc;
  std::vector<float> px, py, pxr, vc;
  std::vector<int32_t> lev;
  for (PointT* p : vpMapPoints) {  // std::set iteration order, src/matcher.cpp:226
    mps.push_back(p);
    iv.push_back(PT::track_in_view(p) ? 1 : 0);
    bad.push_back(PT::is_bad(p) ? 1 : 0);
    lk.push_back(PT::num_obs(p) > 0 ? 1 : 0);
    float t[5];
    int l;
    PT::tracking(p, t, &l);  // mTrackProjX/Y/XR, mTrackViewCos ; mnTrackScaleLevel
    px.push_back(t[0]); py.push_back(t[1]); pxr.push_back(t[2]); vc.push_back(t[3]);
    lev.push_back(iv.back() ? l : 0);
    desc.resize(desc.size() + 32);
    PT::descriptor(p, &desc[desc.size() - 32]);
  }
  lorb_local_points L;
  L.n = (int32_t)n; L.track_in_view = iv.data(); L.is_bad = bad.data(); L.locked = lk.data();
  L.proj_x = px.data(); L.proj_y = py.data(); L.proj_xr = pxr.data(); L.pred_level = lev.data();
  L.view_cos = vc.data(); L.desc = desc.data();
  lorb_keypoints kv = k.view();
  std::vector<int32_t> assign(kv.n + 1);
  int32_t nm = 0;
  check(ctx, lorb_search_by_projection_local(ctx, &fp, &kv, st.data(), &L, th, assign.data(), &nm),
        "lorb_search_by_projection_local");
  for (int32_t j = 0; j < kv.n; ++j)
    if (assign[j] >= 0) FT::set_map_point(F, j, mps[assign[j]]);
  return (size_t)nm;
}

// ---- BA::ProjectPoseOptimization(Frame*), src/bundle_adjust.cpp:158-202 -------------------
template <class FrameT>
void ProjectPoseOptimization(lorb_ctx* ctx, FrameT* F) {
  using FT = FrameTraits<FrameT>;
  using P = typename FT::point_type;
  using PT = PointTraits<P>;
  std::vector<float> pts, obs;
  for (size_t i = 0; i < FT::num_keypoints(F); ++i) {
    P* p = FT::map_point(F, i);
    if (!p) continue;
    float X[3], x, y, a;
    int o;
    PT::pos(p, X);
    FT::keypoint(F, i, &x, &y, &o, &a);  // GetKp2d(i) = mvKeysUn[i].pt
    pts.insert(pts.end(), X, X + 3);
    obs.push_back(x);
    obs.push_back(y);
  }
  lorb_frame_params fp = frame_params(F);
  float rt[6];
  FT::pose_vectors(F, rt, rt + 3);  // mRvec, mTvec
  const float intr[4] = {fp.fx, fp.fx /* PoseCost quirk: v uses fx, src/bundle_adjust.cpp:51 */, fp.cx, fp.cy};
  const int32_t res_off[2] = {0, (int32_t)(obs.size() / 2)};
  lorb_pose_problem_batch b;
  b.n_frames = 1; b.res_off = res_off; b.intr = intr; b.pose_init = rt; b.pts3d = pts.data(); b.obs2d = obs.data();
  lorb_lm_options opt;
  lorb_lm_options_default(&opt);
  double pose[6];
  lorb_ba_summary s;
  check(ctx, lorb_ba_pose_only(ctx, &b, &opt, pose, nullptr, &s), "lorb_ba_pose_only");
  const float R[3] = {(float)pose[0], (float)pose[1], (float)pose[2]};
  const float T[3] = {(float)pose[3], (float)pose[4], (float)pose[5]};
  FT::set_pose(F, T, R);  // Frame::SetPose(T, R) -> Rodrigues -> mTcw (src/frame.cpp:577-594)
}

// ---- BA::LocalPoseOptimization(Frame*), src/bundle_adjust.cpp:207-330 ---------------------
// Observation source: the reference reads GetKps2d()[idx] (src/bundle_adjust.cpp:285,295),
// which is empty on the live path (UB); we use GetKp2d(idx) as ProjectPoseOptimization does
// (the one intentional divergence).
template <class FrameT>
void LocalPoseOptimization(lorb_ctx* ctx, FrameT* cur) {
  using FT = FrameTraits<FrameT>;
  using P = typename FT::point_type;
  using PT = PointTraits<P>;
  std::vector<FrameT*> frames{cur};
  for (FrameT* f : FT::covisible_frames(cur))
    if (!FT::is_bad(f)) frames.push_back(f);
  std::map<FrameT*, int> frame_idx;
  for (size_t i = 0; i < frames.size(); ++i) frame_idx.emplace(frames[i], (int)i);
  std::vector<P*> points;  // union in first-seen order (std::find dedup, :224-241)
  std::set<P*> seen;
  for (FrameT* f : frames)
    for (size_t i = 0; i < FT::num_keypoints(f); ++i) {
      P* p = FT::map_point(f, i);
      if (!p || PT::is_bad(p)) continue;
      if (seen.insert(p).second) points.push_back(p);
    }
  std::vector<float> pose_init(6 * frames.size()), point_init(3 * points.size()), fixed, uv;
  for (size_t i = 0; i < frames.size(); ++i) FT::pose_vectors(frames[i], &pose_init[6 * i], &pose_init[6 * i + 3]);
  std::vector<int32_t> op, of;
  std::map<FrameT*, int> fixed_idx;
  for (size_t pi = 0; pi < points.size(); ++pi) {
    P* p = points[pi];
    PT::pos(p, &point_init[3 * pi]);
    for (auto& ob : PT::observations(p)) {  // std::map<Frame*, size_t> order
      FrameT* f = ob.first;
      if (FT::is_bad(f)) continue;
      float x, y, a;
      int o;
      FT::keypoint(f, ob.second, &x, &y, &o, &a);
      auto it = frame_idx.find(f);
      int code;
      if (it != frame_idx.end()) {
        code = it->second;
      } else {
        auto jt = fixed_idx.find(f);
        if (jt == fixed_idx.end()) {
          jt = fixed_idx.emplace(f, (int)fixed_idx.size()).first;
          fixed.resize(fixed.size() + 6);
          FT::pose_vectors(f, &fixed[fixed.size() - 6], &fixed[fixed.size() - 3]);
        }
        code = -1 - jt->second;
      }
      op.push_back((int32_t)pi);
      of.push_back(code);
      uv.push_back(x);
      uv.push_back(y);
    }
  }
  lorb_frame_params fp = frame_params(cur);
  lorb_ba_window w;
  w.n_poses = (int32_t)frames.size(); w.n_fixed = (int32_t)fixed_idx.size();
  w.n_points = (int32_t)points.size(); w.n_obs = (int32_t)op.size();
  w.fx = fp.fx; w.fy = fp.fy; w.cx = fp.cx; w.cy = fp.cy;
  w.pose_init = pose_init.data(); w.fixed_pose = fixed.data(); w.point_init = point_init.data();
  w.obs_point = op.data(); w.obs_frame = of.data(); w.obs_uv = uv.data();
  lorb_lm_options opt;
  lorb_lm_options_default(&opt);
  std::vector<double> po(6 * frames.size() + 1), pt(3 * points.size() + 1);
  double* pp = po.data();
  double* qq = pt.data();
  lorb_ba_summary s;
  // the thread's solver: the window's device-built plan stays resident between calls (no per-call
  // plan construction; lorb_c.h lorb_ba_solver_solve)
  check(ctx, lorb_ba_solver_solve(thread_ba_solver(ctx), &w, &opt, pp, qq, &s), "lorb_ba_solver_solve");
  for (size_t i = 0; i < frames.size(); ++i) {  // float write-back, :317-329
    const float R[3] = {(float)po[6 * i], (float)po[6 * i + 1], (float)po[6 * i + 2]};
    const float T[3] = {(float)po[6 * i + 3], (float)po[6 * i + 4], (float)po[6 * i + 5]};
    FT::set_pose(frames[i], T, R);
  }
  for (size_t i = 0; i < points.size(); ++i) {
    const float X[3] = {(float)pt[3 * i], (float)pt[3 * i + 1], (float)pt[3 * i + 2]};
    PT::set_pos(points[i], X);
  }
}

// ---- the callers either side of the path ---------------------------------

// One camera's ORBextractor::mvImagePyramid packed into one buffer (levels are separate cv::Mat
// ROIs in the reference; the C-ABI takes one buffer + per-level offsets).
struct PyramidPack {
  std::vector<uint8_t> buf;
  lorb_image_pyramid view;
};
template <class FrameT>
PyramidPack pack_pyramid(FrameT* F, int side /* 0 left, 1 right */) {
  using FT = FrameTraits<FrameT>;
  PyramidPack p;
  std::memset(&p.view, 0, sizeof(p.view));
  const int L = FT::num_levels(F);
  p.view.n_levels = L;
  std::vector<const uint8_t*> src(L);
  std::vector<int> sstep(L);
  size_t off = 0;
  for (int l = 0; l < L; ++l) {
    int rows, cols;
    FT::pyramid_level(F, side, l, &src[l], &rows, &cols, &sstep[l]);
    p.view.offset[l] = (int64_t)off; p.view.rows[l] = rows; p.view.cols[l] = cols; p.view.step[l] = cols;
    off += (size_t)rows * cols;
  }
  p.buf.resize(off > 0 ? off : 1);
  for (int l = 0; l < L; ++l)
    for (int r = 0; r < p.view.rows[l]; ++r)
      std::memcpy(&p.buf[p.view.offset[l] + (size_t)r * p.view.cols[l]], src[l] + (size_t)r * sstep[l], p.view.cols[l]);
  p.view.data = p.buf.data();
  return p;
}

// ---- Frame::ComputeStereoMatches, src/frame.cpp:125-333 (§8f row 2) ------------------------
// Reads mvKeys / mvKeysRight (distorted, :178, :206), both descriptor matrices and both
// pyramids; writes mvuRight / mvDepth (:127-128, :310-311, :329-330).
template <class FrameT>
void ComputeStereoMatches(lorb_ctx* ctx, FrameT* F) {
  using FT = FrameTraits<FrameT>;
  const size_t nl = FT::num_keypoints(F), nr = FT::num_right_keypoints(F);
  std::vector<float> lx(nl + 1), ly(nl + 1), rx(nr + 1), ry(nr + 1);
  std::vector<int32_t> lo(nl + 1), ro(nr + 1);
  std::vector<uint8_t> ld(32 * nl + 32), rd(32 * nr + 32);
  for (size_t i = 0; i < nl; ++i) {
    FT::raw_keypoint(F, i, &lx[i], &ly[i], &lo[i]);
    FT::descriptor(F, i, &ld[32 * i]);
  }
  for (size_t i = 0; i < nr; ++i) {
    FT::right_keypoint(F, i, &rx[i], &ry[i], &ro[i]);
    FT::right_descriptor(F, i, &rd[32 * i]);
  }
  const lorb_stereo_keys L{(int32_t)nl, lx.data(), ly.data(), lo.data(), ld.data()};
  const lorb_stereo_keys R{(int32_t)nr, rx.data(), ry.data(), ro.data(), rd.data()};
  const PyramidPack pl = pack_pyramid(F, 0), pr = pack_pyramid(F, 1);
  const lorb_frame_params fp = frame_params(F);
  std::vector<float> uR(nl + 1, -1.0f), depth(nl + 1, -1.0f);
  check(ctx, lorb_compute_stereo_matches(ctx, &fp, &L, &R, &pl.view, &pr.view, uR.data(), depth.data()),
        "lorb_compute_stereo_matches");
  FT::set_stereo(F, uR.data(), depth.data(), nl);
}

// ---- MapPoint::ComputeDescriptor, src/map_point.cpp:69-129, batched (§8f row 4) -----------
// Candidates: the observations in std::map<Frame*, size_t> order, bad frames skipped (:74-81).
// A point with no candidate keeps its descriptor (the reference indexes an empty vector there).
template <class PointT>
void ComputeDescriptors(lorb_ctx* ctx, const std::vector<PointT*>& mps) {
  using PT = PointTraits<PointT>;
  using ObsMap = decltype(PT::observations(std::declval<PointT*>()));
  using FrameT = std::remove_pointer_t<typename std::decay_t<ObsMap>::key_type>;
  using FT = FrameTraits<FrameT>;
  std::vector<int32_t> off(1, 0);
  std::vector<uint8_t> desc;
  for (PointT* p : mps) {
    for (const auto& kv : PT::observations(p)) {
      if (FT::is_bad(kv.first)) continue;
      desc.resize(desc.size() + 32);
      FT::descriptor(kv.first, kv.second, &desc[desc.size() - 32]);
    }
    off.push_back((int32_t)(desc.size() / 32));
  }
  const int32_t n = (int32_t)mps.size();
  std::vector<int32_t> best(n + 1);
  std::vector<uint8_t> out(32 * (size_t)n + 32);
  if (desc.empty()) desc.resize(32);
  check(ctx, lorb_compute_descriptor(ctx, n, off.data(), desc.data(), best.data(), out.data()),
        "lorb_compute_descriptor");
  for (int32_t i = 0; i < n; ++i)
    if (best[i] >= 0) PT::set_descriptor(mps[i], &out[32 * (size_t)i]);
}

// ---- VisualOdometry::EstimatePoseLocal's local-map loop, src/visual_odometry.cpp:173-201 ---
// (§8f row 1).  For every local point neither seen in this frame yet (mnLastFrameSeen == mnId;
// its mbTrackInView was cleared at :168) nor bad: Frame::IsInFrustum(pMP, 0.5) (src/frame.cpp:
// 425-494) writes mbTrackInView and, in view, the tracking fields + IncreaseVisible (:190); then,
// if any point is in view, SearchByProjection(F, localMPs, th) (:197-201).  Returns nMatches.
template <class FrameT, class PointT>
size_t TrackLocalMap(lorb_ctx* ctx, FrameT* F, const std::set<PointT*>& localMPs, float th = 1.0f,
                     float viewing_cos_limit = 0.5f) {
  using FT = FrameTraits<FrameT>;
  using PT = PointTraits<PointT>;
  const lorb_frame_params fp = frame_params(F);
  float T[16];
  FT::Tcw(F, T);
  KeypointsSoA k = gather_keypoints(F);
  std::vector<uint8_t> st = gather_slot_state(F);
  const size_t n = localMPs.size();
  std::vector<PointT*> mps;
  mps.reserve(n);
  std::vector<float> pos(3 * n + 3), nrm(3 * n + 3), maxd(n + 1), mind(n + 1);
  std::vector<uint8_t> desc(32 * n + 32), locked(n + 1), bad(n + 1), inframe(n + 1);
  for (PointT* p : localMPs) {  // std::set iteration order (:175)
    const size_t i = mps.size();
    mps.push_back(p);
    PT::pos(p, &pos[3 * i]);
    PT::normal(p, &nrm[3 * i]);
    PT::distances(p, &maxd[i], &mind[i]);
    PT::descriptor(p, &desc[32 * i]);
    locked[i] = PT::num_obs(p) > 0 ? 1 : 0;
    bad[i] = PT::is_bad(p) ? 1 : 0;
    inframe[i] = PT::last_frame_seen(p) == FT::id(F) ? 1 : 0;
  }
  lorb_map_points_dev M;  // host arrays for the host entry point
  M.n = (int32_t)n; M.pos = pos.data(); M.normal = nrm.data(); M.max_dist = maxd.data(); M.min_dist = mind.data();
  M.desc = desc.data(); M.locked = locked.data(); M.is_bad = bad.data(); M.in_frame = inframe.data();
  lorb_keypoints kv = k.view();
  std::vector<uint8_t> iv(n + 1);
  std::vector<float> tr(4 * n + 4);
  std::vector<int32_t> lev(n + 1), assign(kv.n + 1);
  int32_t nm = 0;
  check(ctx, lorb_track_local_map(ctx, &fp, T, &kv, st.data(), &M, viewing_cos_limit, th, iv.data(), tr.data(),
                                  lev.data(), assign.data(), &nm),
        "lorb_track_local_map");
  size_t nToMatch = 0;
  for (size_t i = 0; i < n; ++i) {
    if (inframe[i] || bad[i]) continue;
    const float t4[4] = {tr[i], tr[n + i], tr[2 * n + i], tr[3 * n + i]};  // planes x, y, xr, viewcos
    PT::set_tracking(mps[i], iv[i] != 0, t4, lev[i]);
    if (iv[i]) { PT::increase_visible(mps[i]); ++nToMatch; }
  }
  if (nToMatch == 0) return 0;
  for (int32_t j = 0; j < kv.n; ++j)
    if (assign[j] >= 0) FT::set_map_point(F, j, mps[assign[j]]);
  return (size_t)nm;
}

}  // namespace lorb
