// integration/Simple_ORB_SLAM/lorb_traits.hpp -- binds lorb/adapters.hpp to the reference's
// own Frame / MapPoint / Map (include/frame.h, include/map_point.h, include/map.h of
// abstract-liu/LORB_SLAM).  Compiled only inside the reference's build (needs OpenCV); see
// INTEGRATION.md.  Every accessor names the reference field it reads.
#pragma once

#include <lorb/adapters.hpp>
#include <lorb/local_mapping.hpp>

#include "frame.h"
#include "map.h"
#include "map_point.h"

namespace lorb {

template <> struct FrameTraits<Simple_ORB_SLAM::Frame> {
  using F = Simple_ORB_SLAM::Frame;
  using point_type = Simple_ORB_SLAM::MapPoint;
  static size_t num_keypoints(F* f) { return f->mnMapPoints; }                   // frame.h:77
  static void keypoint(F* f, size_t i, float* x, float* y, int* o, float* a) {    // mvKeysUn (frame.h:93)
    const cv::KeyPoint& k = f->mvKeysUn[i];
    *x = k.pt.x; *y = k.pt.y; *o = k.octave; *a = k.angle;
  }
  static void descriptor(F* f, size_t i, uint8_t* d) {                             // GetDescriptor (frame.cpp:643)
    cv::Mat m = f->GetDescriptor(i);
    std::memcpy(d, m.ptr<uint8_t>(), 32);
  }
  static bool has_right(F* f) { return f->mvuRight.size() == f->mnMapPoints; }     // frame.h:90
  static float u_right(F* f, size_t i) { return f->mvuRight[i]; }
  static point_type* map_point(F* f, size_t i) { return f->mvpMapPoints[i]; }    // frame.h:80
  // SURVEY §8f row 2 (lorb::ComputeStereoMatches, called as the body of
  // Frame::ComputeStereoMatches).  mDescriptorsRight and the extractors are private
  // (frame.h:126-134): these accessors need `friend struct lorb::FrameTraits<Frame>;` in frame.h
  // and are compiled only with -DLORB_REFERENCE_FRIENDS.  The three drop-in
  // files never call them, so the default build needs the reference headers unchanged.
#ifdef LORB_REFERENCE_FRIENDS
  static void raw_keypoint(F* f, size_t i, float* x, float* y, int* o) {         // mvKeys (frame.h:94)
    const cv::KeyPoint& k = f->mvKeys[i];
    *x = k.pt.x; *y = k.pt.y; *o = k.octave;
  }
  static size_t num_right_keypoints(F* f) { return f->mvKeysRight.size(); }       // frame.h:94
  static void right_keypoint(F* f, size_t i, float* x, float* y, int* o) {
    const cv::KeyPoint& k = f->mvKeysRight[i];
    *x = k.pt.x; *y = k.pt.y; *o = k.octave;
  }
  static void right_descriptor(F* f, size_t i, uint8_t* d) {                       // mDescriptorsRight (frame.h:132)
    std::memcpy(d, f->mDescriptorsRight.ptr<uint8_t>((int)i), 32);
  }
  static int num_levels(F* f) { return (int)f->mpORBextractorLeft->mvImagePyramid.size(); }
  static void pyramid_level(F* f, int side, int l, const uint8_t** d, int* rows, int* cols, int* step) {
    const cv::Mat& m = (side ? f->mpORBextractorRight : f->mpORBextractorLeft)->mvImagePyramid[l];  // ORBextractor.h:85
    *d = m.ptr<uint8_t>(); *rows = m.rows; *cols = m.cols; *step = (int)m.step;
  }
#endif  // LORB_REFERENCE_FRIENDS
  static void set_stereo(F* f, const float* uR, const float* depth, size_t n) {   // mvuRight / mvDepth (frame.h:90-91)
    f->mvuRight.assign(uR, uR + n);
    f->mvDepth.assign(depth, depth + n);
  }
  static void set_map_point(F* f, size_t i, point_type* p) { f->mvpMapPoints[i] = p; }
  static bool outlier(F* f, size_t i) { return f->mvbOutlier[i]; }                // frame.h:92
  static void params(F* f, lorb_frame_params* fp) {                                // frame.h:96-110
    fp->fx = f->fx; fp->fy = f->fy; fp->cx = f->cx; fp->cy = f->cy; fp->bf = f->mbf; fp->b = f->mb;
    fp->min_x = f->mnMinX; fp->max_x = f->mnMaxX; fp->min_y = f->mnMinY; fp->max_y = f->mnMaxY;
    fp->grid_w_inv = static_cast<float>(Simple_ORB_SLAM::FRAME_GRID_COLS) / (f->mnMaxX - f->mnMinX);   // frame.cpp:83
    fp->grid_h_inv = static_cast<float>(Simple_ORB_SLAM::FRAME_GRID_ROWS) / (f->mnMaxY - f->mnMinY);
    fp->n_levels = f->mnScaleLevels; fp->log_scale_factor = f->mfLogScaleFactor;
    for (int i = 0; i < f->mnScaleLevels && i < LORB_MAX_LEVELS; ++i) fp->scale_factors[i] = f->mvScaleFactors[i];
  }
  static void Tcw(F* f, float* T) {                                                // mTcw (frame.h:86)
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) T[4 * r + c] = f->mTcw.at<float>(r, c);
  }
  static void pose_vectors(F* f, float* r, float* t) {                             // mRvec / mTvec
    for (int i = 0; i < 3; ++i) { r[i] = f->mRvec.at<float>(i); t[i] = f->mTvec.at<float>(i); }
  }
  static void set_pose(F* f, const float* t, const float* r) {                     // SetPose(T, R) (frame.cpp:577)
    cv::Mat R = (cv::Mat_<float>(3, 1) << r[0], r[1], r[2]);
    cv::Mat T = (cv::Mat_<float>(3, 1) << t[0], t[1], t[2]);
    f->SetPose(T, R);
  }
  static std::vector<F*> covisible_frames(F* f) { return f->GetCovisibleFrames(); }  // frame.cpp:729
  static bool is_bad(F* f) { return f->IsBad(); }
  static size_t id(F* f) { return f->mnId; }
  static void update_connections(F* f) { f->UpdateConnections(); }                  // frame.cpp:801
  static void map_add_frame(Simple_ORB_SLAM::Map* m, F* f) { m->AddFrame(f); }    // map.cpp:41
};

template <> struct PointTraits<Simple_ORB_SLAM::MapPoint> {
  using P = Simple_ORB_SLAM::MapPoint;
  using F = Simple_ORB_SLAM::Frame;
  static size_t num_obs(P* p) { return p->mnObs; }                                 // map_point.h:54
  static void descriptor(P* p, uint8_t* d) {                                       // map_point.cpp:62
    cv::Mat m = p->GetDescriptor();
    std::memcpy(d, m.ptr<uint8_t>(), 32);
  }
  static void pos(P* p, float* X) { const cv::Point3f q = p->GetPos(); X[0] = q.x; X[1] = q.y; X[2] = q.z; }
  static void set_pos(P* p, const float* X) { p->SetWorldPos(cv::Point3f(X[0], X[1], X[2])); }
  static bool is_bad(P* p) { return p->IsBad(); }
  static bool track_in_view(P* p) { return p->mbTrackInView; }                     // map_point.h:66
  static void tracking(P* p, float* t, int* l) {
    t[0] = p->mTrackProjX; t[1] = p->mTrackProjY; t[2] = p->mTrackProjXR; t[3] = p->mTrackViewCos;
    *l = p->mnTrackScaleLevel;
  }
  static std::map<F*, size_t> observations(P* p) { return p->GetObservations(); }  // map_point.cpp:155
  static bool is_in_frame(P* p, F* f) { return p->IsInFrame(f); }
  static void add_observation(P* p, F* f, size_t i) { p->AddObservation(f, i); }
  static float found_ratio(P* p) { return p->GetFoundRatio(); }
  static void set_bad(P* p) { p->SetBadFlag(); }
  static size_t first_frame_id(P* p) { return p->mnFirstFId; }
  // SURVEY §8f row 1 (lorb::TrackLocalMap)
  static void normal(P* p, float* n) {                                              // GetNormal (map_point.h:48)
    const cv::Mat m = p->GetNormal();
    n[0] = m.at<float>(0); n[1] = m.at<float>(1); n[2] = m.at<float>(2);
  }
  static void distances(P* p, float* mx, float* mn) { *mx = p->mfMaxDistance; *mn = p->mfMinDistance; }  // map_point.h:70
  static size_t last_frame_seen(P* p) { return p->mnLastFrameSeen; }              // map_point.h:69
  static void set_tracking(P* p, bool in_view, const float* t, int level) {       // IsInFrustum (frame.cpp:427, 484-490)
    p->mbTrackInView = in_view;
    if (in_view) {
      p->mTrackProjX = t[0]; p->mTrackProjY = t[1]; p->mTrackProjXR = t[2]; p->mTrackViewCos = t[3];
      p->mnTrackScaleLevel = level;
    }
  }
  static void increase_visible(P* p) { p->IncreaseVisible(); }                     // map_point.cpp:167
  // SURVEY §8f row 4 (lorb::ComputeDescriptors): mDescriptor is private (map_point.h:81), so
  // batching needs `friend struct lorb::PointTraits<MapPoint>;` in map_point.h
  // (-DLORB_REFERENCE_FRIENDS, as above).
#ifdef LORB_REFERENCE_FRIENDS
  static void set_descriptor(P* p, const uint8_t* d) {
    p->mDescriptor = cv::Mat(1, 32, CV_8U);
    std::memcpy(p->mDescriptor.ptr<uint8_t>(), d, 32);
  }
#endif  // LORB_REFERENCE_FRIENDS
};

}  // namespace lorb
