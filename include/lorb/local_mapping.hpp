// lorb/local_mapping.hpp -- LocalMapping (src/local_mapping.cpp:8-113, include/local_mapping.h:15-46)
// over the C-ABI.  Same queue semantics as the reference: VisualOdometry pushes keyframes with
// InsertKeyFrame, the mapper thread runs Run().  Differences, all documented in DESIGN.md:
//   * ProcessNewFrames pops under mFrameLock (the reference pops without the lock,
//     src/local_mapping.cpp:51-54 -- a data race);
//   * Run() can be stopped (RequestFinish) instead of spinning forever;
//   * the reference's commented-out design (AddObservation + UpdateConnections, local BA when
//     the queue drains, src/local_mapping.cpp:28-33,55-74) is available behind
//     set_full_step(true); by default only Map::AddFrame runs, exactly like the reference.
#pragma once

#include <atomic>
#include <list>
#include <mutex>
#include <thread>
#include <vector>

#include "adapters.hpp"

namespace lorb {

template <class FrameT, class MapT>
class LocalMapping {
 public:
  using FT = FrameTraits<FrameT>;
  using PointT = typename FT::point_type;
  using PT = PointTraits<PointT>;

  explicit LocalMapping(MapT* pMap) : mpMap(pMap) {}

  void InsertKeyFrame(FrameT* pF) {  // src/local_mapping.cpp:13-17
    std::unique_lock<std::mutex> lock(mFrameLock);
    mlpNewFrames.push_back(pF);
  }

  bool CheckNewFrame() {  // src/local_mapping.cpp:42-46
    std::unique_lock<std::mutex> lock(mFrameLock);
    return !mlpNewFrames.empty();
  }

  void ProcessNewFrames() {  // src/local_mapping.cpp:49-78
    {
      std::unique_lock<std::mutex> lock(mFrameLock);
      mpCurrFrame = mlpNewFrames.front();
      mlpNewFrames.pop_front();
    }
    if (mbFullStep) {
      // step 1 (commented in the reference): register the keyframe's observations
      for (size_t i = 0; i < FT::num_keypoints(mpCurrFrame); ++i) {
        PointT* p = FT::map_point(mpCurrFrame, i);
        if (!p || PT::is_bad(p)) continue;
        if (!PT::is_in_frame(p, mpCurrFrame)) PT::add_observation(p, mpCurrFrame, i);
        else mvpRecentAddPoints.push_back(p);
      }
      // step 2: covisibility graph
      FT::update_connections(mpCurrFrame);
    }
    FT::map_add_frame(mpMap, mpCurrFrame);  // step 3
    ++mnProcessed;
  }

  // intended semantics of src/local_mapping.cpp:82-108 (its erase-then-increment bug removed)
  void MapPointsCulling() {
    std::vector<PointT*> keep;
    const size_t cur = FT::id(mpCurrFrame);
    for (PointT* p : mvpRecentAddPoints) {
      if (PT::is_bad(p)) continue;
      if (PT::found_ratio(p) < 0.25f) { PT::set_bad(p); continue; }
      if (cur - PT::first_frame_id(p) >= 2 && PT::num_obs(p) < 3) { PT::set_bad(p); continue; }
      if (cur - PT::first_frame_id(p) >= 3) continue;
      keep.push_back(p);
    }
    mvpRecentAddPoints.swap(keep);
  }

  void KeyFramesCulling() {}  // empty in the reference (src/local_mapping.cpp:110-113)

  // src/local_mapping.cpp:19-40
  void Run() {
    while (!mbFinish.load()) {
      if (CheckNewFrame()) {
        ProcessNewFrames();
        if (mbFullStep) MapPointsCulling();
        if (!CheckNewFrame() && mbFullStep) LocalPoseOptimization(thread_ctx(mDevice), mpCurrFrame);
      } else {
        std::this_thread::yield();
      }
    }
  }

  void RequestFinish() { mbFinish.store(true); }
  void set_full_step(bool on) { mbFullStep = on; }
  void set_device(int d) { mDevice = d; }
  size_t processed() const { return mnProcessed.load(); }
  FrameT* current() const { return mpCurrFrame; }

 protected:
  std::mutex mFrameLock;

 private:
  FrameT* mpCurrFrame = nullptr;
  MapT* mpMap;
  std::list<FrameT*> mlpNewFrames;
  std::vector<PointT*> mvpRecentAddPoints;
  std::atomic<bool> mbFinish{false};
  bool mbFullStep = false;
  int mDevice = 0;
  std::atomic<size_t> mnProcessed{0};  // read by other threads (processed())
};

}  // namespace lorb
