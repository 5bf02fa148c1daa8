// Drop-in replacement of the reference's src/local_mapping.cpp (include/local_mapping.h:15-46).
// The reference header is kept unchanged; its members are used as declared.  The pop in
// ProcessNewFrames takes mFrameLock (the reference pops without it -- a race).
#include "../include/local_mapping.h"
#include "lorb_traits.hpp"

namespace Simple_ORB_SLAM {

LocalMapping::LocalMapping(Map* pMap) { mpMap = pMap; }

void LocalMapping::InsertKeyFrame(Frame* pF) {
  std::unique_lock<std::mutex> lock(mFrameLock);
  mlpNewFrames.push_back(pF);
}

void LocalMapping::Run() {
  while (true) {  // the reference's busy loop (src/local_mapping.cpp:21-38)
    if (CheckNewFrame() == true) {
      ProcessNewFrames();
      // MapPointsCulling();                          // commented out in the reference
      if (CheckNewFrame() == false) {
#ifdef LORB_LOCAL_BA
        BA::LocalPoseOptimization(mpCurrFrame);        // src/local_mapping.cpp:32 (opt-in)
#endif
      }
    }
  }
}

bool LocalMapping::CheckNewFrame() {
  std::unique_lock<std::mutex> lock(mFrameLock);
  return (mlpNewFrames.empty() == false);
}

void LocalMapping::ProcessNewFrames() {
  {
    std::unique_lock<std::mutex> lock(mFrameLock);
    mpCurrFrame = mlpNewFrames.front();
    mlpNewFrames.pop_front();
  }
#ifdef LORB_LOCAL_BA
  for (size_t i = 0; i < mpCurrFrame->mnMapPoints; i++) {  // steps 1-2, src/local_mapping.cpp:55-74
    MapPoint* pMP = mpCurrFrame->mvpMapPoints[i];
    if (!pMP || pMP->IsBad()) continue;
    if (pMP->IsInFrame(mpCurrFrame) == false) pMP->AddObservation(mpCurrFrame, i);
    else mvpRecentAddPoints.push_back(pMP);
  }
  mpCurrFrame->UpdateConnections();
#endif
  mpMap->AddFrame(mpCurrFrame);
}

void LocalMapping::MapPointsCulling() {
  std::vector<MapPoint*> keep;
  for (MapPoint* pMP : mvpRecentAddPoints) {
    if (pMP->IsBad()) continue;
    if (pMP->GetFoundRatio() < 0.25f) { pMP->SetBadFlag(); continue; }
    if ((mpCurrFrame->mnId - pMP->mnFirstFId) >= 2 && pMP->mnObs < 3) { pMP->SetBadFlag(); continue; }
    if ((mpCurrFrame->mnId - pMP->mnFirstFId) >= 3) continue;
    keep.push_back(pMP);
  }
  mvpRecentAddPoints.swap(keep);
}

void LocalMapping::KeyFramesCulling() {}

}  // namespace Simple_ORB_SLAM
