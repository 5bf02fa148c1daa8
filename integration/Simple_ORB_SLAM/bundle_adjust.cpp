// Drop-in replacement of the reference's src/bundle_adjust.cpp (include/bundle_adjust.h:12-21):
// the Ceres problems are replaced by liblorb.so's device-resident LM (MI355X, FP64).
#include "../include/bundle_adjust.h"
#include "lorb_traits.hpp"

namespace Simple_ORB_SLAM {

BA::BA() {}

void BA::ProjectPoseOptimization(Frame* pCurrFrame) {
  lorb::ProjectPoseOptimization(lorb::thread_ctx(), pCurrFrame);
}

void BA::LocalPoseOptimization(Frame* pCurrFrame) {
  lorb::LocalPoseOptimization(lorb::thread_ctx(), pCurrFrame);
}

}  // namespace Simple_ORB_SLAM
