// Compile-only TU (tests/test_compile_boundary.py): with the two friend declarations of
// INTEGRATION.md §4 added to the reference's frame.h / map_point.h, the §8f adapters that read
// private members (stereo matching, batched ComputeDescriptor) and the local-map tracking
// adapter instantiate against the reference's own Frame / MapPoint.
#include "lorb_traits.hpp"

namespace Simple_ORB_SLAM {

void lorb_compile_check_rows(Frame* F, const std::set<MapPoint*>& local, const std::vector<MapPoint*>& mps) {
  lorb_ctx* ctx = lorb::thread_ctx();
  lorb::ComputeStereoMatches(ctx, F);                 // src/frame.cpp:125-333
  lorb::ComputeDescriptors(ctx, mps);                 // src/map_point.cpp:69-129
  (void)lorb::TrackLocalMap(ctx, F, local, 1.0f);     // src/visual_odometry.cpp:173-201
}

}  // namespace Simple_ORB_SLAM
