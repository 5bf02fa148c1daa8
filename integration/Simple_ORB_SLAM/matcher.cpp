// Drop-in replacement of the reference's src/matcher.cpp: same class, same signatures
// (include/matcher.h:15-36), bodies routed through lorb/adapters.hpp -> liblorb.so (MI355X).
// Build: add this file instead of src/matcher.cpp, add -I<lorb>/include, link liblorb.so.
#include "../include/matcher.h"
#include "lorb_traits.hpp"

namespace Simple_ORB_SLAM {

const int Matcher::TH_HIGH = LORB_TH_HIGH;        // src/matcher.cpp:6
const int Matcher::TH_LOW = LORB_TH_LOW;          // src/matcher.cpp:7
const int Matcher::HISTO_LENGTH = LORB_HISTO_LENGTH;  // src/matcher.cpp:8

size_t Matcher::SearchByProjection(Frame* currFrame, Frame* prevFrame) {
  return lorb::SearchByProjectionBF(lorb::thread_ctx(), currFrame, prevFrame);
}

size_t Matcher::SearchByProjection(Frame* CurrentFrame, Frame* LastFrame, const float th) {
  return lorb::SearchByProjectionFrame(lorb::thread_ctx(), CurrentFrame, LastFrame, th);
}

size_t Matcher::SearchLocalPoints(Frame* currFrame, std::set<MapPoint*> vpMPs) {
  return lorb::SearchLocalPoints(lorb::thread_ctx(), currFrame, vpMPs);
}

size_t Matcher::SearchByProjection(Frame* F, const std::set<MapPoint*>& vpMapPoints, const float th) {
  return lorb::SearchByProjectionLocal(lorb::thread_ctx(), F, vpMapPoints, th);
}

// Host helpers keep the reference semantics (src/matcher.cpp:369-436)
int Matcher::DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
  const uint32_t* pa = a.ptr<uint32_t>();
  const uint32_t* pb = b.ptr<uint32_t>();
  int dist = 0;
  for (int i = 0; i < 8; i++) dist += __builtin_popcount(pa[i] ^ pb[i]);
  return dist;
}

float Matcher::RadiusByViewingCos(const float& viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

void Matcher::ComputeThreeMaxima(vector<int>* histo, const int L, int& ind1, int& ind2, int& ind3) {
  int max1 = 0, max2 = 0, max3 = 0;
  for (int i = 0; i < L; i++) {
    const int s = (int)histo[i].size();
    if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
    else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
    else if (s > max3) { max3 = s; ind3 = i; }
  }
  if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
  else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

}  // namespace Simple_ORB_SLAM
