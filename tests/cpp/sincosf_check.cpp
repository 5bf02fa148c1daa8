// tests/cpp/sincosf_check.cpp -- TEST: lorb_sincosf.h (the device restatement of libm's cosf / sinf)
// against this machine's libm for every float angle the ORB descriptor forms: (float)deg * factorPI
// for every float deg in [0, 360) (src/ORBextractor.cpp:109, 114-115).  Prints the mismatch count.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../lorb_slam_amd/csrc/lorb_sincosf.h"

int main() {
  const float factorPI = (float)(3.14159265358979323846 / 180.f);
  float lim = 360.0f;
  uint32_t end;
  memcpy(&end, &lim, 4);
  const int T = 8;
  std::vector<long> bad(T, 0), cnt(T, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < T; t++)
    th.emplace_back([&, t] {
      long b = 0, c = 0;
      for (uint32_t u = t; u < end; u += T) {
        float deg;
        memcpy(&deg, &u, 4);
        const float a = deg * factorPI;
        b += (cosf(a) != lorb_cosf(a)) + (sinf(a) != lorb_sinf(a));
        c++;
      }
      bad[t] = b;
      cnt[t] = c;
    });
  for (auto& x : th) x.join();
  long b = 0, n = 0;
  for (int t = 0; t < T; t++) { b += bad[t]; n += cnt[t]; }
  printf("angles %ld mismatches %ld\n", n, b);
  return b != 0;
}
