// Micro: does a kernel take a large by-value argument (the pose-only inputs of a small batch), and
// what does a launch + sync cost with it?  hipcc --offload-arch=gfx950 -O3 kernarg.hip -o kernarg
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
template <int N>
struct Big { float v[N]; };
template <int N>
__global__ void k_sum(Big<N> a, float* out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += 64) s += a.v[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  if (threadIdx.x == 0) *out = s;
}
template <int N>
void run(float* d, float* h) {
  Big<N> a;
  for (int i = 0; i < N; ++i) a.v[i] = (float)(i % 7);
  double want = 0;
  for (int i = 0; i < N; ++i) want += a.v[i];
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int w = 0; w < 20; ++w) { hipLaunchKernelGGL(k_sum<N>, dim3(1), dim3(64), 0, s, a, d); (void)hipStreamSynchronize(s); }
  const int reps = 200;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) {
    a.v[r % N] += 1.0f; a.v[r % N] -= 1.0f;
    hipLaunchKernelGGL(k_sum<N>, dim3(1), dim3(64), 0, s, a, d);
    (void)hipStreamSynchronize(s);
  }
  auto t1 = std::chrono::steady_clock::now();
  (void)hipMemcpy(h, d, 4, hipMemcpyDeviceToHost);
  hipError_t e = hipGetLastError();
  printf("bytes %6d: launch+sync %.2f us, result %.1f (want %.1f), err %s\n", (int)sizeof(a),
         std::chrono::duration<double, std::micro>(t1 - t0).count() / reps, *h, want, hipGetErrorString(e));
  (void)hipStreamDestroy(s);
}
int main() {
  float *d, h = 0;
  (void)hipMalloc(&d, 4);
  run<16>(d, &h);
  run<1000>(d, &h);
  run<2000>(d, &h);
  run<4000>(d, &h);
  run<7000>(d, &h);
  return 0;
}
