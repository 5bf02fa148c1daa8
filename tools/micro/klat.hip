// klat.hip -- duration floor of small kernels in a captured graph (diagnostic for the LM
// iteration's one-wave / short launches; not part of liblorb.so).  A graph of back-to-back launches
// on one stream: empty one-wave kernels, one-wave kernels that chase N dependent loads through a
// buffer the previous launch wrote, and 372 x 512-thread launches doing the same per workgroup.
// Prints the wall time per launch of each graph; run under rocprofv3 --kernel-trace --stats for the
// per-kernel durations.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/klat.hip -o tools/micro/klat
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && p[1] < 0) p[0] = 1;  // one load, never a store
}
// N dependent loads (each index from the previous load), then one store the next launch reads
template <int N>
__global__ void k_chain(int* __restrict__ buf, int stride) {
  int i = (int)(blockIdx.x * 64 + (threadIdx.x & 63)) * 0;
#pragma unroll
  for (int k = 0; k < N; ++k) i = buf[(i + k * stride) & ((1 << 20) - 1)];
  if (threadIdx.x == 0) buf[(blockIdx.x * 977) & ((1 << 20) - 1)] = i & 0;  // keeps the chain (value 0)
}

template <typename F>
static double graph_us(hipStream_t s, int n, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeGlobal) != hipSuccess) return -1;
  for (int i = 0; i < n; ++i) launch(i);
  if (hipStreamEndCapture(s, &g) != hipSuccess) return -1;
  if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return -1;
  (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    best = us < best ? us : best;
  }
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  return best / n;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* buf;
  CK(hipMalloc(&buf, sizeof(int) << 20));
  CK(hipMemset(buf, 0, sizeof(int) << 20));
  const int n = 200;
  printf("empty 1x64:      %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, buf); }));
  printf("chain1 1x64:     %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, s, buf, 4099); }));
  printf("chain3 1x64:     %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, s, buf, 4099); }));
  printf("chain6 1x64:     %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<6>, dim3(1), dim3(64), 0, s, buf, 4099); }));
  printf("empty 372x512:   %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(372), dim3(512), 0, s, buf); }));
  printf("chain1 372x512:  %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<1>, dim3(372), dim3(512), 0, s, buf, 4099); }));
  printf("chain3 372x512:  %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<3>, dim3(372), dim3(512), 0, s, buf, 4099); }));
  printf("chain6 372x512:  %.2f us per launch\n", graph_us(s, n, [&](int) { hipLaunchKernelGGL(k_chain<6>, dim3(372), dim3(512), 0, s, buf, 4099); }));
  return 0;
}
