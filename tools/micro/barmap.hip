// Micro: can the host write device memory directly (fine-grained VRAM through the BAR), and does a
// kernel then read its inputs faster than from mapped pinned host memory?
// hipcc --offload-arch=gfx950 -O3 barmap.hip -o barmap
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>
#include <cstring>
__global__ void k_sum(const float4* __restrict__ in, int n, float* out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) { const float4 v = in[i]; s += v.x + v.y + v.z + v.w; }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
  __shared__ float w[4];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = w[0] + w[1] + w[2] + w[3];
}
static double bench(const char* name, float* hostw, const float4* devr, int n4, float* dout, hipStream_t st, hipEvent_t ev) {
  const int reps = 300;
  double best = 1e9, sum = 0;
  for (int r = 0; r < reps + 20; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 4 * n4; ++i) hostw[i] = (float)((i + r) % 5);
    hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, st, devr, n4, dout);
    (void)hipEventRecord(ev, st);
    while (hipEventQuery(ev) == hipErrorNotReady) {}
    auto t1 = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    if (r >= 20) { sum += us; best = us < best ? us : best; }
  }
  printf("%-44s mean %.2f us  best %.2f us\n", name, sum / reps, best);
  return sum / reps;
}
int main() {
  const int n4 = 256;  // 4 KB
  hipStream_t st; (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev; (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  float* dout; (void)hipMalloc(&dout, 4);
  int lb = 0;
  (void)hipDeviceGetAttribute(&lb, hipDeviceAttributeCanMapHostMemory, 0);
  printf("canMapHostMemory %d\n", lb);
  // 1. mapped pinned host memory (what the pose-only call reads today)
  float* h = nullptr; void* hd = nullptr;
  (void)hipHostMalloc((void**)&h, 4096 * 4, hipHostMallocMapped | hipHostMallocCoherent);
  (void)hipHostGetDevicePointer(&hd, h, 0);
  bench("kernel reads mapped pinned host memory", h, (const float4*)hd, n4, dout, st, ev);
  // 2. fine-grained device memory: host-accessible?
  float* f = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&f, 4096 * 4, hipDeviceMallocFinegrained);
  hipPointerAttribute_t at;
  memset(&at, 0, sizeof(at));
  hipError_t e2 = f ? hipPointerGetAttributes(&at, f) : hipErrorInvalidValue;
  printf("finegrained alloc %s, attrs %s, hostPointer %p devicePointer %p type %d\n", hipGetErrorString(e),
         hipGetErrorString(e2), at.hostPointer, at.devicePointer, (int)at.type);
  if (e == hipSuccess && at.hostPointer) {
    bench("host writes fine-grained VRAM, kernel reads", (float*)at.hostPointer, (const float4*)f, n4, dout, st, ev);
  } else {
    printf("fine-grained VRAM not host-mapped: skipped\n");
  }
  // 3. plain device memory + hipMemcpyAsync H2D from pinned (reference)
  float* dd; (void)hipMalloc(&dd, 4096 * 4);
  {
    const int reps = 300; double sum = 0;
    for (int r = 0; r < reps + 20; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 4 * n4; ++i) h[i] = (float)((i + r) % 5);
      (void)hipMemcpyAsync(dd, h, 4096, hipMemcpyHostToDevice, st);
      hipLaunchKernelGGL(k_sum, dim3(1), dim3(256), 0, st, (const float4*)dd, n4, dout);
      (void)hipEventRecord(ev, st);
      while (hipEventQuery(ev) == hipErrorNotReady) {}
      auto t1 = std::chrono::steady_clock::now();
      if (r >= 20) sum += std::chrono::duration<double, std::micro>(t1 - t0).count();
    }
    printf("%-44s mean %.2f us\n", "pinned H2D copy + kernel", sum / reps);
  }
  return 0;
}
