// micro-benchmark: dependent-chain latency of FP64 VALU ops and v_readlane broadcasts (1 wave)
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffu), l);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
template <int MODE>
__global__ void k(double* out, unsigned long long* cyc, double a, double b) {
  double x = threadIdx.x * 1e-3 + a;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < 1024; ++i) {
    if (MODE == 0) x = fma(x, a, b);                       // dependent DP fma
    if (MODE == 1) x = readlane_d(x, i & 63) * a + b;      // readlane + fma chain
    if (MODE == 2) x = __shfl(x, (threadIdx.x + 1) & 63) * a + b;  // bpermute chain
    if (MODE == 3) { float f = (float)x; f = fmaf(f, (float)a, (float)b); x = f; }
    if (MODE == 4) x = __builtin_amdgcn_rsq(x * x + 1.0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main() {
  double* o; unsigned long long* c; hipMalloc(&o, 64 * 8); hipMalloc(&c, 8);
  const char* names[] = {"fma_f64", "readlane_d+fma", "shfl+fma", "fma_f32(cvt)", "rsq_f64+fma"};
  for (int m = 0; m < 5; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      unsigned long long h = 0;
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (m == 0) k<0><<<1, 64>>>(o, c, 0.999, 1e-3);
      if (m == 1) k<1><<<1, 64>>>(o, c, 0.999, 1e-3);
      if (m == 2) k<2><<<1, 64>>>(o, c, 0.999, 1e-3);
      if (m == 3) k<3><<<1, 64>>>(o, c, 0.999, 1e-3);
      if (m == 4) k<4><<<1, 64>>>(o, c, 0.999, 1e-3);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-16s memtime/iter %.1f   us/iter(event) %.4f\n", names[m], h / 1024.0, ms * 1e3 / 1024.0);
    }
  }
  return 0;
}
