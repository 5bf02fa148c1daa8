// micro: v_mfma_f64_16x16x4f64 issue rate / dependent latency on one wave (cycles per MFMA)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
template <int IND>
__global__ void k(double* out, unsigned long long* cyc, int iters) {
  v4d acc[IND];
  for (int q = 0; q < IND; ++q) acc[q] = v4d{0.0, 0.0, 0.0, (double)q};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int q = 0; q < IND; ++q) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
  double s = 0;
  for (int q = 0; q < IND; ++q) s += acc[q][0] + acc[q][3];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
// VALU f64 FMA rate for comparison
__global__ void kv(double* out, unsigned long long* cyc, int iters) {
  double x[8];
  for (int q = 0; q < 8; ++q) x[q] = q;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = fma(x[q], b, a);
  double s = 0;
  for (int q = 0; q < 8; ++q) s += x[q];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int IND>
void run(double* o, unsigned long long* c, int threads) {
  const int it = 2000;
  k<IND><<<1, threads>>>(o, c, it);
  k<IND><<<1, threads>>>(o, c, it);
  unsigned long long h;
  hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("mfma f64 16x16x4: %d independent chains, %4d threads: %.1f memtime ticks per MFMA per wave\n", IND, threads,
         (double)h / (it * IND));
}
int main() {
  double* o; unsigned long long* c;
  hipMalloc(&o, 1 << 20); hipMalloc(&c, 4096);
  run<1>(o, c, 64); run<2>(o, c, 64); run<4>(o, c, 64); run<8>(o, c, 64);
  run<4>(o, c, 256); run<4>(o, c, 512);
  kv<<<1, 64>>>(o, c, 2000); kv<<<1, 64>>>(o, c, 2000);
  unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("valu f64 fma, 8 chains, 64 threads: %.2f ticks per FMA\n", (double)h / (2000 * 8));
  // memtime tick vs shader clock: a 1M-iteration s_nop-free loop is not needed; report wall time too
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  k<8><<<1, 64>>>(o, c, 200000);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("1.6M MFMA (8 chains): %.3f ms wall, %llu ticks -> %.1f MHz tick, %.2f ns per MFMA\n", ms, h, h / (ms * 1e3), ms * 1e6 / 1.6e6);
  return 0;
}
