// micro: the bsg_tiles step pattern (NTL tiles: 4 chained MFMAs for y, 12 more using y as the B
// operand, the window shift by register moves), one wave, ticks per MFMA
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
template <int NTL, bool SHIFT>
__global__ void k(double* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x;
  double xa[4], la[3][4];
  for (int st = 0; st < 4; ++st) { xa[st] = 1e-3 * (lane + st); for (int t = 0; t < 3; ++t) la[t][st] = -1e-4 * (lane + t); }
  v4d acc[NTL][4];
  for (int q = 0; q < NTL; ++q) for (int t = 0; t < 4; ++t) acc[q][t] = v4d{1e-3 * q, 0.5, 0.25, 1e-3 * t};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    v4d y[NTL];
#pragma unroll
    for (int q = 0; q < NTL; ++q) {
      y[q] = v4d{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int st = 0; st < 4; ++st) y[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[st], acc[q][3][st], y[q], 0, 0, 0);
    }
#pragma unroll
    for (int t = 2; t >= 0; --t)
#pragma unroll
      for (int q = 0; q < NTL; ++q)
#pragma unroll
        for (int st = 0; st < 4; ++st) acc[q][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(la[t][st], y[q][st], acc[q][t], 0, 0, 0);
    if (SHIFT) {
#pragma unroll
      for (int q = 0; q < NTL; ++q) {
        acc[q][3] = acc[q][2] + y[q]; acc[q][2] = acc[q][1]; acc[q][1] = acc[q][0]; acc[q][0] = v4d{0.0, 0.0, 0.0, 0.0};
      }
    } else {
#pragma unroll
      for (int q = 0; q < NTL; ++q) acc[q][3] = acc[q][2] + y[q];
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int q = 0; q < NTL; ++q) for (int t = 0; t < 4; ++t) s += acc[q][t][0] + acc[q][t][3];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int NTL, bool SHIFT>
void run(double* o, unsigned long long* c) {
  const int it = 1000;
  k<NTL, SHIFT><<<1, 64>>>(o, c, it);
  k<NTL, SHIFT><<<1, 64>>>(o, c, it);
  unsigned long long h = 0;
  (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("NTL %d shift %d: %.1f ticks per step, %.1f per MFMA\n", NTL, (int)SHIFT, (double)h / it, (double)h / (it * 16.0 * NTL));
}
int main() {
  double* o; unsigned long long* c;
  (void)hipMalloc(&o, 1 << 20); (void)hipMalloc(&c, 4096);
  run<1, true>(o, c); run<2, true>(o, c); run<3, true>(o, c);
  run<1, false>(o, c); run<3, false>(o, c);
  return 0;
}
