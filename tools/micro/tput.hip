// micro-benchmark: VALU issue throughput of v_xor_b32 vs v_bcnt_u32_b32 (8 independent chains per
// wave, 8 waves per SIMD over the whole chip); reports SIMD-cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed) {
  unsigned r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 2654435761u + i * seed;
  for (int it = 0; it < 4096; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r[i]) : "v"(r[(i + 1) & 7]));
      if (MODE == 1) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(r[i]) : "v"(r[(i + 1) & 7]));
      if (MODE == 2) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r[i]) : "v"(r[(i + 1) & 7]));
      if (MODE == 3) asm volatile("v_min_u32 %0, %1, %0" : "+v"(r[i]) : "v"(r[(i + 1) & 7]));
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += r[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU -> 8 waves per SIMD
  unsigned* o; hipMalloc(&o, sizeof(unsigned) * blocks * 256);
  const char* names[] = {"v_xor_b32", "v_bcnt_u32_b32", "v_add_u32", "v_min_u32"};
  for (int m = 0; m < 4; ++m) {
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (m == 0) k<0><<<blocks, 256>>>(o, 7);
      if (m == 1) k<1><<<blocks, 256>>>(o, 7);
      if (m == 2) k<2><<<blocks, 256>>>(o, 7);
      if (m == 3) k<3><<<blocks, 256>>>(o, 7);
      hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    // wave-instructions per SIMD = 8 waves * 4096 * 8
    const double instr = 8.0 * 4096 * 8;
    printf("%-16s %.3f ms  SIMD-cycles per wave-instruction at 2.4 GHz: %.2f\n", names[m], ms,
           ms * 1e-3 * 2.4e9 / instr);
  }
  return 0;
}
