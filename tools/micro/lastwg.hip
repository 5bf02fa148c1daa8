// lastwg.hip -- cost of a "last workgroup finishes the launch" tail against a second launch
// (diagnostic for folding a one-wave kernel such as k_ba_lm_end into the kernel before it; not part
// of liblorb.so).  N workgroups each write `kw` doubles per thread (the point-group outputs) and one
// partial; then either
//   (a) a second one-wave launch sums the partials, or
//   (b) every workgroup bumps a counter with an agent-scope release RMW and the last one (acquire)
//       sums the partials in the same launch,
//   (c) as (b) with a relaxed RMW after a workgroup-scope release fence and s_waitcnt only (no L2
//       write-back; the partials written with agent-scope relaxed atomic stores, the reader using
//       agent-scope relaxed atomic loads),
// in a captured graph of back-to-back iterations.  Prints the wall time per iteration and checks
// the sums.
//   hipcc -O3 --offload-arch=gfx950 tools/micro/lastwg.hip -o tools/micro/lastwg
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kW = 8;  // doubles written per thread (the bulk output)

__device__ __forceinline__ double wg_sum(double v, double* sh) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += sh[k];
  return s;
}

// the producer: bulk output + one partial per workgroup
template <int MODE>
__global__ __launch_bounds__(256) void k_prod(double* __restrict__ bulk, double* part, unsigned* cnt, double* out,
                                              int it) {
  __shared__ double sh[4];
  __shared__ int s_last;
  const int g = blockIdx.x, t = threadIdx.x;
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < kW; ++k) {
    const double x = (double)(g + t + k + it);
    bulk[((size_t)g * 256 + t) * kW + k] = x;
    v += x;
  }
  const double s = wg_sum(v, sh);
  if (MODE == 0) {
    if (t == 0) part[g] = s;
    return;
  }
  if (t == 0) {
    if (MODE == 1) {
      part[g] = s;
      const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == gridDim.x - 1;
    } else {
      __hip_atomic_store(part + g, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);
      const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == gridDim.x - 1;
    }
  }
  __syncthreads();
  if (!s_last || t >= 64) return;
  if (MODE == 1) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // (agent scope by default on the device)
  double a = 0.0;
  for (int k = t; k < (int)gridDim.x; k += 64)
    a += MODE == 1 ? part[k] : __hip_atomic_load(part + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (t == 0) { out[it] = a; *cnt = 0u; }
}

// the consumer of MODE 0: one wave sums the partials
__global__ __launch_bounds__(64) void k_cons(const double* __restrict__ part, int n, double* out, int it) {
  const int t = threadIdx.x;
  double a = 0.0;
  for (int k = t; k < n; k += 64) a += part[k];
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (t == 0) out[it] = a;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int G = 372, iters = 100;
  double *bulk, *part, *out;
  unsigned* cnt;
  CK(hipMalloc(&bulk, sizeof(double) * G * 256 * kW));
  CK(hipMalloc(&part, sizeof(double) * G));
  CK(hipMalloc(&out, sizeof(double) * iters));
  CK(hipMalloc(&cnt, sizeof(unsigned)));
  CK(hipMemset(cnt, 0, sizeof(unsigned)));
  double expect[iters];
  for (int it = 0; it < iters; ++it) {
    double e = 0.0;
    for (int g = 0; g < G; ++g)
      for (int t = 0; t < 256; ++t)
        for (int k = 0; k < kW; ++k) e += (double)(g + t + k + it);
    expect[it] = e;
  }
  for (int mode = 0; mode < 3; ++mode) {
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int it = 0; it < iters; ++it) {
      if (mode == 0) {
        hipLaunchKernelGGL(k_prod<0>, dim3(G), dim3(256), 0, s, bulk, part, cnt, out, it);
        hipLaunchKernelGGL(k_cons, dim3(1), dim3(64), 0, s, part, G, out, it);
      } else if (mode == 1) {
        hipLaunchKernelGGL(k_prod<1>, dim3(G), dim3(256), 0, s, bulk, part, cnt, out, it);
      } else {
        hipLaunchKernelGGL(k_prod<2>, dim3(G), dim3(256), 0, s, bulk, part, cnt, out, it);
      }
    }
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    double best = 1e30;
    for (int r = 0; r < 6; ++r) {
      CK(hipMemset(out, 0, sizeof(double) * iters));
      CK(hipStreamSynchronize(s));
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r > 0 && us < best) best = us;
    }
    double h[iters];
    CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int it = 0; it < iters; ++it) bad += h[it] != expect[it];
    printf("mode %d (%s): %.2f us per iteration, %d wrong sums\n", mode,
           mode == 0 ? "two launches" : mode == 1 ? "last workgroup, release / acquire" : "last workgroup, coherent atomics",
           best / iters, bad);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
  }
  return 0;
}
