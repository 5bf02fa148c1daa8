// fetch_cal.hip -- calibration of rocprofv3's FETCH_SIZE on gfx950 for the access patterns of the
// BA kernels (diagnostic, not part of liblorb.so).  Every kernel reads each byte of a 96 MB buffer
// exactly once (a 384 MB sweep of another buffer in between evicts L2 and the Infinity Cache), so
// the known byte count divided by FETCH_SIZE (KiB -> bytes) is the correction of that pattern:
//   stream16  16 B per lane, consecutive lanes consecutive (global_load_dwordx4): the guide's case
//   stream8   8 B per lane, consecutive
//   rec96     one 96-byte record per lane (12 doubles, the Schur / lin tile shape) at a permuted
//             record index (records gathered in random order, each once)
//   rec48     one 48-byte record per lane (6 doubles: obs_Q / obs_Jps), permuted
//   line8     8 B per lane, one per 64-byte line, lines in permuted order (scattered scalars)
// and for WRITE_SIZE: wstream16 (16 B per lane, consecutive), wrec96 / wrec48 (one 96- / 48-byte
// record per lane at a permuted slot: the camera-major tiles k_ba_lin writes from point-major threads)
//   hipcc -O3 --offload-arch=gfx950 tools/micro/fetch_cal.hip -o tools/micro/fetch_cal
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o fc --output-format csv -- tools/micro/fetch_cal
#include <hip/hip_runtime.h>

#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr size_t kBytes = 96u << 20;

__global__ void k_stream16(const double2* __restrict__ a, size_t n, double* __restrict__ sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) { const double2 v = a[i]; s += v.x + v.y; }
  if (s == 12345.678) sink[0] = s;
}
__global__ void k_stream8(const double* __restrict__ a, size_t n, double* __restrict__ sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 12345.678) sink[0] = s;
}
template <int R>
__global__ void k_rec(const double* __restrict__ a, const int* __restrict__ perm, size_t nrec, double* __restrict__ sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nrec; i += (size_t)gridDim.x * 256) {
    const double* r = a + (size_t)perm[i] * R;
#pragma unroll
    for (int k = 0; k < R; ++k) s += r[k];
  }
  if (s == 12345.678) sink[0] = s;
}
__global__ void k_line8(const double* __restrict__ a, const int* __restrict__ perm, size_t nline, double* __restrict__ sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nline; i += (size_t)gridDim.x * 256) s += a[(size_t)perm[i] * 8];
  if (s == 12345.678) sink[0] = s;
}
__global__ void k_wstream16(double2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = double2{1.0, (double)i};
}
template <int R>
__global__ void k_wrec(double* __restrict__ a, const int* __restrict__ perm, size_t nrec) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < nrec; i += (size_t)gridDim.x * 256) {
    double* r = a + (size_t)perm[i] * R;
#pragma unroll
    for (int k = 0; k < R; ++k) r[k] = (double)(i + k);
  }
}
__global__ void k_evict(const double2* __restrict__ a, size_t n, double* __restrict__ sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i].x;
  if (s == 12345.678) sink[0] = s;
}

int main() {
  double *a, *ev, *sink;
  int* perm;
  const size_t evb = 384u << 20;
  CK(hipMalloc(&a, kBytes));
  CK(hipMalloc(&ev, evb));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, kBytes));
  CK(hipMemset(ev, 0, evb));
  const size_t nmax = kBytes / 48;
  CK(hipMalloc(&perm, sizeof(int) * nmax));
  std::mt19937 rng(7);
  auto upload_perm = [&](size_t n) -> int {
    std::vector<int> p(n);
    std::iota(p.begin(), p.end(), 0);
    std::shuffle(p.begin(), p.end(), rng);
    CK(hipMemcpy(perm, p.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    return 0;
  };
  const dim3 g(4096), b(256);
  auto evict = [&] { hipLaunchKernelGGL(k_evict, g, b, 0, 0, (const double2*)ev, evb / 16, sink); };
  for (int rep = 0; rep < 2; ++rep) {
    evict();
    hipLaunchKernelGGL(k_stream16, g, b, 0, 0, (const double2*)a, kBytes / 16, sink);
    evict();
    hipLaunchKernelGGL(k_stream8, g, b, 0, 0, a, kBytes / 8, sink);
    if (upload_perm(kBytes / 96)) return 1;
    evict();
    hipLaunchKernelGGL(k_rec<12>, g, b, 0, 0, a, perm, kBytes / 96, sink);
    if (upload_perm(kBytes / 48)) return 1;
    evict();
    hipLaunchKernelGGL(k_rec<6>, g, b, 0, 0, a, perm, kBytes / 48, sink);
    if (upload_perm(kBytes / 64)) return 1;
    evict();
    hipLaunchKernelGGL(k_line8, g, b, 0, 0, a, perm, kBytes / 64, sink);
    evict();
    hipLaunchKernelGGL(k_wstream16, g, b, 0, 0, (double2*)a, kBytes / 16);
    if (upload_perm(kBytes / 96)) return 1;
    evict();
    hipLaunchKernelGGL(k_wrec<12>, g, b, 0, 0, a, perm, kBytes / 96);
    if (upload_perm(kBytes / 48)) return 1;
    evict();
    hipLaunchKernelGGL(k_wrec<6>, g, b, 0, 0, a, perm, kBytes / 48);
    CK(hipDeviceSynchronize());
  }
  // the unique bytes of each kernel (line8 touches every 64-byte line once: a line's bytes)
  printf("known bytes: stream16 %zu stream8 %zu rec96 %zu rec48 %zu line8 %zu (lines) / %zu (used)\n", kBytes, kBytes,
         kBytes / 96 * 96, kBytes / 48 * 48, kBytes, kBytes / 8);
  return 0;
}
