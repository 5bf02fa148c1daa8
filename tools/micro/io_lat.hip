// io_lat.hip -- round-trip latency of the ways a per-frame C-ABI call can move ~30 KB in and ~2 KB
// out (diagnostic for the C1 host calls; not part of liblorb.so).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/io_lat.hip -o tools/micro/io_lat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && p) p[0] += 1; }
struct BigArgs { int v[200]; };
__global__ void k_bigargs(int* p, BigArgs a) { if (threadIdx.x == 0 && p) p[0] += a.v[threadIdx.x]; }

// one workgroup: copy `n` dwords from (mapped host) src to dst, then write `m` dwords back to out
__global__ __launch_bounds__(1024) void k_inout(const int* __restrict__ src, int* __restrict__ dev, int n,
                                                int* __restrict__ out, int m) {
  int acc = 0;
  for (int i = threadIdx.x; i < n; i += 1024) { const int v = src[i]; dev[i] = v; acc += v; }
  __syncthreads();
  for (int i = threadIdx.x; i < m; i += 1024) out[i] = acc + i;
}

static void spin(hipEvent_t ev, hipStream_t s) {
  (void)hipEventRecord(ev, s);
  while (hipEventQuery(ev) == hipErrorNotReady) {
  }
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int IN = 30 * 1024, OUT = 2 * 1024;
  int *d_in, *d_out, *h_pin_in, *h_pin_out;
  CK(hipMalloc(&d_in, IN));
  CK(hipMalloc(&d_out, OUT));
  CK(hipHostMalloc(&h_pin_in, IN));
  CK(hipHostMalloc(&h_pin_out, OUT));
  std::vector<int> pg_in(IN / 4, 1), pg_out(OUT / 4);
  auto bench = [&](const char* name, auto fn) {
    for (int i = 0; i < 50; ++i) fn();
    std::vector<double> t;
    for (int i = 0; i < 400; ++i) {
      const auto a = std::chrono::steady_clock::now();
      fn();
      t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    std::sort(t.begin(), t.end());
    printf("%-58s median %7.2f us  p10 %7.2f  p90 %7.2f\n", name, t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
  };
  bench("empty kernel + hipStreamSynchronize", [&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr); (void)hipStreamSynchronize(s); });
  bench("empty kernel + event spin", [&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr); spin(ev, s); });
  bench("empty kernel + hipStreamQuery spin", [&] {
    hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
  });
  bench("hipEventRecord only", [&] { (void)hipEventRecord(ev, s); });
  (void)hipStreamSynchronize(s);
  bench("5 empty kernels + event spin", [&] { for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr); spin(ev, s); });
  bench("pinned H2D 30KB + event spin", [&] { (void)hipMemcpyAsync(d_in, h_pin_in, IN, hipMemcpyHostToDevice, s); spin(ev, s); });
  bench("pageable H2D 30KB + event spin", [&] { (void)hipMemcpyAsync(d_in, pg_in.data(), IN, hipMemcpyHostToDevice, s); spin(ev, s); });
  bench("pinned D2H 2KB + event spin", [&] { (void)hipMemcpyAsync(h_pin_out, d_out, OUT, hipMemcpyDeviceToHost, s); spin(ev, s); });
  bench("pageable D2H 2KB + event spin", [&] { (void)hipMemcpyAsync(pg_out.data(), d_out, OUT, hipMemcpyDeviceToHost, s); spin(ev, s); });
  bench("pinned H2D + kernel + pinned D2H + spin", [&] {
    (void)hipMemcpyAsync(d_in, h_pin_in, IN, hipMemcpyHostToDevice, s);
    hipLaunchKernelGGL(k_inout, 1, 1024, 0, s, d_in, d_in, IN / 4, d_out, OUT / 4);
    (void)hipMemcpyAsync(h_pin_out, d_out, OUT, hipMemcpyDeviceToHost, s);
    spin(ev, s);
  });
  bench("kernel reads mapped host, writes mapped host + spin", [&] {
    hipLaunchKernelGGL(k_inout, 1, 1024, 0, s, h_pin_in, d_in, IN / 4, h_pin_out, OUT / 4);
    spin(ev, s);
  });
  bench("kernel mapped in/out + 4 empty kernels + spin", [&] {
    hipLaunchKernelGGL(k_inout, 1, 1024, 0, s, h_pin_in, d_in, IN / 4, h_pin_out, OUT / 4);
    for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr);
    spin(ev, s);
  });
  bench("host memcpy 30KB into pinned", [&] { memcpy(h_pin_in, pg_in.data(), IN); });
  // host-side cost of reading a 50 x 50 int matrix column-wise (the device plan build's covisibility
  // fill) from pinned vs pageable memory, and of one launch with 800 bytes of arguments
  {
    int* hp = nullptr;
    CK(hipHostMalloc(&hp, 4 * 2600));
    std::vector<int> pv(2600, 1);
    for (int i = 0; i < 2600; ++i) hp[i] = 1;
    volatile int sink = 0;
    auto colsum = [&](const int* m) { int s = 0; for (int i = 0; i < 50; ++i) for (int j = i + 1; j < 50; ++j) s += m[j * 50 + i]; sink = s; };
    bench("column walk of 50x50 ints, pinned", [&] { colsum(hp); });
    bench("column walk of 50x50 ints, pageable", [&] { colsum(pv.data()); });
    BigArgs ba{};
    bench("launch only (8-byte args)", [&] { hipLaunchKernelGGL(k_empty, 1, 64, 0, s, nullptr); });
    (void)hipStreamSynchronize(s);
    bench("launch only (808-byte args)", [&] { hipLaunchKernelGGL(k_bigargs, 1, 64, 0, s, nullptr, ba); });
    (void)hipStreamSynchronize(s);
    (void)hipHostFree(hp);
  }
  return 0;
}
