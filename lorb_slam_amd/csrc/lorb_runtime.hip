// lorb_runtime.hip -- context, memory and timer entry points of the C-ABI (include/lorb_c.h).
#include "lorb_internal.h"

#include <algorithm>

namespace lorb {

int set_error(lorb_ctx* ctx, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

static int scratch_alloc(lorb_ctx* ctx, int slot, size_t bytes, void** out) {
  if (slot < 0 || slot >= lorb_ctx::kScratch) return set_error(ctx, LORB_E_INVALID, "bad scratch slot %d", slot);
  if (bytes == 0) bytes = 16;
  if (ctx->scratch_sz[slot] < bytes) {
    ctx->up_mirror[slot].clear();
    if (ctx->scratch[slot]) {
      LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
      LORB_HIP(ctx, hipFree(ctx->scratch[slot]));
      ctx->scratch[slot] = nullptr;
      ctx->scratch_sz[slot] = 0;
    }
    size_t want = bytes + bytes / 4;
    LORB_HIP(ctx, hipMalloc(&ctx->scratch[slot], want));
    ctx->scratch_sz[slot] = want;
  }
  *out = ctx->scratch[slot];
  return LORB_OK;
}

int scratch(lorb_ctx* ctx, int slot, size_t bytes, void** out) {
  LORB_TRY(scratch_alloc(ctx, slot, bytes, out));
  ctx->up_mirror[slot].clear();  // kernels may write it: the uploaded bytes are no longer known
  return LORB_OK;
}

int upload(lorb_ctx* ctx, int slot, const void* host, size_t bytes, void** dev) {
  LORB_TRY(scratch_alloc(ctx, slot, bytes, dev));
  if (!bytes) return LORB_OK;
  std::vector<unsigned char>& m = ctx->up_mirror[slot];
  if (m.size() == bytes && std::memcmp(m.data(), host, bytes) == 0) return LORB_OK;  // already resident
  LORB_HIP(ctx, hipMemcpyAsync(*dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
  m.assign(static_cast<const unsigned char*>(host), static_cast<const unsigned char*>(host) + bytes);
  return LORB_OK;
}

// coherent + mapped: kernels read (InPack) and write (OutPack direct) it over PCIe, uncached on the
// GPU side, so a call never sees a line of an earlier call's staging
static int pinned_grow(lorb_ctx* ctx, void** p, void** pdev, size_t* sz, size_t want) {
  if (*sz >= want) return LORB_OK;
  if (*p) {
    LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));  // no pull / direct write still in flight
    (void)hipHostFree(*p);
  }
  *p = nullptr; *pdev = nullptr; *sz = 0;
  want += want / 4;
  want = (want + 255) & ~size_t(255);
  LORB_HIP(ctx, hipHostMalloc(p, want, hipHostMallocMapped | hipHostMallocCoherent));
  LORB_HIP(ctx, hipHostGetDevicePointer(pdev, *p, 0));
  *sz = want;
  return LORB_OK;
}

// InPack's host-to-device move: 16-byte loads of the mapped staging (each lane one PCIe read in
// flight per iteration), stores into the device block
__global__ __launch_bounds__(256) void k_io_pull(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

int InPack::commit(bool mapped) {
  if (!total) return LORB_OK;
  // a call that failed after its commit may have left its copy in flight
  // every host-array call ends waiting for its stream (OutPack::fetch); only a call that failed
  // after its commit can leave a pull in flight
  if (ctx->io_pending) LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  LORB_TRY(pinned_grow(ctx, &ctx->io_in, &ctx->io_in_dev, &ctx->io_in_sz, total));
  unsigned char* h = static_cast<unsigned char*>(ctx->io_in);
  for (const Part& p : parts)
    if (p.bytes) std::memcpy(h + p.off, p.host, p.bytes);
  if (mapped) {
    base = ctx->io_in_dev;
    ctx->io_pending = true;
    return LORB_OK;
  }
  LORB_TRY(scratch(ctx, S_IO_IN, total, &base));
  size_t used = 0;
  for (const Part& p : parts) used = std::max(used, p.off + p.bytes);
  const size_t n16 = (used + 15) / 16;  // total is 256-aligned: the rounded tail stays inside
  if (n16) {
    const unsigned g = (unsigned)std::min<size_t>((n16 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_io_pull, dim3(g), dim3(256), 0, ctx->stream, static_cast<const uint4*>(ctx->io_in_dev),
                       static_cast<uint4*>(base), n16);
    LORB_CHECK_LAUNCH(ctx);
  }
  ctx->io_pending = true;
  return LORB_OK;
}

int OutPack::alloc(bool direct_) {
  direct = direct_;
  LORB_TRY(pinned_grow(ctx, &ctx->io_out, &ctx->io_out_dev, &ctx->io_out_sz, std::max<size_t>(total, 16)));
  hbase = ctx->io_out;
  if (direct) dbase = ctx->io_out_dev;
  else LORB_TRY(scratch(ctx, S_IO_OUT, std::max<size_t>(total, 16), &dbase));
  return LORB_OK;
}

int OutPack::fetch() {
  size_t used = 0;
  for (const Part& p : parts) used = std::max(used, p.off + p.bytes);
  if (used && !direct) LORB_HIP(ctx, hipMemcpyAsync(hbase, dbase, used, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, spin_sync(ctx));
  ctx->io_pending = false;
  return LORB_OK;
}

static hipEvent_t pool_get(lorb_ctx* ctx) {
  if (!ctx->kev_pool.empty()) { hipEvent_t e = ctx->kev_pool.back(); ctx->kev_pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

KernelTimer::KernelTimer(lorb_ctx* c, int kid) : ctx(c), k(kid) {
  if (!ctx->ktime || k < 0 || k >= LORB_K_COUNT) return;
  b = pool_get(ctx); e = pool_get(ctx);
  if (b) (void)hipEventRecord(b, ctx->stream);
}
KernelTimer::~KernelTimer() {
  if (!b || !e) return;
  (void)hipEventRecord(e, ctx->stream);
  ctx->kev[k].emplace_back(b, e);
}

}  // namespace lorb

using namespace lorb;

extern "C" {

int lorb_abi_version(void) { return LORB_ABI_VERSION; }

int lorb_device_count(int* count) {
  if (!count) return LORB_E_INVALID;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *count = 0; return LORB_E_DEVICE; }
  *count = n;
  return LORB_OK;
}

int lorb_create(int device, lorb_ctx** out) {
  if (!out) return LORB_E_INVALID;
  *out = nullptr;
  lorb_ctx* ctx = new (std::nothrow) lorb_ctx();
  if (!ctx) return LORB_E_NOMEM;
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
  for (int i = 0; i < 64 && e == hipSuccess; i++) e = hipEventCreate(&ctx->ev[i]);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->spin_ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    delete ctx;
    return LORB_E_DEVICE;
  }
  *out = ctx;
  return LORB_OK;
}

int lorb_destroy(lorb_ctx* ctx) {
  if (!ctx) return LORB_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->solver) (void)lorb_ba_solver_destroy(ctx->solver);  // its plans use the ctx's stream
  ctx->solver = nullptr;
  for (int i = 0; i < lorb_ctx::kScratch; i++)
    if (ctx->scratch[i]) (void)hipFree(ctx->scratch[i]);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  if (ctx->io_in) (void)hipHostFree(ctx->io_in);
  if (ctx->io_out) (void)hipHostFree(ctx->io_out);
  for (int i = 0; i < 64; i++)
    if (ctx->ev[i]) (void)hipEventDestroy(ctx->ev[i]);
  if (ctx->spin_ev) (void)hipEventDestroy(ctx->spin_ev);
  for (int k = 0; k < LORB_K_COUNT; k++)
    for (auto& pr : ctx->kev[k]) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
  for (auto e : ctx->kev_pool) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return LORB_OK;
}

const char* lorb_last_error(const lorb_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int lorb_sync(lorb_ctx* ctx) {
  if (!ctx) return LORB_E_INVALID;
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_malloc(lorb_ctx* ctx, void** dptr, size_t bytes) {
  if (!ctx || !dptr) return LORB_E_INVALID;
  LORB_HIP(ctx, hipMalloc(dptr, bytes ? bytes : 16));
  return LORB_OK;
}

int lorb_free(lorb_ctx* ctx, void* dptr) {
  if (!ctx) return LORB_E_INVALID;
  if (dptr) LORB_HIP(ctx, hipFree(dptr));
  return LORB_OK;
}

int lorb_memcpy_h2d(lorb_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return LORB_E_INVALID;
  if (!bytes) return LORB_OK;
  LORB_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_memcpy_d2h(lorb_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (!ctx) return LORB_E_INVALID;
  if (!bytes) return LORB_OK;
  LORB_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

int lorb_memset_dev(lorb_ctx* ctx, void* dst, int value, size_t bytes) {
  if (!ctx) return LORB_E_INVALID;
  if (!bytes) return LORB_OK;
  LORB_HIP(ctx, hipMemsetAsync(dst, value, bytes, ctx->stream));
  return LORB_OK;
}

int lorb_timer_mark(lorb_ctx* ctx, int slot) {
  if (!ctx || slot < 0 || slot >= 64) return LORB_E_INVALID;
  LORB_HIP(ctx, hipEventRecord(ctx->ev[slot], ctx->stream));
  return LORB_OK;
}

int lorb_timer_elapsed_ms(lorb_ctx* ctx, int a, int b, float* ms) {
  if (!ctx || !ms || a < 0 || a >= 64 || b < 0 || b >= 64) return LORB_E_INVALID;
  LORB_HIP(ctx, hipEventSynchronize(ctx->ev[b]));
  LORB_HIP(ctx, hipEventElapsedTime(ms, ctx->ev[a], ctx->ev[b]));
  return LORB_OK;
}

int lorb_kernel_timing_enable(lorb_ctx* ctx, int enable) {
  if (!ctx) return LORB_E_INVALID;
  ctx->ktime = enable != 0;
  return LORB_OK;
}

int lorb_kernel_timing_read(lorb_ctx* ctx, int k, double* total_ms, int* launches) {
  if (!ctx || k < 0 || k >= LORB_K_COUNT || !total_ms || !launches) return LORB_E_INVALID;
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  double tot = 0.0;
  for (auto& pr : ctx->kev[k]) {
    float ms = 0.f;
    LORB_HIP(ctx, hipEventElapsedTime(&ms, pr.first, pr.second));
    tot += ms;
    ctx->kev_pool.push_back(pr.first);
    ctx->kev_pool.push_back(pr.second);
  }
  *launches = (int)ctx->kev[k].size();
  ctx->kev[k].clear();
  *total_ms = tot;
  return LORB_OK;
}

void lorb_lm_options_default(lorb_lm_options* o) {
  if (!o) return;
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
}

}  // extern "C"
