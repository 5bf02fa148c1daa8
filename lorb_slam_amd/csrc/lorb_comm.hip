// lorb_comm.hip -- multi-GPU communicator of the sharded local BA.
//
// One process per GPU.  The RCCL transport runs ncclAllReduce on the context's stream (xGMI on
// an MI355X node; stream-ordered and capturable in the LM hipGraph).  The host transport hands a
// staged copy to a caller-supplied all-reduce (used by the CPU-rendezvous tests, where several
// ranks may share one GPU and RCCL cannot run).
#include <rccl/rccl.h>

#include "lorb_internal.h"

namespace lorb {

static ncclRedOp_t nccl_op(int op) { return op == LORB_OP_MAX ? ncclMax : op == LORB_OP_MIN ? ncclMin : ncclSum; }

int comm_allreduce(lorb_comm* c, const double* d_send, double* d_recv, size_t n, int op) {
  lorb_ctx* ctx = c->ctx;
  if (n == 0) return LORB_OK;
  if (c->nranks == 1 && !c->rccl) {  // the identity (RCCL runs even over one rank: in place, no copy)
    if (d_send != d_recv)
      LORB_HIP(ctx, hipMemcpyAsync(d_recv, d_send, n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    return LORB_OK;
  }
  if (c->rccl) {
    const ncclResult_t r = ncclAllReduce(d_send, d_recv, n, ncclFloat64, nccl_op(op),
                                         static_cast<ncclComm_t>(c->nccl), ctx->stream);
    if (r != ncclSuccess) return set_error(ctx, LORB_E_COMM, "ncclAllReduce: %s", ncclGetErrorString(r));
    return LORB_OK;
  }
  if (c->pinned_n < n) {
    if (c->pinned) (void)hipHostFree(c->pinned);
    c->pinned = nullptr;
    c->pinned_n = 0;
    LORB_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&c->pinned), n * sizeof(double)));
    c->pinned_n = n;
  }
  LORB_HIP(ctx, hipMemcpyAsync(c->pinned, d_send, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  if (c->fn(c->user, c->pinned, (int64_t)n, op) != 0) return set_error(ctx, LORB_E_COMM, "host all-reduce callback failed");
  LORB_HIP(ctx, hipMemcpyAsync(d_recv, c->pinned, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return LORB_OK;
}

// host arrays (the plan builds' structure exchanges): over one rank the reduction is the identity;
// over RCCL through a grow-only device buffer of the communicator (no allocation per call)
int comm_allreduce_host(lorb_comm* c, double* h, size_t n, int op) {
  lorb_ctx* ctx = c->ctx;
  if (n == 0 || c->nranks == 1) return LORB_OK;
  if (!c->rccl) return c->fn(c->user, h, (int64_t)n, op) == 0 ? LORB_OK : set_error(ctx, LORB_E_COMM, "host all-reduce callback failed");
  if (c->dbuf_n < n) {
    if (c->dbuf) {
      LORB_HIP(ctx, hipStreamSynchronize(ctx->stream));
      (void)hipFree(c->dbuf);
    }
    c->dbuf = nullptr;
    c->dbuf_n = 0;
    LORB_HIP(ctx, hipMalloc(reinterpret_cast<void**>(&c->dbuf), n * sizeof(double)));
    c->dbuf_n = n;
  }
  int rc = LORB_OK;
  if (hipMemcpyAsync(c->dbuf, h, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream) != hipSuccess) rc = LORB_E_DEVICE;
  if (rc == LORB_OK) rc = comm_allreduce(c, c->dbuf, c->dbuf, n, op);
  if (rc == LORB_OK && hipMemcpyAsync(h, c->dbuf, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    rc = LORB_E_DEVICE;
  if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == LORB_OK) rc = LORB_E_DEVICE;
  return rc == LORB_OK ? LORB_OK : set_error(ctx, rc, "host-array all-reduce failed");
}

}  // namespace lorb

extern "C" {

int lorb_comm_unique_id(void* id_out) {
  if (!id_out) return LORB_E_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return LORB_E_COMM;
  memcpy(id_out, &id, sizeof(id));
  return LORB_OK;
}

int lorb_comm_init_rccl(lorb_ctx* ctx, int32_t nranks, int32_t rank, const void* unique_id, lorb_comm** out) {
  if (!ctx || !out || !unique_id || nranks < 1 || rank < 0 || rank >= nranks) return LORB_E_INVALID;
  *out = nullptr;
  LORB_HIP(ctx, hipSetDevice(ctx->device));
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  ncclComm_t nc = nullptr;
  const ncclResult_t r = ncclCommInitRank(&nc, nranks, id, rank);
  if (r != ncclSuccess) return lorb::set_error(ctx, LORB_E_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
  lorb_comm* c = new (std::nothrow) lorb_comm();
  if (!c) { (void)ncclCommDestroy(nc); return LORB_E_NOMEM; }
  c->ctx = ctx; c->nranks = nranks; c->rank = rank; c->rccl = true; c->nccl = nc;
  *out = c;
  return LORB_OK;
}

int lorb_comm_init_host(lorb_ctx* ctx, int32_t nranks, int32_t rank, lorb_host_allreduce_fn fn, void* user,
                        lorb_comm** out) {
  if (!ctx || !out || !fn || nranks < 1 || rank < 0 || rank >= nranks) return LORB_E_INVALID;
  lorb_comm* c = new (std::nothrow) lorb_comm();
  if (!c) return LORB_E_NOMEM;
  c->ctx = ctx; c->nranks = nranks; c->rank = rank; c->rccl = false; c->fn = fn; c->user = user;
  *out = c;
  return LORB_OK;
}

int lorb_comm_destroy(lorb_comm* c) {
  if (!c) return LORB_OK;
  if (c->ctx && c->ctx->stream) (void)hipStreamSynchronize(c->ctx->stream);
  if (c->rccl && c->nccl) (void)ncclCommDestroy(static_cast<ncclComm_t>(c->nccl));
  if (c->pinned) (void)hipHostFree(c->pinned);
  if (c->dbuf) (void)hipFree(c->dbuf);
  delete c;
  return LORB_OK;
}

int lorb_comm_size(lorb_comm* c, int32_t* nranks, int32_t* rank) {
  if (!c || !nranks) return LORB_E_INVALID;
  if (c->rccl) {
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(static_cast<ncclComm_t>(c->nccl), &n);
    if (e == ncclSuccess) e = ncclCommUserRank(static_cast<ncclComm_t>(c->nccl), &r);
    if (e != ncclSuccess) return lorb::set_error(c->ctx, LORB_E_COMM, "ncclCommCount: %s", ncclGetErrorString(e));
    *nranks = n;
    if (rank) *rank = r;
  } else {
    *nranks = c->nranks;
    if (rank) *rank = c->rank;
  }
  return LORB_OK;
}

int lorb_comm_allreduce_f64(lorb_comm* c, const double* d_send, double* d_recv, int64_t count, int32_t op) {
  if (!c || count < 0 || (count > 0 && (!d_send || !d_recv))) return LORB_E_INVALID;
  return lorb::comm_allreduce(c, d_send, d_recv, (size_t)count, op);
}

}  // extern "C"
