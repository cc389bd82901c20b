// Multi-GPU sharding support: RCCL over xGMI behind the C ABI (include/tmpc.h,
// "multi-GPU" section).  The reference has no distributed path at all -- its
// drivers run independent problems in a multiprocessing.Pool
// (examples/test_multiple.py:123-128); here independent problem
// batches shard across the GPUs of a node, one process per GPU, and RCCL
// carries the only data that crosses GPUs: the initial states broadcast from
// rank 0 and the per-problem result summaries gathered back.
// Collectives run on the context's HIP stream and are synchronous at the ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "../../include/tmpc.h"
#include "tmpc_internal.h"

struct tmpc_comm {
  tmpc_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  int* d_flag = nullptr;   // barrier word
};

static_assert(sizeof(ncclUniqueId) == TMPC_COMM_ID_BYTES, "RCCL unique id size");

#define NCCL_OK(call)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (call);                                                                      \
    if (r_ != ncclSuccess) return tmpc::ctx_fail(c->ctx, "%s failed: %s", #call, ncclGetErrorString(r_)); \
  } while (0)

#define HIPC_OK(call)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return tmpc::ctx_fail(c->ctx, "%s failed: %s", #call, hipGetErrorString(e_)); \
  } while (0)

extern "C" {

int tmpc_comm_get_unique_id(uint8_t* id) {
  if (!id) return -1;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return -2;
  memcpy(id, &u, sizeof(u));
  return 0;
}

int tmpc_comm_create(tmpc_ctx* ctx, int nranks, int rank, const uint8_t* id, tmpc_comm** out) {
  if (!ctx || !id || !out) return -1;
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks)
    return tmpc::ctx_fail(ctx, "tmpc_comm_create: rank %d of %d ranks", rank, nranks);
  tmpc_comm* c = new tmpc_comm();
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  hipSetDevice(tmpc::ctx_device(ctx));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return tmpc::ctx_fail(ctx, "ncclCommInitRank(%d ranks, rank %d) failed: %s", nranks, rank, ncclGetErrorString(r));
  }
  if (hipMalloc(&c->d_flag, sizeof(int)) != hipSuccess) {
    ncclCommDestroy(c->comm);
    delete c;
    return tmpc::ctx_fail(ctx, "tmpc_comm_create: device allocation failed");
  }
  *out = c;
  return 0;
}

void tmpc_comm_destroy(tmpc_comm* c) {
  if (!c) return;
  hipSetDevice(tmpc::ctx_device(c->ctx));
  hipStreamSynchronize(tmpc::ctx_stream(c->ctx));
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->d_flag) hipFree(c->d_flag);
  delete c;
}

int tmpc_comm_size(const tmpc_comm* c, int* nranks, int* rank) {
  if (!c) return -1;
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  return 0;
}

int tmpc_comm_broadcast(tmpc_comm* c, void* d_buf, size_t bytes, int root) {
  if (!c) return -1;
  if (root < 0 || root >= c->nranks) return tmpc::ctx_fail(c->ctx, "broadcast root %d of %d ranks", root, c->nranks);
  hipSetDevice(tmpc::ctx_device(c->ctx));
  hipStream_t s = tmpc::ctx_stream(c->ctx);
  NCCL_OK(ncclBroadcast(d_buf, d_buf, bytes, ncclChar, root, c->comm, s));
  HIPC_OK(hipStreamSynchronize(s));
  return 0;
}

int tmpc_comm_allgather(tmpc_comm* c, const void* d_send, void* d_recv, size_t bytes_per_rank) {
  if (!c) return -1;
  hipSetDevice(tmpc::ctx_device(c->ctx));
  hipStream_t s = tmpc::ctx_stream(c->ctx);
  NCCL_OK(ncclAllGather(d_send, d_recv, bytes_per_rank, ncclChar, c->comm, s));
  HIPC_OK(hipStreamSynchronize(s));
  return 0;
}

int tmpc_comm_allreduce_max_f64(tmpc_comm* c, double* d_buf, size_t count) {
  if (!c) return -1;
  hipSetDevice(tmpc::ctx_device(c->ctx));
  hipStream_t s = tmpc::ctx_stream(c->ctx);
  NCCL_OK(ncclAllReduce(d_buf, d_buf, count, ncclFloat64, ncclMax, c->comm, s));
  HIPC_OK(hipStreamSynchronize(s));
  return 0;
}

int tmpc_comm_barrier(tmpc_comm* c) {
  if (!c) return -1;
  hipSetDevice(tmpc::ctx_device(c->ctx));
  hipStream_t s = tmpc::ctx_stream(c->ctx);
  // every rank's stream work issued so far completes before its contribution
  HIPC_OK(hipMemsetAsync(c->d_flag, 0, sizeof(int), s));
  NCCL_OK(ncclAllReduce(c->d_flag, c->d_flag, 1, ncclInt32, ncclSum, c->comm, s));
  HIPC_OK(hipStreamSynchronize(s));
  return 0;
}

}  // extern "C"
