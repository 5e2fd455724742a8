// Multi-GPU exchange step over RCCL (xGMI): the all-gather of the per-rank
// partial multiexp records (BH_PARTIAL_BYTES each).  Elliptic-curve addition is
// not an RCCL reduction operator, so the "reduce" is an all-gather of the
// affine partial sums followed by the host-side sum in bh_proof_from_partials.
// The reference has no multi-device path; this is the MI355X
// replacement for its single-process rayon fan-out (prover.rs:233-307).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "api_internal.h"

struct bh_comm {
  bh_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  uint8_t* d_send = nullptr;
  uint8_t* d_recv = nullptr;
  double* d_val = nullptr;  // bh_comm_allreduce_max
};

extern "C" {

bh_status bh_comm_unique_id(uint8_t out[128]) {
  if (!out) return BH_ERR_INVALID_ARGUMENT;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return BH_ERR_HIP;
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  memcpy(out, &id, sizeof id);
  return BH_OK;
}

bh_status bh_comm_init(bh_ctx* ctx, const uint8_t id[128], int nranks, int rank, bh_comm** out) {
  if (!ctx || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks) return BH_ERR_INVALID_ARGUMENT;
  BH_TRY_HIP(hipSetDevice(ctx->device));
  bh_comm* c = new bh_comm();
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    fprintf(stderr, "bh_comm_init(rank %d of %d, device %d): ncclCommInitRank: %s\n", rank, nranks, ctx->device,
            ncclGetErrorString(r));
    delete c;
    return BH_ERR_HIP;
  }
  if (hipMalloc(&c->d_send, BH_PARTIAL_BYTES) != hipSuccess ||
      hipMalloc(&c->d_recv, (size_t)BH_PARTIAL_BYTES * nranks) != hipSuccess ||
      hipMalloc(&c->d_val, sizeof(double)) != hipSuccess) {
    ncclCommDestroy(c->comm);
    delete c;
    return BH_ERR_OUT_OF_MEMORY;
  }
  *out = c;
  return BH_OK;
}

bh_status bh_comm_allgather_partials(bh_comm* c, const uint8_t* partial, uint8_t* all_out) {
  if (!c || !partial || !all_out) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(c->ctx->mu);
  BH_TRY_HIP(hipSetDevice(c->ctx->device));
  hipStream_t st = c->ctx->stream;
  BH_TRY_HIP(hipMemcpyAsync(c->d_send, partial, BH_PARTIAL_BYTES, hipMemcpyHostToDevice, st));
  if (ncclAllGather(c->d_send, c->d_recv, BH_PARTIAL_BYTES, ncclUint8, c->comm, st) != ncclSuccess) return BH_ERR_HIP;
  BH_TRY_HIP(hipMemcpyAsync(all_out, c->d_recv, (size_t)BH_PARTIAL_BYTES * c->nranks, hipMemcpyDeviceToHost, st));
  BH_TRY_HIP(hipStreamSynchronize(st));
  return BH_OK;
}

// every rank's nbytes record, rank order (small host records: rank metadata, timings)
bh_status bh_comm_allgather(bh_comm* c, const uint8_t* in, size_t nbytes, uint8_t* all_out) {
  if (!c || !in || !all_out || nbytes == 0) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(c->ctx->mu);
  BH_TRY_HIP(hipSetDevice(c->ctx->device));
  hipStream_t st = c->ctx->stream;
  bh::DevBuf d;
  BH_TRY_HIP(d.alloc(nbytes * (size_t)(c->nranks + 1)));
  uint8_t* ds = d.as<uint8_t>();
  uint8_t* dr = ds + nbytes;
  BH_TRY_HIP(hipMemcpyAsync(ds, in, nbytes, hipMemcpyHostToDevice, st));
  if (ncclAllGather(ds, dr, nbytes, ncclUint8, c->comm, st) != ncclSuccess) return BH_ERR_HIP;
  BH_TRY_HIP(hipMemcpyAsync(all_out, dr, nbytes * (size_t)c->nranks, hipMemcpyDeviceToHost, st));
  BH_TRY_HIP(hipStreamSynchronize(st));
  return BH_OK;
}

// max over ranks of *inout, every rank receiving it; completes only when every rank has
// reached it, so it doubles as the barrier of a timed region
bh_status bh_comm_allreduce_max(bh_comm* c, double* inout) {
  if (!c || !inout) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(c->ctx->mu);
  BH_TRY_HIP(hipSetDevice(c->ctx->device));
  hipStream_t st = c->ctx->stream;
  BH_TRY_HIP(hipMemcpyAsync(c->d_val, inout, sizeof(double), hipMemcpyHostToDevice, st));
  if (ncclAllReduce(c->d_val, c->d_val, 1, ncclFloat64, ncclMax, c->comm, st) != ncclSuccess) return BH_ERR_HIP;
  BH_TRY_HIP(hipMemcpyAsync(inout, c->d_val, sizeof(double), hipMemcpyDeviceToHost, st));
  BH_TRY_HIP(hipStreamSynchronize(st));
  return BH_OK;
}

// what RCCL itself reports for this communicator: out = {rank count, this rank, HIP device}
bh_status bh_comm_info(const bh_comm* c, int out[3]) {
  if (!c || !out) return BH_ERR_INVALID_ARGUMENT;
  if (ncclCommCount(c->comm, &out[0]) != ncclSuccess || ncclCommUserRank(c->comm, &out[1]) != ncclSuccess ||
      ncclCommCuDevice(c->comm, &out[2]) != ncclSuccess)
    return BH_ERR_HIP;
  return BH_OK;
}

}  // extern "C"

namespace bh {

// Smallest rank count that distributes the H block.  2: at N = 2 a rank's replicated H (~8 % of
// the proof's VALU work) was the largest non-shrinking cost; distributing it took the one-GPU
// rehearsal from 35.2 to 33.7 ms per rank (1.66x -> 1.73x, profiles/r03_ab_dist_h_N2.txt).
size_t dist_h_min_ranks() { return 2; }

static bh_status comm_exchange(bh_comm* c, const uint32_t* send, uint32_t* recv, size_t C, size_t M, int nvec,
                        hipStream_t st) {
  const size_t bytes = C * 32;
  for (int v = 0; v < nvec; v++) {  // own chunk: a device copy
    const size_t off = ((size_t)v * M + (size_t)c->rank * C) * 8;
    BH_TRY_HIP(hipMemcpyAsync(recv + off, send + off, bytes, hipMemcpyDeviceToDevice, st));
  }
  if (ncclGroupStart() != ncclSuccess) return BH_ERR_HIP;
  for (int v = 0; v < nvec; v++)
    for (int p = 0; p < c->nranks; p++) {
      if (p == c->rank) continue;
      const uint32_t* s = send + ((size_t)v * M + (size_t)p * C) * 8;
      uint32_t* r = recv + ((size_t)v * M + (size_t)p * C) * 8;
      if (ncclSend(s, bytes, ncclUint8, p, c->comm, st) != ncclSuccess ||
          ncclRecv(r, bytes, ncclUint8, p, c->comm, st) != ncclSuccess) {
        ncclGroupEnd();
        return BH_ERR_HIP;
      }
    }
  if (ncclGroupEnd() != ncclSuccess) return BH_ERR_HIP;
  return BH_OK;
}

int comm_rank(const bh_comm* c) { return c->rank; }
int comm_size(const bh_comm* c) { return c->nranks; }

namespace {
struct RcclExchanger : Exchanger {
  bh_comm* c;
  explicit RcclExchanger(bh_comm* cc) : c(cc) {}
  int rank() const override { return c->rank; }
  int size() const override { return c->nranks; }
  bh_status exchange(const uint32_t* send, uint32_t* recv, size_t C, size_t M, int nvec, hipStream_t st) override {
    return comm_exchange(c, send, recv, C, M, nvec, st);
  }
};
}  // namespace

std::unique_ptr<Exchanger> rccl_exchanger(bh_comm* c) { return std::unique_ptr<Exchanger>(new RcclExchanger(c)); }

}  // namespace bh

extern "C" {

bh_status bh_comm_destroy(bh_comm* c) {
  if (!c) return BH_OK;
  (void)hipSetDevice(c->ctx->device);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->d_send) (void)hipFree(c->d_send);
  if (c->d_recv) (void)hipFree(c->d_recv);
  if (c->d_val) (void)hipFree(c->d_val);
  delete c;
  return BH_OK;
}

bh_status bh_ctx_synchronize(bh_ctx* ctx) {
  if (!ctx) return BH_ERR_INVALID_ARGUMENT;
  BH_TRY_HIP(hipSetDevice(ctx->device));
  BH_TRY_HIP(hipDeviceSynchronize());
  return BH_OK;
}

int bh_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
