// Distributed H pipeline (the prover.rs:210-231 block split over N ranks).
//
// With m = N*M, rank r owns the strided residue class {N*j + r} ("S") or, after a transform,
// the N chunks {M*t + q : q in [r*C, (r+1)*C)}, C = M/N ("B").  Every NTT of the H block is
// one local M-point NTT, one all-to-all of C-element chunks and N-point DFTs done in
// registers (four-step decomposition); the ifft -> coset_fft pair shares one kernel between
// its two all-to-alls.  Each rank ends with h[M*t + q] for its own q chunk, which is exactly
// the index set of its share of the h multiexp: no further exchange is needed.
//
// The exchange is a callback so the same phases run over RCCL (bh_prove_witness_partial_comm)
// or, for tests and rehearsal, with N virtual ranks on one device
// (bh_prove_witness_partials_local).
#pragma once
#include "kinfo.h"
#include <functional>

#include "api_internal.h"

namespace bh {

struct DistH {
  int N = 0, rank = 0, L = 0, Lm = 0;  // m = 2^L, M = 2^Lm = m / N
  size_t M = 0, C = 0;
  DevBuf work, recv;  // 3*M packed Fr each, [vec][peer][C]
  DevBuf hbuf, hidx;  // this rank's h scalars (canonical, M) and their global indices
};

// send[vec*M + p*C ...] goes to rank p, which stores it at recv[vec*M + me*C ...]
using HExchange = std::function<bh_status(const uint32_t* send, uint32_t* recv, int nvec, hipStream_t st)>;

bool dist_h_eligible(int N, int L);
bh_status dist_h_init(bh_ctx* ctx, DistH& d, int N, int rank, int L);
// phases; exchange k runs between phase k and k+1 with the buffers returned here
bh_status dist_h_phase1(bh_ctx* ctx, DistH& d, const uint32_t* abc_full, hipStream_t st);  // send work -> recv
bh_status dist_h_phase2(bh_ctx* ctx, DistH& d, hipStream_t st);                            // send work -> recv
bh_status dist_h_phase3(bh_ctx* ctx, DistH& d, hipStream_t st);                            // send recv[0] -> work[0]
bh_status dist_h_final(bh_ctx* ctx, DistH& d, hipStream_t st);                             // -> hbuf, hidx
// the distributed-H unit's kernels (scratch budget, scratch.cpp)
void dist_kernels(std::vector<KernInfo>& v);
// whole pipeline with an exchange callback, stream-ordered on st
bh_status dist_h_run(bh_ctx* ctx, DistH& d, const uint32_t* abc_full, const HExchange& ex, hipStream_t st);

}  // namespace bh
