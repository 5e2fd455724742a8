// Asynchronous multiexp: the reference's plugin seam is
//   multiexp(pool, bases, density_map, exponents) -> Waiter<Result<G, SynthesisError>>
// (multiexp.rs:252-281, Waiter = multicore.rs:94-110), and create_proof keeps eight of them in
// flight before waiting on any (prover.rs:233-307).  bh_multiexp_submit enqueues one multiexp on
// a stream and workspace of its own -- no context-wide lock is held while the GPU works -- and
// bh_multiexp_wait is the host-side event sync plus the W-window Horner combine
// (multiexp.rs:244-249).  Several submitted multiexps overlap on the device (sorts of one
// beside accumulations of another), as the reference's rayon tasks do on the CPU.
#include <string.h>

#include <algorithm>

#include "api_internal.h"

using namespace bh;

// One in-flight multiexp's private resources, recycled through the context's free list.
struct bh_job_slot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  DevBuf raw, scalars, dwords, idx, dtmp, dscan;
  MsmWorkspace<G1Ops> ws1;
  MsmWorkspace<G2Ops> ws2;
  ~bh_job_slot() {
    if (st) (void)hipStreamSynchronize(st);
    ws1.release();
    ws2.release();
    if (done) (void)hipEventDestroy(done);
    if (st) (void)hipStreamDestroy(st);
  }
};

struct bh_job {
  std::shared_ptr<bh_job_registry> reg;  // keeps the slot bookkeeping alive past bh_ctx_destroy
  int device = 0;
  int window_override = 0;
  bh_job_slot* slot = nullptr;
  int group = BH_G1;
  MsmShape sh{};
  bool empty = false;      // n == 0: the identity
  bool detached = false;   // the context was destroyed before wait (the slot was released with it)
  bh_status status = BH_OK;  // deferred error (the reference reports it from wait())
};

namespace {

bh_status take_slot(bh_job_registry& reg, bh_job_slot** out) {
  {
    std::lock_guard<std::mutex> lk(reg.mu);
    if (!reg.free_slots.empty()) {
      *out = reg.free_slots.back();
      reg.free_slots.pop_back();
      return BH_OK;
    }
  }
  std::unique_ptr<bh_job_slot> s(new bh_job_slot());
  BH_TRY_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
  BH_TRY_HIP(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
  *out = s.release();
  std::lock_guard<std::mutex> lk(reg.mu);
  reg.all_slots.push_back(*out);
  return BH_OK;
}

// back to the free list, or -- the context is gone -- released
void give_slot(bh_job_registry& reg, bh_job_slot* s) {
  {
    std::lock_guard<std::mutex> lk(reg.mu);
    if (reg.alive) {
      reg.free_slots.push_back(s);
      return;
    }
    reg.all_slots.erase(std::remove(reg.all_slots.begin(), reg.all_slots.end(), s), reg.all_slots.end());
  }
  delete s;
}

template <class C>
bh_status enqueue_msm(bh_job* job, MsmWorkspace<C>& ws, const bh_srs* bases, size_t base_offset, size_t n,
                      const int32_t* d_idx) {
  job->sh = msm_shape(n, job->window_override);
  fit_segments<C>(job->sh, n);
  BH_TRY_HIP(msm_window_sums<C>(ws, job->slot->st, bases->pts.as<uint32_t>(), job->slot->scalars.as<uint32_t>(), n,
                                d_idx, (uint32_t)base_offset, job->sh, nullptr));
  return BH_OK;
}

}  // namespace

// bh_ctx_destroy: every job not yet waited for is detached and its slot released (after its
// stream drains); slots a waiter currently holds are released by that waiter (give_slot)
void bh_ctx_release_jobs(bh_ctx* ctx) {
  std::vector<bh_job_slot*> dead;
  {
    std::lock_guard<std::mutex> lk(ctx->jobs->mu);
    bh_job_registry& reg = *ctx->jobs;
    reg.alive = false;
    for (bh_job* j : reg.pending) {
      j->detached = true;
      if (j->slot) dead.push_back(j->slot);
      j->slot = nullptr;
    }
    reg.pending.clear();
    for (bh_job_slot* s : reg.free_slots) dead.push_back(s);
    reg.free_slots.clear();
    for (bh_job_slot* s : dead)
      reg.all_slots.erase(std::remove(reg.all_slots.begin(), reg.all_slots.end(), s), reg.all_slots.end());
  }
  for (bh_job_slot* s : dead) delete s;  // ~bh_job_slot drains the slot's stream first
}

extern "C" {

bh_status bh_multiexp_submit(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint64_t* density_words,
                             size_t density_len, const uint64_t* exponents, size_t n, int scalar_format,
                             bh_job** out) {
  if (!ctx || !bases || !out || (n && !exponents)) return BH_ERR_INVALID_ARGUMENT;
  if (scalar_format != BH_SCALARS_CANONICAL && scalar_format != BH_SCALARS_MONTGOMERY) return BH_ERR_INVALID_ARGUMENT;
  if (density_words && density_len != n) return BH_ERR_DENSITY_SIZE_MISMATCH;  // the reference asserts
  if (n > 0x7fffffffull || !bases->ctx || bases->ctx->device != ctx->device) return BH_ERR_INVALID_ARGUMENT;
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<bh_job> job(new bh_job());
  job->reg = ctx->jobs;
  job->device = ctx->device;
  job->window_override = ctx->window_override;
  job->group = bases->group;
  // Source semantics (EOF / identity base): decided on the host from the density map and, only
  // when an identity base is reachable, the exponents; reported by wait() like the reference
  std::vector<uint64_t> canon;
  const uint64_t* ex_c = exponents;
  if (scalar_format == BH_SCALARS_MONTGOMERY && !bases->identity_idx.empty()) {
    canon.resize(n * 4);
    for (size_t i = 0; i < n; i++) {
      Fr x;
      memcpy(x.v, exponents + 4 * i, 32);
      fr_to_canonical(x, &canon[4 * i]);
    }
    ex_c = canon.data();
  }
  job->status = multiexp_check(bases, base_offset, density_words, n, ex_c, true);
  if (job->status || n == 0) {
    job->empty = true;
    *out = job.release();
    return BH_OK;
  }
  bh_status s = take_slot(*job->reg, &job->slot);
  if (s) return s;
  bh_job_slot* sl = job->slot;
  auto fail = [&](bh_status e) {
    (void)hipStreamSynchronize(sl->st);
    give_slot(*job->reg, sl);
    return e;
  };
  // the caller's buffers are read before submit returns (pageable copies complete on return)
  if (sl->raw.alloc(n * 32) || sl->scalars.alloc(n * 32)) return fail(BH_ERR_OUT_OF_MEMORY);
  if (hipMemcpyAsync(sl->raw.p, exponents, n * 32, hipMemcpyHostToDevice, sl->st)) return fail(BH_ERR_HIP);
  if (scalars_prepare(sl->raw.as<uint32_t>(), sl->scalars.as<uint32_t>(), n,
                      scalar_format == BH_SCALARS_MONTGOMERY ? 1 : 0, 0, sl->st))
    return fail(BH_ERR_HIP);
  const int32_t* d_idx = nullptr;
  if (density_words) {
    const size_t nw = (n + 63) / 64;
    if (sl->dwords.alloc(nw * 8) || sl->idx.alloc(n * 4) || sl->dtmp.alloc((nw + 1) * 4) ||
        sl->dscan.alloc(scan_scratch_words(nw + 1) * 4 + 64))
      return fail(BH_ERR_OUT_OF_MEMORY);
    if (hipMemcpyAsync(sl->dwords.p, density_words, nw * 8, hipMemcpyHostToDevice, sl->st)) return fail(BH_ERR_HIP);
    if (density_index(sl->dwords.as<uint64_t>(), n, (uint32_t)base_offset, sl->idx.as<int32_t>(),
                      sl->dtmp.as<uint32_t>(), sl->dscan.as<uint32_t>(), sl->st))
      return fail(BH_ERR_HIP);
    d_idx = sl->idx.as<int32_t>();
  }
  s = bases->group == BH_G1 ? enqueue_msm<G1Ops>(job.get(), sl->ws1, bases, base_offset, n, d_idx)
                            : enqueue_msm<G2Ops>(job.get(), sl->ws2, bases, base_offset, n, d_idx);
  if (s) return fail(s);
  if (hipEventRecord(sl->done, sl->st)) return fail(BH_ERR_HIP);
  {
    std::lock_guard<std::mutex> lk(job->reg->mu);
    job->reg->pending.push_back(job.get());
  }
  *out = job.release();
  return BH_OK;
}

bh_status bh_multiexp_wait(bh_job* job, uint8_t* out) {
  if (!job) return BH_ERR_INVALID_ARGUMENT;
  std::unique_ptr<bh_job> j(job);
  if (j->empty) {
    if (j->status) return j->status;
    if (!out) return BH_ERR_INVALID_ARGUMENT;
    if (j->group == BH_G1) g1_to_uncompressed(jac_to_affine(jac_identity<Fp>()), out);
    else g2_to_uncompressed(jac_to_affine(jac_identity<bh::Fp2>()), out);
    return BH_OK;
  }
  bh_job_slot* sl = nullptr;
  {
    std::lock_guard<std::mutex> lk(j->reg->mu);
    auto& pend = j->reg->pending;
    pend.erase(std::remove(pend.begin(), pend.end(), j.get()), pend.end());
    if (!j->detached) sl = j->slot;
  }
  if (!sl) return BH_ERR_INVALID_ARGUMENT;  // its context was destroyed: no result exists
  (void)hipSetDevice(j->device);
  const hipError_t e = hipEventSynchronize(sl->done);  // Waiter::wait: a host-side event sync
  bh_status s = e == hipSuccess ? BH_OK : BH_ERR_HIP;
  if (!s && out) {
    if (j->group == BH_G1) g1_to_uncompressed(jac_to_affine(combine_g1(sl->ws1.host_window_sums, j->sh)), out);
    else g2_to_uncompressed(jac_to_affine(combine_g2(sl->ws2.host_window_sums, j->sh)), out);
  }
  give_slot(*j->reg, sl);
  if (!out && !s) return BH_ERR_INVALID_ARGUMENT;
  return s;
}

}  // extern "C"
