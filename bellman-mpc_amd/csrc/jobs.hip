// Asynchronous multiexp: the reference's plugin seam is
//   multiexp(pool, bases, density_map, exponents) -> Waiter<Result<G, SynthesisError>>
// (multiexp.rs:252-281, Waiter = multicore.rs:94-110), and create_proof keeps eight of them in
// flight before waiting on any (prover.rs:233-307).  bh_multiexp_submit enqueues one multiexp on
// a stream and workspace of its own -- no context-wide lock is held while the GPU works -- and
// bh_multiexp_wait is the host-side event sync plus the W-window Horner combine
// (multiexp.rs:244-249).  Several submitted multiexps overlap on the device (sorts of one
// beside accumulations of another), as the reference's rayon tasks do on the CPU.
#include <string.h>

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
  bh_ctx* ctx = nullptr;
  bh_job_slot* slot = nullptr;
  int group = BH_G1;
  MsmShape sh{};
  bool empty = false;     // n == 0: the identity
  bh_status status = BH_OK;  // deferred error (the reference reports it from wait())
};

namespace {

bh_status take_slot(bh_ctx* ctx, bh_job_slot** out) {
  {
    std::lock_guard<std::mutex> lk(ctx->jobs_mu);
    if (!ctx->free_slots.empty()) {
      *out = ctx->free_slots.back();
      ctx->free_slots.pop_back();
      return BH_OK;
    }
  }
  std::unique_ptr<bh_job_slot> s(new bh_job_slot());
  BH_TRY_HIP(hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking));
  BH_TRY_HIP(hipEventCreateWithFlags(&s->done, hipEventDisableTiming));
  *out = s.release();
  std::lock_guard<std::mutex> lk(ctx->jobs_mu);
  ctx->all_slots.push_back(*out);
  return BH_OK;
}

void give_slot(bh_ctx* ctx, bh_job_slot* s) {
  std::lock_guard<std::mutex> lk(ctx->jobs_mu);
  ctx->free_slots.push_back(s);
}

template <class C>
bh_status enqueue_msm(bh_job* job, MsmWorkspace<C>& ws, const bh_srs* bases, size_t base_offset, size_t n,
                      const int32_t* d_idx) {
  bh_ctx* ctx = job->ctx;
  job->sh = msm_shape(n, ctx->window_override);
  fit_segments<C>(job->sh, n);
  BH_TRY_HIP(msm_window_sums<C>(ws, job->slot->st, bases->pts.as<uint32_t>(), job->slot->scalars.as<uint32_t>(), n,
                                d_idx, (uint32_t)base_offset, job->sh, nullptr));
  return BH_OK;
}

}  // namespace

void bh_ctx_release_jobs(bh_ctx* ctx) {
  std::lock_guard<std::mutex> lk(ctx->jobs_mu);
  for (bh_job_slot* s : ctx->all_slots) delete s;
  ctx->all_slots.clear();
  ctx->free_slots.clear();
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
  job->ctx = ctx;
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
  bh_status s = take_slot(ctx, &job->slot);
  if (s) return s;
  bh_job_slot* sl = job->slot;
  auto fail = [&](bh_status e) {
    (void)hipStreamSynchronize(sl->st);
    give_slot(ctx, sl);
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
  *out = job.release();
  return BH_OK;
}

bh_status bh_multiexp_wait(bh_job* job, uint8_t* out) {
  if (!job) return BH_ERR_INVALID_ARGUMENT;
  std::unique_ptr<bh_job> j(job);
  bh_ctx* ctx = j->ctx;
  if (j->empty) {
    if (j->status) return j->status;
    if (!out) return BH_ERR_INVALID_ARGUMENT;
    if (j->group == BH_G1) g1_to_uncompressed(jac_to_affine(jac_identity<Fp>()), out);
    else g2_to_uncompressed(jac_to_affine(jac_identity<bh::Fp2>()), out);
    return BH_OK;
  }
  bh_job_slot* sl = j->slot;
  const hipError_t e = hipEventSynchronize(sl->done);  // Waiter::wait: a host-side event sync
  bh_status s = e == hipSuccess ? BH_OK : BH_ERR_HIP;
  if (!s && out) {
    if (j->group == BH_G1) g1_to_uncompressed(jac_to_affine(combine_g1(sl->ws1.host_window_sums, j->sh)), out);
    else g2_to_uncompressed(jac_to_affine(combine_g2(sl->ws2.host_window_sums, j->sh)), out);
  }
  give_slot(ctx, sl);
  if (!out && !s) return BH_ERR_INVALID_ARGUMENT;
  return s;
}

}  // extern "C"
