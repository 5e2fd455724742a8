// Asynchronous multiexp: the reference's plugin seam is
//   multiexp(pool, bases, density_map, exponents) -> Waiter<Result<G, SynthesisError>>
// (multiexp.rs:252-281, Waiter = multicore.rs:94-110), and create_proof keeps eight of them in
// flight before waiting on any (prover.rs:233-307).  bh_multiexp_submit enqueues one multiexp on
// a workspace of its own -- no context-wide lock is held while the GPU works -- and
// bh_multiexp_wait is the host-side event sync plus the W-window Horner combine
// (multiexp.rs:244-249).  The jobs use the prover's stream layout (no stream of their own, so
// the context's hardware-queue budget does not grow with the jobs in flight): the digit sorts on
// the high-priority sort stream, the accumulations back to back on the main stream in submit
// order, each reduction tail on one of the tail streams -- so several submitted multiexps overlap
// on the device (sorts and tails of some beside the accumulation of another) as create_proof's
// do in bh_prove, and as the reference's rayon tasks do on the CPU.
#include <string.h>

#include <algorithm>
#include <atomic>

#include "api_internal.h"

using namespace bh;

// One in-flight multiexp's private resources, recycled through the context's free list.
struct bh_job_slot {
  hipEvent_t uploaded = nullptr, sorted = nullptr, accumulated = nullptr, done = nullptr;
  uint64_t use = 0;  // bumped each time the slot is taken (bh_job_registry::SortRec validity)
  uint64_t last_key = 0;  // job_key() of the last multiexp this slot ran (take_slot's match)
  DevBuf raw, scalars, dwords, idx, dtmp, dscan, dscan2, dspan;
  MsmWorkspace<G1Ops> ws1;
  MsmWorkspace<G2Ops> ws2;
  ~bh_job_slot() {  // (its last use was waited for, or the context's streams were drained)
    ws1.release();
    ws2.release();
    for (hipEvent_t e : {uploaded, sorted, accumulated, done})
      if (e) (void)hipEventDestroy(e);
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
  // what the device reads until the job is done: a Parameters window table, a bh_scalars vector
  std::shared_ptr<DevBuf> table_hold;
  std::shared_ptr<bh_scalar_buf> scalars_hold;
  bool deferred = false;   // enqueued by the scalars' producer (bh_multiexp_submit_scalars)
  bh_status status = BH_OK;  // deferred error (the reference reports it from wait())
};

namespace {

// The shape of a multiexp for slot reuse: a slot whose buffers were sized by the same kind of
// job (same bases, offset, length) needs no reallocation -- and a reallocation is a hipFree, which
// waits for the whole device (the submit would block behind every multiexp in flight).
uint64_t job_key(const bh_srs* bases, size_t base_offset, size_t n) {
  uint64_t h = (uint64_t)(uintptr_t)bases * 0x9e3779b97f4a7c15ull;
  h ^= (base_offset + 0x632be59bd9b4e019ull) + (h << 6) + (h >> 2);
  h ^= (n + 0x85ebca77c2b2ae63ull) + (h << 6) + (h >> 2);
  return h | 1u;
}

bh_status take_slot(bh_job_registry& reg, bh_job_slot** out, uint64_t key) {
  {
    std::lock_guard<std::mutex> lk(reg.mu);
    if (!reg.free_slots.empty()) {
      // the slot that last ran this kind of job, else the most recently freed one
      auto it = std::find_if(reg.free_slots.rbegin(), reg.free_slots.rend(),
                             [key](const bh_job_slot* sl) { return sl->last_key == key; });
      auto pos = it != reg.free_slots.rend() ? std::next(it).base() : std::prev(reg.free_slots.end());
      *out = *pos;
      reg.free_slots.erase(pos);
      (*out)->use++;
      (*out)->last_key = key;
      return BH_OK;
    }
  }
  std::unique_ptr<bh_job_slot> s(new bh_job_slot());
  s->last_key = key;
  for (hipEvent_t* e : {&s->uploaded, &s->sorted, &s->accumulated, &s->done})
    BH_TRY_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
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
    reg.sorts.erase(std::remove_if(reg.sorts.begin(), reg.sorts.end(),
                                   [s](const bh_job_registry::SortRec& r) { return r.slot == s; }),
                    reg.sorts.end());
  }
  delete s;
}

// A multiexp over a Parameters vector whose window table (bh_params_prepare) covers the bases
// it consumes runs like the prover's: every digit window into one shared bucket set at the
// table's c (2^16 set scalars and up; smaller ones use plain windows, as the prover does).
struct JobStreams {
  hipStream_t sort, acc, tail;
  uint64_t key = 0;        // bh_scalar_buf::id of the scalars (0: a private copy, never shared)
  uint64_t dens_hash = 0;  // of the density words (0: full density)
};

uint64_t words_hash(const uint64_t* w, size_t nw) {
  uint64_t h = 0x9e3779b97f4a7c15ull ^ nw;
  for (size_t i = 0; i < nw; i++) {
    h ^= w[i] + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
  }
  return h;
}

template <class C>
bh_status enqueue_msm(bh_ctx* ctx, bh_job* job, MsmWorkspace<C>& ws, const bh_srs* bases, size_t base_offset, size_t n,
                      size_t set, const uint64_t* density_words, const uint32_t* d_scalars, bool tables,
                      const JobStreams& st) {
  const uint32_t* pts = bases->pts.as<uint32_t>();
  bool tab = false;
  if (tables && set >= TABLE_MIN_USED) {
    std::lock_guard<std::mutex> lk(bases->win_mu);
    if (bases->win_c && bases->win_covers(bases->win_c, base_offset, base_offset + set)) {
      job->sh = msm_shape_table(n, bases->win_c);
      job->sh.rec = bases->win_rec;
      job->table_hold = bases->win;
      pts = bases->win_global();
      tab = true;
    }
  }
  if (!tab) job->sh = msm_shape(n, job->window_override);
  fit_segments_E<C>(job->sh, seg_entries(n, set, job->sh.W));
  bh_job_slot* sl = job->slot;
  bool copied = false;
  if (st.key) {  // the same digits already sorted by a recent job: copy its entries
    bh_job_registry& reg = *job->reg;
    std::lock_guard<std::mutex> lk(reg.mu);  // (the source slot cannot be taken again meanwhile)
    for (const auto& r : reg.sorts) {
      if (r.scalars_id != st.key || r.dens_hash != st.dens_hash || r.n != n || r.base_offset != base_offset ||
          r.c != job->sh.c || r.W != job->sh.W || r.NB != job->sh.NB || r.Wb != job->sh.Wb ||
          r.pre != job->sh.pre || r.slot->use != r.use || r.slot == sl)
        continue;
      const uint32_t *e, *cn, *of;
      if (r.group == BH_G1) { e = r.slot->ws1.entries; cn = r.slot->ws1.counts; of = r.slot->ws1.offsets; }
      else { e = r.slot->ws2.entries; cn = r.slot->ws2.counts; of = r.slot->ws2.offsets; }
      BH_TRY_HIP(ws.reserve_shape(n, job->sh));
      const size_t nbt = (size_t)job->sh.Wb * job->sh.NB;
      // stream order on the sort stream: after the source's sort, before any later reuse of it
      BH_TRY_HIP(hipMemcpyAsync(ws.counts, cn, (nbt + 1) * 4, hipMemcpyDeviceToDevice, st.sort));
      BH_TRY_HIP(hipMemcpyAsync(ws.offsets, of, (nbt + 1) * 4, hipMemcpyDeviceToDevice, st.sort));
      BH_TRY_HIP(hipMemcpyAsync(ws.entries, e, n * (size_t)job->sh.W * 4, hipMemcpyDeviceToDevice, st.sort));
      copied = true;
      break;
    }
  }
  if (!copied) {
    // the density map's base-index map (the sort is its only reader)
    const int32_t* d_idx = nullptr;
    if (density_words) {
      const size_t nw = (n + 63) / 64;
      if (sl->dwords.alloc(nw * 8) || sl->idx.alloc(n * 4) || sl->dtmp.alloc((nw + 1) * 4) ||
          sl->dscan.alloc(scan_scratch_words(nw + 1) * 4 + 64))
        return BH_ERR_OUT_OF_MEMORY;
      // (pageable: the copy is staged before the call returns, on the copy stream so that it
      // never waits behind compute)
      BH_TRY_HIP(hipMemcpyAsync(sl->dwords.p, density_words, nw * 8, hipMemcpyHostToDevice, ctx->h2d));
      BH_TRY_HIP(hipEventRecord(sl->uploaded, ctx->h2d));
      BH_TRY_HIP(hipStreamWaitEvent(st.sort, sl->uploaded, 0));
      BH_TRY_HIP(density_index(sl->dwords.as<uint64_t>(), n, (uint32_t)base_offset, sl->idx.as<int32_t>(),
                               sl->dtmp.as<uint32_t>(), sl->dscan.as<uint32_t>(), st.sort));
      d_idx = sl->idx.as<int32_t>();
    }
    // a sparser density map over a vector already sorted under FULL density with the same digit
    // geometry (a_aux and b_g1_aux over l's aux sort): compact those sorted entries through this
    // map (the prover's derived sort) instead of sorting again
    bool derived = false;
    if (st.key && d_idx) {
      bh_job_registry& reg = *job->reg;
      std::lock_guard<std::mutex> lk(reg.mu);  // (the source slot cannot be taken again meanwhile)
      for (const auto& r : reg.sorts) {
        if (r.scalars_id != st.key || r.dens_hash != 0 || r.n != n || r.c != job->sh.c || r.W != job->sh.W ||
            r.NB != job->sh.NB || r.Wb != job->sh.Wb || r.pre != job->sh.pre || r.slot->use != r.use || r.slot == sl)
          continue;
        const uint32_t *e, *of;
        if (r.group == BH_G1) { e = r.slot->ws1.entries; of = r.slot->ws1.offsets; }
        else { e = r.slot->ws2.entries; of = r.slot->ws2.offsets; }
        BH_TRY_HIP(ws.reserve_shape(n, job->sh));
        const size_t nbt = (size_t)job->sh.Wb * job->sh.NB, Emax = n * (size_t)job->sh.W;
        BH_TRY_HIP(sl->dscan2.alloc(derive_scratch_words(Emax) * 4));
        BH_TRY_HIP(derive_sorted(e, of, nbt, Emax, job->sh.pre, (uint32_t)job->sh.W, (uint32_t)r.base_offset, d_idx,
                                 reinterpret_cast<uint32_t*>(ws.recs), sl->dscan2.as<uint32_t>(), ws.entries,
                                 ws.counts, ws.offsets, st.sort));
        derived = true;
        break;
      }
    }
    if (!derived) BH_TRY_HIP(msm_sort<C>(ws, st.sort, d_scalars, n, d_idx, (uint32_t)base_offset, job->sh));
    if (st.key) {
      bh_job_registry& reg = *job->reg;
      std::lock_guard<std::mutex> lk(reg.mu);
      bh_job_registry::SortRec r;
      r.scalars_id = st.key; r.dens_hash = st.dens_hash; r.n = n; r.base_offset = base_offset;
      r.c = job->sh.c; r.W = job->sh.W; r.NB = job->sh.NB; r.Wb = job->sh.Wb; r.pre = job->sh.pre;
      r.slot = sl; r.group = job->group; r.use = sl->use;
      reg.sorts.push_back(r);
      if (reg.sorts.size() > 16) reg.sorts.erase(reg.sorts.begin());
    }
  }
  // the longest bucket span, read on the device by the tail (no host wait before its enqueue)
  const size_t nbt = (size_t)job->sh.Wb * job->sh.NB;
  BH_TRY_HIP(sl->dspan.alloc(MAX_SPAN_BLOCKS * 4));
  BH_TRY_HIP(max_span(ws.counts, ws.offsets, nbt, (uint32_t)job->sh.S, sl->dspan.as<uint32_t>(), nullptr, st.sort));
  BH_TRY_HIP(hipEventRecord(sl->sorted, st.sort));
  BH_TRY_HIP(hipStreamWaitEvent(st.acc, sl->sorted, 0));
  BH_TRY_HIP(msm_accumulate<C>(ws, st.acc, pts, n, job->sh, nullptr));
  BH_TRY_HIP(hipEventRecord(sl->accumulated, st.acc));
  BH_TRY_HIP(hipStreamWaitEvent(st.tail, sl->accumulated, 0));
  BH_TRY_HIP(msm_back<C>(ws, st.tail, n, job->sh, ws.host_window_sums, -1, nullptr, sl->dspan.as<uint32_t>()));
  BH_TRY_HIP(hipEventRecord(sl->done, st.tail));
  return BH_OK;
}

size_t density_set(const uint64_t* density_words, size_t n) {
  if (!density_words) return n;
  size_t set = 0;
  for (size_t w = 0; w < n / 64; w++) set += (size_t)__builtin_popcountll(density_words[w]);
  if (n % 64) set += (size_t)__builtin_popcountll(density_words[n / 64] & ((1ull << (n % 64)) - 1ull));
  return set;
}

// Common device work of both submits, on the job's slot stream (scalars already ordered before
// it: d_scalars): the density map, the multiexp, the completion event.  On failure the slot
// goes back and the job is left without one.
// G2 jobs accumulate on the small-multiexp stream (stream2, idle under the seam), so a G2
// accumulation runs beside the G1 ones as bh_prove's first accumulation does, instead of queueing
// behind them on the main stream (create_proof submits b_g2_aux last: prover.rs:298-307).  G1 jobs
// alternate between the main stream and stream5, as bh_prove's accumulation lanes do, so
// consecutive G1 accumulations do not wait at a stream barrier for each other's last blocks.
JobStreams job_streams(bh_ctx* ctx, bool g2) {
  static std::atomic<unsigned> rr{0}, lane{0};
  hipStream_t acc = ctx->stream2;
  if (!g2) acc = (ctx->stream5 && (lane.fetch_add(1) & 1)) ? ctx->stream5 : ctx->stream;
  return JobStreams{ctx->stream3, acc, ctx->tstream[rr.fetch_add(1) % bh_ctx::TAIL_STREAMS]};
}

// the slot back after a failed enqueue: whatever was enqueued for it has drained first
void fail_slot(bh_ctx* ctx, bh_job* job) {
  (void)hipStreamSynchronize(ctx->h2d);
  (void)hipStreamSynchronize(ctx->stream3);
  (void)hipStreamSynchronize(ctx->stream);
  (void)hipStreamSynchronize(ctx->stream2);
  if (ctx->stream5) (void)hipStreamSynchronize(ctx->stream5);
  for (hipStream_t t : ctx->tstream) (void)hipStreamSynchronize(t);
  give_slot(*job->reg, job->slot);
  job->slot = nullptr;
}

bh_status enqueue_job(bh_ctx* ctx, bh_job* job, const bh_srs* bases, size_t base_offset,
                      const uint64_t* density_words, size_t n, const uint32_t* d_scalars, uint64_t scalars_id) {
  bh_job_slot* sl = job->slot;
  JobStreams js = job_streams(ctx, bases->group != BH_G1);
  js.key = scalars_id;
  if (scalars_id && density_words) js.dens_hash = words_hash(density_words, (n + 63) / 64) | 1u;
  auto fail = [&](bh_status e) {
    fail_slot(ctx, job);
    return e;
  };
  const size_t set = density_set(density_words, n);
  // window tables as the prover uses them: not under a forced window size (bh_ctx_set_window)
  const bool tables = ctx->tables && !job->window_override;
  bh_status s = bases->group == BH_G1
                    ? enqueue_msm<G1Ops>(ctx, job, sl->ws1, bases, base_offset, n, set, density_words, d_scalars,
                                         tables, js)
                    : enqueue_msm<G2Ops>(ctx, job, sl->ws2, bases, base_offset, n, set, density_words, d_scalars,
                                         tables, js);
  if (s) return fail(s);
  return BH_OK;
}

void add_pending(bh_job* job) {
  std::lock_guard<std::mutex> lk(job->reg->mu);
  job->reg->pending.push_back(job);
}

bh_status submit_check(bh_ctx* ctx, const bh_srs* bases, const uint64_t* density_words, size_t density_len,
                       size_t n) {
  if (density_words && density_len != n) return BH_ERR_DENSITY_SIZE_MISMATCH;  // the reference asserts
  if (n > 0x7fffffffull || !bases->ctx || bases->ctx->device != ctx->device) return BH_ERR_INVALID_ARGUMENT;
  return scratch_check(ctx);  // rather than an abort inside the runtime
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
    reg.sorts.clear();
    for (bh_job_slot* s : reg.free_slots) dead.push_back(s);
    reg.free_slots.clear();
    for (bh_job_slot* s : dead)
      reg.all_slots.erase(std::remove(reg.all_slots.begin(), reg.all_slots.end(), s), reg.all_slots.end());
  }
  for (bh_job_slot* s : dead) delete s;  // (bh_ctx_destroy drained the context's streams first)
}

extern "C" {

bh_status bh_multiexp_submit(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint64_t* density_words,
                             size_t density_len, const uint64_t* exponents, size_t n, int scalar_format,
                             bh_job** out) {
  if (!ctx || !bases || !out || (n && !exponents)) return BH_ERR_INVALID_ARGUMENT;
  if (scalar_format != BH_SCALARS_CANONICAL && scalar_format != BH_SCALARS_MONTGOMERY) return BH_ERR_INVALID_ARGUMENT;
  bh_status s = submit_check(ctx, bases, density_words, density_len, n);
  if (s) return s;
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
  if ((s = take_slot(*job->reg, &job->slot, job_key(bases, base_offset, n)))) return s;
  bh_job_slot* sl = job->slot;
  // the caller's buffers are read before submit returns (pageable copies complete on return)
  bool ok = !sl->raw.alloc(n * 32) && !sl->scalars.alloc(n * 32);
  ok = ok && !hipMemcpyAsync(sl->raw.p, exponents, n * 32, hipMemcpyHostToDevice, ctx->h2d);
  ok = ok && !hipEventRecord(sl->uploaded, ctx->h2d) && !hipStreamWaitEvent(ctx->stream3, sl->uploaded, 0);
  ok = ok && !scalars_prepare(sl->raw.as<uint32_t>(), sl->scalars.as<uint32_t>(), n,
                              scalar_format == BH_SCALARS_MONTGOMERY ? 1 : 0, 0, ctx->stream3);
  if (!ok) {
    fail_slot(ctx, job.get());
    return BH_ERR_HIP;
  }
  if ((s = enqueue_job(ctx, job.get(), bases, base_offset, density_words, n, sl->scalars.as<uint32_t>(), 0)))
    return s;
  add_pending(job.get());
  *out = job.release();
  return BH_OK;
}

// The same over a device-resident scalar vector: nothing crosses PCIe but the density words, and
// the job's stream waits on the device for the vector (e.g. h still being computed)
bh_status bh_multiexp_submit_scalars(bh_ctx* ctx, const bh_srs* bases, size_t base_offset,
                                     const uint64_t* density_words, size_t density_len, const bh_scalars* exps,
                                     bh_job** out) {
  if (!ctx || !bases || !out || !exps || !exps->buf) return BH_ERR_INVALID_ARGUMENT;
  const size_t n = exps->n;
  bh_status s = submit_check(ctx, bases, density_words, density_len, n);
  if (s) return s;
  if (exps->buf->device != ctx->device) return BH_ERR_INVALID_ARGUMENT;
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<bh_job> job(new bh_job());
  job->reg = ctx->jobs;
  job->device = ctx->device;
  job->window_override = ctx->window_override;
  job->group = bases->group;
  job->status = multiexp_check(bases, base_offset, density_words, n, nullptr, false);
  if (job->status == BH_ERR_UNEXPECTED_IDENTITY) {  // the exponents decide: read them back (rare)
    std::vector<uint64_t> host(n * 4);
    exps->buf->wait_enqueued();
    if (exps->buf->status) return exps->buf->status;
    BH_TRY_HIP(hipEventSynchronize(exps->buf->ready));
    BH_TRY_HIP(hipMemcpy(host.data(), exps->buf->d.p, n * 32, hipMemcpyDeviceToHost));
    job->status = multiexp_check(bases, base_offset, density_words, n, host.data(), true);
  }
  if (job->status || n == 0) {
    job->empty = true;
    *out = job.release();
    return BH_OK;
  }
  if ((s = take_slot(*job->reg, &job->slot, job_key(bases, base_offset, n)))) return s;
  job->scalars_hold = exps->buf;
  bh_scalar_buf* buf = exps->buf.get();
  const uint32_t* d_sc = buf->d.as<uint32_t>();
  bh_job* jp = job.get();
  // the device work, after the vector's producer: now, or -- `ready` not yet recorded (h still
  // uploading) -- run by the producer right after it records it
  auto work = [ctx, jp, bases, base_offset, n, d_sc, buf](const uint64_t* dens, bh_status up) {
    bh_status e = up;
    if (!e && hipStreamWaitEvent(ctx->stream3, buf->ready, 0)) e = BH_ERR_HIP;  // the sort reads it first
    if (!e) e = enqueue_job(ctx, jp, bases, base_offset, dens, n, d_sc, buf->id);
    else {
      give_slot(*jp->reg, jp->slot);
      jp->slot = nullptr;
    }
    if (e) {  // reported by wait, like the Source errors
      jp->status = e;
      jp->empty = true;
    }
  };
  if (buf->owner != ctx) {
    // the producer thread runs deferred enqueues on its own context's streams, and only that
    // context's teardown waits for it: a vector still being produced by ANOTHER context is first
    // waited for here (its producer has then enqueued H, stream-ordered behind `ready`), and the
    // job takes the non-deferred path below
    buf->wait_enqueued();
  }
  {
    std::unique_lock<std::mutex> lk(buf->mu);
    if (!buf->enqueued) {
      std::vector<uint64_t> dens;  // the caller's density words are read before submit returns
      if (density_words) dens.assign(density_words, density_words + (n + 63) / 64);
      buf->deferred.push_back([work, dens = std::move(dens)](bh_status up) {
        work(dens.empty() ? nullptr : dens.data(), up);
      });
      jp->deferred = true;
      lk.unlock();
      add_pending(jp);
      *out = job.release();
      return BH_OK;
    }
  }
  work(density_words, buf->status);
  add_pending(jp);
  *out = job.release();
  return BH_OK;
}

bh_status bh_multiexp_wait(bh_job* job, uint8_t* out) {
  if (!job) return BH_ERR_INVALID_ARGUMENT;
  std::unique_ptr<bh_job> j(job);
  if (j->deferred) j->scalars_hold->wait_enqueued();  // its device work is enqueued (or failed)
  bh_job_slot* sl = nullptr;
  {
    std::lock_guard<std::mutex> lk(j->reg->mu);
    auto& pend = j->reg->pending;
    pend.erase(std::remove(pend.begin(), pend.end(), j.get()), pend.end());
    if (!j->detached) sl = j->slot;
  }
  if (j->empty) {
    if (j->status) return j->status;
    if (!out) return BH_ERR_INVALID_ARGUMENT;
    if (j->group == BH_G1) g1_to_uncompressed(jac_to_affine(jac_identity<Fp>()), out);
    else g2_to_uncompressed(jac_to_affine(jac_identity<bh::Fp2>()), out);
    return BH_OK;
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
