// EvaluationDomain with its coefficients resident in HBM (include/bellman_hip.h, bh_evdom_*):
// the reference's EvaluationDomain (domain.rs:21-190) keeps `coeffs` private behind
// AsRef/AsMut/into_coeffs, so a binding may hold them on the device for the whole H block of
// create_proof (prover.rs:210-231: three from_coeffs, ifft + coset_fft each, mul_assign,
// sub_assign, divide_by_z_on_coset, icoset_fft, into_coeffs) instead of moving 2 x m x 32 B over
// PCIe per call (bh_fft & co.).
//
// A domain's logical value is V = k * g^(e*i) (.) T(S): S the stored packed device values (in
// natural or bit-reversed order), T an optional PENDING transform (not yet launched), k a host
// constant and e a power of the multiplicative generator g, by natural index i.  The methods
// only move (k, e, T): ifft multiplies k by m^-1, coset_fft / icoset_fft add +-1 to e,
// divide_by_z_on_coset multiplies k by Z(g)^-1, and a transform is launched when the NEXT one
// (or a pointwise op, or a read) needs it -- with (k, e) folded into its storing pass's
// post-scale (ntt.hip: factor by natural index).  Transforms alternate DIF (natural in,
// bit-reversed out) and DIT (bit-reversed in, natural out) according to the stored order, so no
// permutation pass runs in the reference's H sequence; it launches exactly the 7 transforms of
// the fused H pipeline plus one pointwise product and one difference, and into_scalars writes h
// as canonical scalars from icoset_fft's storing pass (the SCALARS epilogue).  A constant k
// commutes with transforms; only a pending e without a transform to carry it costs a scale pass.
#include <string.h>

#include "api_internal.h"

using namespace bh;

struct bh_evdom {
  bh_ctx* ctx = nullptr;
  int L = 0;
  size_t m = 1;
  // coefficients (packed device Fr), permute / download scratch, the post-scale table of the
  // next launch (built on ctx->stream before it), events; pooled by the context when freed
  std::unique_ptr<EvdomBufs> b;
  DevBuf glo, ghi;  // generic g^(e*i) tables (|e| >= 2, or an arbitrary distribute_powers base)
  bool rev = false; // S is stored in bit-reversed order
  int pend = 0;     // pending transform: 0 none, 1 forward (omega), 2 inverse (omega^-1)
  Fr k;             // pending constant factor
  int e = 0;        // pending power of the generator, by natural index
  bool consumed = false;
  // the asynchronous upload (from_coeffs / write): b->landed on bg.cst; b->idle orders an upload
  // behind the compute still reading the buffer (a write-back, or a pooled buffer's last owner)
  std::mutex mu;
  std::condition_variable cv;
  bool enqueued = true;   // the upload thread has read the host buffer and recorded `landed`
  bool waited = true;     // ctx->stream already waits for `landed`
  bh_status up_status = BH_OK;
};

namespace {

Fr fr_u64(uint64_t v) {
  uint64_t x[4] = {v, 0, 0, 0};
  return from_int<4>(x);
}
const Fr& gen() {  // F::multiplicative_generator() of bls12_381's Fr (= 7), as ctx_domain uses
  static const Fr g = fr_u64(7);
  return g;
}
const Fr& gen_inv() {
  static const Fr g = inv(fr_u64(7));
  return g;
}
const Fr& fr32() {  // bls12_381 Montgomery words read as device values are x / 32
  static const Fr v = fr_u64(32);
  return v;
}
FrConst dev_const(const Fr& x) {  // multiplier for the device kernels: y -> y * x
  FrConst c;
  fr_to_dev_limbs(x, c.v);
  return c;
}
Fr mont_in(const uint64_t g[4]) {  // a bls12_381 Montgomery value (R = 2^256) as a host Fr
  Fr r;
  memcpy(r.v, g, 32);
  return r;
}

// the upload thread of a context (DomainUploads in api_internal.h), started on first use
void dup_push(bh_ctx* ctx, std::function<void()> job) {
  auto& u = ctx->dup;
  std::lock_guard<std::mutex> lk(u.mu);
  if (!u.th.joinable()) {
    u.th = std::thread([&u] {
      for (;;) {
        std::function<void()> f;
        {
          std::unique_lock<std::mutex> l(u.mu);
          u.cv.wait(l, [&] { return u.stop || !u.q.empty(); });
          if (u.q.empty()) return;  // stop, drained
          f = std::move(u.q.front());
          u.q.pop_front();
        }
        f();
      }
    });
  }
  u.q.push_back(std::move(job));
  u.cv.notify_all();
}

// queue the upload of len bls12_381-Montgomery values into d->buf (zero padding to m); the stored
// words are then the device values x / 32 (k = 32).  wait_idle: behind d's compute so far.
bh_status start_upload(bh_evdom* d, const uint64_t* coeffs, size_t len, bool record_idle, bool wait_idle) {
  bh_ctx* ctx = d->ctx;
  if (record_idle) BH_TRY_HIP(hipEventRecord(d->b->idle, ctx->stream));
  wait_idle = wait_idle || record_idle;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    d->enqueued = false;
    d->waited = false;
    d->up_status = BH_OK;
  }
  d->rev = false;
  d->pend = 0;
  d->k = fr32();
  d->e = 0;
  d->consumed = false;
  dup_push(ctx, [d, ctx, coeffs, len, wait_idle] {
    auto run = [&]() -> bh_status {
      std::lock_guard<std::mutex> lk(ctx->bg.mu);
      BH_TRY_HIP(hipSetDevice(ctx->device));
      bh_status s = bg_init(ctx);
      if (s) return s;
      hipStream_t cst = ctx->bg.cst;
      if (wait_idle) BH_TRY_HIP(hipStreamWaitEvent(cst, d->b->idle, 0));
      uint32_t* dst = d->b->buf.as<uint32_t>();
      if (d->m > len) BH_TRY_HIP(hipMemsetAsync(dst + len * 8, 0, (d->m - len) * 32, cst));
      if (len && (s = bg_copy(ctx, dst, coeffs, len * 32))) return s;
      BH_TRY_HIP(hipEventRecord(d->b->landed, cst));
      return BH_OK;
    };
    const bh_status s = run();
    if (s) (void)hipEventRecord(d->b->landed, nullptr);  // (nothing to wait for)
    {
      std::lock_guard<std::mutex> lk(d->mu);
      d->up_status = s;
      d->enqueued = true;
    }
    d->cv.notify_all();
  });
  return BH_OK;
}

// host wait until the upload has been enqueued (the caller's buffer is free again)
bh_status wait_enqueued(bh_evdom* d) {
  std::unique_lock<std::mutex> lk(d->mu);
  d->cv.wait(lk, [&] { return d->enqueued; });
  return d->up_status;
}

// ctx->stream waits for the coefficients to land (caller holds ctx->mu)
bh_status ensure_landed(bh_evdom* d) {
  if (d->waited) return d->up_status;
  bh_status s = wait_enqueued(d);
  if (s) return s;
  BH_TRY_HIP(hipStreamWaitEvent(d->ctx->stream, d->b->landed, 0));
  d->waited = true;
  return BH_OK;
}

// factor(i) = k * g^(e*i) as split tables for the device (lo[i & mask] * hi[i >> bits]; bits < 0:
// the constant hi[0]); false when it is 1.  The tables are built on ctx->stream (stream order
// keeps a rebuild behind the launch that read the previous one).
bool factor_tables(bh_evdom* d, Domain* D, const Fr& k, int e, const uint32_t** lo, const uint32_t** hi,
                   int* bits, bh_status* st) {
  *st = BH_OK;
  if (e == 0 && k == Fr::one()) return false;
  bh_ctx* ctx = d->ctx;
  const int L = d->L;
  const size_t nhi = (size_t)1 << (L > D->lo_bits ? L - D->lo_bits : 0);
  auto alloc = [&](size_t n) -> bool {
    if (d->b->post.alloc(n * 36) != hipSuccess) { *st = BH_ERR_OUT_OF_MEMORY; return false; }
    return true;
  };
  if (e == 0) {  // gpow_hi[0] = g^0 = 1, times k
    if (!alloc(1)) return false;
    launch_table_scale(d->b->post.as<uint32_t>(), D->gpow_hi.as<uint32_t>(), 1, dev_const(k), ctx->stream);
    *lo = nullptr;
    *hi = d->b->post.as<uint32_t>();
    *bits = -1;
  } else if (e == 1) {  // gpow: g^i
    if (!alloc(nhi)) return false;
    launch_table_scale(d->b->post.as<uint32_t>(), D->gpow_hi.as<uint32_t>(), nhi, dev_const(k), ctx->stream);
    *lo = D->gpow_lo.as<uint32_t>();
    *hi = d->b->post.as<uint32_t>();
    *bits = D->lo_bits;
  } else if (e == -1) {  // icoset: m^-1 g^-i, so k * m
    if (!alloc(nhi)) return false;
    launch_table_scale(d->b->post.as<uint32_t>(), D->icoset_hi.as<uint32_t>(), nhi, dev_const(mul(k, fr_u64(d->m))),
                       ctx->stream);
    *lo = D->icoset_lo.as<uint32_t>();
    *hi = d->b->post.as<uint32_t>();
    *bits = D->lo_bits;
  } else {  // (g^e)^i from the host: an unusual chain of distribute_powers calls
    Fr b = Fr::one();
    for (int q = 0; q < (e > 0 ? e : -e); q++) b = mul(b, e > 0 ? gen() : gen_inv());
    if ((*st = upload_split_table(ctx, d->glo, d->ghi, b, k, L, D->lo_bits))) return false;
    *lo = d->glo.as<uint32_t>();
    *hi = d->ghi.as<uint32_t>();
    *bits = D->lo_bits;
  }
  if (hipGetLastError() != hipSuccess) { *st = BH_ERR_HIP; return false; }
  return true;
}

// launch the pending transform with (k, e) in its storing pass (and the given epilogue)
bh_status flush_transform(bh_evdom* d, Domain* D, const NttEpilogue& epi = NttEpilogue()) {
  if (!d->pend) return BH_OK;
  const uint32_t *lo = nullptr, *hi = nullptr;
  int bits = 0;
  bh_status s;
  if (!factor_tables(d, D, d->k, d->e, &lo, &hi, &bits, &s) && s) return s;
  const uint32_t* lv = (d->pend == 1 ? D->lv_fwd : D->lv_inv).as<uint32_t>();
  launch_ntt(d->b->buf.as<uint32_t>(), d->L, !d->rev, lv, lo, hi, bits, d->ctx->stream, nullptr, epi);
  BH_TRY_HIP(hipGetLastError());
  d->rev = !d->rev;
  d->pend = 0;
  d->k = Fr::one();
  d->e = 0;
  return BH_OK;
}

// no pending transform and no pending power: V = k * S
bh_status settle(bh_evdom* d, Domain* D) {
  bh_status s = flush_transform(d, D);
  if (s || d->e == 0) return s;
  const uint32_t *lo = nullptr, *hi = nullptr;
  int bits = 0;
  if (!factor_tables(d, D, d->k, d->e, &lo, &hi, &bits, &s) && s) return s;
  launch_scale(d->b->buf.as<uint32_t>(), d->m, lo, hi, bits, nullptr, d->ctx->stream, d->rev ? d->L : -1);
  BH_TRY_HIP(hipGetLastError());
  d->k = Fr::one();
  d->e = 0;
  return BH_OK;
}

// V = S: settle, then a constant scale pass if k != 1
bh_status materialize(bh_evdom* d, Domain* D) {
  bh_status s = settle(d, D);
  if (s || d->k == Fr::one()) return s;
  const uint32_t *lo = nullptr, *hi = nullptr;
  int bits = 0;
  if (!factor_tables(d, D, d->k, 0, &lo, &hi, &bits, &s) && s) return s;
  launch_scale(d->b->buf.as<uint32_t>(), d->m, lo, hi, bits, nullptr, d->ctx->stream, -1);
  BH_TRY_HIP(hipGetLastError());
  d->k = Fr::one();
  return BH_OK;
}

// stored order of `o` flipped to `rev` (its value unchanged)
bh_status reorder(bh_evdom* o, bool rev) {
  if (o->rev == rev || o->L == 0) { o->rev = rev; return BH_OK; }
  BH_TRY_HIP(o->b->tmp.alloc(o->m * 32));
  launch_permute(o->b->buf.as<uint32_t>(), o->b->tmp.as<uint32_t>(), o->L, nullptr, nullptr, 0, o->ctx->stream);
  BH_TRY_HIP(hipGetLastError());
  std::swap(o->b->buf.p, o->b->tmp.p);
  std::swap(o->b->buf.bytes, o->b->tmp.bytes);
  o->rev = rev;
  return BH_OK;
}

// common prologue: the context's lock, device, domain tables, landed coefficients
struct Op {
  std::unique_lock<std::mutex> lk;
  Domain* D = nullptr;
  bh_status s = BH_OK;
  explicit Op(bh_evdom* d) : lk(d->ctx->mu) {
    if (d->consumed) { s = BH_ERR_INVALID_ARGUMENT; return; }
    if (hipSetDevice(d->ctx->device) != hipSuccess) { s = BH_ERR_HIP; return; }
    if ((s = ctx_domain(d->ctx, d->L, &D))) return;
    s = ensure_landed(d);
  }
};

// the next transform: the pending one is launched first; a pending power that no transform can
// carry (a coset shift BEFORE this transform) is applied by a scale pass; k stays pending
bh_status begin_transform(bh_evdom* d, Domain* D, int dir) {
  bh_status s = flush_transform(d, D);
  if (s) return s;
  if (d->e != 0 && (s = settle(d, D))) return s;
  d->pend = dir;
  return BH_OK;
}

// distribute_powers(b) (domain.rs:101-113): coefficient i times b^i
bh_status distribute(bh_evdom* d, Domain* D, const Fr& b) {
  if (b == gen()) { d->e++; return BH_OK; }
  if (b == gen_inv()) { d->e--; return BH_OK; }
  bh_status s = settle(d, D);
  if (s) return s;
  if ((s = upload_split_table(d->ctx, d->glo, d->ghi, b, Fr::one(), d->L, D->lo_bits))) return s;
  launch_scale(d->b->buf.as<uint32_t>(), d->m, d->glo.as<uint32_t>(), d->ghi.as<uint32_t>(), D->lo_bits, nullptr,
               d->ctx->stream, d->rev ? d->L : -1);
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

}  // namespace

extern "C" {

bh_status bh_evdom_from_coeffs(bh_ctx* ctx, const uint64_t* coeffs, size_t len, bh_evdom** out) {
  if (!ctx || !out || (len && !coeffs)) return BH_ERR_INVALID_ARGUMENT;
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(len, &m, &L);  // domain.rs:51-60
  if (s) return s;
  std::unique_ptr<bh_evdom> d(new bh_evdom());
  d->ctx = ctx;
  d->L = (int)L;
  d->m = m;
  bool pooled = false;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    BH_TRY_HIP(hipSetDevice(ctx->device));
    Domain* D;
    if ((s = ctx_domain(ctx, (int)L, &D))) return s;  // tables built here, not on the first transform
    // a freed domain's buffers (the smallest that fits, at most 4x): its upload then waits for
    // that domain's last work on ctx->stream (b->idle), not for a hipMalloc / hipFree
    auto& pool = ctx->evdom_pool;
    size_t best = pool.size();
    for (size_t i = 0; i < pool.size(); i++) {
      const size_t have = pool[i]->buf.bytes;
      if (have >= m * 32 && have <= 4 * m * 32 + 4096 && (best == pool.size() || have < pool[best]->buf.bytes))
        best = i;
    }
    if (best < pool.size()) {
      d->b = std::move(pool[best]);
      pool.erase(pool.begin() + (long)best);
      pooled = true;
    } else {
      d->b.reset(new EvdomBufs());
      BH_TRY_HIP(d->b->buf.alloc(m * 32));
      BH_TRY_HIP(hipEventCreateWithFlags(&d->b->landed, hipEventDisableTiming));
      BH_TRY_HIP(hipEventCreateWithFlags(&d->b->idle, hipEventDisableTiming));
    }
  }
  if ((s = start_upload(d.get(), coeffs, len, false, pooled))) return s;
  *out = d.release();
  return BH_OK;
}

bh_status bh_evdom_size(const bh_evdom* d, size_t* m, uint32_t* log_m) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  if (m) *m = d->m;
  if (log_m) *log_m = (uint32_t)d->L;
  return BH_OK;
}

// fft / ifft (domain.rs:81-99): ifft = the transform over omega^-1, then m^-1
bh_status bh_evdom_fft(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  return begin_transform(d, op.D, 1);
}
bh_status bh_evdom_ifft(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  bh_status s = begin_transform(d, op.D, 2);
  if (!s) d->k = mul(d->k, op.D->minv);
  return s;
}
// coset_fft = distribute_powers(g) + fft; icoset_fft = ifft + distribute_powers(g^-1) (domain.rs:115-127)
bh_status bh_evdom_coset_fft(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  bh_status s = distribute(d, op.D, gen());
  return s ? s : begin_transform(d, op.D, 1);
}
bh_status bh_evdom_icoset_fft(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  bh_status s = begin_transform(d, op.D, 2);
  if (s) return s;
  d->k = mul(d->k, op.D->minv);
  return distribute(d, op.D, gen_inv());
}
bh_status bh_evdom_distribute_powers(bh_evdom* d, const uint64_t g_mont[4]) {
  if (!d || !g_mont) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  return distribute(d, op.D, mont_in(g_mont));
}
// divide_by_z_on_coset (domain.rs:139-151): times Z(g)^-1 = (g^m - 1)^-1, a constant
bh_status bh_evdom_divide_by_z_on_coset(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  d->k = mul(d->k, op.D->zinv);
  return BH_OK;
}

// mul_assign / sub_assign (domain.rs:153-189): both sides settled, the other one stored in this
// one's order; mul_assign multiplies the pending constants, sub_assign folds a differing one in
static bh_status pointwise(bh_evdom* d, bh_evdom* o, int op_kind) {
  if (!d || !o || d->ctx != o->ctx) return BH_ERR_INVALID_ARGUMENT;
  if (d->m != o->m) return BH_ERR_INVALID_ARGUMENT;  // (the reference asserts equal lengths)
  Op op(d);
  if (op.s) return op.s;
  if (o->consumed) return BH_ERR_INVALID_ARGUMENT;
  bh_status s = ensure_landed(o);
  if (s) return s;
  if ((s = settle(d, op.D))) return s;
  if (o != d && (s = settle(o, op.D))) return s;
  if ((s = reorder(o, d->rev))) return s;
  hipStream_t st = d->ctx->stream;
  if (op_kind == 0) {
    launch_pointwise(d->b->buf.as<uint32_t>(), o->b->buf.as<uint32_t>(), nullptr, d->m, 0, nullptr, st);
    d->k = mul(d->k, o->k);
  } else if (d->k == o->k) {
    launch_pointwise(d->b->buf.as<uint32_t>(), o->b->buf.as<uint32_t>(), nullptr, d->m, 1, nullptr, st);
  } else {
    if (o->k.is_zero() && (s = materialize(o, op.D))) return s;
    // k_d S_d - k_o S_o = k_o ((k_d / k_o) S_d - S_o)
    launch_scale_sub(d->b->buf.as<uint32_t>(), o->b->buf.as<uint32_t>(), d->m, dev_const(mul(d->k, inv(o->k))), st);
    d->k = o->k;
  }
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}
bh_status bh_evdom_mul_assign(bh_evdom* d, bh_evdom* other) { return pointwise(d, other, 0); }
bh_status bh_evdom_sub_assign(bh_evdom* d, bh_evdom* other) { return pointwise(d, other, 1); }

// as_ref / into_coeffs: natural order, bls12_381 Montgomery; the domain keeps its state
bh_status bh_evdom_read(bh_evdom* d, uint64_t* out, size_t len) {
  if (!d || (len && !out) || len > (d ? d->m : 0)) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  if (!len) return BH_OK;
  bh_status s = settle(d, op.D);
  if (s) return s;
  hipStream_t st = d->ctx->stream;
  BH_TRY_HIP(d->b->tmp.alloc(d->m * 32));
  uint32_t* t = d->b->tmp.as<uint32_t>();
  const uint32_t* src = d->b->buf.as<uint32_t>();
  if (d->rev && d->L) {
    launch_permute(src, t, d->L, nullptr, nullptr, 0, st);
    src = t;
  }
  // device value y (y * 2^261) -> y * 2^256 words = the device form of y / 32, reduced; times k
  launch_fr_convert(src, t, len, dev_const(mul(d->k, inv(fr32()))), 1, st);
  BH_TRY_HIP(hipGetLastError());
  BH_TRY_HIP(hipMemcpyAsync(out, t, len * 32, hipMemcpyDeviceToHost, st));
  BH_TRY_HIP(hipStreamSynchronize(st));
  return BH_OK;
}

bh_status bh_evdom_write(bh_evdom* d, const uint64_t* coeffs, size_t len) {
  if (!d || (len && !coeffs) || len > (d ? d->m : 0)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(d->ctx->mu);
  BH_TRY_HIP(hipSetDevice(d->ctx->device));
  (void)wait_enqueued(d);  // a previous upload into the same buffer is replaced (its status too)
  return start_upload(d, coeffs, len, true, true);
}

// prover.rs:226-231 without the round trip: into_coeffs, truncate, to_le_bits -> a device vector
bh_status bh_evdom_into_scalars(bh_evdom* d, size_t len, bh_scalars** out) {
  if (!d || !out || len > (d ? d->m : 0)) return BH_ERR_INVALID_ARGUMENT;
  Op op(d);
  if (op.s) return op.s;
  std::shared_ptr<bh_scalar_buf> buf;
  bh_status s = new_scalar_buf(d->ctx, len, &buf);
  if (s) return s;
  hipStream_t st = d->ctx->stream;
  if (len) {
    if (d->pend) {  // the pending transform's storing pass writes the scalars (natural order)
      NttEpilogue epi;
      epi.kind = NttEpilogue::SCALARS;
      epi.out = buf->d.as<uint32_t>();
      epi.n_out = (uint32_t)len;
      if ((s = flush_transform(d, op.D, epi))) return s;
    } else {
      if ((s = materialize(d, op.D))) return s;
      BH_TRY_HIP(scalars_prepare(d->b->buf.as<uint32_t>(), buf->d.as<uint32_t>(), len, 2, d->rev ? d->L : 0, st));
    }
  }
  BH_TRY_HIP(hipEventRecord(buf->ready, st));
  d->consumed = true;
  *out = new bh_scalars{len, std::move(buf)};
  return BH_OK;
}

bh_status bh_evdom_sync(bh_evdom* d) {
  if (!d) return BH_ERR_INVALID_ARGUMENT;
  return wait_enqueued(d);
}

// (the reference drops b and c right after their use, prover.rs:221-224: no host wait here)
bh_status bh_evdom_free(bh_evdom* d) {
  if (!d) return BH_OK;
  const bh_status us = wait_enqueued(d);  // the upload thread is done with d
  {
    bh_ctx* ctx = d->ctx;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    bool ok = true;
    // the buffers go to the context's pool behind d's last work: the upload (waited on the
    // stream if no method did) and everything enqueued on ctx->stream
    if (!d->waited && !us) ok = hipStreamWaitEvent(ctx->stream, d->b->landed, 0) == hipSuccess;
    if (us) ok = ok && hipEventSynchronize(d->b->landed) == hipSuccess;
    ok = ok && hipEventRecord(d->b->idle, ctx->stream) == hipSuccess;
    if (ok) {
      auto& pool = ctx->evdom_pool;
      pool.push_back(std::move(d->b));
      if (pool.size() > 6) pool.erase(pool.begin());  // (hipFree: waits for the device; rare)
    } else {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipStreamSynchronize(ctx->bg.cst);
    }
    d->b.reset();
    if (d->glo.p || d->ghi.p) {  // (generic tables: rare, freed synchronously)
      d->glo.release();
      d->ghi.release();
    }
  }
  delete d;
  return BH_OK;
}

}  // extern "C"
