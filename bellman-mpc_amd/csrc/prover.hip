// Groth16 prover core on the device: Parameters handling (groth16/mod.rs:224-477)
// and create_proof after synthesis (groth16/prover.rs:206-349).
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <thread>

#include "api_internal.h"
#include "crs.h"
#include "dist_h.h"

using namespace bh;

namespace {

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool take(size_t n, const uint8_t** out) {
    if ((size_t)(end - p) < n) return false;
    *out = p;
    p += n;
    return true;
  }
  bool u32be(uint32_t* v) {
    const uint8_t* b;
    if (!take(4, &b)) return false;
    *v = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
    return true;
  }
};

// VerifyingKey::read uses from_uncompressed (checked), groth16/mod.rs:161-222
bh_status read_g1_vk(Reader& r, AffinePt<Fp>* out, bool reject_identity) {
  const uint8_t* b;
  if (!r.take(96, &b)) return BH_ERR_INVALID_ENCODING;
  if (g1_from_uncompressed(b, out, true, true) != 0) return BH_ERR_INVALID_ENCODING;
  if (reject_identity && out->infinity) return BH_ERR_INVALID_ENCODING;
  return BH_OK;
}
bh_status read_g2_vk(Reader& r, AffinePt<bh::Fp2>* out) {
  const uint8_t* b;
  if (!r.take(192, &b)) return BH_ERR_INVALID_ENCODING;
  if (g2_from_uncompressed(b, out, true, true) != 0) return BH_ERR_INVALID_ENCODING;
  return BH_OK;
}

bh_status read_vec(bh_ctx* ctx, Reader& r, int group, int checked, bh_srs* out) {
  uint32_t len;
  if (!r.u32be(&len)) return BH_ERR_INVALID_ENCODING;
  const size_t pb = group == BH_G1 ? 96 : 192;
  const uint8_t* b;
  if (!r.take((size_t)len * pb, &b)) return BH_ERR_INVALID_ENCODING;
  // Parameters::read rejects points at infinity in every vector (mod.rs:309-318)
  bh_status s = srs_from_bytes(ctx, group, b, len, checked, true, out);
  if (s == BH_ERR_NOT_ON_CURVE) return BH_ERR_INVALID_ENCODING;
  return s;
}

void write_vec(const bh_srs& v, std::vector<uint8_t>& out) {
  const size_t n = v.n;
  out.push_back((uint8_t)(n >> 24)); out.push_back((uint8_t)(n >> 16));
  out.push_back((uint8_t)(n >> 8)); out.push_back((uint8_t)n);
  if (!n) return;
  const int words = v.group == BH_G1 ? 24 : 48;
  std::vector<uint32_t> w(n * words);
  (void)hipMemcpy(w.data(), v.pts.p, n * words * 4, hipMemcpyDeviceToHost);
  std::vector<char> inf(n, 0);
  for (size_t k : v.identity_idx) inf[k] = 1;
  const size_t pb = v.group == BH_G1 ? 96 : 192;
  const size_t base = out.size();
  out.resize(base + n * pb);
  for (size_t i = 0; i < n; i++) {
    const uint32_t* d = &w[i * words];
    uint8_t* o = &out[base + i * pb];
    if (v.group == BH_G1) {
      g1_to_uncompressed(AffinePt<Fp>{fp_from_dev_words_g1(d), fp_from_dev_words_g1(d + 12), inf[i] != 0}, o);
    } else {
      g2_to_uncompressed(AffinePt<bh::Fp2>{bh::Fp2{fp_from_dev_words(d), fp_from_dev_words(d + 12)},
                                           bh::Fp2{fp_from_dev_words(d + 24), fp_from_dev_words(d + 36)}, inf[i] != 0},
                         o);
    }
  }
}

inline size_t popcount_words(const std::vector<uint64_t>& w, size_t nbits) {
  size_t c = 0;
  for (size_t i = 0; i < nbits / 64; i++) c += (size_t)__builtin_popcountll(w[i]);
  if (nbits % 64) c += (size_t)__builtin_popcountll(w[nbits / 64] & ((1ull << (nbits % 64)) - 1ull));
  return c;
}

// ---- the complete assignment on the device (prover.rs:206-231 hands create_proof host
// Vecs).  witness_host: argument checks, sizes, host copies of the density maps and their
// prefix counts, device buffers; witness_device: the staged copies and format conversions on
// stream st, in the order the prover needs them -- density maps, inputs, aux (then up stage
// 1: every multiexp's sort can start), a, b, c (stage 2: the H block can start).
bh_status witness_host(bh_ctx* ctx, bh_witness* w, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                       size_t nc, const uint64_t* inputs, size_t ni, const uint64_t* aux, size_t na,
                       const uint64_t* a_aux_density, const uint64_t* b_input_density,
                       const uint64_t* b_aux_density) {
  if ((nc && (!a || !b || !c)) || (ni && !inputs) || (na && !aux)) return BH_ERR_INVALID_ARGUMENT;
  if ((na && (!a_aux_density || !b_aux_density)) || (ni && !b_input_density)) return BH_ERR_INVALID_ARGUMENT;
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(nc, &m, &L);  // EvaluationDomain::from_coeffs, prover.rs:211-213
  if (s) return s;
  w->ctx = ctx;
  w->num_constraints = nc; w->m = m; w->log_m = (int)L; w->num_inputs = ni; w->num_aux = na;
  BH_TRY_HIP(w->abc.alloc(3 * m * 32));
  BH_TRY_HIP(w->inputs.alloc(std::max<size_t>(ni, 1) * 32));
  BH_TRY_HIP(w->aux.alloc(std::max<size_t>(na, 1) * 32));
  w->a_aux_words = (na + 63) / 64;
  w->b_in_words = (ni + 63) / 64;
  w->b_aux_words = (na + 63) / 64;
  w->a_aux_density.assign(a_aux_density ? a_aux_density : nullptr, a_aux_density ? a_aux_density + w->a_aux_words : nullptr);
  w->b_input_density.assign(b_input_density ? b_input_density : nullptr,
                            b_input_density ? b_input_density + w->b_in_words : nullptr);
  w->b_aux_density.assign(b_aux_density ? b_aux_density : nullptr, b_aux_density ? b_aux_density + w->b_aux_words : nullptr);
  auto prefix = [](const std::vector<uint64_t>& d, size_t words) {
    std::vector<size_t> pc(words + 1, 0);
    for (size_t k = 0; k < words; k++) pc[k + 1] = pc[k] + (size_t)__builtin_popcountll(d[k]);
    return pc;
  };
  w->h_inputs.resize(ni * 4);
  for (size_t i = 0; i < ni; i++) {  // bls12_381 Montgomery -> canonical
    Fr x;
    memcpy(x.v, inputs + 4 * i, 32);
    fr_to_canonical(x, &w->h_inputs[4 * i]);
  }
  w->a_aux_prefix = prefix(w->a_aux_density, w->a_aux_words);
  w->b_aux_prefix = prefix(w->b_aux_density, w->b_aux_words);
  w->a_aux_total = popcount_words(w->a_aux_density, na);
  w->b_in_total = popcount_words(w->b_input_density, ni);
  w->b_aux_total = popcount_words(w->b_aux_density, na);
  const size_t tw = w->a_aux_words + w->b_in_words + w->b_aux_words;
  BH_TRY_HIP(w->dens.alloc(std::max<size_t>(tw, 1) * 8));
  return BH_OK;
}

// Caller (pageable) bytes -> device on the copy stream st: the pinned staging ring (memcpy
// workers + DMA).  (One hipMemcpyAsync from the pageable buffer -- the runtime's own staging, 56
// GB/s in tools/microbench/h2dbench.cpp against ~50 for the ring -- was within noise for bh_prove,
// profiles/r05_ab_dropin_h_uploader.txt, and removed.)
hipError_t upload_host(bh_ctx* ctx, void* dst, const void* src, size_t bytes, hipStream_t st) {
  return ctx->ring.copy(ctx_pool(ctx), dst, src, bytes, st);
}

bh_status witness_device_impl(bh_ctx* ctx, bh_witness* w, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                              const uint64_t* inputs, const uint64_t* aux, hipStream_t st, UploadSync* up) {
  uint64_t* d = w->dens.as<uint64_t>();
  if (w->a_aux_words)
    BH_TRY_HIP(hipMemcpyAsync(d, w->a_aux_density.data(), w->a_aux_words * 8, hipMemcpyHostToDevice, st));
  if (w->b_in_words)
    BH_TRY_HIP(hipMemcpyAsync(d + w->a_aux_words, w->b_input_density.data(), w->b_in_words * 8,
                              hipMemcpyHostToDevice, st));
  if (w->b_aux_words)
    BH_TRY_HIP(hipMemcpyAsync(d + w->a_aux_words + w->b_in_words, w->b_aux_density.data(), w->b_aux_words * 8,
                              hipMemcpyHostToDevice, st));
  HostPool& pool = ctx_pool(ctx);
  const size_t ni = w->num_inputs, na = w->num_aux, nc = w->num_constraints, m = w->m;
  uint32_t* abc = w->abc.as<uint32_t>();
  if (up) {
    // asynchronous (bh_prove): DMA only -- a conversion kernel on this stream would wait for
    // CUs behind the running accumulations and stall the copies queued after it; the
    // prover's own streams convert (compute_msms: aux/inputs before the sorts, a/b/c into
    // the H block's buffer)
    w->raw = true;
    if (ni) BH_TRY_HIP(upload_host(ctx, w->inputs.p, inputs, ni * 32, st));
    if (na) BH_TRY_HIP(upload_host(ctx, w->aux.p, aux, na * 32, st));
    BH_TRY_HIP(hipEventRecord(up->ev[0], st));
    up->set(1);
    const uint64_t* src[3] = {a, b, c};
    for (int v = 0; v < 3; v++) {
      if (nc) BH_TRY_HIP(upload_host(ctx, abc + (size_t)v * m * 8, src[v], nc * 32, st));
      if (up->vec[v]) BH_TRY_HIP(hipEventRecord(up->vec[v], st));
      if (up->on_vector) {
        const bh_status hs = (bh_status)up->on_vector(v);
        if (hs) return hs;
      }
    }
    BH_TRY_HIP(hipEventRecord(up->ev[1], st));
    up->set(2);
    return BH_OK;
  }
  w->raw = false;
  if (ni) {
    BH_TRY_HIP(ctx->ring.copy(pool, w->inputs.p, inputs, ni * 32, st));
    BH_TRY_HIP(scalars_prepare(w->inputs.as<uint32_t>(), w->inputs.as<uint32_t>(), ni, 1, 0, st));
  }
  if (na) {
    BH_TRY_HIP(ctx->ring.copy(pool, w->aux.p, aux, na * 32, st));
    BH_TRY_HIP(scalars_prepare(w->aux.as<uint32_t>(), w->aux.as<uint32_t>(), na, 1, 0, st));
  }
  bh_status s;
  if ((s = upload_fr_staged(ctx, a, nc, m, abc, st))) return s;
  if ((s = upload_fr_staged(ctx, b, nc, m, abc + m * 8, st))) return s;
  if ((s = upload_fr_staged(ctx, c, nc, m, abc + 2 * m * 8, st))) return s;
  return BH_OK;
}

// the density index maps of a device-resident witness, once (density_index: a base index per
// set bit, -1 per clear one), stream-ordered on st after the density words' upload
bh_status witness_index_maps(bh_ctx* ctx, bh_witness* w, hipStream_t st) {
  const size_t ni = w->num_inputs, na = w->num_aux;
  const size_t maxn = std::max({w->m, ni, na, (size_t)1});
  BH_TRY_HIP(w->idx3.alloc((2 * na + ni + 1) * 4));
  BH_TRY_HIP(ctx->dtmp.alloc((maxn / 64 + 2) * 4));
  BH_TRY_HIP(ctx->dscan.alloc(scan_scratch_words(maxn / 64 + 2) * 4 + 64));
  const uint64_t* dens = w->dens.as<uint64_t>();
  int32_t* ia = w->idx3.as<int32_t>();
  if (na) BH_TRY_HIP(density_index(dens, na, (uint32_t)ni, ia, ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(), st));
  if (ni) BH_TRY_HIP(density_index(dens + w->a_aux_words, ni, 0, ia + na, ctx->dtmp.as<uint32_t>(),
                                   ctx->dscan.as<uint32_t>(), st));
  if (na) BH_TRY_HIP(density_index(dens + w->a_aux_words + w->b_in_words, na, (uint32_t)w->b_in_total, ia + na + ni,
                                   ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(), st));
  w->idx_ready = true;
  return BH_OK;
}

// always leaves `up` in a final stage (2, or -1 with the status) so that no waiter hangs
bh_status witness_device(bh_ctx* ctx, bh_witness* w, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                         const uint64_t* inputs, const uint64_t* aux, hipStream_t st, UploadSync* up) {
  bh_status s = witness_device_impl(ctx, w, a, b, c, inputs, aux, st, up);
  if (s && up) up->set(-1, s);
  return s;
}

}  // namespace

extern "C" {

bh_status bh_params_load(bh_ctx* ctx, const uint8_t* bytes, size_t len, int checked, bh_params** out) {
  if (!ctx || !bytes || !out) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<bh_params> p(new bh_params());
  p->ctx = ctx;
  Reader r{bytes, bytes + len};
  bh_status s;
  if ((s = read_g1_vk(r, &p->alpha_g1, false))) return s;
  if ((s = read_g1_vk(r, &p->beta_g1, false))) return s;
  if ((s = read_g2_vk(r, &p->beta_g2))) return s;
  if ((s = read_g2_vk(r, &p->gamma_g2))) return s;
  if ((s = read_g1_vk(r, &p->delta_g1, false))) return s;
  if ((s = read_g2_vk(r, &p->delta_g2))) return s;
  uint32_t ic_len;
  if (!r.u32be(&ic_len)) return BH_ERR_INVALID_ENCODING;
  p->ic.resize(ic_len);
  for (uint32_t i = 0; i < ic_len; i++)
    if ((s = read_g1_vk(r, &p->ic[i], true))) return s;
  if ((s = read_vec(ctx, r, BH_G1, checked, &p->h))) return s;
  if ((s = read_vec(ctx, r, BH_G1, checked, &p->l))) return s;
  if ((s = read_vec(ctx, r, BH_G1, checked, &p->a))) return s;
  if ((s = read_vec(ctx, r, BH_G1, checked, &p->b_g1))) return s;
  if ((s = read_vec(ctx, r, BH_G2, checked, &p->b_g2))) return s;
  *out = p.release();
  return BH_OK;
}

bh_status bh_params_free(bh_params* p) {
  delete p;
  return BH_OK;
}

bh_status bh_params_sizes(const bh_params* p, size_t out[6]) {
  if (!p || !out) return BH_ERR_INVALID_ARGUMENT;
  out[0] = p->h.n; out[1] = p->l.n; out[2] = p->a.n; out[3] = p->b_g1.n; out[4] = p->b_g2.n; out[5] = p->ic.size();
  return BH_OK;
}

// Parameters::write (groth16/mod.rs:260-290)
bh_status bh_params_write(const bh_params* p, uint8_t* out, size_t cap, size_t* written) {
  if (!p || !written) return BH_ERR_INVALID_ARGUMENT;
  std::vector<uint8_t> v;
  uint8_t b[192];
  g1_to_uncompressed(p->alpha_g1, b); v.insert(v.end(), b, b + 96);
  g1_to_uncompressed(p->beta_g1, b); v.insert(v.end(), b, b + 96);
  g2_to_uncompressed(p->beta_g2, b); v.insert(v.end(), b, b + 192);
  g2_to_uncompressed(p->gamma_g2, b); v.insert(v.end(), b, b + 192);
  g1_to_uncompressed(p->delta_g1, b); v.insert(v.end(), b, b + 96);
  g2_to_uncompressed(p->delta_g2, b); v.insert(v.end(), b, b + 192);
  const size_t n = p->ic.size();
  v.push_back((uint8_t)(n >> 24)); v.push_back((uint8_t)(n >> 16)); v.push_back((uint8_t)(n >> 8)); v.push_back((uint8_t)n);
  for (const auto& ic : p->ic) { g1_to_uncompressed(ic, b); v.insert(v.end(), b, b + 96); }
  write_vec(p->h, v);
  write_vec(p->l, v);
  write_vec(p->a, v);
  write_vec(p->b_g1, v);
  write_vec(p->b_g2, v);
  *written = v.size();
  if (!out) return BH_OK;  // size query
  if (cap < v.size()) return BH_ERR_INVALID_ARGUMENT;
  memcpy(out, v.data(), v.size());
  return BH_OK;
}

bh_status bh_witness_upload(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c, size_t nc,
                            const uint64_t* inputs, size_t ni, const uint64_t* aux, size_t na,
                            const uint64_t* a_aux_density, const uint64_t* b_input_density,
                            const uint64_t* b_aux_density, bh_witness** out) {
  if (!ctx || !out) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<bh_witness> w(new bh_witness());
  bh_status s = witness_host(ctx, w.get(), a, b, c, nc, inputs, ni, aux, na, a_aux_density, b_input_density,
                             b_aux_density);
  if (s) return s;
  if ((s = witness_device(ctx, w.get(), a, b, c, inputs, aux, ctx->h2d, nullptr))) return s;
  if ((s = witness_index_maps(ctx, w.get(), ctx->h2d))) return s;
  BH_TRY_HIP(hipStreamSynchronize(ctx->h2d));
  *out = w.release();
  return BH_OK;
}

bh_status bh_witness_free(bh_witness* w) {
  delete w;
  return BH_OK;
}

}  // extern "C"

namespace {

struct VkHost {
  AffinePt<Fp> alpha_g1, beta_g1, delta_g1;
  AffinePt<bh::Fp2> beta_g2, delta_g2;
};

// shard k of n items: [k*n/N, (k+1)*n/N)
inline void shard_range(size_t n, size_t k, size_t N, size_t* lo, size_t* hi) {
  *lo = (size_t)((unsigned __int128)n * k / N);
  *hi = (size_t)((unsigned __int128)n * (k + 1) / N);
}

// The 8 multiexps of create_proof (prover.rs:233-307) restricted to scalar shard
// ---- SRS window tables.  A multiexp over a fixed base vector can trade HBM for work: with
// T[i*W + w] = 2^(c*w) * P_i resident, every digit window adds into ONE set of 2^(c-1)
// buckets, so the window size is no longer tied to W bucket reductions and c can grow
// (c = 20 at 2^22 points: 13 instead of 16 additions per scalar).  Tables are built once
// per (vector, c) -- a function of the CRS only, like Parameters::read -- and cost
// n * ceil(256/c) points, each padded to whole 128-byte lines so one gather is one (G1)
// or two (G2) lines (7 GB for a 2^22-point G1 vector at c = 20, 14 GB for b_g2).
constexpr size_t SMALL_JOB = 4096;                   // run whole on a side stream (latency-bound)

int table_c_for(size_t used_per_shard) {
  return used_per_shard >= TABLE_MIN_USED ? msm_table_c(used_per_shard) : 0;
}

// ---- Bucket shards.  With N > 1 ranks a table multiexp (one shared set of 2^(c-1) buckets)
// is split by BUCKET range instead of scalar range: every rank reads all the scalars, keeps the
// digits that fall in its range of buckets, accumulates and reduces only those, and the ranks'
// parts sum to the multiexp like scalar shards do (bh_proof_from_partials).  Against a scalar
// shard of n/N points, which needs its own smaller window (c = 16 at 2^19 points: 16 windows
// against 13) and still reduces a whole bucket set of its own, each rank keeps one GPU's c = 20
// and 1/N of its bucket reduction.  The ranges come from the digit distribution of uniformly
// distributed scalars (bucket_cdf); a skewed witness (e.g. many small values) stays correct, its
// ranks just do unequal work.  Measured in the one-GPU rehearsal at 2^22 (round 5,
// profiles/r05_ab_bucket_shards.txt) it is no faster than scalar shards: each rank's G1
// accumulations take ~12 % less time, but every rank sorts all the scalars (8x the partition
// scan), and its bucket range holds as many continuation partials per bucket as a c = 16 shard's
// buckets do, so the reductions do not shrink.  Off by default; BH_SHARD_BUCKETS=1 (read per
// proof, on every rank alike) selects it.
bool bucket_shards_on() {
  const char* e = getenv("BH_SHARD_BUCKETS");
  return e && e[0] == '1';
}

// Expected digits per scalar in buckets [0, b) of a shared-bucket table of W c-bit signed
// windows (digit_at): the W - 1 lower windows spread |d| in [1, 2^(c-1)] evenly over the
// NB = 2^(c-1) buckets; the top window holds t + carry with t <= T = (r - 1) >> (c * (W - 1))
// (r: the Fr modulus, 0x73eda753299d7d48... in its top 64 bits), so its digits fill buckets
// [0, T + 1) evenly.
double bucket_cdf(int c, int W, double b) {
  const double NB = (double)((size_t)1 << (c - 1));
  const int top_shift = c * (W - 1);
  double T1 = NB;  // (a top window below bit 192: treated like the others)
  if (top_shift >= 192 && top_shift < 256) T1 = (double)(0x73eda753299d7d48ull >> (top_shift - 192)) + 1.0;
  if (T1 > NB) T1 = NB;
  return (W - 1) * b / NB + std::min(b, T1) / T1;
}

// Bucket shards for a proof with na aux scalars on N ranks, co_ranks of them side by side on
// each device?  The same answer on every rank (a function of the shape only): every rank sorts all
// na scalars of the four aux multiexps, so its workspaces (entries + partition records, 12 B per
// digit, and the continuation partials) do not shrink with N -- ~5 GB per rank at 2^22.  Scalar
// shards when co_ranks of them would take over a quarter of the device (8 virtual ranks at 2^24).
bool bucket_shards_use(int device, size_t na, size_t nshards, int co_ranks) {
  if (nshards < 2 || !bucket_shards_on()) return false;
  size_t total = 0;
  if (hipDeviceTotalMem(&total, device) != hipSuccess || total == 0) return false;
  const double ws = 4.0 * (double)na * 16.0 * 12.0 * 1.6;  // (16: the most windows of a table size)
  return (double)std::max(co_ranks, 1) * ws <= (double)total / 4.0;
}

// Rank `shard` of N: its bucket range [lo, hi), granule-aligned, balancing the expected
// accumulation (used * bucket_cdf) plus the reduction (3 additions per bucket).  False when the bucket set is too small to give every rank several granules.
bool bucket_shard_range(int c, size_t used, size_t shard, size_t N, uint32_t* lo, uint32_t* hi) {
  const int W = (256 + c - 1) / c;
  const uint32_t NB = 1u << (c - 1);
  const uint32_t G = std::max<uint32_t>(BUCKET_SHARD_GRANULE, NB >> 12);  // (sort partition width)
  if ((size_t)NB < 4 * N * G) return false;
  constexpr double kw = 3.0;
  auto cost = [&](double b) { return (double)used * bucket_cdf(c, W, b) + kw * b; };
  const double total = cost(NB);
  auto bound = [&](size_t k) -> uint32_t {
    if (k == 0) return 0;
    if (k >= N) return NB;
    const double target = total * (double)k / (double)N;
    double a = 0, z = NB;
    for (int it = 0; it < 64; it++) {
      const double m = 0.5 * (a + z);
      (cost(m) < target ? a : z) = m;
    }
    uint32_t g = (uint32_t)std::llround(a / G);
    g = std::max<uint32_t>(g, (uint32_t)k);                      // every rank keeps >= one granule
    g = std::min<uint32_t>(g, NB / G - (uint32_t)(N - k));
    return g * G;
  };
  *lo = bound(shard);
  *hi = bound(shard + 1);
  return *hi > *lo;
}

// Window table of c-bit windows over the bases [lo, hi) of srs (a shard's slice, or the whole
// vector): kept if the resident table already covers them at this c, else rebuilt for exactly
// [lo, hi).  Skipped (plain windows, same results) when HBM is short -- reported once.
bool table_wanted(const bh_srs* srs, int c, size_t lo, size_t hi) {
  if (c == 0 || hi <= lo || srs->win_covers(c, lo, hi)) return false;
  if (srs->skip_c == c && srs->skip_lo == lo && srs->skip_hi == hi) return false;  // HBM short last time
  if (!srs->identity_idx.empty() || srs->n == 0 || hi > srs->n) return false;
  return (unsigned __int128)hi * ((256 + c - 1) / c) < ((size_t)1 << 31);
}

bh_status ensure_table(bh_ctx* ctx, bh_srs* srs, int c, size_t lo, size_t hi) {
  if (c == 0 || hi <= lo || srs->win_covers(c, lo, hi)) return BH_OK;
  if (!srs->identity_idx.empty() || srs->n == 0 || hi > srs->n) return BH_OK;  // identities: plain windows only
  const int W = (256 + c - 1) / c;
  if ((unsigned __int128)hi * W >= ((size_t)1 << 31)) return BH_OK;  // entry encoding limit (global index)
  const bool g2 = srs->group == BH_G2;
  const uint32_t rec = g2 ? G2_TABLE_REC : G1_TABLE_REC;  // 224 / 112-byte raw-limb points in whole 128-byte lines
  const size_t n = hi - lo;
  const size_t bytes = n * W * rec * 4;
  const size_t chunk = std::min<size_t>(n, (size_t)1 << 19);
  const size_t scratch = g2 ? window_table_scratch_bytes<G2Ops>(chunk, W) : window_table_scratch_bytes<G1Ops>(chunk, W);
  {
    // a fresh buffer: multiexp jobs still reading the old table keep it alive until their wait
    std::lock_guard<std::mutex> lk(srs->win_mu);
    srs->win = std::make_shared<DevBuf>();
    srs->win_c = 0;
    srs->win_lo = srs->win_hi = 0;
  }
  size_t free_b = 0, total_b = 0;
  BH_TRY_HIP(hipMemGetInfo(&free_b, &total_b));
  if (bytes + scratch + ((size_t)4 << 30) > free_b) {  // keep 4 GB headroom
    if (srs->skip_c != c || srs->skip_lo != lo || srs->skip_hi != hi)
      fprintf(stderr, "bellman_hip: window table skipped (%.2f GB needed, %.2f GB free): plain windows\n",
              (bytes + scratch) / 1e9, free_b / 1e9);
    srs->skip_c = c; srs->skip_lo = lo; srs->skip_hi = hi;
    return BH_OK;
  }
  BH_TRY_HIP(srs->win->alloc(bytes));
  DevBuf tmp;
  BH_TRY_HIP(tmp.alloc(scratch));
  const uint32_t* pts = srs->pts.as<uint32_t>() + lo * (g2 ? 48 : 24);
  if (g2) BH_TRY_HIP(window_table<G2Ops>(pts, n, c, W, srs->win->as<uint32_t>(), rec, tmp.p, chunk, ctx->stream));
  else BH_TRY_HIP(window_table<G1Ops>(pts, n, c, W, srs->win->as<uint32_t>(), rec, tmp.p, chunk, ctx->stream));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  std::lock_guard<std::mutex> lk(srs->win_mu);
  srs->win_c = c;
  srs->win_W = W;
  srs->win_rec = (int)rec;
  srs->win_lo = lo;
  srs->win_hi = hi;
  return BH_OK;
}

// BH_ACC_EVENTS=0: no timing events around the accumulations (A/B of their cost; the
// accumulation timings of bh_last_timings then read 0)
bool acc_events_on() {  // (read per proof: tests/test_gpu_parity.py runs both modes)
  const char* e = getenv("BH_ACC_EVENTS");
  return !(e && e[0] == '0');
}

// One multiexp of create_proof (prover.rs:233-307) as planned for a shard.
struct Job {
  bool g2 = false;
  const bh_srs* srs = nullptr;  // bases: a Parameters vector, or a gathered h share
  const uint32_t* sc = nullptr; // device scalars (canonical, packed)
  size_t n = 0;                 // full query length (sharded below)
  const int32_t* idx = nullptr; // device density map (global base index, -1 = absent) or null
  size_t used = 0;              // density-set scalars (roofline accounting)
  int out = 0;                  // result slot: G1 0..5 / G2 0..1
  bool is_h = false;            // h: needs the H pipeline
  bool presharded = false;      // n/idx are this shard's already (distributed H)
  // host view for base ranges: dense (prefix == null) scalar i uses base boff + i; with a
  // density map the set bits before i count the bases consumed
  const std::vector<uint64_t>* hdens = nullptr;
  const std::vector<size_t>* prefix = nullptr;
  size_t boff = 0;
  // filled by plan_shard
  size_t lo = 0, hi = 0;    // this shard's scalars
  size_t blo = 0, bhi = 0;  // the bases they consume
  int table_c = 0;          // window size of this job's table (0: plain windows)
  uint32_t bk_lo = 0, bk_hi = 0;  // bucket shard (MsmShape::bk_lo): every scalar, these buckets
};

inline size_t dens_before(const Job& J, size_t i) {
  if (!J.prefix) return i;
  const size_t k = i / 64, r = i % 64;
  size_t c = (*J.prefix)[k];
  if (r) c += (size_t)__builtin_popcountll((*J.hdens)[k] & ((1ull << r) - 1ull));
  return c;
}

// The shape of the distributed-H share of rank `rank` of N at m = 2^L (dist_h.h): position
// p = t*C + u holds h[M*t + rank*C + u]; the last rank's last position is the truncated
// coefficient m-1 (prover.rs:227), so its share has M-1 scalars.
struct ShareGeom {
  int N = 0, rank = 0, L = 0;
  size_t M = 0, C = 0;
  size_t used() const { return rank == N - 1 ? M - 1 : M; }
};

// h bases of a share, gathered into share order (built once per Parameters, N, rank, L)
bh_status ensure_h_share(bh_ctx* ctx, bh_params* params, const ShareGeom& g, bh_srs** out) {
  auto key = std::make_tuple(g.N, g.rank, g.L);
  auto it = params->h_shares.find(key);
  if (it != params->h_shares.end()) { *out = it->second.get(); return BH_OK; }
  std::unique_ptr<bh_srs> sh(new bh_srs());
  sh->ctx = ctx;
  sh->group = BH_G1;
  sh->n = g.used();
  BH_TRY_HIP(sh->pts.alloc(std::max<size_t>(sh->n, 1) * 96));
  const uint8_t* src = params->h.pts.as<uint8_t>();
  uint8_t* dst = sh->pts.as<uint8_t>();
  for (int t = 0; t < g.N; t++) {
    const size_t k0 = (size_t)t * g.M + (size_t)g.rank * g.C;
    const size_t cnt = std::min(g.C, params->h.n > k0 ? params->h.n - k0 : 0);
    if (cnt) BH_TRY_HIP(hipMemcpyAsync(dst + (size_t)t * g.C * 96, src + k0 * 96, cnt * 96, hipMemcpyDeviceToDevice,
                                       ctx->stream));
  }
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  *out = sh.get();
  params->h_shares[key] = std::move(sh);
  return BH_OK;
}

// ---- The public-input multiexps (a_inputs, b_g1_inputs, b_g2_inputs: prover.rs:262-307 over
// the input assignment) are a few terms for any circuit with few public inputs -- 2 for the
// MiMC chain, at most 1 per rank of an N-GPU run.  On the device each would still run a full
// sort and bucket reduction on the side streams, beside the accumulations; a host thread
// computes them (double-and-add, bellman's own per-term cost) while the device works.
constexpr size_t HOST_INPUT_MSM_MAX = 64;

// the first n points of a device vector, on the host (device Montgomery -> host Montgomery)
template <bool G2>
bh_status read_head(const bh_srs& v, size_t n, std::vector<typename std::conditional<G2, AffinePt<bh::Fp2>, AffinePt<Fp>>::type>* out) {
  const size_t words = G2 ? 48 : 24;
  std::vector<uint32_t> w(std::max<size_t>(n, 1) * words);
  if (n) BH_TRY_HIP(hipMemcpy(w.data(), v.pts.p, n * words * 4, hipMemcpyDeviceToHost));
  out->resize(n);
  for (size_t i = 0; i < n; i++) {
    const uint32_t* d = &w[i * words];
    if constexpr (G2)
      (*out)[i] = AffinePt<bh::Fp2>{bh::Fp2{fp_from_dev_words(d), fp_from_dev_words(d + 12)},
                                    bh::Fp2{fp_from_dev_words(d + 24), fp_from_dev_words(d + 36)}, false};
    else
      (*out)[i] = AffinePt<Fp>{fp_from_dev_words_g1(d), fp_from_dev_words_g1(d + 12), false};
  }
  return BH_OK;
}

// shard [lo, hi) of the input multiexps -> r_a (a_inputs), r_b1 (b_g1_inputs), r_b2 (b_g2_inputs)
bh_status host_input_msms(int device, bh_params* p, const bh_witness* w, size_t lo, size_t hi, Jac<Fp>* r_a,
                          Jac<Fp>* r_b1, Jac<bh::Fp2>* r_b2) {
  *r_a = jac_identity<Fp>();
  *r_b1 = jac_identity<Fp>();
  *r_b2 = jac_identity<bh::Fp2>();
  if (hi <= lo) return BH_OK;
  const auto bit = [&](size_t i) { return (w->b_input_density[i / 64] >> (i % 64)) & 1ull; };
  size_t nb = 0;  // b bases consumed before lo, and the total up to hi
  for (size_t i = 0; i < lo; i++) nb += bit(i);
  size_t nb_hi = nb;
  for (size_t i = lo; i < hi; i++) nb_hi += bit(i);
  // The cache only grows (a rank never shrinks what another one read), and this rank's points are
  // copied out under the lock: N rank threads share one bh_params (run_ranks), with different
  // [lo, hi) ranges, and a concurrent refill may reallocate the vectors.
  std::vector<AffinePt<Fp>> a_pts, b1_pts;
  std::vector<AffinePt<bh::Fp2>> b2_pts;
  {
    std::lock_guard<std::mutex> lk(p->head_mu);
    if (p->h_a_head.size() < hi || p->h_b1_head.size() < nb_hi || p->h_b2_head.size() < nb_hi) {
      if (hipSetDevice(device) != hipSuccess) return BH_ERR_HIP;
      const size_t na = std::max(hi, p->h_a_head.size());
      const size_t nb2 = std::max(nb_hi, std::max(p->h_b1_head.size(), p->h_b2_head.size()));
      bh_status s;
      if ((s = read_head<false>(p->a, na, &p->h_a_head))) return s;
      if ((s = read_head<false>(p->b_g1, nb2, &p->h_b1_head))) return s;
      if ((s = read_head<true>(p->b_g2, nb2, &p->h_b2_head))) return s;
    }
    a_pts.assign(p->h_a_head.begin() + lo, p->h_a_head.begin() + hi);
    b1_pts.assign(p->h_b1_head.begin() + nb, p->h_b1_head.begin() + nb_hi);
    b2_pts.assign(p->h_b2_head.begin() + nb, p->h_b2_head.begin() + nb_hi);
  }
  for (size_t i = lo, j = 0; i < hi; i++) {
    const uint64_t* k = &w->h_inputs[4 * i];
    *r_a = jac_add(*r_a, jac_mul(jac_from_affine(a_pts[i - lo]), k, 4));
    if (bit(i)) {
      *r_b1 = jac_add(*r_b1, jac_mul(jac_from_affine(b1_pts[j]), k, 4));
      *r_b2 = jac_add(*r_b2, jac_mul(jac_from_affine(b2_pts[j]), k, 4));
      j++;
    }
  }
  return BH_OK;
}

// Caller holds params->mu: exclusively with build = true (tables and shares are rebuilt in
// place), shared otherwise.
// Plan the 8 multiexps of shard `shard` of `nshards`: scalar ranges, the base ranges they
// consume and the window table each one uses; with build = true the tables (slices of the
// Parameters vectors, or a gathered h share) are made resident first.  share: the
// distributed-H geometry when h comes from the distributed pipeline (then the h job covers
// the share, not a range).  Device pointers may be null when only tables are prepared.
bh_status plan_shard(bh_ctx* ctx, const bh_params* params_c, const bh_witness* w, size_t shard, size_t nshards,
                     const ShareGeom* share, const uint32_t* hbuf, const int32_t* hidx, const int32_t* idx_aaux,
                     const int32_t* idx_bin, const int32_t* idx_baux, bool build, Job jobs[8]) {
  bh_params* params = const_cast<bh_params*>(params_c);  // tables are a cache of the CRS
  const size_t m = w->m, ni = w->num_inputs, na = w->num_aux;
  const uint32_t* inputs = w->inputs.as<uint32_t>();
  const uint32_t* aux = w->aux.as<uint32_t>();
  const bool tables = ctx->tables && !ctx->window_override;
  Job hjob;
  hjob.srs = &params->h; hjob.sc = ctx->hbuf.as<uint32_t>(); hjob.n = m - 1; hjob.used = m - 1; hjob.out = 0;
  hjob.is_h = true;
  if (share) {
    hjob.presharded = true;
    hjob.sc = hbuf;
    hjob.used = share->used();
    const int c = tables ? table_c_for(share->used()) : 0;
    bh_srs* sh = nullptr;
    if (c && !params->h.win_covers(c, 0, m - 1)) {
      // no full-vector table at this c (the per-rank case): a table over the share's own bases
      auto it = params->h_shares.find(std::make_tuple(share->N, share->rank, share->L));
      if (it != params->h_shares.end()) sh = it->second.get();
      else if (build) {
        bh_status s = ensure_h_share(ctx, params, *share, &sh);
        if (s) return s;
      }
    }
    if (sh) {
      hjob.srs = sh;
      hjob.n = share->used();
      hjob.idx = nullptr;  // position p of the share = base p of the gathered vector
    } else {
      hjob.n = share->M;
      hjob.idx = hidx;  // global indices into the full h vector (-1: truncated coefficient)
    }
  }
  auto mk = [](bool g2, const bh_srs* srs, const uint32_t* sc, size_t n, const int32_t* idx, size_t used, int out,
               const std::vector<uint64_t>* hd, const std::vector<size_t>* pf, size_t boff) {
    Job j;
    j.g2 = g2; j.srs = srs; j.sc = sc; j.n = n; j.idx = idx; j.used = used; j.out = out;
    j.hdens = hd; j.prefix = pf; j.boff = boff;
    return j;
  };
  // G2 first (the longest tail gets the most overlap), then b_g1_aux whose sorted digits are
  // a copy of b_g2_aux's (so both are ready at the first accumulation for the price of one
  // sort), h last so the H pipeline has the most slack
  jobs[0] = mk(true, &params->b_g2, aux, na, idx_baux, w->b_aux_total, 1, &w->b_aux_density, &w->b_aux_prefix,
               w->b_in_total);                                                                         // b_g2_aux
  jobs[1] = mk(false, &params->b_g1, aux, na, idx_baux, w->b_aux_total, 5, &w->b_aux_density, &w->b_aux_prefix,
               w->b_in_total);                                                                         // b_g1_aux
  // (b_g1_aux first, b_g2_aux copying its sort: N = 8 +0.2 ms per rank, r03_ab_g1_first.txt; removed)
  jobs[2] = mk(false, &params->l, aux, na, nullptr, na, 1, nullptr, nullptr, 0);                       // l
  jobs[3] = mk(false, &params->a, aux, na, idx_aaux, w->a_aux_total, 3, &w->a_aux_density, &w->a_aux_prefix,
               ni);                                                                                    // a_aux
  jobs[4] = hjob;                                                                                      // h
  jobs[5] = mk(false, &params->a, inputs, ni, nullptr, ni, 2, nullptr, nullptr, 0);                   // a_inputs
  jobs[6] = mk(false, &params->b_g1, inputs, ni, idx_bin, w->b_in_total, 4, nullptr, nullptr, 0);     // b_g1_inputs
  jobs[7] = mk(true, &params->b_g2, inputs, ni, idx_bin, w->b_in_total, 0, nullptr, nullptr, 0);      // b_g2_inputs
  // the large aux multiexps (b_g2_aux, b_g1_aux, l, a_aux) are bucket shards when N > 1
  const bool bshard = tables && bucket_shards_use(ctx->device, na, nshards, ctx->co_ranks);
  for (int j = 0; j < 8; j++) {
    Job& J = jobs[j];
    J.table_c = 0;
    J.bk_lo = J.bk_hi = 0;
    if (bshard && j <= 3 && !J.is_h && J.n && J.used >= TABLE_MIN_USED) {
      const int c = table_c_for(J.used);
      if (c && bucket_shard_range(c, J.used, shard, nshards, &J.bk_lo, &J.bk_hi)) {
        J.lo = 0; J.hi = J.n;
        J.blo = J.boff; J.bhi = J.boff + dens_before(J, J.n);
        J.table_c = c;
        continue;
      }
      J.bk_lo = J.bk_hi = 0;
    }
    if (J.presharded) { J.lo = 0; J.hi = J.n; }
    else shard_range(J.n, shard, nshards, &J.lo, &J.hi);
    if (J.hi == J.lo) continue;
    const size_t used = (size_t)((unsigned __int128)J.used * (J.hi - J.lo) / std::max<size_t>(J.n, 1));
    if (J.idx && !J.prefix && J.presharded) {  // h share over the full vector: any base may be used
      J.blo = 0; J.bhi = J.srs->n;
    } else if (j >= 5) {  // the public-input multiexps: tiny, plain windows
      J.blo = J.boff; J.bhi = J.boff;
    } else {
      J.blo = J.boff + dens_before(J, J.lo);
      J.bhi = J.boff + dens_before(J, J.hi);
    }
    if (tables && used >= TABLE_MIN_USED) J.table_c = table_c_for(used);
  }
  if (build) {
    for (int j = 0; j < 8; j++) {
      const Job& J = jobs[j];
      if (!J.table_c) continue;
      bh_status s = ensure_table(ctx, const_cast<bh_srs*>(J.srs), J.table_c, J.blo, J.bhi);
      if (s) return s;
    }
  }
  return BH_OK;
}

// would plan_shard(build = true) change anything resident?
bool plan_needs_build(const bh_params* params, const Job jobs[8], const ShareGeom* share, bool tables) {
  if (share && tables) {
    const int c = table_c_for(share->used());
    const size_t m_1 = params->h.n;
    if (c && !params->h.win_covers(c, 0, m_1) &&
        !params->h_shares.count(std::make_tuple(share->N, share->rank, share->L)))
      return true;
  }
  for (int j = 0; j < 8; j++)
    if (jobs[j].table_c && table_wanted(jobs[j].srs, jobs[j].table_c, jobs[j].blo, jobs[j].bhi)) return true;
  return false;
}

// Full-vector tables at the window size of one of nshards shards (bh_params_prepare): every
// shard's slice is covered, so one device can run all N shards (rehearsal, partials_local).
bh_status prepare_tables_full(bh_ctx* ctx, bh_params* params, size_t m, size_t na, size_t a_aux_used,
                              size_t b_aux_used, size_t nshards, int co_ranks = 1) {
  if (!ctx->tables || ctx->window_override) return BH_OK;
  const size_t N = std::max<size_t>(nshards, 1);
  bh_status s;
  // bucket shards (plan_shard) keep one GPU's window size for the aux vectors
  const size_t Naux = bucket_shards_use(ctx->device, na, N, co_ranks) ? 1 : N;
  auto full = [&](bh_srs* v, size_t used) {
    return ensure_table(ctx, v, table_c_for(used / (v == &params->h ? N : Naux)), 0, v->n);
  };
  if ((s = full(&params->h, m - 1))) return s;
  if ((s = full(&params->l, na))) return s;
  if ((s = full(&params->a, a_aux_used))) return s;
  if ((s = full(&params->b_g1, b_aux_used))) return s;
  return full(&params->b_g2, b_aux_used);
}

// BH_PROVER_SERIAL=1: one stream (per-kernel profiling only)
bool prover_serial() {  // (read per proof: tests/test_gpu_parity.py runs both modes)
  const char* e = getenv("BH_PROVER_SERIAL");
  return e && e[0] == '1';
}

// resident threads of the G1 bucket reduction (k_reduce_blocks) on every CU (full) or on the
// CU-masked tail streams' quarter of them
size_t reduce_resident_threads(bh_ctx* ctx, bool full) {
  // occupancy is a property of the kernel (one code object for every device); the CU count is
  // the context's device's, read once per device (contexts on several devices, concurrently)
  static const size_t per_cu = reduce_blocks_resident_per_cu_g1();
  static std::once_flag once[64];
  static int ncu[64];
  const int d = ctx->device & 63;
  std::call_once(once[d], [&] {
    if (hipDeviceGetAttribute(&ncu[d], hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) ncu[d] = 1;
  });
  const int cus = full ? ncu[d] : std::max(1, ncu[d] / 4);
  return per_cu * (size_t)std::max(cus, 1);
}

// When an exchanger is given (RCCL ranks, or the one-device emulation's virtual ranks) and
// the rank count qualifies, the H block is distributed (dist_h.h): this rank's h multiexp then
// covers the share of h it ends with instead of the range [shard*(m-1)/N, ...).

// `shard` of `nshards`: res1 = [h, l, a_inputs, a_aux, b_g1_inputs, b_g1_aux],
// res2 = [b_g2_inputs, b_g2_aux].  Error checks cover the full (unsharded) query.
// bh_prove_batch's pipelined lanes (set by the lane thread around one proof): after_accs once
// the proof has enqueued everything but its reduction tails, before_tails / after_tails around
// the tails' enqueue (proof order on the shared tail streams)
struct LaneHooks {
  std::function<void()> after_accs, before_tails, after_tails;
};
thread_local LaneHooks t_lane;

bh_status compute_msms(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t shard, size_t nshards,
                       Jac<Fp> res1[6], Jac<bh::Fp2> res2[2], Exchanger* ex = nullptr, bool may_build = true,
                       UploadSync* up = nullptr) {
  const auto t0 = std::chrono::steady_clock::now();
  if (bh_status sc = scratch_check(ctx)) return sc;  // rather than an abort inside the runtime
  bh_params* mparams = const_cast<bh_params*>(params);
  // The proof reads the Parameters' window tables under a shared lock (taken below).  Declared
  // before the drain guard so that on an error return the streams are drained BEFORE the lock
  // is released: another context must not rebuild a table that kernels of this failed proof
  // may still be reading.
  std::shared_lock<std::shared_mutex> prd(mparams->mu, std::defer_lock);
  // an error return in the middle of enqueueing leaves kernels running on the streams below,
  // reading workspaces the next call reuses: drain every stream before returning one
  struct DrainOnError {
    bh_ctx* c;
    bool ok = false;
    ~DrainOnError() { if (!ok) ctx_sync_all(c); }
  } drain{ctx};
  const size_t m = w->m, ni = w->num_inputs, na = w->num_aux;
  const int L = w->log_m;
  bh_status s;
  Domain* D;
  if ((s = ctx_domain(ctx, L, &D))) return s;
  const size_t maxn = std::max({m, ni, na, (size_t)1});
  BH_TRY_HIP(ctx->staging.alloc(3 * m * 32));
  BH_TRY_HIP(ctx->hbuf.alloc(m * 32));
  BH_TRY_HIP(ctx->idx.alloc(maxn * 4));
  BH_TRY_HIP(ctx->dtmp.alloc((maxn / 64 + 2) * 4));
  BH_TRY_HIP(ctx->dscan.alloc(scan_scratch_words(maxn / 64 + 2) * 4 + 64));
  BH_TRY_HIP(ctx->dspan.alloc(8 * MAX_SPAN_BLOCKS * 4));

  // ---- error semantics (prover.rs:309-343 order: delta check, then the waits)
  const uint64_t* dens = w->dens.as<uint64_t>();
  const uint64_t* d_a_aux = dens;
  const uint64_t* d_b_in = dens + w->a_aux_words;
  const uint64_t* d_b_aux = dens + w->a_aux_words + w->b_in_words;
  if (params->delta_g1.infinity || params->delta_g2.infinity) return BH_ERR_UNEXPECTED_IDENTITY;
  {
    // bases are validated at load (no identities), so only EOF is possible here
    struct Q { const bh_srs* srs; size_t off; const std::vector<uint64_t>* dens; size_t n; };
    const Q qs[] = {
        {&params->a, 0, nullptr, ni},                          // a_inputs
        {&params->a, ni, &w->a_aux_density, na},               // a_aux
        {&params->b_g1, 0, &w->b_input_density, ni},           // b_g1_inputs
        {&params->b_g1, w->b_in_total, &w->b_aux_density, na}, // b_g1_aux
        {&params->b_g2, 0, &w->b_input_density, ni},           // b_g2_inputs
        {&params->b_g2, w->b_in_total, &w->b_aux_density, na}, // b_g2_aux
        {&params->h, 0, nullptr, m - 1},                       // h
        {&params->l, 0, nullptr, na},                          // l
    };
    for (const Q& q : qs) {
      s = multiexp_check(q.srs, q.off, q.dens ? q.dens->data() : nullptr, q.n, nullptr, false);
      if (s) return s;
    }
  }
  // Streams, all ordered after whatever ran before on ctx->stream:
  //   stream    : the bucket accumulations back to back (VALU-bound critical path);
  //   stream4   : the H pipeline (after the first accumulation, or first when distributed);
  //   stream3   : density maps, then every multiexp's sort (memory-bound, runs ahead);
  //   stream2   : the small (public-input) multiexps, whole;
  //   tstream[q % 5]: the reduction tail of the q-th large multiexp.
  // Each multiexp has its own workspace, so the only dependencies are the events below.
  hipStream_t sA = ctx->stream, sT = ctx->stream2, sS = ctx->stream3, sH = ctx->stream4;
  hipStream_t tails[8];
  for (int q = 0; q < 8; q++) tails[q] = ctx->tstream[q % bh_ctx::TAIL_STREAMS];
  const bool serial = prover_serial();
  if (serial) {
    sT = sS = sH = sA;
    for (auto& t : tails) t = sA;
  }
  // The last multiexp's reduction tail runs when every accumulation is done, alone at the end of
  // the critical path: on the CU-masked tail streams (a quarter of the CUs) its 2^19-bucket
  // reduction needed two rounds of resident blocks.  So it runs on the
  // small-multiexp stream (high priority, every CU), with its bucket reduction shaped for one round
  // of the whole GPU (not on a pipelined batch lane, whose next proof's first accumulation would
  // queue behind it).
  const bool last_full = !serial && !ctx->borrowed_streams && ctx->cu_masked;
  hipEvent_t* jev = ctx->jev;  // [2j,2j+1] accumulate timing, [16+j] sorted, [24+j] accumulated,
                               // [32] start, [33] density maps ready
  BH_TRY_HIP(hipEventRecord(jev[32], sA));
  // ordered after whatever this context ran before on its main stream -- except on a pipelined
  // batch lane (borrowed streams): there the main stream holds the previous proof's
  // accumulations, which this proof's density maps and sorts must not wait for (they read only
  // this lane's own witness and workspaces)
  if (!ctx->borrowed_streams) {
    BH_TRY_HIP(hipStreamWaitEvent(sS, jev[32], 0));
    BH_TRY_HIP(hipStreamWaitEvent(sT, jev[32], 0));
  }

  // ---- the 8 multiexps (prover.rs:233-307)
  // (a resident witness carries its maps from bh_witness_upload; bh_prove's is rebuilt per call)
  if (!w->idx_ready) BH_TRY_HIP(ctx->idx3.alloc((2 * na + ni + 1) * 4));
  int32_t* idx_aaux = w->idx_ready ? const_cast<int32_t*>(w->idx3.as<int32_t>()) : ctx->idx3.as<int32_t>();
  int32_t* idx_bin = idx_aaux + na;
  int32_t* idx_baux = idx_bin + ni;
  // distributed H: this rank ends with its own share of h (dist_h.h), no range split
  DistH* dh = nullptr;
  if (ex && dist_h_eligible((int)nshards, L) && nshards >= dist_h_min_ranks()) {
    if (!ctx->dist) ctx->dist = new DistH();
    if ((s = dist_h_init(ctx, *ctx->dist, (int)nshards, (int)shard, L))) return s;
    dh = ctx->dist;
  }
  ShareGeom geom;
  if (dh) {
    geom.N = dh->N; geom.rank = dh->rank; geom.L = L; geom.M = dh->M; geom.C = dh->C;
  }
  const ShareGeom* sg = dh ? &geom : nullptr;
  const uint32_t* sh_buf = dh ? dh->hbuf.as<uint32_t>() : nullptr;
  const int32_t* sh_idx = dh ? dh->hidx.as<int32_t>() : nullptr;
  // The proof reads the Parameters' window tables under a shared lock for its whole duration;
  // tables it wants but lacks are built first under the exclusive lock (a proof of another
  // shape may have replaced them).
  Job jobs[8];
  prd.lock();
  if ((s = plan_shard(ctx, params, w, shard, nshards, sg, sh_buf, sh_idx, idx_aaux, idx_bin, idx_baux, false, jobs)))
    return s;
  if (may_build && plan_needs_build(params, jobs, sg, ctx->tables && !ctx->window_override)) {
    prd.unlock();
    {
      std::unique_lock<std::shared_mutex> pwr(mparams->mu);
      if ((s = plan_shard(ctx, params, w, shard, nshards, sg, sh_buf, sh_idx, idx_aaux, idx_bin, idx_baux, true,
                          jobs)))
        return s;
    }
    prd.lock();
    if ((s = plan_shard(ctx, params, w, shard, nshards, sg, sh_buf, sh_idx, idx_aaux, idx_bin, idx_baux, false,
                        jobs)))
      return s;
  }
  // the public-input multiexps on a host thread (HOST_INPUT_MSM_MAX); BH_HOST_INPUTS=0: on the
  // device like the others (A/B experiments)
  // (read per proof: tests run the device branch of small input counts with BH_HOST_INPUTS=0)
  const bool host_inputs_on = [] {
    const char* e = getenv("BH_HOST_INPUTS");
    return !(e && e[0] == '0');
  }();
  const bool host_in = host_inputs_on && jobs[5].hi - jobs[5].lo <= HOST_INPUT_MSM_MAX;
  struct HostInputs {
    std::thread th;
    bh_status st = BH_OK;
    Jac<Fp> a, b1;
    Jac<bh::Fp2> b2;
    ~HostInputs() { if (th.joinable()) th.join(); }
  } hin;
  if (host_in)
    hin.th = std::thread([&hin, ctx, mparams, w, lo = jobs[5].lo, hi = jobs[5].hi] {
      hin.st = host_input_msms(ctx->device, mparams, w, lo, hi, &hin.a, &hin.b1, &hin.b2);
    });
  if (up) {  // witness still uploading (bh_prove): density maps, inputs and aux first
    if (!up->wait(1)) return up->status;
    BH_TRY_HIP(hipStreamWaitEvent(sS, up->ev[0], 0));
    if (w->raw) {  // bls12_381 Montgomery -> canonical scalars, here rather than on the copy stream
      uint32_t* in = const_cast<uint32_t*>(w->inputs.as<uint32_t>());
      uint32_t* ax = const_cast<uint32_t*>(w->aux.as<uint32_t>());
      if (ni) BH_TRY_HIP(scalars_prepare(in, in, ni, 1, 0, sS));
      if (na) BH_TRY_HIP(scalars_prepare(ax, ax, na, 1, 0, sS));
    }
  }
  if (na && !w->idx_ready) BH_TRY_HIP(density_index(d_a_aux, na, (uint32_t)ni, idx_aaux, ctx->dtmp.as<uint32_t>(),
                                   ctx->dscan.as<uint32_t>(), sS));
  if (ni && !w->idx_ready)
    BH_TRY_HIP(density_index(d_b_in, ni, 0, idx_bin, ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(), sS));
  if (na && !w->idx_ready) BH_TRY_HIP(density_index(d_b_aux, na, (uint32_t)w->b_in_total, idx_baux, ctx->dtmp.as<uint32_t>(),
                                   ctx->dscan.as<uint32_t>(), sS));
  MsmShape shapes[8];
  bool use_table[8] = {false};
  size_t los[8], his[8];
  int n_table = 0, n_large = 0;
  for (int j = 0; j < 8; j++) {
    los[j] = jobs[j].lo;
    his[j] = jobs[j].hi;
    if (his[j] == los[j]) continue;
    const bh_srs* srs = jobs[j].srs;
    use_table[j] = jobs[j].table_c && srs->win_covers(jobs[j].table_c, jobs[j].blo, jobs[j].bhi);
    if (jobs[j].bk_hi && !use_table[j]) {
      // a bucket shard without its window table (HBM short when it was to be built): another rank
      // may well have its table, so a plain-window stand-in here would not sum with the other
      // ranks' parts -- refuse (bucket shards are opt-in, BH_SHARD_BUCKETS=1)
      fprintf(stderr, "bellman_hip: bucket shard without its window table (HBM short): set BH_SHARD_BUCKETS=0\n");
      return BH_ERR_OUT_OF_MEMORY;
    }
    shapes[j] = use_table[j] ? msm_shape_table(his[j] - los[j], srs->win_c)
                             : msm_shape(his[j] - los[j], ctx->window_override);
    if (use_table[j]) shapes[j].rec = srs->win_rec;
    if (jobs[j].bk_hi) {
      MsmShape& sh = shapes[j];
      sh.bk_lo = jobs[j].bk_lo;
      sh.bk_hi = jobs[j].bk_hi;
      // reduction geometry: L * BT divides the granule (BUCKET_SHARD_GRANULE), and at least as many
      // reduction threads as one GPU's whole bucket set gets (msm_shape_table: 16 384), since a
      // shard's buckets hold as many continuation partials each (a round-5 rank of 8: G2 with 8 192
      // threads was a 4.6 ms reduction at the end of the proof)
      const uint32_t BT = reduce_block_max(jobs[j].g2);
      while (sh.L > 1 && ((uint32_t)sh.L * BT > BUCKET_SHARD_GRANULE || sh.red_nb() / (uint32_t)sh.L < 16384u))
        sh.L >>= 1;
      // segments sized for the range's expected entries (the grid still covers every position)
      const double f = bucket_cdf(sh.c, sh.W, sh.bk_hi) - bucket_cdf(sh.c, sh.W, sh.bk_lo);
      const size_t E = std::max<size_t>((size_t)((double)jobs[j].used * f), 1);
      if (jobs[j].g2) fit_segments_E<G2Ops>(sh, E);
      else fit_segments_E<G1Ops>(sh, E);
    } else {
      // segments sized for the entries the density set gives (the grid still covers n * W positions)
      const size_t nj = his[j] - los[j];
      const size_t used_j = (size_t)((unsigned __int128)jobs[j].used * nj / std::max<size_t>(jobs[j].n, 1));
      const size_t E = seg_entries(nj, used_j, shapes[j].W);
      if (jobs[j].g2) fit_segments_E<G2Ops>(shapes[j], E);
      else fit_segments_E<G1Ops>(shapes[j], E);
    }
    if (jobs[j].table_c) n_large++;
    if (use_table[j]) n_table++;
  }
  // ---- H (prover.rs:210-234), device resident.  Where it is enqueued: see 'H placement' below;
  // only h's sort waits for it.
  auto enqueue_h = [&](hipEvent_t after) -> bh_status {
    if (up && up->on_vector) {
      // bh_prove: the uploading thread enqueues H on sH vector by vector, each behind its own
      // upload; only h's sort (enqueued on sH right after this) needs the host to wait until
      // that enqueue is done
      if (!up->wait(2)) return up->status;
      return BH_OK;
    }
    BH_TRY_HIP(hipStreamWaitEvent(sH, after, 0));
    hipEventRecord(ctx->ev[0], sH);
    if (dh) {  // three all-to-alls (RCCL, or the emulation's device copies), stream-ordered on sH
      const size_t chunk = dh->C, M = dh->M;
      HExchange hx = [ex, chunk, M](const uint32_t* send, uint32_t* recv, int nvec, hipStream_t st) {
        return ex->exchange(send, recv, chunk, M, nvec, st);
      };
      bh_status hs = dist_h_run(ctx, *dh, w->abc.as<uint32_t>(), hx, sH);
      if (hs) return hs;
      hipEventRecord(ctx->ev[1], sH);
      return BH_OK;
    }
    uint32_t* abc = ctx->staging.as<uint32_t>();
    if (up) {  // a, b, c still uploading (bh_prove)
      if (!up->wait(2)) return up->status;
      BH_TRY_HIP(hipStreamWaitEvent(sH, up->ev[1], 0));
    }
    const uint32_t* src = w->abc.as<uint32_t>();  // the first passes read the witness in place
    if (w->raw) {  // convert into the H block's buffer (bls12_381 -> device Montgomery), zero padding
      const size_t nc = w->num_constraints;
      for (int v = 0; v < 3; v++) {
        if (nc) launch_fr_convert(w->abc.as<uint32_t>() + (size_t)v * m * 8, abc + (size_t)v * m * 8, nc,
                                  fr_to_dev_const(), 0, sH);
        if (m > nc) BH_TRY_HIP(hipMemsetAsync(abc + ((size_t)v * m + nc) * 8, 0, (m - nc) * 32, sH));
      }
      BH_TRY_HIP(hipGetLastError());
      src = nullptr;
    }
    // ... and the last one writes h as canonical scalars in natural order, truncated to m-1
    // (prover.rs:227-231)
    bh_status hs = run_h_pipeline(ctx, D, abc, sH, src, ctx->hbuf.as<uint32_t>());
    if (hs) return hs;
    hipEventRecord(ctx->ev[1], sH);
    return BH_OK;
  };
  // Two multiexps with the same scalars, density map, range and digit geometry (b_g1_aux and
  // b_g2_aux: prover.rs:282-307 both use the aux assignment under b_aux_density) have
  // identical sorted entries, so the second one copies the first one's instead of sorting.
  auto same_digits = [&](int i, int j) {
    const MsmShape &a = shapes[i], &b = shapes[j];
    return jobs[i].sc == jobs[j].sc && jobs[i].idx == jobs[j].idx && los[i] == los[j] && his[i] == his[j] &&
           a.c == b.c && a.W == b.W && a.NB == b.NB && a.Wb == b.Wb && a.pre == b.pre && a.bk_lo == b.bk_lo &&
           a.bk_hi == b.bk_hi;
  };
  // ... and one over a sparser density map (a_aux, b_aux under l's dense one) compacts it
  auto derivable = [&](int i, int j) {
    const MsmShape &a = shapes[i], &b = shapes[j];
    return jobs[i].sc == jobs[j].sc && !jobs[i].idx && jobs[j].idx && !jobs[i].is_h && los[i] == los[j] &&
           his[i] == his[j] && a.c == b.c && a.W == b.W && a.NB == b.NB && a.Wb == b.Wb && a.pre == b.pre &&
           a.bk_lo == b.bk_lo && a.bk_hi == b.bk_hi;
  };
  int sorted_from[8];
  for (int j = 0; j < 8; j++) sorted_from[j] = -1;
  auto sort_job = [&](int j, hipStream_t st) -> bh_status {
    const Job& J = jobs[j];
    const size_t n = his[j] - los[j];
    const int32_t* ix = J.idx ? J.idx + los[j] : nullptr;
    const uint32_t* sc = J.sc + los[j] * 8;
    int src = -1;
    for (int i = 0; i < 8 && src < 0; i++)
      if (i != j && sorted_from[i] == i && same_digits(i, j)) src = i;
    int dsrc = -1;  // a fully dense sort over the same scalars and digits to compact from
    for (int i = 0; i < 8 && src < 0 && dsrc < 0; i++)
      if (i != j && sorted_from[i] == i && derivable(i, j)) dsrc = i;
    if (dsrc >= 0) {
      const MsmShape& sh = shapes[j];
      const size_t nbt = (size_t)sh.Wb * sh.NB, Emax = n * (size_t)sh.W;
      const auto& S = jobs[dsrc];
      const uint32_t* se = S.g2 ? ctx->pw2[S.out].entries : ctx->pw1[S.out].entries;
      const uint32_t* so = S.g2 ? ctx->pw2[S.out].offsets : ctx->pw1[S.out].offsets;
      uint32_t *de, *dc, *dof, *pos;
      if (J.g2) {
        BH_TRY_HIP(ctx->pw2[J.out].reserve_shape(n, sh));
        de = ctx->pw2[J.out].entries; dc = ctx->pw2[J.out].counts; dof = ctx->pw2[J.out].offsets;
        pos = reinterpret_cast<uint32_t*>(ctx->pw2[J.out].recs);
      } else {
        BH_TRY_HIP(ctx->pw1[J.out].reserve_shape(n, sh));
        de = ctx->pw1[J.out].entries; dc = ctx->pw1[J.out].counts; dof = ctx->pw1[J.out].offsets;
        pos = reinterpret_cast<uint32_t*>(ctx->pw1[J.out].recs);
      }
      BH_TRY_HIP(ctx->dscan2.alloc(derive_scratch_words(Emax) * 4));
      BH_TRY_HIP(hipStreamWaitEvent(st, jev[16 + dsrc], 0));
      BH_TRY_HIP(derive_sorted(se, so, nbt, Emax, sh.pre, (uint32_t)sh.W, (uint32_t)los[dsrc], ix, pos,
                               ctx->dscan2.as<uint32_t>(), de, dc, dof, st, sh.bucket_shard() ? sh.bk_lo : 0u,
                               sh.bucket_shard() ? sh.bk_hi : 0u));
      sorted_from[j] = j;  // a sort of its own from here on (copies may take it)
    } else if (src >= 0) {
      const MsmShape& sh = shapes[j];
      const size_t nbt = (size_t)sh.Wb * sh.NB;
      const uint32_t *e, *cn, *of;
      if (jobs[src].g2) { e = ctx->pw2[jobs[src].out].entries; cn = ctx->pw2[jobs[src].out].counts; of = ctx->pw2[jobs[src].out].offsets; }
      else { e = ctx->pw1[jobs[src].out].entries; cn = ctx->pw1[jobs[src].out].counts; of = ctx->pw1[jobs[src].out].offsets; }
      uint32_t *de, *dc, *dof;
      if (J.g2) {
        BH_TRY_HIP(ctx->pw2[J.out].reserve_shape(n, sh));
        de = ctx->pw2[J.out].entries; dc = ctx->pw2[J.out].counts; dof = ctx->pw2[J.out].offsets;
      } else {
        BH_TRY_HIP(ctx->pw1[J.out].reserve_shape(n, sh));
        de = ctx->pw1[J.out].entries; dc = ctx->pw1[J.out].counts; dof = ctx->pw1[J.out].offsets;
      }
      BH_TRY_HIP(hipStreamWaitEvent(st, jev[16 + src], 0));
      BH_TRY_HIP(hipMemcpyAsync(dc, cn, (nbt + 1) * 4, hipMemcpyDeviceToDevice, st));
      BH_TRY_HIP(hipMemcpyAsync(dof, of, (nbt + 1) * 4, hipMemcpyDeviceToDevice, st));
      BH_TRY_HIP(hipMemcpyAsync(de, e, n * (size_t)sh.W * 4, hipMemcpyDeviceToDevice, st));
      sorted_from[j] = src;
    } else {
      if (J.g2) BH_TRY_HIP(msm_sort<G2Ops>(ctx->pw2[J.out], st, sc, n, ix, (uint32_t)los[j], shapes[j]));
      else BH_TRY_HIP(msm_sort<G1Ops>(ctx->pw1[J.out], st, sc, n, ix, (uint32_t)los[j], shapes[j]));
      sorted_from[j] = j;
    }
    // continuation-tree depth of this multiexp (read by its tail, so it launches only the
    // levels that can do work)
    const MsmShape& shj = shapes[j];
    // (a bucket shard: over its own buckets, the only ones its sort set)
    const uint32_t* cnt = (J.g2 ? ctx->pw2[J.out].counts : ctx->pw1[J.out].counts) + shj.red_lo();
    const uint32_t* off = (J.g2 ? ctx->pw2[J.out].offsets : ctx->pw1[J.out].offsets) + shj.red_lo();
    BH_TRY_HIP(max_span(cnt, off, (size_t)shj.Wb * shj.red_nb(), (uint32_t)shj.S,
                        ctx->dspan.as<uint32_t>() + (size_t)j * MAX_SPAN_BLOCKS, ctx->host_spans + (size_t)j * MAX_SPAN_BLOCKS,
                        st));
    BH_TRY_HIP(hipEventRecord(jev[16 + j], st));
    return BH_OK;
  };
  auto acc_job = [&](int j, hipStream_t st) -> bh_status {
    const Job& J = jobs[j];
    const size_t n = his[j] - los[j];
    BH_TRY_HIP(hipStreamWaitEvent(st, jev[16 + j], 0));
    MsmTiming tm;
    tm.ev_acc_begin = acc_events_on() ? jev[2 * j] : nullptr;
    tm.ev_acc_end = acc_events_on() ? jev[2 * j + 1] : nullptr;
    const uint32_t* bases = use_table[j] ? J.srs->win_global() : J.srs->pts.as<uint32_t>();
    if (J.g2) BH_TRY_HIP(msm_accumulate<G2Ops>(ctx->pw2[J.out], st, bases, n, shapes[j], &tm));
    else BH_TRY_HIP(msm_accumulate<G1Ops>(ctx->pw1[J.out], st, bases, n, shapes[j], &tm));
    BH_TRY_HIP(hipEventRecord(jev[24 + j], st));
    return BH_OK;
  };
  auto tail_job = [&](int j, hipStream_t st) -> bh_status {
    const Job& J = jobs[j];
    const size_t n = his[j] - los[j];
    BH_TRY_HIP(hipStreamWaitEvent(st, jev[24 + j], 0));
    // entries = mixed additions of this multiexp (offsets[nbt]), for the VALU roofline
    // (copied here, off the accumulation stream)
    const uint32_t* offs = J.g2 ? ctx->pw2[J.out].offsets : ctx->pw1[J.out].offsets;
    BH_TRY_HIP(hipMemcpyAsync(&ctx->host_counts[j], offs + (size_t)shapes[j].Wb * shapes[j].NB, 4,
                              hipMemcpyDeviceToHost, st));
    // The longest bucket span picks the continuation fold: the tail kernels read the sort's span
    // words on the device, so enqueueing a tail never waits for its sort (a pipelined batch hands
    // the streams on to the next proof without waiting for this one's h sort, which follows H)
    const int span = -1;
    const uint32_t* dspan = n >= SMALL_JOB ? ctx->dspan.as<uint32_t>() + (size_t)j * MAX_SPAN_BLOCKS : nullptr;
    if (J.g2)
      BH_TRY_HIP(msm_back<G2Ops>(ctx->pw2[J.out], st, n, shapes[j], ctx->host_out2 + 128 * J.out, span, jev[24 + j],
                                 dspan));
    else
      BH_TRY_HIP(msm_back<G1Ops>(ctx->pw1[J.out], st, n, shapes[j], ctx->host_out1 + 128 * J.out, span, jev[24 + j],
                                 dspan));
    return BH_OK;
  };
  // the H stream follows the density maps and sorts enqueued so far -- unless the uploading
  // thread is enqueueing H on it vector by vector (bh_prove): those kernels are ordered behind
  // their uploads already, and a wait issued here would land between them at a random point
  // (jev[33] = the density maps: the small multiexps' stream waits on it below)
  BH_TRY_HIP(hipEventRecord(jev[33], sS));
  if (!(up && up->on_vector)) BH_TRY_HIP(hipStreamWaitEvent(sH, jev[33], 0));
  int big[8], nbig = 0, small[8], nsmall = 0;
  hipStream_t acc_stream[8] = {};  // the stream each large multiexp's accumulation was enqueued on
  for (int j = 0; j < 8; j++) {
    const size_t n = his[j] - los[j];
    if (!n || (host_in && j >= 5)) continue;
    if (n < SMALL_JOB && !jobs[j].is_h) small[nsmall++] = j;
    else big[nbig++] = j;
  }
  // Large ones: sorts run ahead on stream3, accumulations back to back on the main stream,
  // each reduction tail on a stream of its own (the tails are latency-bound chains of point
  // additions: several run side by side at little cost, and none waits behind another).
  int h_pos = nbig;
  for (int q = 0; q < nbig; q++)
    if (jobs[big[q]].is_h) h_pos = q;
  // The last accumulated multiexp's reduction tail runs alone on an idle GPU, at the end of
  // the critical path: give its bucket reduction more, shorter chains (fewer buckets per
  // thread: 2L + 2 log2(BT) + log2(L) serial point operations in k_reduce_blocks), while
  // the earlier tails, which share the SIMDs with accumulations, keep the work-lean shape.
  // (Tried and removed: the last multiexp accumulated and reduced as two bucket halves so the
  // lower half's reduction runs beside the upper half's accumulation, +0.8 ms per 2^22 proof,
  // profiles/r03_ab_last_halves.txt; fewer rounds for the last accumulation, within noise.)
  if (nbig > 0) {
    MsmShape& sl = shapes[big[nbig - 1]];
    // one round of resident k_reduce_blocks blocks on the CUs the last tail runs on
    const int last_threads =
        last_full ? (int)std::min<size_t>(reduce_resident_threads(ctx, true), 1 << 20) : 65536;
    const int nb = (int)sl.red_nb();
    int L = sl.L;
    while (L > 1 && (size_t)sl.Wb * (size_t)(nb / L) < (size_t)last_threads) L >>= 1;
    sl.L = L;
  }
  // H placement.  A resident witness enqueues H first, running beside everything: since the G2
  // accumulation keeps ZZ/ZZZ in LDS (268 registers, msm_impl.cuh accumulate_lds) H's NTT passes
  // co-reside with it (same-box A/B at 2^22: 55.1-55.3 ms per proof against 57.4-58.2 with H after
  // the first accumulation, profiles/r04_ab_hmode_g2.txt).  Other placements were measured and
  // removed: H enqueued after the first accumulation's launch, between the first sorts and the first
  // accumulation, from a helper host thread, or held on the device until the first sort is done
  // (N = 8 rehearsal within 0.1 ms or slower, profiles/r03_ab_hmode_N8.txt, r03_ab_hmode_more_N8.txt,
  // r05_ab_sched_knobs_N1_2_8.txt).  From host buffers (bh_prove) the uploading thread enqueues H
  // vector by vector behind each upload (on_vector); here only h's own sort and accumulation wait on
  // the host for that enqueue, so they are enqueued last.
  bool h_late = up != nullptr;
  // the small multiexps run whole on their own stream, after the density maps
  BH_TRY_HIP(hipStreamWaitEvent(sT, jev[33], 0));
  auto run_small = [&]() -> bh_status {
    for (int i = 0; i < nsmall; i++) {
      bh_status e = sort_job(small[i], sT);
      if (!e) e = acc_job(small[i], sT);
      if (!e) e = tail_job(small[i], sT);
      if (e) return e;
    }
    return BH_OK;
  };
  // Host enqueue order follows the critical path: the first two sorts (a sort running beside
  // a whole-GPU accumulation only gets CUs as its workgroups retire, so the second one would
  // not be ready when the first accumulation ends), the first accumulation, H, the remaining
  // sorts (h's after H), every accumulation, the small multiexps, then the tails.
  // Sort order = accumulation order (b_g2_aux sorted, b_g1_aux copied, l sorted, a_aux
  // compacted from l, h): putting l first so that b_g2_aux could be compacted from it would
  // lengthen the start-up (measured +2 ms at 2^22), so only later sorts are derived.
  // h's digit sort reads the H block's output: on a replicated H it runs on the H stream right
  // behind it, so the sort stream never waits for H (a pipelined batch's next proof queues its
  // density maps and sorts there, behind this proof's); distributed H (CU-masked stream) keeps it
  // on the sort stream after an event wait
  auto sort_h_or = [&](int j) -> bh_status {
    if (!jobs[j].is_h) return sort_job(j, sS);
    if (!dh) return sort_job(j, sH);
    BH_TRY_HIP(hipStreamWaitEvent(sS, ctx->ev[1], 0));
    return sort_job(j, sS);
  };
  int sorder[8];
  const int ns = nbig;
  for (int q = 0; q < nbig; q++) sorder[q] = big[q];
  // every sort up to those of the first two accumulations runs ahead of the first accumulation
  int pre_sorts = 0;
  for (int r = 0; r < ns; r++)
    if (sorder[r] == big[0] || (nbig > 1 && h_pos != 1 && sorder[r] == big[1])) pre_sorts = r + 1;
  bool h_in_pre = false;
  for (int r = 0; r < pre_sorts; r++) h_in_pre = h_in_pre || jobs[sorder[r]].is_h;
  if (h_in_pre) h_late = false;  // h's own sort is among the first: H first
  if (!h_late && (s = enqueue_h(jev[33]))) return s;

  for (int r = 0; r < pre_sorts; r++) {
    if ((s = sort_h_or(sorder[r]))) return s;
  }
  // The first accumulation (G2: 268 registers, one wave per SIMD) runs on the small-multiexp
  // stream (idle when the public-input multiexps are on the host), so the G1 accumulations start
  // beside it instead of after it: same-box A/B at 2^22 54.66-55.17 against 55.01-55.45 ms
  // (profiles/r04_ab_first_acc_stream.txt).
  const bool first_own = nsmall == 0 && !serial;
  if (nbig > 0) {
    // wait for the last pre-sort that is a real sort: a trailing copy of another multiexp's
    // entries (b_g1_aux from b_g2_aux) is ~0.15 ms of blits that can run beside the accumulation
    int wait_j = big[0];
    for (int r = 0; r < pre_sorts; r++)
      if (sorted_from[sorder[r]] == sorder[r]) wait_j = sorder[r];
    hipStream_t s0 = first_own ? sT : sA;
    BH_TRY_HIP(hipStreamWaitEvent(s0, jev[16 + wait_j], 0));
    if ((s = acc_job(big[0], s0))) return s;
    acc_stream[0] = s0;
  }
  // With the first accumulation on its own stream, the second one (G1: b_g1_aux, whose sorted
  // entries are a copy among the first sorts) is enqueued right behind it, before the remaining
  // sorts: those are ~20-40 host enqueues (~0.7 ms per rank at N = 8 in the round-5 kernel
  // trace, 1.6 ms at N = 2), during which the G2 accumulation ran alone on its one wave per SIMD.
  int q_first = 1;
  if (nbig > 1 && !jobs[big[1]].is_h && first_own) {
    bool pre = false;  // its sort is among the pre-sorts (enqueued above)
    for (int r = 0; r < pre_sorts; r++) pre = pre || sorder[r] == big[1];
    if (pre) {
      if ((s = acc_job(big[1], sA))) return s;
      acc_stream[1] = sA;
      q_first = 2;
    }
  }
  const auto t_acc0 = std::chrono::steady_clock::now();
  const auto t_h = std::chrono::steady_clock::now();
  for (int r = pre_sorts; r < ns; r++) {
    if (h_late && jobs[sorder[r]].is_h) continue;  // behind H, enqueued below
    if ((s = sort_h_or(sorder[r]))) return s;
  }
  const auto t_sorts = std::chrono::steady_clock::now();
  // Accumulation lanes: the accumulations after the first two go to whichever of three accumulation
  // streams (the first one's, the main one, stream5) has the least queued work (mixed additions, a G2
  // one weighted 2.75x).  Consecutive accumulations on one stream are separated by a barrier (the
  // next kernel dispatches only once the last block of the previous one is done: ~0.12 ms between
  // them in the round-5 traces), and in that moment other streams' pending kernels take the freed
  // slots (round-5 drop-in trace: 1.4 and 2.9 ms of main-stream idle before a_aux and h).  Two lanes
  // (round 5): rehearsal N = 8 9.85-9.92 against 10.05-10.23 ms per rank (profiles/r05_ab_acc_lanes.txt);
  // with the G2 accumulation holding one lane for most of the proof, the G1 ones still ran back to
  // back on the other, so round 6 adds a third: the 2^22 bench 54.4-54.6 against 54.8-55.0 ms, bh_prove
  // 58.7-58.9 against 59.5-59.7, N = 2 30.4 against 30.8-31.2 ms per rank, N = 1 and 8 within noise
  // (profiles/r06_ab_acc_lanes3.txt).
  const bool multi_lane = first_own && !ctx->borrowed_streams && nbig > 2;
  auto acc_cost = [&](int j) {
    const double e = (double)jobs[j].used * (double)(shapes[j].W ? shapes[j].W : 1);
    return jobs[j].g2 ? 2.75 * e : e;
  };
  double lane_load[3] = {nbig > 0 ? acc_cost(big[0]) : 0.0, 0.0, 0.0};  // [0] sT, [1] sA, [2] stream5
  for (int q = 1; q < q_first; q++) lane_load[1] += acc_cost(big[q]);
  bool h_done = !h_late;
  for (int q = q_first; q < nbig; q++) {
    if (!h_done && jobs[big[q]].is_h) {
      if ((s = enqueue_h(jev[33]))) return s;
      if ((s = sort_h_or(big[q]))) return s;
      h_done = true;
    }
    hipStream_t sq = sA;
    if (multi_lane) {
      int l = lane_load[0] < lane_load[1] ? 0 : 1;
      if (lane_load[2] < lane_load[l]) l = 2;
      lane_load[l] += acc_cost(big[q]);
      sq = l == 0 ? sT : l == 1 ? sA : ctx->stream5;
    }
    if ((s = acc_job(big[q], sq))) return s;
    acc_stream[q] = sq;
  }
  if (!h_done && (s = enqueue_h(jev[33]))) return s;  // (no large h job: H still runs)
  if ((s = run_small())) return s;
  // The host waits below are on events of THIS proof's work (not stream syncs): on a pipelined
  // batch lane the streams soon hold the next proof's work behind it.
  // ev[10..13]: small multiexps, sorts, accumulations, H; ev[2+q]: tail q
  BH_TRY_HIP(hipEventRecord(ctx->ev[10], sT));
  BH_TRY_HIP(hipEventRecord(ctx->ev[11], sS));
  BH_TRY_HIP(hipEventRecord(ctx->ev[12], sA));
  BH_TRY_HIP(hipEventRecord(ctx->ev[13], sH));
  // pipelined batch lanes: the next proof may enqueue its start-up and accumulations now (they
  // queue behind these on every stream); this proof's tails go in only after the previous
  // proof's (a tail stream would otherwise hold them behind the next proof's tails)
  const auto t_hand = std::chrono::steady_clock::now();
  if (t_lane.after_accs) t_lane.after_accs();
  if (t_lane.before_tails) t_lane.before_tails();
  // The last tail right behind its own accumulation, on that lane (every CU): with three lanes
  // (round 6) the first accumulation's stream may still be running the G2 tail below, which held
  // the last tail back 0.9 ms at N = 8 (profiles/r06_n8_rank0_timeline.txt, second trace).
  if (last_full && nbig > 0 && nsmall == 0) tails[nbig - 1] = multi_lane ? acc_stream[nbig - 1] : sT;
  // The G2 multiexp's reduction tail (continuation fold + reduction of G2 buckets, each addition
  // ~3x a G1 one) on the first accumulation's stream, every CU, right behind the G2 accumulation,
  // rather than on a quarter-CU tail stream: with three accumulation lanes the G1 accumulations end
  // earlier and at N = 8 that latency-bound tail (2.9 + 1.6 + 0.8 ms on 64 CUs) became the rank's
  // critical path (profiles/r06_n8_rank0_timeline.txt).  Same-box A/B: the 2^22 bench 53.9-54.0 against 54.3-54.8
  // ms, bh_prove 57.9-58.2 against 58.4-58.9, rehearsal N = 1 / 2 / 8 at or below the base
  // (profiles/r06_ab_g2_tail.txt).  (On a pipelined batch lane the streams are shared: tail streams.)
  // (only where no later accumulation queued on that stream: the tail would wait for it)
  if (!serial && !ctx->borrowed_streams)
    for (int q = 0; q + 1 < nbig; q++) {
      if (!jobs[big[q]].g2 || !acc_stream[q]) continue;
      bool later = false;
      for (int r = q + 1; r < nbig; r++) later = later || acc_stream[r] == acc_stream[q];
      if (!later) tails[q] = acc_stream[q];
    }
  for (int q = 0; q < nbig; q++) {
    if ((s = tail_job(big[q], tails[q]))) return s;
    BH_TRY_HIP(hipEventRecord(ctx->ev[2 + q], tails[q]));
  }
  const auto t_enq = std::chrono::steady_clock::now();
  if (t_lane.after_tails) t_lane.after_tails();
  float g1_acc_ms = 0, g2_acc_ms = 0;
  size_t g1_pairs = 0, g2_pairs = 0, g1_adds = 0, g2_adds = 0;
  int g1_launches = 0, g2_launches = 0;
  for (int i = 0; i < 6; i++) res1[i] = jac_identity<Fp>();
  for (int i = 0; i < 2; i++) res2[i] = jac_identity<bh::Fp2>();
  // Each multiexp's host combine runs as soon as its own tail stream is done (its window sums
  // are on the host), while later tails still run: only the last one's stays on the critical
  // path.  The small multiexps (stream sT) finish first.
  int order[8], nord = 0;
  for (int i = 0; i < nsmall; i++) order[nord++] = small[i];
  for (int q = 0; q < nbig; q++) order[nord++] = big[q];
  for (int o = 0; o < nord; o++) {
    const int j = order[o];
    const Job& J = jobs[j];
    if (o == 0 || o == nsmall) BH_TRY_HIP(hipEventSynchronize(ctx->ev[10]));
    if (o >= nsmall) BH_TRY_HIP(hipEventSynchronize(ctx->ev[2 + (o - nsmall)]));
    float t = 0;
    if (acc_events_on()) (void)hipEventElapsedTime(&t, jev[2 * j], jev[2 * j + 1]);
    const size_t pairs = (size_t)((unsigned __int128)J.used * (his[j] - los[j]) / std::max<size_t>(J.n, 1));
    if (J.g2) {
      res2[J.out] = combine_g2(ctx->host_out2 + 128 * J.out, shapes[j]);
      g2_acc_ms += t; g2_launches++; g2_pairs += pairs; g2_adds += ctx->host_counts[j];
    } else {
      res1[J.out] = combine_g1(ctx->host_out1 + 128 * J.out, shapes[j]);
      g1_acc_ms += t; g1_launches++; g1_pairs += pairs; g1_adds += ctx->host_counts[j];
    }
  }
  for (int e = 10; e <= 13; e++) BH_TRY_HIP(hipEventSynchronize(ctx->ev[e]));
  if (host_in) {
    hin.th.join();
    if (hin.st) return hin.st;
    res1[jobs[5].out] = hin.a;
    res1[jobs[6].out] = hin.b1;
    res2[jobs[7].out] = hin.b2;
  }
  const auto t_gpu = std::chrono::steady_clock::now();

  const auto t1 = std::chrono::steady_clock::now();
  static const bool host_timing = getenv("BH_HOST_TIMING") != nullptr;
  if (host_timing) {
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    fprintf(stderr, "compute_msms host: ctx %p start %.3f ms (monotonic), first accumulation enqueued %.3f ms, H %.3f, sorts %.3f, accumulations handed on %.3f, enqueue done %.3f, gpu and combines done %.3f, after %.3f\n",
            (void*)ctx, std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count(), ms(t0, t_acc0), ms(t0, t_h),
            ms(t0, t_sorts), ms(t0, t_hand), ms(t0, t_enq), ms(t0, t_gpu), ms(t_gpu, t1));
  }
  float h_ms = 0;
  hipEventElapsedTime(&h_ms, ctx->ev[0], ctx->ev[1]);
  ctx->last_timings[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
  ctx->last_timings[1] = h_ms;
  ctx->last_timings[2] = g1_acc_ms;
  ctx->last_timings[3] = g1_launches;
  ctx->last_timings[4] = (double)g1_pairs;
  ctx->last_timings[5] = g2_acc_ms;
  ctx->last_timings[6] = g2_launches;
  ctx->last_timings[7] = (double)g2_pairs;
  ctx->last_timings[8] = (double)g1_adds;
  ctx->last_timings[9] = (double)g2_adds;
  ctx->last_timings[10] = n_table;
  ctx->last_timings[11] = n_large;
  // [21] / [22]: wall time during which at least one G1 / G2 accumulation ran (the union of the
  // launches' event intervals): with two accumulation lanes G1 launches overlap, so the summed
  // launch time ([2]) counts that time twice
  ctx->last_timings[21] = ctx->last_timings[22] = 0;
  if (acc_events_on()) {
    for (int g = 0; g < 2; g++) {
      std::vector<std::pair<float, float>> iv;
      for (int q = 0; q < nbig; q++) {
        const int j = big[q];
        if (jobs[j].g2 != (g == 1)) continue;
        float a = 0, b = 0;
        if (hipEventElapsedTime(&a, jev[32], jev[2 * j]) == hipSuccess &&
            hipEventElapsedTime(&b, jev[32], jev[2 * j + 1]) == hipSuccess)
          iv.push_back({a, b});
      }
      std::sort(iv.begin(), iv.end());
      double tot = 0, cs = -1e30, ce = -1e30;
      for (const auto& x : iv) {
        if (x.first > ce) { if (ce > cs) tot += ce - cs; cs = x.first; ce = x.second; }
        else ce = std::max(ce, (double)x.second);
      }
      if (ce > cs) tot += ce - cs;
      ctx->last_timings[21 + g] = tot;
    }
  }
  // bytes of the window tables this proof's multiexps read (each distinct table once): for a
  // shard, its own slices and h share only, not whatever else the Parameters keep resident
  size_t tb = 0;
  for (int j = 0; j < 8; j++) {
    if (!use_table[j]) continue;
    bool seen = false;
    for (int q = 0; q < j; q++) seen |= use_table[q] && jobs[q].srs == jobs[j].srs;
    if (!seen) tb += jobs[j].srs->win->bytes;
  }
  ctx->last_timings[12] = (double)tb;
  drain.ok = true;
  return BH_OK;
}

// proof assembly (prover.rs:315-349) -> Proof::write (groth16/mod.rs:42-48)
// The terms of A, B and C that depend only on the verifying key and r, s (5 of the 7 scalar
// multiplications): computed on a host thread while the device works.
struct AssemblePre {
  uint64_t rc[4], sc[4];
  Jac<Fp> g_a, g_c;
  Jac<bh::Fp2> g_b;
};

AssemblePre assemble_pre(const VkHost& vk, const uint64_t r_in[4], const uint64_t s_in[4]) {
  AssemblePre p;
  Fr r = fr_from_canonical(r_in), sv = fr_from_canonical(s_in);
  uint64_t rsc[4];
  fr_to_canonical(r, p.rc);
  fr_to_canonical(sv, p.sc);
  fr_to_canonical(mul(r, sv), rsc);
  const Jac<Fp> d1 = jac_from_affine(vk.delta_g1);
  const Jac<bh::Fp2> d2 = jac_from_affine(vk.delta_g2);
  p.g_a = jac_add(jac_mul(d1, p.rc, 4), jac_from_affine(vk.alpha_g1));
  p.g_b = jac_add(jac_mul(d2, p.sc, 4), jac_from_affine(vk.beta_g2));
  p.g_c = jac_mul(d1, rsc, 4);
  p.g_c = jac_add(p.g_c, jac_mul(jac_from_affine(vk.alpha_g1), p.sc, 4));
  p.g_c = jac_add(p.g_c, jac_mul(jac_from_affine(vk.beta_g1), p.rc, 4));
  return p;
}

void assemble_finish(const AssemblePre& p, const Jac<Fp> r1[6], const Jac<bh::Fp2> r2[2], uint8_t proof_out[192]) {
  Jac<Fp> g_a = p.g_a, g_c = p.g_c;
  Jac<bh::Fp2> g_b = p.g_b;
  Jac<Fp> a_answer = jac_add(r1[2], r1[3]);
  g_a = jac_add(g_a, a_answer);
  a_answer = jac_mul(a_answer, p.sc, 4);
  g_c = jac_add(g_c, a_answer);
  Jac<Fp> b1_answer = jac_add(r1[4], r1[5]);
  Jac<bh::Fp2> b2_answer = jac_add(r2[0], r2[1]);
  g_b = jac_add(g_b, b2_answer);
  b1_answer = jac_mul(b1_answer, p.rc, 4);
  g_c = jac_add(g_c, b1_answer);
  g_c = jac_add(g_c, r1[0]);
  g_c = jac_add(g_c, r1[1]);
  g1_to_compressed(jac_to_affine(g_a), proof_out);
  g2_to_compressed(jac_to_affine(g_b), proof_out + 48);
  g1_to_compressed(jac_to_affine(g_c), proof_out + 144);
}

void assemble(const VkHost& vk, const Jac<Fp> r1[6], const Jac<bh::Fp2> r2[2], const uint64_t r_in[4],
              const uint64_t s_in[4], uint8_t proof_out[192]) {
  assemble_finish(assemble_pre(vk, r_in, s_in), r1, r2, proof_out);
}

// assemble_pre on its own host thread, started before the device work is enqueued (~0.1 ms of
// the ~0.2 ms assembly leaves the critical path); computed inline if no thread can be started.
struct AssemblePreThread {
  VkHost vk;
  uint64_t r[4], s[4];
  AssemblePre pre;
  std::thread th;
  AssemblePreThread(const VkHost& v, const uint64_t r_in[4], const uint64_t s_in[4]) : vk(v) {
    memcpy(r, r_in, sizeof r);
    memcpy(s, s_in, sizeof s);
    try {
      th = std::thread([this] { pre = assemble_pre(vk, r, s); });
    } catch (...) {
      pre = assemble_pre(vk, r, s);
    }
  }
  const AssemblePre& get() {
    if (th.joinable()) th.join();
    return pre;
  }
  ~AssemblePreThread() {
    if (th.joinable()) th.join();
  }
};

VkHost vk_of(const bh_params* p) {
  return VkHost{p->alpha_g1, p->beta_g1, p->delta_g1, p->beta_g2, p->delta_g2};
}

constexpr size_t PARTIAL_BYTES = 6 * 96 + 2 * 192;

void write_partial(const Jac<Fp> r1[6], const Jac<bh::Fp2> r2[2], uint8_t* out) {
  for (int i = 0; i < 6; i++) g1_to_uncompressed(jac_to_affine(r1[i]), out + 96 * i);
  for (int i = 0; i < 2; i++) g2_to_uncompressed(jac_to_affine(r2[i]), out + 576 + 192 * i);
}

// N virtual ranks of one device, one host thread each: the all-to-all as device copies.
struct LocalGroup {
  explicit LocalGroup(int n) : N(n), send(n, nullptr), ready(n, nullptr), copied(n, nullptr) {}
  int N;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  size_t gen = 0;
  bool aborted = false;
  std::vector<const uint32_t*> send;
  std::vector<hipEvent_t> ready, copied;
  // false if a rank failed (its peers must not wait for it)
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const size_t g = gen;
    if (++arrived == N) {
      arrived = 0;
      gen++;
      cv.notify_all();
      return true;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

struct LocalExchanger : Exchanger {
  LocalGroup* g;
  int r;
  LocalExchanger(LocalGroup* gg, int rr) : g(gg), r(rr) {}
  int rank() const override { return r; }
  int size() const override { return g->N; }
  bh_status exchange(const uint32_t* send, uint32_t* recv, size_t C, size_t M, int nvec, hipStream_t st) override {
    g->send[r] = send;
    BH_TRY_HIP(hipEventRecord(g->ready[r], st));
    if (!g->barrier()) return BH_ERR_HIP;  // every rank's send buffer is final once its event fires
    for (int p = 0; p < g->N; p++) {
      if (p != r) BH_TRY_HIP(hipStreamWaitEvent(st, g->ready[p], 0));
      for (int v = 0; v < nvec; v++)  // chunk r of p's send -> chunk p of my recv
        BH_TRY_HIP(hipMemcpyAsync(recv + ((size_t)v * M + (size_t)p * C) * 8,
                                  g->send[p] + ((size_t)v * M + (size_t)r * C) * 8, C * 32, hipMemcpyDeviceToDevice,
                                  st));
    }
    BH_TRY_HIP(hipEventRecord(g->copied[r], st));
    if (!g->barrier()) return BH_ERR_HIP;
    // my send buffer is rewritten later on this stream: only after every peer has copied from it
    for (int p = 0; p < g->N; p++)
      if (p != r) BH_TRY_HIP(hipStreamWaitEvent(st, g->copied[p], 0));
    return BH_OK;
  }
};

// Rehearsal of ONE rank of an N-rank run on one device: the all-to-alls move this rank's own
// chunks only (the same copy volume per rank as the real exchange, minus the link), so the
// device work and its timing are those of the rank, the data is not (the result is discarded).
struct SelfExchanger : Exchanger {
  int r, n;
  SelfExchanger(int rr, int nn) : r(rr), n(nn) {}
  int rank() const override { return r; }
  int size() const override { return n; }
  bh_status exchange(const uint32_t* send, uint32_t* recv, size_t C, size_t M, int nvec, hipStream_t st) override {
    for (int v = 0; v < nvec; v++)
      BH_TRY_HIP(hipMemcpyAsync(recv + (size_t)v * M * 8, send + (size_t)v * M * 8, M * 32, hipMemcpyDeviceToDevice,
                                st));
    return BH_OK;
  }
};

inline int dev_of(const bh_ctx* c) { return c ? c->device : -1; }
// Parameters and witnesses live in one device's HBM: a context of another device cannot use them
bool same_device(const bh_ctx* ctx, const bh_params* p, const bh_witness* w) {
  return (!p || dev_of(p->ctx) == ctx->device) && (!w || dev_of(w->ctx) == ctx->device);
}

// compute_msms, and on failure wait for whatever it had already enqueued on the context's
// streams (the next call reuses the same workspaces)
bh_status compute_msms_sync(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t shard, size_t nshards,
                            Jac<Fp> res1[6], Jac<bh::Fp2> res2[2], Exchanger* ex = nullptr, bool may_build = true,
                            UploadSync* up = nullptr) {
  bh_status s = compute_msms(ctx, params, w, shard, nshards, res1, res2, ex, may_build, up);
  if (s) ctx_sync_all(ctx);
  return s;
}

// N ranks of one device, one context and one host thread each, running exactly the per-rank
// code of bh_prove_witness_partial_comm with a LocalExchanger in place of RCCL.  With
// prebuilt = false each rank's tables are built first, rank after rank (a rank must never
// build while its peers wait for it inside an exchange); the threads themselves never build.
bh_status run_ranks(const std::vector<bh_ctx*>& ctxs, const std::vector<const bh_params*>& ps, const bh_witness* w,
                    uint8_t* partials_out, bool build_first) {
  const int N = (int)ctxs.size();
  if (build_first) {
    for (int k = 0; k < N; k++) {
      bh_ctx* v = ctxs[k];
      std::lock_guard<std::mutex> vl(v->mu);
      BH_TRY_HIP(hipSetDevice(v->device));
      ShareGeom geom;
      const bool dist = dist_h_eligible(N, w->log_m) && (size_t)N >= dist_h_min_ranks();
      if (dist) {
        geom.N = N; geom.rank = k; geom.L = w->log_m; geom.M = w->m / N; geom.C = geom.M / N;
      }
      std::unique_lock<std::shared_mutex> pwr(const_cast<bh_params*>(ps[k])->mu);
      Job jobs[8];
      bh_status s = plan_shard(v, ps[k], w, (size_t)k, (size_t)N, dist ? &geom : nullptr, nullptr, nullptr, nullptr,
                               nullptr, nullptr, true, jobs);
      if (s) return s;
    }
  }
  LocalGroup grp(N);
  struct EvGuard {
    LocalGroup& g;
    ~EvGuard() {
      for (int k = 0; k < g.N; k++) {
        if (g.ready[k]) (void)hipEventDestroy(g.ready[k]);
        if (g.copied[k]) (void)hipEventDestroy(g.copied[k]);
      }
    }
  } guard{grp};
  for (int k = 0; k < N; k++) {
    BH_TRY_HIP(hipEventCreateWithFlags(&grp.ready[k], hipEventDisableTiming));
    BH_TRY_HIP(hipEventCreateWithFlags(&grp.copied[k], hipEventDisableTiming));
  }
  std::vector<bh_status> st(N, BH_OK);
  std::vector<std::thread> th;
  for (int k = 0; k < N; k++)
    th.emplace_back([&, k] {
      bh_ctx* v = ctxs[k];
      std::lock_guard<std::mutex> vl(v->mu);
      if (hipSetDevice(v->device) != hipSuccess) { st[k] = BH_ERR_HIP; grp.abort(); return; }
      LocalExchanger ex(&grp, k);
      Jac<Fp> r1[6];
      Jac<bh::Fp2> r2[2];
      st[k] = compute_msms_sync(v, ps[k], w, (size_t)k, (size_t)N, r1, r2, &ex, false);
      if (st[k]) { grp.abort(); return; }
      write_partial(r1, r2, partials_out + (size_t)k * PARTIAL_BYTES);
    });
  for (auto& t : th) t.join();
  for (int k = 0; k < N; k++)
    if (st[k]) return st[k];
  return BH_OK;
}

}  // namespace

extern "C" {

bh_status bh_params_prepare(bh_ctx* ctx, bh_params* params, const bh_witness* w, size_t nshards) {
  if (!ctx || !params || !w || nshards == 0) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_lock<std::shared_mutex> pwr(params->mu);
  return prepare_tables_full(ctx, params, w->m, w->num_aux, w->a_aux_total, w->b_aux_total, nshards);
}

bh_status bh_params_prepare_shard(bh_ctx* ctx, bh_params* params, const bh_witness* w, size_t shard, size_t nshards,
                                  int distributed_h) {
  if (!ctx || !params || !w || nshards == 0 || shard >= nshards) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  ShareGeom geom;
  const bool dist = distributed_h && dist_h_eligible((int)nshards, w->log_m) && nshards >= dist_h_min_ranks();
  if (dist) {
    geom.N = (int)nshards; geom.rank = (int)shard; geom.L = w->log_m;
    geom.M = w->m / nshards; geom.C = geom.M / nshards;
  }
  std::unique_lock<std::shared_mutex> pwr(params->mu);
  Job jobs[8];
  return plan_shard(ctx, params, w, shard, nshards, dist ? &geom : nullptr, nullptr, nullptr, nullptr, nullptr,
                    nullptr, true, jobs);
}

bh_status bh_prove_witness(bh_ctx* ctx, const bh_params* params, const bh_witness* w, const uint64_t r_in[4],
                           const uint64_t s_in[4], uint8_t proof_out[192]) {
  if (!ctx || !params || !w || !r_in || !s_in || !proof_out) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  AssemblePreThread pre(vk_of(params), r_in, s_in);
  bh_status s = compute_msms_sync(ctx, params, w, 0, 1, r1, r2);
  if (s) return s;
  const auto t0 = std::chrono::steady_clock::now();
  assemble_finish(pre.get(), r1, r2, proof_out);
  const double asm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ctx->last_timings[0] += asm_ms;
  if (getenv("BH_HOST_TIMING")) fprintf(stderr, "assemble %.3f ms\n", asm_ms);
  return BH_OK;
}

bh_status bh_shard_range(size_t n, size_t shard, size_t nshards, size_t* lo, size_t* hi) {
  if (!lo || !hi || nshards == 0 || shard >= nshards) return BH_ERR_INVALID_ARGUMENT;
  shard_range(n, shard, nshards, lo, hi);
  return BH_OK;
}

bh_status bh_prove_witness_partial(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t shard,
                                   size_t nshards, uint8_t partial_out[960]) {
  if (!ctx || !params || !w || !partial_out || nshards == 0 || shard >= nshards) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  bh_status s = compute_msms_sync(ctx, params, w, shard, nshards, r1, r2);
  if (s) return s;
  write_partial(r1, r2, partial_out);
  return BH_OK;
}

bh_status bh_prove_witness_partial_comm(bh_ctx* ctx, const bh_params* params, const bh_witness* w, bh_comm* comm,
                                        uint8_t partial_out[960]) {
  if (!ctx || !params || !w || !comm || !partial_out) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  std::unique_ptr<Exchanger> ex = rccl_exchanger(comm);
  bh_status s = compute_msms_sync(ctx, params, w, (size_t)ex->rank(), (size_t)ex->size(), r1, r2, ex.get());
  if (s) return s;
  write_partial(r1, r2, partial_out);
  return BH_OK;
}

bh_status bh_prove_witness_partials_local(bh_ctx* ctx, const bh_params* params, const bh_witness* w,
                                          size_t nshards, uint8_t* partials_out) {
  if (!ctx || !params || !w || !partials_out || nshards == 0 || nshards > 64) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  const int N = (int)nshards;
  while ((int)ctx->vranks.size() < N) {
    bh_ctx* v = nullptr;
    bh_status s = bh_ctx_create(ctx->device, &v);
    if (s) return s;
    ctx->vranks.push_back(v);
  }
  std::vector<bh_ctx*> ctxs(ctx->vranks.begin(), ctx->vranks.begin() + N);
  for (bh_ctx* v : ctxs) {
    v->tables = ctx->tables;
    v->window_override = ctx->window_override;
    v->co_ranks = N;
  }
  // one Parameters for every rank: tables covering every shard (full vectors at the shard's
  // window size) are built once up front
  {
    std::unique_lock<std::shared_mutex> pwr(const_cast<bh_params*>(params)->mu);
    bh_status s = prepare_tables_full(ctx, const_cast<bh_params*>(params), w->m, w->num_aux, w->a_aux_total,
                                      w->b_aux_total, nshards, N);
    if (s) return s;
  }
  std::vector<const bh_params*> ps(N, params);
  return run_ranks(ctxs, ps, w, partials_out, false);
}

bh_status bh_rehearse_rank(bh_ctx* ctx, const bh_params* params, const bh_witness* w, size_t rank, size_t nranks,
                           double* ms) {
  if (!ctx || !params || !w || nranks == 0 || rank >= nranks) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, w)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  SelfExchanger ex((int)rank, (int)nranks);
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  const auto t0 = std::chrono::steady_clock::now();
  bh_status s = compute_msms_sync(ctx, params, w, rank, nranks, r1, r2, &ex);
  if (s) return s;
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return BH_OK;
}

// default pipelined lanes of bh_prove_batch: two (a third adds nothing, profiles/r04_ab_c5_lanes.txt)
static int batch_lanes() { return 2; }

bh_status bh_prove_batch(bh_ctx* ctx, const bh_params* params, const bh_witness* const* ws, size_t k,
                         const uint64_t r_in[4], const uint64_t s_in[4], int lanes, uint8_t* proofs_out) {
  if (!ctx || !params || !ws || !r_in || !s_in || !proofs_out || lanes < 0 || lanes > 16) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, nullptr)) return BH_ERR_INVALID_ARGUMENT;
  for (size_t i = 0; i < k; i++)
    if (!ws[i] || !same_device(ctx, nullptr, ws[i])) return BH_ERR_INVALID_ARGUMENT;
  if (k == 0) return BH_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  // Throughput mode (BASELINE.json configs[4]): independent proofs (r, s fixed, prover.rs:158-173)
  // on `lanes` contexts of this device, each driven by a host thread through a share of the
  // batch, so one proof's start-up (sorts, H) and reduction tails fill the bubbles of
  // another's accumulations; proofs_out[i] is exactly bh_prove_witness(ws[i]).
  // lanes = 0: the default, BATCH_LANES pipelined lanes
  const int L = (int)std::min<size_t>(lanes ? (size_t)lanes : (size_t)batch_lanes(), k);
  if (L == 1) {
    // one lane: the proofs back to back on this context, each one's start-up and last tail
    // exposed (2^20 proofs: 17.98 ms each, BENCH r03 before the pipelined lanes)
    // r and s are shared by the batch: their terms of A, B, C once, beside the first proof
    AssemblePreThread pre(vk_of(params), r_in, s_in);
    for (size_t i = 0; i < k; i++) {
      Jac<Fp> r1[6];
      Jac<bh::Fp2> r2[2];
      bh_status st1 = compute_msms_sync(ctx, params, ws[i], 0, 1, r1, r2, nullptr, true);
      if (st1) return st1;
      assemble_finish(pre.get(), r1, r2, proofs_out + 192 * i);
    }
    return BH_OK;
  }
  // Pipelined lanes (the reference's Worker::compute fan-out, multicore.rs:33-76): L contexts that
  // borrow THIS context's streams (ctx_create_lane: own workspaces, events and buffers, no extra
  // hardware queue), driven by L host threads that take turns in proof order.  Proof i+1 is
  // enqueued as soon as proof i's device work is (t_enqueued_hook), so its density maps, sorts and
  // H sit in the streams behind proof i's accumulations and run beside proof i's last reduction
  // tail and host combine; stream order keeps the accumulations proof after proof.
  // (Round 2's lanes were contexts with streams of their own: 19.8 ms per 2^20 proof with two,
  // slower than one lane -- every extra context added 13 streams to the queue budget.)
  while ((int)ctx->lanes.size() < L) {
    bh_ctx* v = nullptr;
    bh_status st = ctx_create_lane(ctx, &v);
    if (st) return st;
    ctx->lanes.push_back(v);
  }
  for (int l = 0; l < L; l++) {
    ctx->lanes[l]->tables = ctx->tables;
    ctx->lanes[l]->window_override = ctx->window_override;
  }
  {  // every table the batch needs, built once before the lanes start (they never build)
    std::unique_lock<std::shared_mutex> pwr(const_cast<bh_params*>(params)->mu);
    for (size_t i = 0; i < k; i++) {
      bool seen = false;
      for (size_t j = 0; j < i && !seen; j++)
        seen = ws[j]->m == ws[i]->m && ws[j]->num_aux == ws[i]->num_aux && ws[j]->a_aux_total == ws[i]->a_aux_total &&
               ws[j]->b_aux_total == ws[i]->b_aux_total;
      if (seen) continue;
      Job jobs[8];
      bh_status st = plan_shard(ctx->lanes[0], params, ws[i], 0, 1, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, true, jobs);
      if (st) return st;
    }
  }
  const AssemblePre pre = assemble_pre(vk_of(params), r_in, s_in);
  // two turnstiles in proof order: turn[0] = the next proof allowed to start enqueueing, turn[1] =
  // the next proof allowed to enqueue its reduction tails
  std::mutex turn_mu;
  std::condition_variable turn_cv;
  size_t turn[2] = {0, 0};
  std::atomic<bool> failed{false};
  auto pass = [&](int t, size_t i) {
    {
      std::lock_guard<std::mutex> lk(turn_mu);
      if (turn[t] == i) turn[t] = i + 1;
    }
    turn_cv.notify_all();
  };
  auto await = [&](int t, size_t i) {
    std::unique_lock<std::mutex> lk(turn_mu);
    turn_cv.wait(lk, [&] { return turn[t] == i; });
  };
  // proof i is over on this lane: both turns handed on (no-ops where its hooks already did;
  // an early error still hands the tail turn on after the previous proof's, in order)
  auto close = [&](size_t i) {
    {
      std::unique_lock<std::mutex> lk(turn_mu);
      if (turn[0] == i) turn[0] = i + 1;
      turn_cv.notify_all();
      turn_cv.wait(lk, [&] { return turn[1] >= i; });
      if (turn[1] == i) turn[1] = i + 1;
    }
    turn_cv.notify_all();
  };
  std::vector<bh_status> st(L, BH_OK);
  std::vector<std::thread> th;
  for (int l = 0; l < L; l++)
    th.emplace_back([&, l] {
      bh_ctx* v = ctx->lanes[l];
      std::lock_guard<std::mutex> vl(v->mu);
      if (hipSetDevice(v->device) != hipSuccess) st[l] = BH_ERR_HIP;
      for (size_t i = (size_t)l; i < k; i += (size_t)L) {
        await(0, i);
        if (st[l] || failed) {  // a failed lane still passes its turns: no thread waits forever
          close(i);
          continue;
        }
        t_lane.after_accs = [&pass, i] { pass(0, i); };
        t_lane.before_tails = [&await, i] { await(1, i); };
        t_lane.after_tails = [&pass, i] { pass(1, i); };
        Jac<Fp> r1[6];
        Jac<bh::Fp2> r2[2];
        st[l] = compute_msms_sync(v, params, ws[i], 0, 1, r1, r2, nullptr, false);
        t_lane = LaneHooks();
        close(i);
        if (st[l]) {
          failed = true;
          continue;
        }
        assemble_finish(pre, r1, r2, proofs_out + 192 * i);
      }
    });
  for (auto& t : th) t.join();
  for (int l = 0; l < L; l++)
    if (st[l]) return st[l];
  return BH_OK;
}

bh_status bh_prove_witness_partials_ranks(bh_ctx* const* ctxs, const bh_params* const* params, const bh_witness* w,
                                          size_t nranks, uint8_t* partials_out) {
  if (!ctxs || !params || !w || !partials_out || nranks == 0 || nranks > 64) return BH_ERR_INVALID_ARGUMENT;
  std::vector<bh_ctx*> cs(ctxs, ctxs + nranks);
  std::vector<const bh_params*> ps(params, params + nranks);
  for (size_t k = 0; k < nranks; k++) {
    if (!cs[k] || !ps[k] || cs[k]->device != cs[0]->device || !same_device(cs[k], ps[k], w))
      return BH_ERR_INVALID_ARGUMENT;
    for (size_t j = 0; j < k; j++)
      if (cs[j] == cs[k]) return BH_ERR_INVALID_ARGUMENT;  // one context per rank
  }
  return run_ranks(cs, ps, w, partials_out, true);
}

bh_status bh_vk_write(const bh_params* p, uint8_t* out, size_t cap, size_t* written) {
  if (!p || !written) return BH_ERR_INVALID_ARGUMENT;
  const size_t need = 96 * 3 + 192 * 3 + 4 + 96 * p->ic.size();
  *written = need;
  if (!out) return BH_OK;
  if (cap < need) return BH_ERR_INVALID_ARGUMENT;
  uint8_t* o = out;
  g1_to_uncompressed(p->alpha_g1, o); o += 96;
  g1_to_uncompressed(p->beta_g1, o); o += 96;
  g2_to_uncompressed(p->beta_g2, o); o += 192;
  g2_to_uncompressed(p->gamma_g2, o); o += 192;
  g1_to_uncompressed(p->delta_g1, o); o += 96;
  g2_to_uncompressed(p->delta_g2, o); o += 192;
  const size_t n = p->ic.size();
  o[0] = (uint8_t)(n >> 24); o[1] = (uint8_t)(n >> 16); o[2] = (uint8_t)(n >> 8); o[3] = (uint8_t)n; o += 4;
  for (const auto& ic : p->ic) { g1_to_uncompressed(ic, o); o += 96; }
  return BH_OK;
}

// Host-only: sum the per-shard partial multiexps (the all-gathered 960-byte records,
// shard order) and assemble the proof.  vk: VerifyingKey::write bytes.
bh_status bh_proof_from_partials(const uint8_t* vk_bytes, size_t vk_len, const uint8_t* partials, size_t nshards,
                                 const uint64_t r[4], const uint64_t s[4], uint8_t proof_out[192]) {
  if (!vk_bytes || !partials || !nshards || !r || !s || !proof_out) return BH_ERR_INVALID_ARGUMENT;
  if (vk_len < 96 * 3 + 192 * 3) return BH_ERR_INVALID_ENCODING;
  // on-curve checks only: the VK comes from bh_vk_write of loaded (checked) Parameters and
  // the partials are sums of subgroup points; this runs once per multi-GPU proof
  VkHost vk;
  AffinePt<bh::Fp2> gamma;
  const uint8_t* p = vk_bytes;
  if (g1_from_uncompressed(p, &vk.alpha_g1, true)) return BH_ERR_INVALID_ENCODING;
  if (g1_from_uncompressed(p + 96, &vk.beta_g1, true)) return BH_ERR_INVALID_ENCODING;
  if (g2_from_uncompressed(p + 192, &vk.beta_g2, true)) return BH_ERR_INVALID_ENCODING;
  if (g2_from_uncompressed(p + 384, &gamma, true)) return BH_ERR_INVALID_ENCODING;
  if (g1_from_uncompressed(p + 576, &vk.delta_g1, true)) return BH_ERR_INVALID_ENCODING;
  if (g2_from_uncompressed(p + 672, &vk.delta_g2, true)) return BH_ERR_INVALID_ENCODING;
  if (vk.delta_g1.infinity || vk.delta_g2.infinity) return BH_ERR_UNEXPECTED_IDENTITY;  // prover.rs:309-313
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  for (int i = 0; i < 6; i++) r1[i] = jac_identity<Fp>();
  for (int i = 0; i < 2; i++) r2[i] = jac_identity<bh::Fp2>();
  for (size_t k = 0; k < nshards; k++) {
    const uint8_t* q = partials + k * PARTIAL_BYTES;
    for (int i = 0; i < 6; i++) {
      AffinePt<Fp> a;
      if (g1_from_uncompressed(q + 96 * i, &a, true)) return BH_ERR_INVALID_ENCODING;
      r1[i] = jac_add(r1[i], jac_from_affine(a));
    }
    for (int i = 0; i < 2; i++) {
      AffinePt<bh::Fp2> a;
      if (g2_from_uncompressed(q + 576 + 192 * i, &a, true)) return BH_ERR_INVALID_ENCODING;
      r2[i] = jac_add(r2[i], jac_from_affine(a));
    }
  }
  assemble(vk, r1, r2, r, s, proof_out);
  return BH_OK;
}

bh_status bh_prove(bh_ctx* ctx, const bh_params* params, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                   size_t nc, const uint64_t* inputs, size_t ni, const uint64_t* aux, size_t na,
                   const uint64_t* a_aux_density, const uint64_t* b_input_density, const uint64_t* b_aux_density,
                   const uint64_t r[4], const uint64_t s[4], uint8_t proof_out[192]) {
  if (!ctx || !params || !r || !s || !proof_out) return BH_ERR_INVALID_ARGUMENT;
  if (!same_device(ctx, params, nullptr)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  // the witness streams in on the copy stream while the proof is enqueued: its sorts start
  // once aux has landed, the H block once a, b, c have (pinned ring + memcpy threads)
  if (!ctx->dropin) ctx->dropin = new bh_witness();
  bh_witness* w = ctx->dropin;
  bh_status st = witness_host(ctx, w, a, b, c, nc, inputs, ni, aux, na, a_aux_density, b_input_density,
                              b_aux_density);
  if (st) return st;
  UploadSync up;
  struct EvGuard {
    UploadSync& u;
    ~EvGuard() {
      for (auto e : u.ev) if (e) (void)hipEventDestroy(e);
      for (auto e : u.vec) if (e) (void)hipEventDestroy(e);
      if (u.t0) (void)hipEventDestroy(u.t0);
    }
  } evg{up};
  BH_TRY_HIP(hipEventCreate(&up.t0));
  BH_TRY_HIP(hipEventCreate(&up.ev[0]));
  BH_TRY_HIP(hipEventCreate(&up.ev[1]));
  for (auto& e : up.vec) BH_TRY_HIP(hipEventCreate(&e));
  // H from the uploading thread: each of a, b, c is converted and transformed on the H stream
  // as soon as its own upload has landed (stream order behind vec[v]), so H starts ~1/3 of the
  // a, b, c upload after aux and runs beside the first accumulations, and no host thread that
  // enqueues the multiexps ever waits for the upload of a, b, c (prover.rs:210-231).  (One stream,
  // BH_PROVER_SERIAL: compute_msms enqueues H after the whole upload.)
  const bool h_uploader = !prover_serial();
  Domain* D = nullptr;
  if (h_uploader) {
    // everything the H stages touch, allocated before the uploading thread can enqueue them
    if ((st = ctx_domain(ctx, w->log_m, &D))) return st;
    BH_TRY_HIP(ctx->staging.alloc(3 * w->m * 32));
    BH_TRY_HIP(ctx->hbuf.alloc(w->m * 32));
    up.on_vector = [ctx, w, D, &up](int v) -> int {
      hipStream_t sH = ctx->stream4;
      const size_t m = w->m, nc = w->num_constraints;
      uint32_t* abc = ctx->staging.as<uint32_t>();
      BH_TRY_HIP(hipStreamWaitEvent(sH, up.vec[v], 0));
      if (v == 0) BH_TRY_HIP(hipEventRecord(ctx->ev[0], sH));
      // the ifft's first pass reads the uploaded bls12_381-Montgomery words in place (their radix
      // folded into its scale, run_h_vector); only the padding is written first.  (A conversion
      // kernel first, round 5's first scheme, waited for slots beside the accumulations: 9.5 ms
      // for a trivial kernel in the round-5 drop-in trace.)
      uint32_t* raw = const_cast<uint32_t*>(w->abc.as<uint32_t>());
      if (m > nc) BH_TRY_HIP(hipMemsetAsync(raw + ((size_t)v * m + nc) * 8, 0, (m - nc) * 32, sH));
      bh_status hs = run_h_vector(ctx, D, abc, sH, raw, v, true);
      if (hs) return hs;
      if (v == 2) {
        // the last pass writes h as canonical scalars, natural order, truncated to m-1 (prover.rs:227-231)
        if ((hs = run_h_final(ctx, D, abc, sH, ctx->hbuf.as<uint32_t>()))) return hs;
        BH_TRY_HIP(hipEventRecord(ctx->ev[1], sH));
      }
      return BH_OK;
    };
  }
  BH_TRY_HIP(hipEventRecord(up.t0, ctx->h2d));
  bh_status ust = BH_OK;
  std::thread uploader([&] {
    if (hipSetDevice(ctx->device) != hipSuccess) { ust = BH_ERR_HIP; up.set(-1, ust); return; }
    ust = witness_device(ctx, w, a, b, c, inputs, aux, ctx->h2d, &up);
  });
  Jac<Fp> r1[6];
  Jac<bh::Fp2> r2[2];
  AssemblePreThread pre(vk_of(params), r, s);
  st = compute_msms_sync(ctx, params, w, 0, 1, r1, r2, nullptr, true, &up);
  uploader.join();
  (void)hipStreamSynchronize(ctx->h2d);
  if (st || ust) {
    // compute_msms' drain may have run before the uploader finished enqueueing H on the H
    // stream (staging, hbuf): drain every stream once more so no later call races those kernels
    ctx_sync_all(ctx);
    return st ? st : ust;
  }
  // upload landing times from the call's start (bh_last_stats [13..16): aux, a, b, c) and, from
  // compute_msms, the H block's end ([12] stays the table bytes)
  {
    float t = 0;
    ctx->last_timings[13] = hipEventElapsedTime(&t, up.t0, up.ev[0]) == hipSuccess ? t : -1;
    for (int v = 0; v < 3; v++)
      ctx->last_timings[14 + v] = hipEventElapsedTime(&t, up.t0, up.vec[v]) == hipSuccess ? t : -1;
    ctx->last_timings[17] = hipEventElapsedTime(&t, up.t0, ctx->ev[1]) == hipSuccess ? t : -1;
  }
  assemble_finish(pre.get(), r1, r2, proof_out);
  ctx->last_timings[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return BH_OK;
}

bh_status bh_last_timings(const bh_ctx* ctx, double out[10]) {
  if (!ctx || !out) return BH_ERR_INVALID_ARGUMENT;
  memcpy(out, ctx->last_timings, 10 * sizeof(double));
  return BH_OK;
}

bh_status bh_last_stats(const bh_ctx* ctx, double* out, size_t n) {
  if (!ctx || (n && !out)) return BH_ERR_INVALID_ARGUMENT;
  const size_t have = sizeof ctx->last_timings / sizeof(double);
  for (size_t i = 0; i < n; i++) out[i] = i < have ? ctx->last_timings[i] : 0.0;
  return BH_OK;
}

}  // extern "C"
