// Groth16 prover core on the device: Parameters handling (groth16/mod.rs:224-477)
// and create_proof after synthesis (groth16/prover.rs:206-349).
#include <string.h>

#include <chrono>

#include "api_internal.h"

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
  if (g1_from_uncompressed(b, out, true) != 0) return BH_ERR_INVALID_ENCODING;
  if (reject_identity && out->infinity) return BH_ERR_INVALID_ENCODING;
  return BH_OK;
}
bh_status read_g2_vk(Reader& r, AffinePt<bh::Fp2>* out) {
  const uint8_t* b;
  if (!r.take(192, &b)) return BH_ERR_INVALID_ENCODING;
  if (g2_from_uncompressed(b, out, true) != 0) return BH_ERR_INVALID_ENCODING;
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
      g1_to_uncompressed(AffinePt<Fp>{fp_from_dev_words(d), fp_from_dev_words(d + 12), inf[i] != 0}, o);
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
  if (!ctx || !out || (nc && (!a || !b || !c)) || (ni && !inputs) || (na && !aux)) return BH_ERR_INVALID_ARGUMENT;
  if ((na && (!a_aux_density || !b_aux_density)) || (ni && !b_input_density)) return BH_ERR_INVALID_ARGUMENT;
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(nc, &m, &L);  // EvaluationDomain::from_coeffs, prover.rs:211-213
  if (s) return s;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::unique_ptr<bh_witness> w(new bh_witness());
  w->ctx = ctx;
  w->num_constraints = nc; w->m = m; w->log_m = (int)L; w->num_inputs = ni; w->num_aux = na;
  BH_TRY_HIP(w->abc.alloc(3 * m * 32));
  uint32_t* abc = w->abc.as<uint32_t>();
  if ((s = upload_fr(ctx, a, nc, m, abc))) return s;
  if ((s = upload_fr(ctx, b, nc, m, abc + m * 8))) return s;
  if ((s = upload_fr(ctx, c, nc, m, abc + 2 * m * 8))) return s;
  BH_TRY_HIP(w->inputs.alloc(std::max<size_t>(ni, 1) * 32));
  BH_TRY_HIP(w->aux.alloc(std::max<size_t>(na, 1) * 32));
  if (ni) {
    BH_TRY_HIP(hipMemcpyAsync(w->inputs.p, inputs, ni * 32, hipMemcpyHostToDevice, ctx->stream));
    BH_TRY_HIP(scalars_prepare(w->inputs.as<uint32_t>(), w->inputs.as<uint32_t>(), ni, 1, 0, ctx->stream));
  }
  if (na) {
    BH_TRY_HIP(hipMemcpyAsync(w->aux.p, aux, na * 32, hipMemcpyHostToDevice, ctx->stream));
    BH_TRY_HIP(scalars_prepare(w->aux.as<uint32_t>(), w->aux.as<uint32_t>(), na, 1, 0, ctx->stream));
  }
  w->a_aux_words = (na + 63) / 64;
  w->b_in_words = (ni + 63) / 64;
  w->b_aux_words = (na + 63) / 64;
  w->a_aux_density.assign(a_aux_density ? a_aux_density : nullptr, a_aux_density ? a_aux_density + w->a_aux_words : nullptr);
  w->b_input_density.assign(b_input_density ? b_input_density : nullptr,
                            b_input_density ? b_input_density + w->b_in_words : nullptr);
  w->b_aux_density.assign(b_aux_density ? b_aux_density : nullptr, b_aux_density ? b_aux_density + w->b_aux_words : nullptr);
  w->a_aux_total = popcount_words(w->a_aux_density, na);
  w->b_in_total = popcount_words(w->b_input_density, ni);
  w->b_aux_total = popcount_words(w->b_aux_density, na);
  const size_t tw = w->a_aux_words + w->b_in_words + w->b_aux_words;
  BH_TRY_HIP(w->dens.alloc(std::max<size_t>(tw, 1) * 8));
  uint64_t* d = w->dens.as<uint64_t>();
  if (w->a_aux_words)
    BH_TRY_HIP(hipMemcpyAsync(d, w->a_aux_density.data(), w->a_aux_words * 8, hipMemcpyHostToDevice, ctx->stream));
  if (w->b_in_words)
    BH_TRY_HIP(hipMemcpyAsync(d + w->a_aux_words, w->b_input_density.data(), w->b_in_words * 8,
                              hipMemcpyHostToDevice, ctx->stream));
  if (w->b_aux_words)
    BH_TRY_HIP(hipMemcpyAsync(d + w->a_aux_words + w->b_in_words, w->b_aux_density.data(), w->b_aux_words * 8,
                              hipMemcpyHostToDevice, ctx->stream));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  *out = w.release();
  return BH_OK;
}

bh_status bh_witness_free(bh_witness* w) {
  delete w;
  return BH_OK;
}

bh_status bh_prove_witness(bh_ctx* ctx, const bh_params* params, const bh_witness* w, const uint64_t r_in[4],
                           const uint64_t s_in[4], uint8_t proof_out[192]) {
  if (!ctx || !params || !w || !r_in || !s_in || !proof_out) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
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
  // ---- H (prover.rs:210-234), device resident
  hipEventRecord(ctx->ev[0], ctx->stream);
  uint32_t* abc = ctx->staging.as<uint32_t>();
  BH_TRY_HIP(hipMemcpyAsync(abc, w->abc.p, 3 * m * 32, hipMemcpyDeviceToDevice, ctx->stream));
  if ((s = run_h_pipeline(ctx, D, abc))) return s;
  // truncate to m-1 and convert to canonical scalars in natural order (prover.rs:227-231)
  BH_TRY_HIP(scalars_prepare(abc, ctx->hbuf.as<uint32_t>(), m - 1, 2, L, ctx->stream));
  hipEventRecord(ctx->ev[1], ctx->stream);

  float g1_acc_ms = 0, g2_acc_ms = 0;
  size_t g1_pairs = 0, g2_pairs = 0;
  int g1_launches = 0, g2_launches = 0;
  auto cnt = [](size_t n, int& launches, size_t& pairs, size_t used) { if (n) { launches++; pairs += used; } };

  Jac<Fp> h, l, a_in, a_aux, b1_in, b1_aux;
  Jac<bh::Fp2> b2_in, b2_aux;
  const uint32_t* inputs = w->inputs.as<uint32_t>();
  const uint32_t* aux = w->aux.as<uint32_t>();
  int32_t* idx = ctx->idx.as<int32_t>();
  // h: FullDensity over params.h (prover.rs:233)
  if ((s = msm_g1_device(ctx, &params->h, 0, ctx->hbuf.as<uint32_t>(), m - 1, nullptr, &h, &g1_acc_ms))) return s;
  cnt(m - 1, g1_launches, g1_pairs, m - 1);
  // l: FullDensity over aux (prover.rs:252-257)
  if ((s = msm_g1_device(ctx, &params->l, 0, aux, na, nullptr, &l, &g1_acc_ms))) return s;
  cnt(na, g1_launches, g1_pairs, na);
  // a_inputs / a_aux (prover.rs:259-275)
  if ((s = msm_g1_device(ctx, &params->a, 0, inputs, ni, nullptr, &a_in, &g1_acc_ms))) return s;
  cnt(ni, g1_launches, g1_pairs, ni);
  if (na) {
    BH_TRY_HIP(density_index(d_a_aux, na, (uint32_t)ni, idx, ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(),
                             ctx->stream));
  }
  if ((s = msm_g1_device(ctx, &params->a, ni, aux, na, idx, &a_aux, &g1_acc_ms))) return s;
  cnt(na, g1_launches, g1_pairs, w->a_aux_total);
  // b_g1 (prover.rs:277-296)
  if (ni) {
    BH_TRY_HIP(density_index(d_b_in, ni, 0, idx, ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(), ctx->stream));
  }
  if ((s = msm_g1_device(ctx, &params->b_g1, 0, inputs, ni, idx, &b1_in, &g1_acc_ms))) return s;
  cnt(ni, g1_launches, g1_pairs, w->b_in_total);
  if ((s = msm_g2_device(ctx, &params->b_g2, 0, inputs, ni, idx, &b2_in, &g2_acc_ms))) return s;
  cnt(ni, g2_launches, g2_pairs, w->b_in_total);
  if (na) {
    BH_TRY_HIP(density_index(d_b_aux, na, (uint32_t)w->b_in_total, idx, ctx->dtmp.as<uint32_t>(),
                             ctx->dscan.as<uint32_t>(), ctx->stream));
  }
  if ((s = msm_g1_device(ctx, &params->b_g1, w->b_in_total, aux, na, idx, &b1_aux, &g1_acc_ms))) return s;
  cnt(na, g1_launches, g1_pairs, w->b_aux_total);
  // b_g2 (prover.rs:298-307)
  if ((s = msm_g2_device(ctx, &params->b_g2, w->b_in_total, aux, na, idx, &b2_aux, &g2_acc_ms))) return s;
  cnt(na, g2_launches, g2_pairs, w->b_aux_total);

  // ---- assembly (prover.rs:315-349)
  Fr r = fr_from_canonical(r_in), sv = fr_from_canonical(s_in);
  uint64_t rc[4], sc[4], rsc[4];
  fr_to_canonical(r, rc);
  fr_to_canonical(sv, sc);
  fr_to_canonical(mul(r, sv), rsc);
  const Jac<Fp> d1 = jac_from_affine(params->delta_g1);
  const Jac<bh::Fp2> d2 = jac_from_affine(params->delta_g2);
  Jac<Fp> g_a = jac_add(jac_mul(d1, rc, 4), jac_from_affine(params->alpha_g1));
  Jac<bh::Fp2> g_b = jac_add(jac_mul(d2, sc, 4), jac_from_affine(params->beta_g2));
  Jac<Fp> g_c = jac_mul(d1, rsc, 4);
  g_c = jac_add(g_c, jac_mul(jac_from_affine(params->alpha_g1), sc, 4));
  g_c = jac_add(g_c, jac_mul(jac_from_affine(params->beta_g1), rc, 4));
  Jac<Fp> a_answer = jac_add(a_in, a_aux);
  g_a = jac_add(g_a, a_answer);
  a_answer = jac_mul(a_answer, sc, 4);
  g_c = jac_add(g_c, a_answer);
  Jac<Fp> b1_answer = jac_add(b1_in, b1_aux);
  Jac<bh::Fp2> b2_answer = jac_add(b2_in, b2_aux);
  g_b = jac_add(g_b, b2_answer);
  b1_answer = jac_mul(b1_answer, rc, 4);
  g_c = jac_add(g_c, b1_answer);
  g_c = jac_add(g_c, h);
  g_c = jac_add(g_c, l);
  // Proof::write: compressed A || B || C (groth16/mod.rs:42-48)
  g1_to_compressed(jac_to_affine(g_a), proof_out);
  g2_to_compressed(jac_to_affine(g_b), proof_out + 48);
  g1_to_compressed(jac_to_affine(g_c), proof_out + 144);

  const auto t1 = std::chrono::steady_clock::now();
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
  return BH_OK;
}

bh_status bh_prove(bh_ctx* ctx, const bh_params* params, const uint64_t* a, const uint64_t* b, const uint64_t* c,
                   size_t nc, const uint64_t* inputs, size_t ni, const uint64_t* aux, size_t na,
                   const uint64_t* a_aux_density, const uint64_t* b_input_density, const uint64_t* b_aux_density,
                   const uint64_t r[4], const uint64_t s[4], uint8_t proof_out[192]) {
  bh_witness* w = nullptr;
  bh_status st = bh_witness_upload(ctx, a, b, c, nc, inputs, ni, aux, na, a_aux_density, b_input_density,
                                   b_aux_density, &w);
  if (st) return st;
  st = bh_prove_witness(ctx, params, w, r, s, proof_out);
  bh_witness_free(w);
  return st;
}

bh_status bh_last_timings(const bh_ctx* ctx, double out[8]) {
  if (!ctx || !out) return BH_ERR_INVALID_ARGUMENT;
  memcpy(out, ctx->last_timings, sizeof ctx->last_timings);
  return BH_OK;
}

}  // extern "C"
