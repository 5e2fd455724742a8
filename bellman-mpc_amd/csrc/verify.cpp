// Groth16 verification on the host: verify_proof (verifier.rs:11-62) and the batch verifier
// (verifier/batch.rs:95-169), over a BLS12-381 optimal-ate pairing written from its published
// definition (the reference's pairing lives in the external crate bls12_381 0.6.0):
//   * tower Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u (Fp6 = Fp2[v]/(v^3 - xi), v = w^2);
//   * G2 on the M-type sextic twist y^2 = x^3 + 4 xi, untwisted by (x, y) -> (x / w^2, y / w^3);
//   * Miller loop over |x|, x = -0xd201000000010000, affine line functions evaluated at P and
//     scaled by w^3 (an Fp4 factor, killed by the final exponentiation), vertical lines dropped;
//   * final exponentiation f^((p^12 - 1) / r) by square-and-multiply.
// The sign of x only inverts every pairing value, so the product-equals-one checks below (the
// form both reference verifiers use) are unaffected.  Proofs are decoded like Proof::read
// (groth16/mod.rs:50-103: compressed, torsion-checked, identity rejected), verifying keys like
// VerifyingKey::read (mod.rs:174-222).  Host-only code: no device is needed.
#include <string.h>

#include <vector>

#include "api_internal.h"

using namespace bh;

namespace {

// ---------------------------------------------------------------- Fp12 = Fp2[w]/(w^6 - xi)
struct Fp12 {
  Fp2 c[6];
};

inline Fp2 mul_xi(const Fp2& a) {  // (a0 + a1 u)(1 + u), u^2 = -1
  return Fp2{sub(a.c0, a.c1), add(a.c0, a.c1)};
}

Fp12 f12_one() {
  Fp12 r;
  r.c[0] = Fp2::one();
  for (int i = 1; i < 6; i++) r.c[i] = Fp2::zero();
  return r;
}

bool f12_is_one(const Fp12& a) {
  if (!(a.c[0] == Fp2::one())) return false;
  for (int i = 1; i < 6; i++)
    if (!(a.c[i] == Fp2::zero())) return false;
  return true;
}

Fp12 f12_mul(const Fp12& a, const Fp12& b) {
  Fp2 t[11];
  for (auto& x : t) x = Fp2::zero();
  for (int i = 0; i < 6; i++) {
    if (a.c[i] == Fp2::zero()) continue;
    for (int j = 0; j < 6; j++) {
      if (b.c[j] == Fp2::zero()) continue;
      t[i + j] = add(t[i + j], mul(a.c[i], b.c[j]));
    }
  }
  Fp12 r;
  for (int k = 0; k < 5; k++) r.c[k] = add(t[k], mul_xi(t[k + 6]));
  r.c[5] = t[5];
  return r;
}

// (p^12 - 1) / r, little-endian 64-bit words (4314 bits), computed exactly (p, r of BLS12-381)
const uint64_t FINAL_EXP[68] = {
    0xc0bcb9b55df57510ull, 0x25f98630e68bfb24ull, 0x4406fbc8fbd5f489ull, 0x8e2f8491d12191a0ull,
    0x3e9d71650a6f8069ull, 0x226c2f011d4cab80ull, 0x67f67c4717489119ull, 0xaf3f881bd88592d7ull,
    0x1a67e49eeed2161dull, 0xe5b78c7869aeb218ull, 0xf6539314043f7bbcull, 0x73f62537f2701aaeull,
    0xaff1c910e9622d2aull, 0x6283313492caa9d4ull, 0x2e2f3ec2bea83d19ull, 0xa4c7e79fb02faa73ull,
    0x6c49637fd7961be1ull, 0x08e88adce8817745ull, 0x35de3f7a36399917ull, 0x9c1d9f7c31759c36ull,
    0xfa9e13c24ea820b0ull, 0x3fc56947a403577dull, 0xa4c1b6dcfc5cceb7ull, 0x1bbd81367066bca6ull,
    0x0418a3ef0bc62775ull, 0x49bf9b71a9f9e010ull, 0x511291097db60b17ull, 0x498345c6e5308f1cull,
    0x6d8823b19dadd7c2ull, 0x92004cedd556952cull, 0x4c6bec3ec03ef195ull, 0x0a1fad20044ce6adull,
    0xc55d3109cd15948dull, 0x334f46c02c3f0bd0ull, 0x3b5a62eb34c05739ull, 0x724538411d1676a5ull,
    0x127a1b5ad0463434ull, 0x61a474c5c85b0129ull, 0x8dfc8e2886ef965eull, 0x96532fef459f1243ull,
    0x40ee7169cdc10412ull, 0x9c40a68eb74bb22aull, 0x25118790f4684d0bull, 0x596bc293c8d4c01full,
    0x1064837f27611212ull, 0x077ffb10bf24dde4ull, 0xc49f570bcd2b01f3ull, 0x1a0c5bf24c374693ull,
    0x350da5359bc73ab6ull, 0xd2670d93e4d7acddull, 0xd39099b86e1ab656ull, 0x19328148978e2b0dull,
    0xb113f414386b0e88ull, 0x07a0dce2630d9aa4ull, 0xa927e7bb93753318ull, 0xe347aa68ad49466full,
    0x1c0ad0d6106feaf4ull, 0xc872ee83ff3a0f0full, 0x074e43b9a660835cull, 0xc0aadff5e9cfee9aull,
    0x30698e8cc7deada9ull, 0xd1073776ab353f2cull, 0x17848517badc3a43ull, 0x7363baa13f8d14a9ull,
    0xd4977b3f7d4507d0ull, 0x496a1c0a89ee0193ull, 0xdcc825b7e1bda9c0ull, 0x0000000002ee1db5ull,
};

Fp12 final_exponentiation(const Fp12& f) {
  Fp12 r = f12_one();
  bool started = false;
  for (int i = 67; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      if (started) r = f12_mul(r, r);
      if ((FINAL_EXP[i] >> b) & 1) {
        r = started ? f12_mul(r, f) : f;
        started = true;
      }
    }
  return r;
}

// ---------------------------------------------------------------- Miller loop
constexpr uint64_t X_ABS = 0xd201000000010000ull;

// line through T with slope lam (twist coordinates) at P, times w^3:
// (lam*xt - yt) - lam*xp w^2 + yp w^3
Fp12 line(const Fp2& lam, const Fp2& xt, const Fp2& yt, const AffinePt<Fp>& p) {
  Fp12 l;
  for (auto& x : l.c) x = Fp2::zero();
  l.c[0] = sub(mul(lam, xt), yt);
  l.c[2] = neg(Fp2{mul(lam.c0, p.x), mul(lam.c1, p.x)});
  l.c[3] = Fp2{p.y, Fp::zero()};
  return l;
}

struct Pair {
  AffinePt<Fp> p;
  AffinePt<Fp2> q;
};

Fp12 multi_miller_loop(const std::vector<Pair>& pairs) {
  std::vector<Pair> terms;
  for (const Pair& t : pairs)
    if (!t.p.infinity && !t.q.infinity) terms.push_back(t);
  std::vector<Fp2> xt(terms.size()), yt(terms.size());
  for (size_t i = 0; i < terms.size(); i++) { xt[i] = terms[i].q.x; yt[i] = terms[i].q.y; }
  const Fp2 three = add(add(Fp2::one(), Fp2::one()), Fp2::one());
  Fp12 f = f12_one();
  for (int bit = 62; bit >= 0; bit--) {  // below the leading one of |x|
    f = f12_mul(f, f);
    for (size_t i = 0; i < terms.size(); i++) {  // doubling step
      const Fp2 lam = mul(mul(three, sqr(xt[i])), inv(add(yt[i], yt[i])));
      f = f12_mul(f, line(lam, xt[i], yt[i], terms[i].p));
      const Fp2 x3 = sub(sqr(lam), add(xt[i], xt[i]));
      yt[i] = sub(mul(lam, sub(xt[i], x3)), yt[i]);
      xt[i] = x3;
    }
    if ((X_ABS >> bit) & 1) {
      for (size_t i = 0; i < terms.size(); i++) {  // addition step (T + Q)
        const Fp2 &xq = terms[i].q.x, &yq = terms[i].q.y;
        const Fp2 lam = mul(sub(yq, yt[i]), inv(sub(xq, xt[i])));
        f = f12_mul(f, line(lam, xt[i], yt[i], terms[i].p));
        const Fp2 x3 = sub(sub(sqr(lam), xt[i]), xq);
        yt[i] = sub(mul(lam, sub(xt[i], x3)), yt[i]);
        xt[i] = x3;
      }
    }
  }
  return f;
}

bool pairing_product_is_one(const std::vector<Pair>& pairs) {
  return f12_is_one(final_exponentiation(multi_miller_loop(pairs)));
}

// ---------------------------------------------------------------- decompression
// big-integer exponents derived from p: (p + 1) / 4, (p - 3) / 4, (p - 1) / 2
struct PExps {
  uint64_t p1_4[6], p3_4[6], p1_2[6];
  PExps() {
    const uint64_t* P = hostc::FP_P;
    auto shr = [](const uint64_t* x, int s, uint64_t* out) {
      for (int i = 0; i < 6; i++) out[i] = (x[i] >> s) | (i + 1 < 6 ? x[i + 1] << (64 - s) : 0);
    };
    uint64_t t[6];
    memcpy(t, P, sizeof t);
    t[0] += 1;  // p is odd: no carry
    shr(t, 2, p1_4);
    memcpy(t, P, sizeof t);
    t[0] -= 3;  // p = 3 mod 4, low word >= 3: no borrow
    shr(t, 2, p3_4);
    memcpy(t, P, sizeof t);
    t[0] -= 1;
    shr(t, 1, p1_2);
  }
};
const PExps& pexps() {
  static const PExps e;
  return e;
}

Fp2 fp2_pow(const Fp2& a, const uint64_t* e, int words) {
  Fp2 r = Fp2::one();
  for (int i = words - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = sqr(r);
      if ((e[i] >> b) & 1) r = mul(r, a);
    }
  return r;
}

bool fp_sqrt(const Fp& a, Fp* out) {  // p = 3 mod 4
  const Fp y = pow_vartime(a, pexps().p1_4, 6);
  if (!(sqr(y) == a)) return false;
  *out = y;
  return true;
}

bool fp2_sqrt(const Fp2& a, Fp2* out) {  // p = 3 mod 4 algorithm over Fp2 = Fp[u]/(u^2 + 1)
  if (a == Fp2::zero()) { *out = a; return true; }
  const Fp2 a1 = fp2_pow(a, pexps().p3_4, 6);
  const Fp2 alpha = mul(sqr(a1), a);
  const Fp2 x0 = mul(a1, a);
  Fp2 x;
  if (alpha == neg(Fp2::one())) {
    x = Fp2{neg(x0.c1), x0.c0};  // u * x0
  } else {
    x = mul(fp2_pow(add(Fp2::one(), alpha), pexps().p1_2, 6), x0);
  }
  if (!(sqr(x) == a)) return false;
  *out = x;
  return true;
}

// G1Affine::from_compressed + Proof::read's identity rejection
bh_status g1_from_compressed(const uint8_t* in, AffinePt<Fp>* out) {
  const uint8_t flags = in[0] >> 5;
  if (!(flags & 0x4)) return BH_ERR_INVALID_ENCODING;  // compression flag
  if (flags & 0x2) return BH_ERR_INVALID_ENCODING;     // the identity ("point at infinity")
  Fp x;
  if (!fp_from_be(in, &x, 0xE0)) return BH_ERR_INVALID_ENCODING;
  Fp y;
  if (!fp_sqrt(add(mul(sqr(x), x), CurveB<Fp>::b()), &y)) return BH_ERR_INVALID_ENCODING;
  if (fp_lex_largest(y) != ((flags & 0x1) != 0)) y = neg(y);
  out->x = x; out->y = y; out->infinity = false;
  if (!in_subgroup(*out)) return BH_ERR_NOT_IN_SUBGROUP;
  return BH_OK;
}

bh_status g2_from_compressed(const uint8_t* in, AffinePt<Fp2>* out) {
  const uint8_t flags = in[0] >> 5;
  if (!(flags & 0x4)) return BH_ERR_INVALID_ENCODING;
  if (flags & 0x2) return BH_ERR_INVALID_ENCODING;
  Fp2 x;
  if (!fp_from_be(in, &x.c1, 0xE0) || !fp_from_be(in + 48, &x.c0)) return BH_ERR_INVALID_ENCODING;
  Fp2 y;
  if (!fp2_sqrt(add(mul(sqr(x), x), CurveB<Fp2>::b()), &y)) return BH_ERR_INVALID_ENCODING;
  const bool lex = fp_lex_largest(y.c1) || (y.c1.is_zero() && fp_lex_largest(y.c0));
  if (lex != ((flags & 0x1) != 0)) y = neg(y);
  out->x = x; out->y = y; out->infinity = false;
  if (!in_subgroup(*out)) return BH_ERR_NOT_IN_SUBGROUP;
  return BH_OK;
}

struct Proof {
  AffinePt<Fp> a, c;
  AffinePt<Fp2> b;
};

bh_status proof_read(const uint8_t* in, Proof* p) {  // Proof::read, groth16/mod.rs:50-103
  bh_status s;
  if ((s = g1_from_compressed(in, &p->a))) return s;
  if ((s = g2_from_compressed(in + 48, &p->b))) return s;
  return g1_from_compressed(in + 144, &p->c);
}

struct Vk {
  AffinePt<Fp> alpha_g1, beta_g1, delta_g1;
  AffinePt<Fp2> beta_g2, gamma_g2, delta_g2;
  std::vector<AffinePt<Fp>> ic;
};

bh_status vk_read(const uint8_t* in, size_t len, Vk* vk) {  // VerifyingKey::read, mod.rs:174-222
  size_t o = 0;
  auto g1 = [&](AffinePt<Fp>* out, bool no_identity) -> bh_status {
    if (len - o < 96) return BH_ERR_UNEXPECTED_EOF;
    const int r = g1_from_uncompressed(in + o, out, true, true);
    o += 96;
    if (r == -3) return BH_ERR_NOT_IN_SUBGROUP;
    if (r) return BH_ERR_INVALID_ENCODING;
    return (no_identity && out->infinity) ? BH_ERR_INVALID_ENCODING : BH_OK;
  };
  auto g2 = [&](AffinePt<Fp2>* out) -> bh_status {
    if (len - o < 192) return BH_ERR_UNEXPECTED_EOF;
    const int r = g2_from_uncompressed(in + o, out, true, true);
    o += 192;
    if (r == -3) return BH_ERR_NOT_IN_SUBGROUP;
    return r ? BH_ERR_INVALID_ENCODING : BH_OK;
  };
  bh_status s;
  if ((s = g1(&vk->alpha_g1, false)) || (s = g1(&vk->beta_g1, false)) || (s = g2(&vk->beta_g2)) ||
      (s = g2(&vk->gamma_g2)) || (s = g1(&vk->delta_g1, false)) || (s = g2(&vk->delta_g2)))
    return s;
  if (len - o < 4) return BH_ERR_UNEXPECTED_EOF;
  const uint32_t n = ((uint32_t)in[o] << 24) | ((uint32_t)in[o + 1] << 16) | ((uint32_t)in[o + 2] << 8) | in[o + 3];
  o += 4;
  if ((size_t)n > (len - o) / 96) return BH_ERR_UNEXPECTED_EOF;
  vk->ic.resize(n);
  for (uint32_t i = 0; i < n; i++)
    if ((s = g1(&vk->ic[i], true))) return s;
  return BH_OK;
}

AffinePt<Fp> neg_pt(AffinePt<Fp> p) { if (!p.infinity) p.y = neg(p.y); return p; }
AffinePt<Fp2> neg_pt(AffinePt<Fp2> q) { if (!q.infinity) q.y = neg(q.y); return q; }

// canonical public inputs (little-endian u64 x 4 each), reduced mod r like Fr::from_repr's
// callers would have to: a word >= r is an invalid Fr
bool canonical_ok(const uint64_t* x) { return !geq_p<4>(x); }

}  // namespace

extern "C" {

bh_status bh_verify_proof(const uint8_t* vk_bytes, size_t vk_len, const uint8_t* proof, const uint64_t* inputs,
                          size_t num_inputs, int* valid) {
  if (!vk_bytes || !proof || !valid || (num_inputs && !inputs)) return BH_ERR_INVALID_ARGUMENT;
  *valid = 0;
  Vk vk;
  bh_status s = vk_read(vk_bytes, vk_len, &vk);
  if (s) return s;
  if (num_inputs + 1 != vk.ic.size()) return BH_ERR_INVALID_ARGUMENT;  // VerificationError::InvalidVerifyingKey
  Proof pf;
  if ((s = proof_read(proof, &pf))) return s;
  // acc = ic[0] + sum_i inputs[i] * ic[i+1]  (verifier.rs:33-40)
  Jac<Fp> acc = jac_from_affine(vk.ic[0]);
  for (size_t i = 0; i < num_inputs; i++) {
    if (!canonical_ok(inputs + 4 * i)) return BH_ERR_INVALID_ARGUMENT;
    acc = jac_add(acc, jac_mul(jac_from_affine(vk.ic[i + 1]), inputs + 4 * i, 4));
  }
  // e(A, B) e(acc, -gamma) e(C, -delta) == e(alpha, beta)  (verifier.rs:42-57), as one product
  // with e(-alpha, beta) so that a single final exponentiation decides
  const std::vector<Pair> pairs = {{pf.a, pf.b},
                                   {jac_to_affine(acc), neg_pt(vk.gamma_g2)},
                                   {pf.c, neg_pt(vk.delta_g2)},
                                   {neg_pt(vk.alpha_g1), vk.beta_g2}};
  *valid = pairing_product_is_one(pairs) ? 1 : 0;
  return BH_OK;
}

bh_status bh_verify_batch(const uint8_t* vk_bytes, size_t vk_len, const uint8_t* proofs, const uint64_t* inputs,
                          size_t num_inputs, size_t k, const uint64_t* z, int* valid) {
  if (!vk_bytes || !valid || (k && (!proofs || !z)) || (k && num_inputs && !inputs)) return BH_ERR_INVALID_ARGUMENT;
  *valid = 0;
  Vk vk;
  bh_status s = vk_read(vk_bytes, vk_len, &vk);
  if (s) return s;
  if (num_inputs + 1 != vk.ic.size()) return BH_ERR_INVALID_ARGUMENT;
  // batch.rs:110-165: per item a random nonzero z; Miller-loop terms (z A_i, -B_i), and the
  // accumulated (acc_Delta, delta), (Psi, gamma), (acc_Y alpha, beta); all valid iff the
  // product's final exponentiation is one
  std::vector<Pair> ml;
  std::vector<Fr> acc_gamma(vk.ic.size(), Fr::zero());
  Jac<Fp> acc_delta = jac_identity<Fp>();
  Fr acc_y = Fr::zero();
  for (size_t j = 0; j < k; j++) {
    const uint64_t* zj = z + 4 * j;
    if (!canonical_ok(zj)) return BH_ERR_INVALID_ARGUMENT;
    const Fr zf = fr_from_canonical(zj);
    if (zf.is_zero()) return BH_ERR_INVALID_ARGUMENT;  // the spec requires z != 0
    Proof pf;
    if ((s = proof_read(proofs + 192 * j, &pf))) return s;
    ml.push_back({jac_to_affine(jac_mul(jac_from_affine(pf.a), zj, 4)), neg_pt(pf.b)});
    acc_gamma[0] = add(acc_gamma[0], zf);
    for (size_t i = 0; i < num_inputs; i++) {
      const uint64_t* ai = inputs + 4 * (j * num_inputs + i);
      if (!canonical_ok(ai)) return BH_ERR_INVALID_ARGUMENT;
      acc_gamma[i + 1] = add(acc_gamma[i + 1], mul(zf, fr_from_canonical(ai)));
    }
    acc_delta = jac_add(acc_delta, jac_mul(jac_from_affine(pf.c), zj, 4));
    acc_y = add(acc_y, zf);
  }
  ml.push_back({jac_to_affine(acc_delta), vk.delta_g2});
  Jac<Fp> psi = jac_identity<Fp>();
  for (size_t i = 0; i < vk.ic.size(); i++) {
    uint64_t w[4];
    fr_to_canonical(acc_gamma[i], w);
    psi = jac_add(psi, jac_mul(jac_from_affine(vk.ic[i]), w, 4));
  }
  ml.push_back({jac_to_affine(psi), vk.gamma_g2});
  uint64_t yw[4];
  fr_to_canonical(acc_y, yw);
  ml.push_back({jac_to_affine(jac_mul(jac_from_affine(vk.alpha_g1), yw, 4)), vk.beta_g2});
  *valid = pairing_product_is_one(ml) ? 1 : 0;
  return BH_OK;
}

}  // extern "C"
