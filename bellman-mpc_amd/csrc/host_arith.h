// Host-side BLS12-381 arithmetic for the parts of create_proof that are
// O(1) per proof: combining the per-window bucket sums the GPU returns
// (multiexp.rs:244-249 Horner step), the proof assembly with r, s
// (prover.rs:315-349), affine normalisation and the zcash encodings used by
// Proof::write / Parameters::write (groth16/mod.rs:42-48, 260-290).
// 64-bit limbs, Montgomery R = 2^384 (Fp) / 2^256 (Fr) -- the bls12_381 layout.
#pragma once
#include <stdint.h>
#include <string.h>
#include "constants.h"

namespace bh {

typedef unsigned __int128 u128;

// ------------------------------------------------------------ generic Montgomery
template <int N>
struct MontCfg;
template <>
struct MontCfg<6> {
  static const uint64_t* p() { return hostc::FP_P; }
  static uint64_t inv() { return hostc::FP_INV; }
  static const uint64_t* r2() { return hostc::FP_R2; }
  static const uint64_t* one() { return hostc::FP_ONE; }
};
template <>
struct MontCfg<4> {
  static const uint64_t* p() { return hostc::FR_Q; }
  static uint64_t inv() { return hostc::FR_INV; }
  static const uint64_t* r2() { return hostc::FR_R2; }
  static const uint64_t* one() { return hostc::FR_ONE; }
};

template <int N>
struct F {
  uint64_t v[N];
  static F zero() { F r; memset(r.v, 0, sizeof r.v); return r; }
  static F one() { F r; memcpy(r.v, MontCfg<N>::one(), sizeof r.v); return r; }
  bool is_zero() const { uint64_t d = 0; for (int i = 0; i < N; i++) d |= v[i]; return d == 0; }
  bool operator==(const F& o) const { return memcmp(v, o.v, sizeof v) == 0; }
  bool operator!=(const F& o) const { return !(*this == o); }
};

template <int N>
static inline bool geq_p(const uint64_t* a) {
  const uint64_t* p = MontCfg<N>::p();
  for (int i = N - 1; i >= 0; i--) {
    if (a[i] != p[i]) return a[i] > p[i];
  }
  return true;
}
template <int N>
static inline void sub_p(uint64_t* a) {
  const uint64_t* p = MontCfg<N>::p();
  uint64_t b = 0;
  for (int i = 0; i < N; i++) {
    u128 t = (u128)a[i] - p[i] - b;
    a[i] = (uint64_t)t;
    b = (uint64_t)(t >> 64) & 1;
  }
}

template <int N>
static inline F<N> add(const F<N>& a, const F<N>& b) {
  F<N> r;
  uint64_t c = 0;
  for (int i = 0; i < N; i++) {
    u128 t = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)t;
    c = (uint64_t)(t >> 64);
  }
  if (c || geq_p<N>(r.v)) sub_p<N>(r.v);
  return r;
}
template <int N>
static inline F<N> sub(const F<N>& a, const F<N>& b) {
  F<N> r;
  uint64_t br = 0;
  for (int i = 0; i < N; i++) {
    u128 t = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  if (br) {
    const uint64_t* p = MontCfg<N>::p();
    uint64_t c = 0;
    for (int i = 0; i < N; i++) {
      u128 t = (u128)r.v[i] + p[i] + c;
      r.v[i] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
  }
  return r;
}
template <int N>
static inline F<N> neg(const F<N>& a) { return sub(F<N>::zero(), a); }

template <int N>
static inline F<N> mul(const F<N>& a, const F<N>& b) {  // CIOS
  const uint64_t* p = MontCfg<N>::p();
  const uint64_t inv = MontCfg<N>::inv();
  uint64_t t[N + 2] = {0};
  for (int i = 0; i < N; i++) {
    uint64_t c = 0;
    for (int j = 0; j < N; j++) {
      u128 s = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    u128 s = (u128)t[N] + c;
    t[N] = (uint64_t)s;
    t[N + 1] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * inv;
    s = (u128)m * p[0] + t[0];
    c = (uint64_t)(s >> 64);
    for (int j = 1; j < N; j++) {
      s = (u128)m * p[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
    s = (u128)t[N] + c;
    t[N - 1] = (uint64_t)s;
    t[N] = t[N + 1] + (uint64_t)(s >> 64);
  }
  F<N> r;
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  if (t[N] || geq_p<N>(r.v)) sub_p<N>(r.v);
  return r;
}
template <int N>
static inline F<N> sqr(const F<N>& a) { return mul(a, a); }

// raw little-endian integer (< p) -> Montgomery
template <int N>
static inline F<N> from_int(const uint64_t* x) {
  F<N> a, r2;
  memcpy(a.v, x, sizeof a.v);
  memcpy(r2.v, MontCfg<N>::r2(), sizeof r2.v);
  return mul(a, r2);
}
template <int N>
static inline void to_int(const F<N>& a, uint64_t* out) {
  F<N> one = F<N>::zero();
  one.v[0] = 1;
  F<N> r = mul(a, one);
  memcpy(out, r.v, sizeof r.v);
}
template <int N>
static inline F<N> pow_vartime(const F<N>& a, const uint64_t* e, int ewords) {
  F<N> r = F<N>::one();
  for (int i = ewords - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = sqr(r);
      if ((e[i] >> b) & 1) r = mul(r, a);
    }
  return r;
}
template <int N>
static inline F<N> inv(const F<N>& a) {  // Fermat
  uint64_t e[N];
  memcpy(e, MontCfg<N>::p(), sizeof e);
  // p - 2 (p odd, low limb >= 2)
  e[0] -= 2;
  return pow_vartime(a, e, N);
}

typedef F<6> Fp;
typedef F<4> Fr;

// ------------------------------------------------------------ Fp2
struct Fp2 {
  Fp c0, c1;
  static Fp2 zero() { return Fp2{Fp::zero(), Fp::zero()}; }
  static Fp2 one() { return Fp2{Fp::one(), Fp::zero()}; }
  bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  bool operator==(const Fp2& o) const { return c0 == o.c0 && c1 == o.c1; }
};
static inline Fp2 add(const Fp2& a, const Fp2& b) { return Fp2{add(a.c0, b.c0), add(a.c1, b.c1)}; }
static inline Fp2 sub(const Fp2& a, const Fp2& b) { return Fp2{sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
static inline Fp2 neg(const Fp2& a) { return Fp2{neg(a.c0), neg(a.c1)}; }
static inline Fp2 mul(const Fp2& a, const Fp2& b) {
  Fp t0 = mul(a.c0, b.c0), t1 = mul(a.c1, b.c1);
  Fp t2 = mul(add(a.c0, a.c1), add(b.c0, b.c1));
  return Fp2{sub(t0, t1), sub(sub(t2, t0), t1)};
}
static inline Fp2 sqr(const Fp2& a) { return mul(a, a); }
static inline Fp2 inv(const Fp2& a) {
  Fp t = inv(add(sqr(a.c0), sqr(a.c1)));
  return Fp2{mul(a.c0, t), neg(mul(a.c1, t))};
}

// ------------------------------------------------------------ curves (Jacobian)
template <class T>
struct Jac {
  T X, Y, Z;
};

template <class T>
struct CurveB;
template <>
struct CurveB<Fp> {
  static Fp b() { uint64_t four[6] = {4, 0, 0, 0, 0, 0}; return from_int<6>(four); }
};
template <>
struct CurveB<Fp2> {
  static Fp2 b() { uint64_t four[6] = {4, 0, 0, 0, 0, 0}; Fp f = from_int<6>(four); return Fp2{f, f}; }
};

template <class T>
static inline T tzero();
template <>
inline Fp tzero<Fp>() { return Fp::zero(); }
template <>
inline Fp2 tzero<Fp2>() { return Fp2::zero(); }
template <class T>
static inline T tone();
template <>
inline Fp tone<Fp>() { return Fp::one(); }
template <>
inline Fp2 tone<Fp2>() { return Fp2::one(); }

template <class T>
static inline Jac<T> jac_identity() { return Jac<T>{tone<T>(), tone<T>(), tzero<T>()}; }
template <class T>
static inline bool jac_is_identity(const Jac<T>& p) { return p.Z.is_zero(); }

template <class T>
static inline Jac<T> jac_dbl(const Jac<T>& p) {
  if (p.Z.is_zero() || p.Y.is_zero()) return jac_identity<T>();
  T A = sqr(p.X), B = sqr(p.Y), C = sqr(B);
  T D = sub(sqr(add(p.X, B)), add(A, C));
  D = add(D, D);
  T E = add(add(A, A), A);
  T Fv = sqr(E);
  Jac<T> r;
  r.X = sub(Fv, add(D, D));
  T C8 = add(C, C); C8 = add(C8, C8); C8 = add(C8, C8);
  r.Y = sub(mul(E, sub(D, r.X)), C8);
  T yz = mul(p.Y, p.Z);
  r.Z = add(yz, yz);
  return r;
}

template <class T>
static inline Jac<T> jac_add(const Jac<T>& p, const Jac<T>& q) {
  if (p.Z.is_zero()) return q;
  if (q.Z.is_zero()) return p;
  T Z1Z1 = sqr(p.Z), Z2Z2 = sqr(q.Z);
  T U1 = mul(p.X, Z2Z2), U2 = mul(q.X, Z1Z1);
  T S1 = mul(mul(p.Y, q.Z), Z2Z2), S2 = mul(mul(q.Y, p.Z), Z1Z1);
  if (U1 == U2) {
    if (S1 == S2) return jac_dbl(p);
    return jac_identity<T>();
  }
  T H = sub(U2, U1);
  T I = sqr(add(H, H));
  T J = mul(H, I);
  T r = sub(S2, S1);
  r = add(r, r);
  T V = mul(U1, I);
  Jac<T> o;
  o.X = sub(sub(sqr(r), J), add(V, V));
  T S1J = mul(S1, J);
  o.Y = sub(mul(r, sub(V, o.X)), add(S1J, S1J));
  o.Z = mul(sub(sqr(add(p.Z, q.Z)), add(Z1Z1, Z2Z2)), H);
  return o;
}

template <class T>
static inline Jac<T> jac_neg(const Jac<T>& p) { return Jac<T>{p.X, neg(p.Y), p.Z}; }

// scalar given as little-endian 64-bit words of its canonical value
template <class T>
static inline Jac<T> jac_mul(const Jac<T>& p, const uint64_t* k, int words) {
  Jac<T> acc = jac_identity<T>();
  for (int i = words - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      acc = jac_dbl(acc);
      if ((k[i] >> b) & 1) acc = jac_add(acc, p);
    }
  return acc;
}

template <class T>
struct AffinePt {
  T x, y;
  bool infinity;
};

template <class T>
static inline AffinePt<T> jac_to_affine(const Jac<T>& p) {
  AffinePt<T> a;
  if (p.Z.is_zero()) {
    a.x = tzero<T>(); a.y = tzero<T>(); a.infinity = true;
    return a;
  }
  T zi = inv(p.Z), zi2 = sqr(zi);
  a.x = mul(p.X, zi2);
  a.y = mul(p.Y, mul(zi2, zi));
  a.infinity = false;
  return a;
}
template <class T>
static inline Jac<T> jac_from_affine(const AffinePt<T>& a) {
  if (a.infinity) return jac_identity<T>();
  return Jac<T>{a.x, a.y, tone<T>()};
}

// XYZZ (x = X/ZZ, y = Y/ZZZ) -> Jacobian without inversion: with s = ZZ*ZZZ,
// X' = x s^2 = X*ZZ*ZZZ^2, Y' = y s^3 = Y*ZZ^3*ZZZ^2, Z' = s.
template <class T>
static inline Jac<T> xyzz_to_jac(const T& X, const T& Y, const T& ZZ, const T& ZZZ) {
  if (ZZ.is_zero()) return jac_identity<T>();
  T zzz2 = sqr(ZZZ);
  Jac<T> r;
  r.X = mul(mul(X, ZZ), zzz2);
  T zz3 = mul(sqr(ZZ), ZZ);
  r.Y = mul(mul(Y, zz3), zzz2);
  r.Z = mul(ZZ, ZZZ);
  return r;
}

// ------------------------------------------------------------ conversions / encodings
// Device packed words (12 x u32 per Fp, value = x * 2^406 mod p, canonical) -> host Montgomery
static inline Fp fp_from_dev_words(const uint32_t* w) {
  Fp a;
  for (int i = 0; i < 6; i++) a.v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  // a = x*2^406 (raw); host Montgomery of x = a * 2^-22 = mont_mul(a, 2^362 mod p)
  static Fp K = [] {
    uint64_t two[6] = {2, 0, 0, 0, 0, 0};
    Fp t = from_int<6>(two);
    uint64_t e[1] = {362};
    Fp k = pow_vartime(t, e, 1);  // Montgomery(2^362)
    uint64_t raw[6];
    to_int(k, raw);               // canonical 2^362 mod p
    Fp out; memcpy(out.v, raw, sizeof raw);
    return out;
  }();
  return mul(a, K);
}
// Device packed words of a field whose device Montgomery radix is 2^rlog (G1's form, R = 2^(N*BITS)
// of its limb configuration: 2^390 for the balanced 13 x 30-bit digits) -> host Montgomery:
// a * 2^-(rlog - 384) = mont_mul(a, 2^(768 - rlog) mod p)
template <int RLOG>
static inline Fp fp_from_dev_words_r(const uint32_t* w) {
  Fp a;
  for (int i = 0; i < 6; i++) a.v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  static Fp K = [] {
    uint64_t two[6] = {2, 0, 0, 0, 0, 0};
    Fp t = from_int<6>(two);
    uint64_t e[1] = {768 - RLOG};
    Fp k = pow_vartime(t, e, 1);  // Montgomery(2^(768 - RLOG))
    uint64_t raw[6];
    to_int(k, raw);               // canonical
    Fp out; memcpy(out.v, raw, sizeof raw);
    return out;
  }();
  return mul(a, K);
}
// host Montgomery -> device packed words (x * 2^406 mod p)
static inline void fp_to_dev_words(const Fp& x, uint32_t* w) {
  static Fp K = [] {
    uint64_t two[6] = {2, 0, 0, 0, 0, 0};
    Fp t = from_int<6>(two);
    uint64_t e[1] = {406};
    Fp k = pow_vartime(t, e, 1);
    uint64_t raw[6];
    to_int(k, raw);
    Fp out; memcpy(out.v, raw, sizeof raw);
    return out;
  }();
  Fp d = mul(x, K);  // x*2^384 * 2^406 * 2^-384 = x*2^406 (as raw value)
  for (int i = 0; i < 6; i++) { w[2 * i] = (uint32_t)d.v[i]; w[2 * i + 1] = (uint32_t)(d.v[i] >> 32); }
}

static inline void fp_to_be(const Fp& a, uint8_t* out48) {
  uint64_t raw[6];
  to_int(a, raw);
  for (int i = 0; i < 6; i++)
    for (int b = 0; b < 8; b++) out48[47 - (8 * i + b)] = (uint8_t)(raw[i] >> (8 * b));
}
// returns false if >= p
static inline bool fp_from_be(const uint8_t* in48, Fp* out, uint8_t flag_mask = 0) {
  uint64_t raw[6] = {0};
  for (int i = 0; i < 48; i++) {
    uint8_t byte = in48[i];
    if (i == 0) byte &= (uint8_t)~flag_mask;
    raw[(47 - i) / 8] |= (uint64_t)byte << (8 * ((47 - i) % 8));
  }
  if (geq_p<6>(raw)) return false;
  *out = from_int<6>(raw);
  return true;
}
static inline bool fp_lex_largest(const Fp& a) {
  // a > (p-1)/2  on canonical values
  uint64_t raw[6], half[6];
  to_int(a, raw);
  uint64_t c = 0;
  for (int i = 5; i >= 0; i--) {
    half[i] = (hostc::FP_P[i] >> 1) | c;
    c = hostc::FP_P[i] << 63;
  }
  for (int i = 5; i >= 0; i--)
    if (raw[i] != half[i]) return raw[i] > half[i];
  return false;
}

static inline void g1_to_compressed(const AffinePt<Fp>& a, uint8_t* out48) {
  if (a.infinity) { memset(out48, 0, 48); out48[0] = 0xC0; return; }
  fp_to_be(a.x, out48);
  out48[0] |= 0x80;
  if (fp_lex_largest(a.y)) out48[0] |= 0x20;
}
static inline void g1_to_uncompressed(const AffinePt<Fp>& a, uint8_t* out96) {
  if (a.infinity) { memset(out96, 0, 96); out96[0] = 0x40; return; }
  fp_to_be(a.x, out96);
  fp_to_be(a.y, out96 + 48);
}
static inline void g2_to_compressed(const AffinePt<Fp2>& a, uint8_t* out96) {
  if (a.infinity) { memset(out96, 0, 96); out96[0] = 0xC0; return; }
  fp_to_be(a.x.c1, out96);
  fp_to_be(a.x.c0, out96 + 48);
  out96[0] |= 0x80;
  bool lex = fp_lex_largest(a.y.c1) || (a.y.c1.is_zero() && fp_lex_largest(a.y.c0));
  if (lex) out96[0] |= 0x20;
}
static inline void g2_to_uncompressed(const AffinePt<Fp2>& a, uint8_t* out192) {
  if (a.infinity) { memset(out192, 0, 192); out192[0] = 0x40; return; }
  fp_to_be(a.x.c1, out192);
  fp_to_be(a.x.c0, out192 + 48);
  fp_to_be(a.y.c1, out192 + 96);
  fp_to_be(a.y.c0, out192 + 144);
}

template <class T>
static inline bool on_curve(const AffinePt<T>& a) {
  if (a.infinity) return true;
  return sqr(a.y) == add(mul(sqr(a.x), a.x), CurveB<T>::b());
}

// [r]P == O (torsion-freeness, part of G1Affine/G2Affine::from_uncompressed)
template <class T>
static inline bool in_subgroup(const AffinePt<T>& p) {
  static const uint64_t R[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                                0x73eda753299d7d48ull};
  return p.infinity || jac_is_identity(jac_mul(jac_from_affine(p), R, 4));
}

// G1Affine::from_uncompressed_unchecked semantics (+ on-curve check when check_curve,
// + subgroup check when check_subgroup); returns 0 ok, -1 invalid encoding, -2 not on
// curve, -3 not in the subgroup
static inline int g1_from_uncompressed(const uint8_t* in96, AffinePt<Fp>* out, bool check_curve,
                                       bool check_subgroup = false) {
  uint8_t flags = in96[0] >> 5;
  if (flags & 0x4) return -1;  // compression flag set
  if (flags & 0x1) return -1;  // sort flag set
  if (flags & 0x2) {           // infinity
    for (int i = 0; i < 96; i++) {
      uint8_t b = (i == 0) ? (in96[0] & 0x1F) : in96[i];
      if (b) return -1;
    }
    out->infinity = true; out->x = Fp::zero(); out->y = Fp::zero();
    return 0;
  }
  if (!fp_from_be(in96, &out->x, 0xE0)) return -1;
  if (!fp_from_be(in96 + 48, &out->y)) return -1;
  out->infinity = false;
  if (check_curve && !on_curve(*out)) return -2;
  if (check_subgroup && !in_subgroup(*out)) return -3;
  return 0;
}
static inline int g2_from_uncompressed(const uint8_t* in192, AffinePt<Fp2>* out, bool check_curve,
                                       bool check_subgroup = false) {
  uint8_t flags = in192[0] >> 5;
  if (flags & 0x4) return -1;
  if (flags & 0x1) return -1;
  if (flags & 0x2) {
    for (int i = 0; i < 192; i++) {
      uint8_t b = (i == 0) ? (in192[0] & 0x1F) : in192[i];
      if (b) return -1;
    }
    out->infinity = true; out->x = Fp2::zero(); out->y = Fp2::zero();
    return 0;
  }
  if (!fp_from_be(in192, &out->x.c1, 0xE0)) return -1;
  if (!fp_from_be(in192 + 48, &out->x.c0)) return -1;
  if (!fp_from_be(in192 + 96, &out->y.c1)) return -1;
  if (!fp_from_be(in192 + 144, &out->y.c0)) return -1;
  out->infinity = false;
  if (check_curve && !on_curve(*out)) return -2;
  if (check_subgroup && !in_subgroup(*out)) return -3;
  return 0;
}

// ------------------------------------------------------------ Fr helpers
// canonical little-endian u64x4 -> Montgomery
static inline Fr fr_from_canonical(const uint64_t* x) { return from_int<4>(x); }
static inline void fr_to_canonical(const Fr& a, uint64_t* out) { to_int(a, out); }

}  // namespace bh
