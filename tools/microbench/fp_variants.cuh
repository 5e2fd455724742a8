// Fp representations tried for G1 in round 3 and measured against the library's 14 x 29-bit form
// (tools/microbench/fp30bench.hip): 13 x 30-bit limbs with separated
// product / reduction scans, and 13 balanced (signed) 30-bit digits with one interleaved scan.
// Both are exact (fp30bench cross-checks them word for word against the library) but neither
// is faster inside the prover's kernels, so the library keeps 14 x 29 bits.
#pragma once
#include "../../bellman-mpc_amd/csrc/field.cuh"
#include "fp30_constants.h"

template <> struct Packed<Fp30Cfg> { static constexpr int W = 12; };

// ---- Separated scans (configs with C::SEPARATED: 13 limbs of 30 bits for G1's Fp).  A column of
// 30-bit limb products holds up to 13 terms < 2^60 (< 2^63.7), so the product and its Montgomery
// reduction cannot share one 64-bit column accumulator as the 29-bit FIPS form does; they run as
// two scans instead: t = a*b normalised to 2N limbs, then t + m*p column by column (t_k < 2^31
// plus at most 13 terms m_i p_j).  13^2 + 13^2 = 338 v_mad_u64_u32 per product against 392 for
// 14 x 29 bits, for one more normalisation (an and + shift per column).
template <class C>
BH_DEV Fe<C> fe_redc_sep(const uint32_t (&t)[2 * C::N]) {
  constexpr int N = C::N;
  Fe<C> r;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    acc += t[k];
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) acc += (uint64_t)m[i] * C::P[k - i];
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      acc += (uint64_t)m[k] * C::P[0];
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc + t[2 * N - 1];
  return r;
}

template <class C>
BH_DEV Fe<C> fe_mul_sep(const Fe<C>& a, const Fe<C>& b) {
  constexpr int N = C::N;
  static_assert(N * ((1ull << (2 * C::BITS)) >> 32) < (1ull << 32), "a product column must fit 64 bits");
  uint32_t t[2 * N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) acc += (uint64_t)a.v[i] * b.v[k - i];
    t[k] = (uint32_t)acc & C::MASK;
    acc >>= C::BITS;
  }
  t[2 * N - 1] = (uint32_t)acc;
  return fe_redc_sep<C>(t);
}

// (a*b + c*d) R^-1: the two product scans side by side (a column of both would overflow), their
// limbs summed (< 2^31) into one reduction
template <class C>
BH_DEV Fe<C> fe_mul2_sep(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d) {
  constexpr int N = C::N;
  uint32_t t[2 * N];
  uint64_t acc = 0, acd = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acd += (uint64_t)c.v[i] * d.v[k - i];
    }
    t[k] = ((uint32_t)acc & C::MASK) + ((uint32_t)acd & C::MASK);
    acc >>= C::BITS;
    acd >>= C::BITS;
  }
  t[2 * N - 1] = (uint32_t)acc + (uint32_t)acd;
  return fe_redc_sep<C>(t);
}

// square: cross products once against 2a (limbs < 2^31: at most 6 cross terms < 2^61 and one
// square < 2^60 per column)
template <class C>
BH_DEV Fe<C> fe_sqr_sep(const Fe<C>& a) {
  constexpr int N = C::N;
  uint32_t t[2 * N], a2[N];
#pragma unroll
  for (int i = 0; i < N; i++) a2[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      const int j = k - i;
      if (i < j) acc += (uint64_t)a.v[i] * a2[j];
      else if (i == j) acc += (uint64_t)a.v[i] * a.v[i];
    }
    t[k] = (uint32_t)acc & C::MASK;
    acc >>= C::BITS;
  }
  t[2 * N - 1] = (uint32_t)acc;
  return fe_redc_sep<C>(t);
}


template <class C>
struct FpSepOps : FpOpsT<C> {  // FpOpsT with the separated-scan products
  using T = Fe<C>;
  static BH_DEV T mul(const T& a, const T& b) { return fe_mul_sep<C>(a, b); }
  static BH_DEV T sqr(const T& a) { return fe_sqr_sep<C>(a); }
  template <uint32_t K> static BH_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return fe_mul2_sep<C>(a, b, fe_neg<C, K>(c), d);
  }
};
using Fp30Ops = FpSepOps<Fp30Cfg>;

// ---------------------------------------------------------------- balanced-digit Fp (G1)
// Fp in 13 signed digits of 30 bits, each in [-2^29, 2^29) (Fp30sCfg, R = 2^390), values kept as
// signed integers of small magnitude (every product ends in (-p/2, 0.6p); sums of a few stay far
// below 128p).  Digit products are at most 2^58 in magnitude, so one signed 64-bit column
// accumulator takes a product column AND its Montgomery reduction (at most 27 terms, < 2^62.8):
// the interleaved (FIPS) scan of the 29-bit form with 13^2 + 13^2 = 338 v_mad_i64_i32 per product
// instead of 392, and no K*p offsets on subtraction (values may be negative).  Output digits and
// the m_k are sign-extended 30-bit fields (v_bfe_i32).
template <class C>
struct FeS {
  int32_t v[C::N];
};

template <class C>
BH_DEV int32_t sext_digit(uint32_t x) {
  return __builtin_amdgcn_sbfe((int32_t)x, 0, C::BITS);
}

template <class C>
BH_DEV FeS<C> fes_zero() {
  FeS<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = 0;
  return r;
}

template <class C>
BH_DEV FeS<C> fes_one() {
  FeS<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = C::ONE[i];
  return r;
}

template <class C>
BH_DEV FeS<C> fes_mul(const FeS<C>& a, const FeS<C>& b) {
  constexpr int N = C::N;
  FeS<C> r;
  int32_t m[N];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) acc += (int64_t)a.v[i] * b.v[k - i];
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) acc += (int64_t)m[i] * C::P[k - i];
    if (k < N) {
      m[k] = sext_digit<C>((uint32_t)acc * C::INV);
      acc += (int64_t)m[k] * C::P[0];  // the low BITS bits are now zero
    } else {
      const int32_t d = sext_digit<C>((uint32_t)acc);
      r.v[k - N] = d;
      acc -= d;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (int32_t)acc;
  return r;
}

// a^2: cross products once against 2a (|2a_i| <= 2^30: at most 6 cross terms of 2^59, one square
// and 14 reduction terms of 2^58 per column, < 2^62.8)
template <class C>
BH_DEV FeS<C> fes_sqr(const FeS<C>& a) {
  constexpr int N = C::N;
  FeS<C> r;
  int32_t m[N], a2[N];
#pragma unroll
  for (int i = 0; i < N; i++) a2[i] = a.v[i] * 2;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      const int j = k - i;
      if (i < j) acc += (int64_t)a.v[i] * a2[j];
      else if (i == j) acc += (int64_t)a.v[i] * a.v[i];
    }
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) acc += (int64_t)m[i] * C::P[k - i];
    if (k < N) {
      m[k] = sext_digit<C>((uint32_t)acc * C::INV);
      acc += (int64_t)m[k] * C::P[0];
    } else {
      const int32_t d = sext_digit<C>((uint32_t)acc);
      r.v[k - N] = d;
      acc -= d;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (int32_t)acc;
  return r;
}

// (a*b + c*d) R^-1 with one reduction: c*d runs in a second accumulator (a column of all three
// would reach 2^63.3) whose low digit moves into the first one every column
template <class C>
BH_DEV FeS<C> fes_mul2(const FeS<C>& a, const FeS<C>& b, const FeS<C>& c, const FeS<C>& d) {
  constexpr int N = C::N;
  FeS<C> r;
  int32_t m[N];
  int64_t acc = 0, acd = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      acc += (int64_t)a.v[i] * b.v[k - i];
      acd += (int64_t)c.v[i] * d.v[k - i];
    }
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) acc += (int64_t)m[i] * C::P[k - i];
    const int32_t t = sext_digit<C>((uint32_t)acd);
    acd = (acd - t) >> C::BITS;
    acc += t;
    if (k < N) {
      m[k] = sext_digit<C>((uint32_t)acc * C::INV);
      acc += (int64_t)m[k] * C::P[0];
    } else {
      const int32_t dd = sext_digit<C>((uint32_t)acc);
      r.v[k - N] = dd;
      acc -= dd;
    }
    acc >>= C::BITS;
    if (k == 2 * N - 2) acc += acd;
  }
  r.v[N - 1] = (int32_t)acc;
  return r;
}

// a + b and a - b, renormalised to balanced digits (the top digit keeps the carry)
template <class C>
BH_DEV FeS<C> fes_add(const FeS<C>& a, const FeS<C>& b) {
  FeS<C> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N - 1; i++) {
    const int32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = sext_digit<C>((uint32_t)s);
    c = (s - r.v[i]) >> C::BITS;
  }
  r.v[C::N - 1] = a.v[C::N - 1] + b.v[C::N - 1] + c;
  return r;
}
template <class C>
BH_DEV FeS<C> fes_sub(const FeS<C>& a, const FeS<C>& b) {
  FeS<C> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N - 1; i++) {
    const int32_t s = a.v[i] - b.v[i] + c;
    r.v[i] = sext_digit<C>((uint32_t)s);
    c = (s - r.v[i]) >> C::BITS;
  }
  r.v[C::N - 1] = a.v[C::N - 1] - b.v[C::N - 1] + c;
  return r;
}
template <class C>
BH_DEV FeS<C> fes_neg(const FeS<C>& a) {  // digit-wise: a balanced form of -a (a digit may be 2^29)
  FeS<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = -a.v[i];
  return r;
}

// balanced digits of k*p for |k| < 2^(BITS-1): the digit-wise comparison target of fes_is_zero
template <class C>
BH_DEV bool fes_is_zero(const FeS<C>& x) {
  const int32_t k = sext_digit<C>((uint32_t)x.v[0] * C::P0INV);  // x = k p  =>  k = x0 / p mod 2^BITS
  if (k >= 128 || k <= -128) return false;
  int64_t carry = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < C::N - 1; i++) {
    const int64_t t = (int64_t)C::P[i] * k + carry;
    const int32_t d = sext_digit<C>((uint32_t)t);
    diff |= (uint32_t)(d ^ x.v[i]);
    carry = (t - d) >> C::BITS;
  }
  diff |= (uint32_t)((int32_t)((int64_t)C::P[C::N - 1] * k + carry) ^ x.v[C::N - 1]);
  return diff == 0;
}

// balanced <-> unsigned BITS-bit limbs (value >= 0 and < 2^(BITS*N))
template <class C, class CU>
BH_DEV Fe<CU> fes_to_unsigned(const FeS<C>& x) {
  Fe<CU> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    const int32_t s = x.v[i] + c;
    r.v[i] = (uint32_t)s & C::MASK;
    c = s >> C::BITS;
  }
  return r;
}
template <class C, class CU>
BH_DEV FeS<C> fes_from_unsigned(const Fe<CU>& x) {
  FeS<C> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N - 1; i++) {
    const int32_t s = (int32_t)x.v[i] + c;
    r.v[i] = sext_digit<C>((uint32_t)s);
    c = (s - r.v[i]) >> C::BITS;
  }
  r.v[C::N - 1] = (int32_t)x.v[C::N - 1] + c;
  return r;
}

// canonical [0, p) for |x| < 128p (x + 128p, then the unsigned conditional subtractions)
template <class C, class CU>
BH_DEV FeS<C> fes_reduce_full(const FeS<C>& x) {
  FeS<C> kp;
  {
    int64_t carry = 0;
#pragma unroll
    for (int i = 0; i < C::N - 1; i++) {
      const int64_t t = (int64_t)C::P[i] * 128 + carry;
      kp.v[i] = sext_digit<C>((uint32_t)t);
      carry = (t - kp.v[i]) >> C::BITS;
    }
    kp.v[C::N - 1] = (int32_t)((int64_t)C::P[C::N - 1] * 128 + carry);
  }
  Fe<CU> u = fes_to_unsigned<C, CU>(fes_add<C>(x, kp));  // in (0, 256p)
  u = fe_csub<CU, 128>(u);
  u = fe_reduce_full<CU>(u);
  return fes_from_unsigned<C, CU>(u);
}

template <class C>
struct FpSOps {
  using Cf = C;
  using CU = Fp30Cfg;  // the unsigned form of the same limb geometry (packing, final reduction)
  using T = FeS<C>;
  static constexpr uint32_t MB = 2;  // bound bookkeeping of CurveOps (signed values need no K*p)
  static BH_DEV T mul(const T& a, const T& b) { return fes_mul<C>(a, b); }
  static BH_DEV T sqr(const T& a) { return fes_sqr<C>(a); }
  static BH_DEV T add(const T& a, const T& b) { return fes_add<C>(a, b); }
  template <uint32_t K> static BH_DEV T sub(const T& a, const T& b) { return fes_sub<C>(a, b); }
  template <uint32_t K> static BH_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return fes_mul2<C>(a, b, fes_neg<C>(c), d);
  }
  static BH_DEV bool is_zero(const T& a) { return fes_is_zero<C>(a); }
  static BH_DEV T zero() { return fes_zero<C>(); }
  static BH_DEV T one() { return fes_one<C>(); }
  static BH_DEV T reduce(const T& a) { return fes_reduce_full<C, CU>(a); }
  static BH_DEV T neg_canonical(const T& a) { return fes_neg<C>(a); }  // -a (the curve code only multiplies it)
  static BH_DEV T select(bool c, const T& a, const T& b) {
    T r;
#pragma unroll
    for (int i = 0; i < C::N; i++) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
  }
  static constexpr int PACKED_WORDS = 12;
  static BH_DEV T unpack(const uint32_t* w) { return fes_from_unsigned<C, CU>(fe_unpack<CU>(w)); }
  // x must be canonical (reduce) or at least in [0, 2^384)
  static BH_DEV void pack(const T& a, uint32_t* w) { fe_pack<CU>(fes_to_unsigned<C, CU>(a), w); }
};
using Fp30sOps = FpSOps<Fp30sCfg>;
