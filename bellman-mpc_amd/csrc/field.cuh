// Device finite-field arithmetic for BLS12-381 on gfx950.
//
// Representation: N little-endian limbs of 29 bits held in uint32 (DFp: N=14,
// Montgomery R = 2^406; Fr: N=9, R = 2^261).  Products of two limbs are < 2^58,
// so a 64-bit column accumulator absorbs all 2N products of one column of the
// product-scanning (FIPS) Montgomery multiplication with no carry handling:
// every product is a single v_mad_u64_u32 (microbenchmarked on MI355X at
// 77 G DFp-mul/s vs 46 G for 32-bit-limb CIOS, tools/microbench/fpbench.hip).
//
// Lazy reduction: because R/p >= 2^25 (DFp) and R/q >= 2^6 (Fr), montgomery
// multiplication of inputs a < A*p, b < B*p returns a value < 2p whenever
// A*B < 2^25 (DFp) / 2^6 (Fr).  Additions therefore never reduce; subtraction
// adds a constant multiple K*p.  Values are brought to [0,p) only when they
// leave the device (`reduce_full`) and equality tests use `is_zero` (x ≡ 0 mod
// p for x < 128p) which costs one 32-bit multiply in the common (non-zero) case.
//
// The arithmetic restates the field ops bls12_381 0.6.0 performs for the
// reference hot path (multiexp.rs:39,217,231-232,248; domain.rs:250-257).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "constants.h"

#define BH_DEV __device__ __forceinline__

template <class C>
struct Fe {
  uint32_t v[C::N];
};

// ---------------------------------------------------------------- constexpr K*p limbs
template <class C, uint32_t K>
struct KP {
  struct L { uint32_t v[C::N]; };
  static constexpr L make() {
    L l{};
    uint64_t carry = 0;
    for (int i = 0; i < C::N; i++) {
      uint64_t t = (uint64_t)C::P[i] * K + carry;
      l.v[i] = (uint32_t)(t & C::MASK);
      carry = t >> C::BITS;
    }
    return l;
  }
  static constexpr L value = make();
};

template <class C>
BH_DEV Fe<C> fe_zero() {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = 0;
  return r;
}

template <class C>
BH_DEV Fe<C> fe_one() {  // Montgomery form of 1
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = C::ONE[i];
  return r;
}

// One step of a column chain: acc + a*b as ONE v_mad_u64_u32 with acc as its addend.  Written as
// plain C (acc += (uint64_t)a * b) the compiler's reassociation starts every column on a fresh
// chain of products and adds the carried accumulator afterwards (one 64-bit add per column); as
// an opaque instruction the column stays one chain seeded with the carry (the hazard recogniser
// follows each with an s_nop 0, which is not VALU work, and the chain is latency-bound per wave).
// Measured (profiles/r06_ab_mul_chain.txt): Fr (the NTT, 4 waves per SIMD) -16 VALU per butterfly,
// 2^22 proof -0.2 ms; Fp (the accumulations, 2 waves per SIMD) 5 129 -> 4 745 VALU per G1 madd but
// the proof +1.2 ms and N = 8 +1.2 ms -- the latency costs more than the merges.  So Fr only.
template <class C>
struct MulChain {
  static constexpr bool value = C::N == 9;  // FrCfg
};
template <bool CH>
BH_DEV void mac(uint64_t& acc, uint32_t a, uint32_t b) {
  if (CH) {
    uint64_t r, sc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(a), "v"(b), "v"(acc));
    acc = r;
  } else {
    acc += (uint64_t)a * b;
  }
}
// ... times a modulus limb (a compile-time constant: an SGPR operand)
template <bool CH>
BH_DEV void mac_p(uint64_t& acc, uint32_t m, uint32_t p) {
  if (CH) {
    uint64_t r, sc;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(m), "s"(p), "v"(acc));
    acc = r;
  } else {
    acc += (uint64_t)m * p;
  }
}

// Montgomery product, FIPS column order. Output < 2p (see header).
// A modulus with p = 1 (mod 2^BITS) (Fr) has m_k = -acc mod 2^BITS, so acc + m_k * p_0 is acc
// rounded up to a multiple of 2^BITS: (acc + MASK) >> BITS, no product and no 64-bit m_k.
// DFp keeps two independent chains (a*b and m*p) per column, which the compiler schedules for
// latency; Fr runs each column as one carry-seeded chain of opaque mads (MulChain, above).
template <class C>
BH_DEV Fe<C> fe_mul(const Fe<C>& a, const Fe<C>& b) {
  constexpr int N = C::N;
  constexpr bool P0_ONE = C::P[0] == 1u;
  constexpr bool CH = MulChain<C>::value;
  constexpr bool TWO_CHAINS = N > 9 && !CH;
  Fe<C> r;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t acc2 = 0;
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) mac<CH>(acc, a.v[i], b.v[k - i]);
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) {
      if (TWO_CHAINS) acc2 += (uint64_t)m[i] * C::P[k - i];
      else mac_p<CH>(acc, m[i], C::P[k - i]);
    }
    if (TWO_CHAINS) acc += acc2;
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      if (P0_ONE) {
        acc = (acc + C::MASK) >> C::BITS;
        continue;
      }
      mac_p<CH>(acc, m[k], C::P[0]);
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

// x * R^-1 (fe_mul(x, 1) without the zero products): out of Montgomery form, <= p for x < R
template <class C>
BH_DEV Fe<C> fe_from_mont(const Fe<C>& a) {
  constexpr int N = C::N;
  constexpr bool CH = MulChain<C>::value;
  constexpr bool P0_ONE = C::P[0] == 1u;
  Fe<C> r;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    if (k < N) acc += a.v[k];
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) mac_p<CH>(acc, m[i], C::P[k - i]);
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      if (P0_ONE) {  // as in fe_mul
        acc = (acc + C::MASK) >> C::BITS;
        continue;
      }
      mac_p<CH>(acc, m[k], C::P[0]);
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

// (a*b + c*d) * R^-1 with ONE interleaved Montgomery reduction: every column absorbs the
// products of both pairs and the m*p terms -- at most 3N = 42 products < 2^58 each for DFp,
// so the 64-bit accumulator still needs no carry handling (2^63.4).  Output < 2p when the
// operand bounds (in multiples of p) satisfy A*B + C*D < R/p (2^25 for DFp).
template <class C>
BH_DEV Fe<C> fe_mul2(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d) {
  constexpr int N = C::N;
  static_assert(3 * N < 64, "3N products < 2^58 plus the carry must fit the 64-bit column accumulator");
  constexpr bool CH = MulChain<C>::value;
  Fe<C> r;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      mac<CH>(acc, a.v[i], b.v[k - i]);
      mac<CH>(acc, c.v[i], d.v[k - i]);
    }
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) mac_p<CH>(acc, m[i], C::P[k - i]);
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      mac_p<CH>(acc, m[k], C::P[0]);
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

// Montgomery square: cross products computed once against 2*a (limbs < 2^30).
template <class C>
BH_DEV Fe<C> fe_sqr(const Fe<C>& a) {
  constexpr int N = C::N;
  Fe<C> r;
  constexpr bool CH = MulChain<C>::value;
  uint32_t m[N], a2[N];
#pragma unroll
  for (int i = 0; i < N; i++) a2[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    const int lo = (k < N ? 0 : k - N + 1);
    const int hi = (k < N ? k : N - 1);
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      const int j = k - i;
      if (i < j) mac<CH>(acc, a.v[i], a2[j]);
      else if (i == j) mac<CH>(acc, a.v[i], a.v[i]);
    }
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) mac_p<CH>(acc, m[i], C::P[k - i]);
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      mac_p<CH>(acc, m[k], C::P[0]);
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

// a + b (no modular reduction; caller tracks the bound)
template <class C>
BH_DEV Fe<C> fe_add(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = s & C::MASK;
    c = s >> C::BITS;
  }
  return r;
}

// a + K*p - b   (requires b < K*p)
template <class C, uint32_t K>
BH_DEV Fe<C> fe_sub(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    int32_t s = (int32_t)(a.v[i] + KP<C, K>::value.v[i]) - (int32_t)b.v[i] + c;
    r.v[i] = (uint32_t)s & C::MASK;
    c = s >> C::BITS;  // arithmetic shift: -1, 0 or +1
  }
  return r;
}

// K*p - a (requires a < K*p)
template <class C, uint32_t K>
BH_DEV Fe<C> fe_neg(const Fe<C>& a) {
  return fe_sub<C, K>(fe_zero<C>(), a);
}

// conditional subtraction: if x >= K*p then x - K*p
template <class C, uint32_t K>
BH_DEV Fe<C> fe_csub(const Fe<C>& x) {
  Fe<C> t;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    int32_t s = (int32_t)x.v[i] - (int32_t)KP<C, K>::value.v[i] + c;
    t.v[i] = (uint32_t)s & C::MASK;
    c = s >> C::BITS;
  }
  const bool ge = (c >= 0);
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = ge ? t.v[i] : x.v[i];
  return r;
}

// Fully reduce x < 128p into [0, p).
template <class C>
BH_DEV Fe<C> fe_reduce_full(Fe<C> x) {
  x = fe_csub<C, 64>(x);
  x = fe_csub<C, 32>(x);
  x = fe_csub<C, 16>(x);
  x = fe_csub<C, 8>(x);
  x = fe_csub<C, 4>(x);
  x = fe_csub<C, 2>(x);
  x = fe_csub<C, 1>(x);
  return x;
}

// x ≡ 0 (mod p), valid for x < 128p.  x = k*p exactly when the low limb gives
// k = x0 * p^-1 mod 2^29 < 128 and the full comparison with k*p succeeds.
template <class C>
BH_DEV bool fe_is_zero(const Fe<C>& x) {
  const uint32_t k = (x.v[0] * C::P0INV) & C::MASK;
  if (k >= 128u) return false;
  uint64_t carry = 0;
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    uint64_t t = (uint64_t)C::P[i] * k + carry;
    diff |= ((uint32_t)t & C::MASK) ^ x.v[i];
    carry = t >> C::BITS;
  }
  return diff == 0;
}

template <class C>
BH_DEV bool fe_is_zero_canonical(const Fe<C>& x) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < C::N; i++) d |= x.v[i];
  return d == 0;
}

template <class C>
BH_DEV Fe<C> fe_select(bool c, const Fe<C>& a, const Fe<C>& b) {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// ---------------------------------------------------------------- packing
// Packed storage: the (near-)canonical value in W = ceil(29N/32) - 0/1 32-bit words.
// DFp packs into 12 words (value < 2^384), Fr into 8 words (value < 2^256).
template <class C> struct Packed;
template <> struct Packed<FpCfg> { static constexpr int W = 12; };
template <> struct Packed<FrCfg> { static constexpr int W = 8; };

template <class C>
BH_DEV Fe<C> fe_unpack(const uint32_t* w) {
  constexpr int W = Packed<C>::W;
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < C::N; i++) {
    const int bit = i * C::BITS;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t lo = w[wi];
    uint64_t hi = (wi + 1 < W) ? (uint64_t)w[wi + 1] : 0ull;
    r.v[i] = (uint32_t)(((hi << 32) | lo) >> sh) & C::MASK;
  }
  return r;
}

// x must be < 2^(32W) (e.g. fully reduced)
template <class C>
BH_DEV void fe_pack(const Fe<C>& x, uint32_t* w) {
  constexpr int W = Packed<C>::W;
#pragma unroll
  for (int j = 0; j < W; j++) {
    uint64_t acc = 0;
    const int bit0 = j * 32;
#pragma unroll
    for (int i = 0; i < C::N; i++) {
      const int b = i * C::BITS;
      if (b + C::BITS <= bit0 || b >= bit0 + 32) continue;
      if (b >= bit0) acc |= (uint64_t)x.v[i] << (b - bit0);
      else acc |= (uint64_t)x.v[i] >> (bit0 - b);
    }
    w[j] = (uint32_t)acc;
  }
}

// ---------------------------------------------------------------- DFp2 = DFp[u]/(u^2+1)
struct DFp2 {
  Fe<FpCfg> c0, c1;
};

using DFp = Fe<FpCfg>;
using DFr = Fe<FrCfg>;

// Field-generic wrappers so the curve code is written once for DFp (G1) and DFp2 (G2).
// MB = bound (in multiples of p) of a product; is_zero valid below 128p.
template <class Cfg>
struct FpOpsT {
  using Cf = Cfg;
  using T = Fe<Cfg>;
  static constexpr uint32_t MB = 2;
  static BH_DEV T mul(const T& a, const T& b) { return fe_mul<Cfg>(a, b); }
  static BH_DEV T sqr(const T& a) { return fe_sqr<Cfg>(a); }
  static BH_DEV T add(const T& a, const T& b) { return fe_add<Cfg>(a, b); }
  template <uint32_t K> static BH_DEV T sub(const T& a, const T& b) { return fe_sub<Cfg, K>(a, b); }
  // a*b - c*d with c < K*p: one reduction for both products (fe_mul2 of a, b, K*p - c, d); < 2p
  template <uint32_t K> static BH_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return fe_mul2<Cfg>(a, b, fe_neg<Cfg, K>(c), d);
  }
  static BH_DEV bool is_zero(const T& a) { return fe_is_zero<Cfg>(a); }
  static BH_DEV T zero() { return fe_zero<Cfg>(); }
  static BH_DEV T one() { return fe_one<Cfg>(); }
  static BH_DEV T reduce(const T& a) { return fe_reduce_full<Cfg>(a); }
  static BH_DEV T neg_canonical(const T& a) {  // p - a for a in [0,p], result in [0,p]
    return fe_csub<Cfg, 1>(fe_sub<Cfg, 1>(fe_zero<Cfg>(), a));
  }
  static BH_DEV T select(bool c, const T& a, const T& b) { return fe_select<Cfg>(c, a, b); }
  static constexpr int PACKED_WORDS = 12;
  static BH_DEV T unpack(const uint32_t* w) { return fe_unpack<Cfg>(w); }
  static BH_DEV void pack(const T& a, uint32_t* w) { fe_pack<Cfg>(a, w); }
};
using FpOps = FpOpsT<FpCfg>;  // 14 x 29-bit limbs


// Fp2 product a*b = (a0 b0 - a1 b1) + (a0 b1 + a1 b0) u with Karatsuba's three column sums
// shared by both halves: per column t0 = sum a0 b0, t1 = sum a1 b1, t2 = sum (a0+a1)(b0+b1);
// c1 += t2 - t0 - t1 (exact: the true value is >= 0 and < 2^63), c0 += t0 - t1 on a signed
// accumulator; both halves get their own interleaved Montgomery reduction.  c0 = (X + M p)/R
// with X > -(128p)^2 lies in (-p/2^11, 2p): one conditional +p makes it >= 0.  Inputs < 128p
// with 29-bit limbs (so a0+a1 limbs < 2^30, products < 2^60, 14-term columns < 2^63.9).
template <class C>
BH_DEV void fe2_mul_kara(const Fe<C>& a0, const Fe<C>& a1, const Fe<C>& b0, const Fe<C>& b1, Fe<C>& r0,
                         Fe<C>& r1) {
  constexpr int N = C::N;
  uint32_t sa[N], sb[N], m0[N], m1[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    sa[i] = a0.v[i] + a1.v[i];
    sb[i] = b0.v[i] + b1.v[i];
  }
  int64_t acc0 = 0;
  uint64_t acc1 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t t0 = 0, t1 = 0, t2 = 0;
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      t0 += (uint64_t)a0.v[i] * b0.v[k - i];
      t1 += (uint64_t)a1.v[i] * b1.v[k - i];
      t2 += (uint64_t)sa[i] * sb[k - i];
    }
    acc0 += (int64_t)(t0 - t1);
    acc1 += t2 - t0 - t1;
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) {
      acc0 += (int64_t)((uint64_t)m0[i] * C::P[k - i]);
      acc1 += (uint64_t)m1[i] * C::P[k - i];
    }
    if (k < N) {
      m0[k] = ((uint32_t)acc0 * C::INV) & C::MASK;
      acc0 += (int64_t)((uint64_t)m0[k] * C::P[0]);
      m1[k] = ((uint32_t)acc1 * C::INV) & C::MASK;
      acc1 += (uint64_t)m1[k] * C::P[0];
    } else {
      r0.v[k - N] = (uint32_t)acc0 & C::MASK;
      r1.v[k - N] = (uint32_t)acc1 & C::MASK;
    }
    acc0 >>= C::BITS;
    acc1 >>= C::BITS;
  }
  r1.v[N - 1] = (uint32_t)acc1;
  // r0's top limb is the signed remainder; add p when it is negative
  const uint32_t neg = (uint32_t)(acc0 >> 63);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N - 1; i++) {
    const uint32_t s = r0.v[i] + (C::P[i] & neg) + c;
    r0.v[i] = s & C::MASK;
    c = s >> C::BITS;
  }
  r0.v[N - 1] = (uint32_t)acc0 + (C::P[N - 1] & neg) + c;
}

// a*b - c*d in Fp2 with ONE Montgomery reduction per half (lazy reduction over both Karatsuba
// products): per column t0 = sum a0 b0, t1 = sum a1 b1, t2 = sum (a0+a1)(b0+b1) and the same
// u0, u1, u2 for c, d; half 0 gets (t0 - t1) - (u0 - u1), half 1 (t2 - t0 - t1) - (u2 - u0 - u1).
// 6 x 196 product mads + 2 x 196 reduction mads instead of 2 x (3 + 2) x 196 for two products and
// a subtraction.  Bounds (column k, in units of 2^58): operand limbs < 2^29 (normalised; values
// < 2^386, so the top limb is < 2^9), so one product's column sum is < 13 and a half's column
// difference lies in (-26, 26); the m*p terms add [0, 7.02) (p's own limbs: max over k of
// (2^29-1) * sum of the p limbs the column meets, computed in DESIGN.md section 4).  The width
// 59.02 < 64 fits 64 bits, but not signed: each accumulator carries BIAS = 28 * 2^58 (a multiple
// of 2^29) and is read as unsigned, in (2, 61.02) * 2^58; the carry out of a column is
// (acc >> 29) - (BIAS >> 29), i.e. the next column starts from (acc >> 29) + (BIAS - (BIAS >> 29)).
// The result (X + M p) / R lies in (-p, 2p) for |X| < 2^25 p^2 (R = 2^406 > 2^25 p): a negative
// half gets + p, leaving [0, 2p).
template <class C>
BH_DEV void fe2_mul_sub_kara(const Fe<C>& a0, const Fe<C>& a1, const Fe<C>& b0, const Fe<C>& b1, const Fe<C>& c0,
                             const Fe<C>& c1, const Fe<C>& d0, const Fe<C>& d1, Fe<C>& r0, Fe<C>& r1) {
  constexpr int N = C::N;
  constexpr uint64_t BIAS = 7ull << 60;  // 28 * 2^58
  constexpr uint64_t NEXT = BIAS - (BIAS >> C::BITS);
  uint32_t m0[N], m1[N], sa[N], sb[N], sc[N], sd[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    sa[i] = a0.v[i] + a1.v[i];
    sb[i] = b0.v[i] + b1.v[i];
    sc[i] = c0.v[i] + c1.v[i];
    sd[i] = d0.v[i] + d1.v[i];
  }
  uint64_t acc0 = BIAS, acc1 = BIAS;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
    uint64_t t0 = 0, t1 = 0, t2 = 0, u0 = 0, u1 = 0, u2 = 0;
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) {
      t0 += (uint64_t)a0.v[i] * b0.v[k - i];
      t1 += (uint64_t)a1.v[i] * b1.v[k - i];
      t2 += (uint64_t)sa[i] * sb[k - i];
      u0 += (uint64_t)c0.v[i] * d0.v[k - i];
      u1 += (uint64_t)c1.v[i] * d1.v[k - i];
      u2 += (uint64_t)sc[i] * sd[k - i];
    }
    // (two's complement: the differences are exact mod 2^64 and the biased sums are in range)
    acc0 += (t0 - t1) - (u0 - u1);
    acc1 += (t2 - t0 - t1) - (u2 - u0 - u1);
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) {
      acc0 += (uint64_t)m0[i] * C::P[k - i];
      acc1 += (uint64_t)m1[i] * C::P[k - i];
    }
    if (k < N) {
      m0[k] = ((uint32_t)acc0 * C::INV) & C::MASK;
      acc0 += (uint64_t)m0[k] * C::P[0];
      m1[k] = ((uint32_t)acc1 * C::INV) & C::MASK;
      acc1 += (uint64_t)m1[k] * C::P[0];
    } else {
      r0.v[k - N] = (uint32_t)acc0 & C::MASK;
      r1.v[k - N] = (uint32_t)acc1 & C::MASK;
    }
    acc0 = (acc0 >> C::BITS) + NEXT;
    acc1 = (acc1 >> C::BITS) + NEXT;
  }
  // top limbs: the signed remainders (acc - BIAS); a negative half gets + p
  const int64_t top0 = (int64_t)(acc0 - BIAS), top1 = (int64_t)(acc1 - BIAS);
  const uint32_t neg0 = (uint32_t)(top0 >> 63), neg1 = (uint32_t)(top1 >> 63);
  uint32_t cy0 = 0, cy1 = 0;
#pragma unroll
  for (int i = 0; i < N - 1; i++) {
    const uint32_t s0 = r0.v[i] + (C::P[i] & neg0) + cy0;
    r0.v[i] = s0 & C::MASK;
    cy0 = s0 >> C::BITS;
    const uint32_t s1 = r1.v[i] + (C::P[i] & neg1) + cy1;
    r1.v[i] = s1 & C::MASK;
    cy1 = s1 >> C::BITS;
  }
  r0.v[N - 1] = (uint32_t)top0 + (C::P[N - 1] & neg0) + cy0;
  r1.v[N - 1] = (uint32_t)top1 + (C::P[N - 1] & neg1) + cy1;
}

constexpr uint32_t bh_pow2_ceil_fp2(uint32_t x) {
  uint32_t r = 1;
  while (r < x) r <<= 1;
  return r;
}

struct Fp2Ops {
  using T = DFp2;
  static constexpr uint32_t MB = 2;
  // Schoolbook over two interleaved reductions (c0 = a0 b0 + (128p - a1) b1, c1 = a0 b1 + a1 b0),
  // or, in translation units that define BH_FP2_KARATSUBA (the G2 bucket accumulation,
  // msm_g2_acc.hip), the column-wise Karatsuba fe2_mul_kara: 3 x 196 product v_mad_u64_u32
  // instead of 4 x 196 (G2 accumulation alone 15.5 -> 14.9 ms per 2^22 proof).  The reduction
  // kernels keep the schoolbook form: Karatsuba's extra live registers raised their spill
  // scratch (k_reduce_blocks<G2> 2352 -> 2648 B/lane, k_cont_seq 32 -> 528) and a test run hit
  // HSA_STATUS_ERROR_OUT_OF_RESOURCES launching k_reduce_window<G2>.  Both forms give < 2p for
  // inputs < 128p (possibly different representatives of the same element).
  static BH_DEV T mul(const T& a, const T& b) {
    T r;
#ifdef BH_FP2_KARATSUBA
    fe2_mul_kara<FpCfg>(a.c0, a.c1, b.c0, b.c1, r.c0, r.c1);
#else
    r.c0 = fe_mul2<FpCfg>(a.c0, b.c0, fe_neg<FpCfg, 128>(a.c1), b.c1);
    r.c1 = fe_mul2<FpCfg>(a.c0, b.c1, a.c1, b.c0);
#endif
    return r;
  }
  static BH_DEV T sqr(const T& a) {
    T r;
    // (a0 + a1)(a0 - a1), (2 a0) a1 ; valid for inputs < 128p, both < 2p
    r.c0 = fe_mul<FpCfg>(fe_add<FpCfg>(a.c0, a.c1), fe_sub<FpCfg, 128>(a.c0, a.c1));
    r.c1 = fe_mul<FpCfg>(fe_add<FpCfg>(a.c0, a.c0), a.c1);
    return r;
  }
  static BH_DEV T add(const T& a, const T& b) {
    return T{fe_add<FpCfg>(a.c0, b.c0), fe_add<FpCfg>(a.c1, b.c1)};
  }
  template <uint32_t K> static BH_DEV T sub(const T& a, const T& b) {
    return T{fe_sub<FpCfg, K>(a.c0, b.c0), fe_sub<FpCfg, K>(a.c1, b.c1)};
  }
  // a*b - c*d (c unused as a bound here: both products are reduced, < MB*p each)
  template <uint32_t K> static BH_DEV T mul_sub(const T& a, const T& b, const T& c, const T& d) {
    return sub<bh_pow2_ceil_fp2(MB)>(mul(a, b), mul(c, d));
  }
  // the same with one reduction per half over both Karatsuba products (fe2_mul_sub_kara): < 2p,
  // for operands whose values are < 2^386 with normalised limbs
  static BH_DEV T mul_sub_lazy(const T& a, const T& b, const T& c, const T& d) {
    T r;
    fe2_mul_sub_kara<FpCfg>(a.c0, a.c1, b.c0, b.c1, c.c0, c.c1, d.c0, d.c1, r.c0, r.c1);
    return r;
  }
  static BH_DEV bool is_zero(const T& a) { return fe_is_zero<FpCfg>(a.c0) && fe_is_zero<FpCfg>(a.c1); }
  static BH_DEV T zero() { return T{fe_zero<FpCfg>(), fe_zero<FpCfg>()}; }
  static BH_DEV T one() { return T{fe_one<FpCfg>(), fe_zero<FpCfg>()}; }
  static BH_DEV T reduce(const T& a) { return T{fe_reduce_full<FpCfg>(a.c0), fe_reduce_full<FpCfg>(a.c1)}; }
  static BH_DEV T neg_canonical(const T& a) { return T{FpOps::neg_canonical(a.c0), FpOps::neg_canonical(a.c1)}; }
  static BH_DEV T select(bool c, const T& a, const T& b) {
    return T{fe_select<FpCfg>(c, a.c0, b.c0), fe_select<FpCfg>(c, a.c1, b.c1)};
  }
  static constexpr int PACKED_WORDS = 24;  // c0 then c1
  static BH_DEV T unpack(const uint32_t* w) { return T{fe_unpack<FpCfg>(w), fe_unpack<FpCfg>(w + 12)}; }
  static BH_DEV void pack(const T& a, uint32_t* w) { fe_pack<FpCfg>(a.c0, w); fe_pack<FpCfg>(a.c1, w + 12); }
};
