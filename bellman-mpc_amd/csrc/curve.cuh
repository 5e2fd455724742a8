// Device group law for BLS12-381 G1 (over Fp) and G2 (over Fp2), a = 0.
//
// Bucket accumulators use extended Jacobian "XYZZ" coordinates
// (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed addition with an affine base
// costs 8M + 2S and needs no inversion (EFD madd-2008-s / add-2008-s /
// dbl-2008-s / mdbl-2008-s).  Exceptional cases (P == Q, P == -Q, identity)
// are handled exactly, so results are canonical group elements and compare
// bit-exactly with bls12_381's projective arithmetic after normalisation.
//
// Bounds (multiples of p, see field.cuh): with MB = product bound of the field,
//   X < XB = MB + K1,  Y < YB = MB + K3,  ZZ, ZZZ < MB
// and every subtraction constant K is chosen >= the subtrahend's bound.
#pragma once
#include "field.cuh"

constexpr uint32_t bh_pow2_ceil(uint32_t x) {
  uint32_t r = 1;
  while (r < x) r <<= 1;
  return r;
}

template <class F>
struct XYZZ {
  typename F::T X, Y, ZZ, ZZZ;
};

template <class F>
struct Affine {
  typename F::T x, y;
};

template <class F>
struct CurveOps {
  using T = typename F::T;
  using P = XYZZ<F>;
  using A = Affine<F>;
  static constexpr uint32_t MB = F::MB;
  static constexpr uint32_t K1 = bh_pow2_ceil(3 * MB);
  static constexpr uint32_t XB = MB + K1;
  static constexpr uint32_t K2 = bh_pow2_ceil(XB);
  static constexpr uint32_t K3 = bh_pow2_ceil(MB);
  static constexpr uint32_t YB = MB + K3;
  static constexpr uint32_t KX = K2;
  static constexpr uint32_t KY = bh_pow2_ceil(YB);
  static_assert(MB + KX < 128 && MB + KY < 128, "is_zero bound");

  static BH_DEV P identity() {
    P r;
    r.X = F::zero(); r.Y = F::zero(); r.ZZ = F::zero(); r.ZZZ = F::zero();
    return r;
  }
  static BH_DEV bool is_identity(const P& p) { return F::is_zero(p.ZZ); }

  static BH_DEV P from_affine(const A& a) {
    P r;
    r.X = a.x; r.Y = a.y; r.ZZ = F::one(); r.ZZZ = F::one();
    return r;
  }

  // 2*(x, y) for an affine point (mdbl-2008-s)
  static BH_DEV P dbl_affine(const A& a) {
    T U = F::add(a.y, a.y);
    T V = F::sqr(U);
    T W = F::mul(U, V);
    T S = F::mul(a.x, V);
    T xx = F::sqr(a.x);
    T M = F::add(F::add(xx, xx), xx);
    P r;
    r.X = F::template sub<K1>(F::sqr(M), F::add(S, S));
    r.Y = F::template sub<K3>(F::mul(M, F::template sub<K2>(S, r.X)), F::mul(W, a.y));
    r.ZZ = V;
    r.ZZZ = W;
    return r;
  }

  // 2*p (dbl-2008-s); identity stays identity (ZZ' = V*ZZ ≡ 0)
  static BH_DEV P dbl(const P& p) {
    T U = F::add(p.Y, p.Y);
    T V = F::sqr(U);
    T W = F::mul(U, V);
    T S = F::mul(p.X, V);
    T xx = F::sqr(p.X);
    T M = F::add(F::add(xx, xx), xx);
    P r;
    r.X = F::template sub<K1>(F::sqr(M), F::add(S, S));
    r.Y = F::template mul_sub<KY>(M, F::template sub<K2>(S, r.X), p.Y, W);
    r.ZZ = F::mul(V, p.ZZ);
    r.ZZZ = F::mul(W, p.ZZZ);
    return r;
  }

  // p + a, a affine and not the identity (madd-2008-s); Y3 = R(Q - X3) - Y1*PPP with one
  // Montgomery reduction for both products over Fp (F::mul_sub).
  // G1 (UNIFIED_MADD): the exceptional cases run through the same instruction stream instead of
  // a separate doubling routine, which the register allocator would otherwise provision for
  // (G1 accumulation 252 -> 178 VGPRs; measured -0.7 ms of G1 accumulation per 2^22 proof):
  //  * p == a: dbl-2008-s of p is this formula with Pd := 2*Y1, R := 3*X1^2 and no PPP term in
  //    X3 (PP = V, PPP = W, Q = S, ZZ3 = ZZ1*V, ZZZ3 = ZZZ1*W);
  //  * p == -a: the identity (the all-zero point, as identity() stores it).
  // No point of G1 or G2 has order 2 (prime-order subgroups), so Y1 != 0 when p == a.
  // G2 keeps the branch to dbl_affine: the unified form measured +1.2 ms of G2 accumulation.
  static constexpr bool UNIFIED_MADD = !std::is_same<F, Fp2Ops>::value;
  static BH_DEV P madd(const P& p, const A& a) {
    if (is_identity(p)) return from_affine(a);
    T U2 = F::mul(a.x, p.ZZ);
    T S2 = F::mul(a.y, p.ZZZ);
    T Pd = F::template sub<KX>(U2, p.X);
    T R = F::template sub<KY>(S2, p.Y);
    bool twice = false, neg = false;
    if (F::is_zero(Pd)) {  // rare: bounds below hold for both substitutions (Pd < 8p, R < 6p)
      if constexpr (!UNIFIED_MADD) {
        if (F::is_zero(R)) return dbl_affine(a);
        return identity();
      }
      twice = F::is_zero(R);
      neg = !twice;
      if (twice) {
        Pd = F::add(p.Y, p.Y);
        const T xx = F::sqr(p.X);
        R = F::add(F::add(xx, xx), xx);
      }
    }
    T PP = F::sqr(Pd);
    T PPP = F::mul(Pd, PP);
    T Q = F::mul(p.X, PP);
    P r;
    const T Q2 = F::add(Q, Q);
    r.X = F::template sub<K1>(F::sqr(R), twice ? Q2 : F::add(PPP, Q2));
    r.Y = F::template mul_sub<KY>(R, F::template sub<K2>(Q, r.X), p.Y, PPP);
    r.ZZ = F::mul(p.ZZ, PP);
    r.ZZZ = F::mul(p.ZZZ, PPP);
    if (neg) r = identity();
    return r;
  }

  // p + q (add-2008-s).  As in madd, p == q takes the same instruction stream: (U1, S1,
  // ZZ1*ZZ2, ZZZ1*ZZZ2) represents p, and its dbl-2008-s is this formula with Pd := 2*S1,
  // R := 3*U1^2 and no PPP term in X3; p == -q gives the identity.  Without a separate doubling
  // routine to provision for, the G2 reduction kernels spill less (k_reduce_blocks<G2> 1760 ->
  // 1124 B/lane of scratch, k_reduce_window<G2> 2128 -> 1916).
  static BH_DEV P add(const P& p, const P& q) {
    if (is_identity(p)) return q;
    if (is_identity(q)) return p;
    T U1 = F::mul(p.X, q.ZZ);
    T U2 = F::mul(q.X, p.ZZ);
    T S1 = F::mul(p.Y, q.ZZZ);
    T S2 = F::mul(q.Y, p.ZZZ);
    T Pd = F::template sub<K3>(U2, U1);
    T R = F::template sub<K3>(S2, S1);
    bool twice = false, neg = false;
    if (F::is_zero(Pd)) {  // rare: Pd = 2*S1 < 4p, R = 3*U1^2 < 6p keep the bounds below
      twice = F::is_zero(R);
      neg = !twice;
      if (twice) {
        Pd = F::add(S1, S1);
        const T uu = F::sqr(U1);
        R = F::add(F::add(uu, uu), uu);
      }
    }
    // ZZ1*ZZ2 and ZZZ1*ZZZ2 before the rest: the four input Z's are dead from here on (fewer live
    // values: the G2 reduction kernels spill less)
    const T ZZ12 = F::mul(p.ZZ, q.ZZ);
    const T ZZZ12 = F::mul(p.ZZZ, q.ZZZ);
    T PP = F::sqr(Pd);
    T PPP = F::mul(Pd, PP);
    T Q = F::mul(U1, PP);
    P r;
    r.ZZ = F::mul(ZZ12, PP);
    r.ZZZ = F::mul(ZZZ12, PPP);
    const T Q2 = F::add(Q, Q);
    r.X = F::template sub<K1>(F::sqr(R), twice ? Q2 : F::add(PPP, Q2));
    r.Y = F::template mul_sub<K3>(R, F::template sub<K2>(Q, r.X), S1, PPP);
    if (neg) r = identity();
    return r;
  }

  // -a for a base about to be added: y -> p - y, left in (0, p] (the formulas take any
  // representative below 128p; a canonical y would cost a conditional subtraction more)
  static BH_DEV A neg_affine(const A& a) {
    A r;
    r.x = a.x;
    r.y = F::template sub<1>(F::zero(), a.y);
    return r;
  }

  // canonical coordinates (each in [0,p)) for hand-off to the host
  static BH_DEV P reduce(const P& p) {
    P r;
    r.X = F::reduce(p.X); r.Y = F::reduce(p.Y); r.ZZ = F::reduce(p.ZZ); r.ZZZ = F::reduce(p.ZZZ);
    return r;
  }
};

// G1's field representation (the host conversions follow G1F::Cf).  13 x 30-bit forms with 338
// instead of 392 limb products per multiplication were measured no faster inside the prover
// (tools/microbench/fp_variants.cuh).
using G1F = FpOps;
using G1Ops = CurveOps<G1F>;
using G2Ops = CurveOps<Fp2Ops>;
