// Modular inversion in Fp (BLS12-381 base field) by Bernstein-Yang divsteps ("safegcd", Fast
// constant-time gcd computation and modular inversion, TCHES 2019), 30 divsteps per batch on
// 32-bit words.  It replaces a Fermat inversion (a^(p-2): ~380 squarings + ~190 products of the
// 14 x 29-bit Montgomery multiplication, ~270 000 VALU instructions) with ~13 batches' worth of
// 32-bit divsteps and 13-limb matrix updates (~20 000), which is what makes per-thread batch
// inversion pay in the batch-affine bucket accumulation (msm_affine.cuh): every accumulation
// thread inverts one product per level.
//
// Representation: signed 30-bit limbs, NL = 13 limbs (390 bits) for the 381-bit modulus; the low
// NL-1 limbs in [0, 2^30) after an update, the top limb signed.  The divsteps are the branch-free
// ones (the same instruction stream on every lane of a wave); the outer loop ends as soon as g = 0
// (a lane that is done idles under the execution mask), at most SG_MAX_BATCHES batches
// (879 divsteps bound 381-bit inputs, Bernstein-Yang theorem 11.2).
//
// Invariant (per batch): f = d x, g = e x (mod p); [f, g] <- T [f, g] / 2^30 and
// [d, e] <- (T [d, e] + p [md, me]) / 2^30 with md, me chosen so the division is exact, which
// keeps d, e in (-2p, p).  At g = 0, f = +-1 and d = +-x^-1.
//
// Header-only and host/device: tests/native/safegcd_test.cpp compiles it with g++ and checks
// x * x^-1 = 1 against Python big integers (tests/test_safegcd.py).
#pragma once
#include <stdint.h>

#include "constants.h"

#if defined(__HIPCC__)
#define BH_HD __host__ __device__ __forceinline__
#else
#define BH_HD inline
#endif

namespace bh {

constexpr int SG_NL = 13;
constexpr int SG_MAX_BATCHES = 32;  // 960 divsteps >= the 879 that bound a 381-bit modulus

struct SgT {
  int32_t u, v, q, r;
};

// 30 branch-free divsteps on the low words of f (odd) and g; zeta = -(delta + 1/2).
BH_HD int32_t sg_divsteps30(int32_t zeta, uint32_t f, uint32_t g, SgT& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < 30; ++i) {
    uint32_t c1 = (uint32_t)(zeta >> 31);  // delta > 0
    const uint32_t c2 = 0u - (g & 1u);      // g odd
    const uint32_t x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;  // g - f (delta > 0) or g + f, when g is odd
    q += y & c2;
    r += z & c2;
    c1 &= c2;  // swap: delta > 0 and g odd
    zeta = (zeta ^ (int32_t)c1) - 1;
    f += g & c1;  // f <- old g
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return zeta;
}

// [d, e] <- (T [d, e] + p [md, me]) / 2^30 (mod p), d, e kept in (-2p, p)
BH_HD void sg_update_de(int32_t* d, int32_t* e, const SgT& t) {
  constexpr int32_t M30 = (int32_t)(0xffffffffu >> 2);
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d[SG_NL - 1] >> 31, se = e[SG_NL - 1] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d[0] + (int64_t)v * e[0];
  int64_t ce = (int64_t)q * d[0] + (int64_t)r * e[0];
  md -= (int32_t)((FpInvCfg::MINV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)M30);
  me -= (int32_t)((FpInvCfg::MINV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)M30);
  cd += (int64_t)FpInvCfg::M30[0] * md;
  ce += (int64_t)FpInvCfg::M30[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < SG_NL; ++i) {
    cd += (int64_t)u * d[i] + (int64_t)v * e[i];
    ce += (int64_t)q * d[i] + (int64_t)r * e[i];
    cd += (int64_t)FpInvCfg::M30[i] * md;
    ce += (int64_t)FpInvCfg::M30[i] * me;
    d[i - 1] = (int32_t)cd & M30;
    cd >>= 30;
    e[i - 1] = (int32_t)ce & M30;
    ce >>= 30;
  }
  d[SG_NL - 1] = (int32_t)cd;
  e[SG_NL - 1] = (int32_t)ce;
}

// [f, g] <- T [f, g] / 2^30 (exact)
BH_HD void sg_update_fg(int32_t* f, int32_t* g, const SgT& t) {
  constexpr int32_t M30 = (int32_t)(0xffffffffu >> 2);
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = (int64_t)u * f[0] + (int64_t)v * g[0];
  int64_t cg = (int64_t)q * f[0] + (int64_t)r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < SG_NL; ++i) {
    cf += (int64_t)u * f[i] + (int64_t)v * g[i];
    cg += (int64_t)q * f[i] + (int64_t)r * g[i];
    f[i - 1] = (int32_t)cf & M30;
    cf >>= 30;
    g[i - 1] = (int32_t)cg & M30;
    cg >>= 30;
  }
  f[SG_NL - 1] = (int32_t)cf;
  g[SG_NL - 1] = (int32_t)cg;
}

// r in (-2p, p) -> (sign < 0 ? -r : r) mod p in [0, p), limbs in [0, 2^30)
BH_HD void sg_normalize(int32_t* r, int32_t sign) {
  constexpr int32_t M30 = (int32_t)(0xffffffffu >> 2);
  int32_t cond = r[SG_NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) r[i] += FpInvCfg::M30[i] & cond;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) r[i] = (r[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < SG_NL - 1; ++i) {
    r[i + 1] += r[i] >> 30;
    r[i] &= M30;
  }
  cond = r[SG_NL - 1] >> 31;
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) r[i] += FpInvCfg::M30[i] & cond;
#pragma unroll
  for (int i = 0; i < SG_NL - 1; ++i) {
    r[i + 1] += r[i] >> 30;
    r[i] &= M30;
  }
}

// x (signed-30 limbs of a value in [0, p)) <- x^-1 mod p; 0 maps to 0
BH_HD void sg_inverse(int32_t* x) {
  int32_t d[SG_NL], e[SG_NL], f[SG_NL], g[SG_NL];
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) {
    d[i] = 0;
    e[i] = 0;
    f[i] = FpInvCfg::M30[i];
    g[i] = x[i];
  }
  e[0] = 1;
  int32_t zeta = -1;  // delta = 1/2
  for (int it = 0; it < SG_MAX_BATCHES; ++it) {
    SgT t;
    zeta = sg_divsteps30(zeta, (uint32_t)f[0], (uint32_t)g[0], t);
    sg_update_de(d, e, t);
    sg_update_fg(f, g, t);
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < SG_NL; ++i) nz |= g[i];
    if (nz == 0) break;
  }
  sg_normalize(d, f[SG_NL - 1]);
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) x[i] = d[i];
}

// 14 x 29-bit limbs (a value < 2^390) <-> 13 x 30-bit limbs
BH_HD void sg_from29(const uint32_t* a, int32_t* s) {
  uint64_t acc = 0;
  int bits = 0, j = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    acc |= (uint64_t)a[i] << bits;
    bits += 29;
    if (bits >= 30 && j < SG_NL) {
      s[j++] = (int32_t)(acc & 0x3fffffffu);
      acc >>= 30;
      bits -= 30;
    }
  }
  while (j < SG_NL) {
    s[j++] = (int32_t)(acc & 0x3fffffffu);
    acc >>= 30;
  }
}
BH_HD void sg_to29(const int32_t* s, uint32_t* a) {
  uint64_t acc = 0;
  int bits = 0, j = 0;
#pragma unroll
  for (int i = 0; i < SG_NL; ++i) {
    acc |= (uint64_t)(uint32_t)s[i] << bits;
    bits += 30;
    while (bits >= 29 && j < 14) {
      a[j++] = (uint32_t)(acc & 0x1fffffffu);
      acc >>= 29;
      bits -= 29;
    }
  }
  while (j < 14) {
    a[j++] = (uint32_t)(acc & 0x1fffffffu);
    acc >>= 29;
  }
}

}  // namespace bh
