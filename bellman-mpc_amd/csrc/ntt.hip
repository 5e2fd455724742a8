// Radix-2 NTT family over BLS12-381 DFr on gfx950 -- the device replacement for
// EvaluationDomain (reference src/domain.rs:42-190) and its best_fft /
// serial_fft / parallel_fft (domain.rs:261-372).
//
// Storage: every DFr value is 8 packed u32 words holding x*2^261 mod r (device
// Montgomery form), kept < 2r.  A transform is ceil(log m / 10) passes; each
// pass stages 1024 elements of one workgroup in LDS (9 limb planes, 36 KB),
// runs up to 10 radix-2 stages there and writes back:
//   DIF (Gentleman-Sande): natural order in  -> bit-reversed order out
//   DIT (Cooley-Tukey)   : bit-reversed in   -> natural order out
// The reference's natural->natural fft is therefore `permute + DIT`, and the
// Groth16 H pipeline (prover.rs:210-231) runs DIF for every inverse transform
// and DIT for every forward one, so no permutation pass is ever needed there;
// the coset factors g^i (distribute_powers, domain.rs:101-113), m^-1
// (domain.rs:88-98) and 1/Z(g) (domain.rs:139-151) are fused into the pass
// that stores the data, indexed by the element's natural index.
#include "ntt.h"
#include "ntt_common.cuh"
#include "msm.h"  // scalars_prepare (one-element epilogue)

namespace bh {

static constexpr int NTT_LG_E = 10;
static constexpr int NTT_E = 1 << NTT_LG_E;  // elements per workgroup
static constexpr int NTT_T = 256;   // threads per workgroup

struct PassArgs {
  int L, t, D;
  const uint32_t* lv;       // per-level twiddles, 9 limbs: lv[2^v + x] = omega_{2^(v+1)}^x, x < 2^v
  const uint32_t* src;      // loads come from src (the first pass may run out of place)
  const uint32_t* post_lo;  // optional post-scale tables
  const uint32_t* post_hi;
  int post_lo_bits;
  NttEpilogue epi;          // what the storing pass writes
};

// ---- limb-wise (carry-free) butterfly arithmetic.  A value handed to fe_mul needs neither
// normalised limbs nor a reduced value: with limbs < 2^31.4 against a twiddle's normalised limbs
// a column holds 9 products < 2^60.4 plus 8 m*p products < 2^58 (< 2^63.8 with the carry), and
// an operand < 12r keeps the product < 2r (12 r^2 < 2^261 r).  So the sums and differences that
// only feed a product skip the carry chain (1-2 VALU per limb instead of 3-4).
// K*r with every limb below the top >= J*(2^29-1), i.e. >= a sum of J normalised limbs: J*2^29
// added to limb i is J taken from limb i+1 (the value is unchanged)
template <uint32_t K, uint32_t J>
struct FrBias {
  struct L { uint32_t v[9]; };
  static constexpr L make() {
    L l{};
    for (int i = 0; i < 9; i++) {
      int64_t c = KP<FrCfg, K>::value.v[i];
      if (i < 8) c += (int64_t)J << 29;
      if (i > 0) c -= J;
      l.v[i] = (uint32_t)c;
    }
    return l;
  }
  static constexpr L value = make();
};
__device__ __forceinline__ DFr lw_add(const DFr& a, const DFr& b) {
  DFr r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + b.v[l];
  return r;
}
// a + K*r - b limb-wise; b's limbs must be sums of at most J normalised limbs (and its top limb
// at most K*r's minus J: b < (K/2) r for the callers' bounds)
template <uint32_t K, uint32_t J>
__device__ __forceinline__ DFr lw_sub(const DFr& a, const DFr& b) {
  DFr r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = a.v[l] + (FrBias<K, J>::value.v[l] - b.v[l]);
  return r;
}
// carry propagation: the same value in normalised limbs (input limbs < 2^31)
__device__ __forceinline__ DFr lw_norm(const DFr& a) {
  DFr r;
  uint32_t c = 0;
#pragma unroll
  for (int l = 0; l < 9; l++) {
    const uint32_t s = a.v[l] + c;
    r.v[l] = l < 8 ? (s & FrCfg::MASK) : s;
    c = s >> FrCfg::BITS;
  }
  return r;
}

// x < 2^261 with normalised limbs below the top one -> x - q*r < 2r, one pass instead of a chain
// of conditional subtractions (fe_csub 16, 8, 4, 2: ~40 VALU each).  r = r8 * 2^232 + r_low with
// 0 < r_low < 2^232 and x < (x8 + 1) * 2^232, so q = floor(x8 / (r8 + 1)) gives q*r <= x and
// x - q*r < (r8 + 1 + q) * 2^232 < 2r (q < 2^29 / r8 = 70).  The quotient comes from one FP64
// fma, exact: (x8 + 1/2) / (r8 + 1) is at least 1/(2(r8 + 1)) ~ 6.6e-8 away from an integer,
// far beyond the product's rounding (< 71 * 2^-52).
__device__ __forceinline__ DFr fr_qreduce(const DFr& x) {
  constexpr double inv = 1.0 / (double)(FrCfg::P[8] + 1u);
  const uint32_t q = (uint32_t)__builtin_fma((double)x.v[8], inv, 0.5 * inv);
  DFr r;
  int64_t c = 0;
#pragma unroll
  for (int l = 0; l < 9; l++) {
    const int64_t t = (int64_t)x.v[l] + c - (int64_t)((uint64_t)q * FrCfg::P[l]);
    r.v[l] = l < 8 ? ((uint32_t)t & FrCfg::MASK) : (uint32_t)t;
    c = t >> FrCfg::BITS;  // arithmetic
  }
  return r;
}

// global element index of (group g, position k) for a DIF pass at stages t..t+D-1
__device__ __forceinline__ uint32_t dif_index(const PassArgs& a, uint32_t g, uint32_t k) {
  const uint32_t s = 1u << (a.L - a.t - a.D);
  const uint32_t lo = g & (s - 1), hi = g >> (a.L - a.t - a.D);
  return (hi << (a.L - a.t)) + k * s + lo;
}
// ... for a DIT pass at stages t..t+D-1 (half sizes 2^t .. 2^(t+D-1))
__device__ __forceinline__ uint32_t dit_index(const PassArgs& a, uint32_t g, uint32_t k) {
  const uint32_t lo = g & ((1u << a.t) - 1), hi = g >> a.t;
  return (hi << (a.t + a.D)) + (k << a.t) + lo;
}

// Twiddles: the butterfly of global stage u with in-level offset x uses omega_{2h}^x where h is
// the stage's pair distance (DIT: h = 2^u, x = (k_low << t) + lo; DIF: h = 2^(L-u-1),
// x = k_low * 2^(L-t-D) + lo).  With one table per level, lanes with consecutive lo
// (consecutive groups) read consecutive entries, and the level-0 stage (h = 1: every twiddle
// is 1) multiplies by nothing.  Entries are stored as the 9 limbs (36 bytes, L2-resident at
// the sizes that matter): an unpack per twiddle (~25 VALU) costs more than the 4 extra bytes.
template <bool DIF>
__global__ void __launch_bounds__(NTT_T) k_ntt_pass(uint32_t* data, PassArgs a) {
  __shared__ uint32_t lds[9 * NTT_E];
  const int D = a.D;
  const int lgG = NTT_LG_E - D;
  const uint32_t G = 1u << lgG;              // groups per workgroup (index math by shifts)
  const uint32_t total_groups = 1u << (a.L - D);
  const uint32_t g0 = blockIdx.x * G;
  const uint32_t stride = DIF ? (1u << (a.L - a.t - D)) : (1u << a.t);  // distance between consecutive lo's
  const bool lo_fast = stride >= G;  // coalesce along lo (groups) or along k
  const uint32_t K = 1u << D;
  // ---- load
  for (uint32_t e = threadIdx.x; e < (uint32_t)NTT_E; e += NTT_T) {
    uint32_t gl, k;
    if (lo_fast) { gl = e & (G - 1); k = e >> lgG; } else { k = e & (K - 1); gl = e >> D; }
    const uint32_t g = g0 + gl;
    if (g >= total_groups) continue;
    const uint32_t idx = DIF ? dif_index(a, g, k) : dit_index(a, g, k);
    DFr x = ld_packed(a.src, idx);
    const uint32_t slot = (k << lgG) + gl;
#pragma unroll
    for (int l = 0; l < 9; l++) lds[l * NTT_E + slot] = x.v[l];
  }
  __syncthreads();
  // ---- D stages: one radix-2 stage when D is odd (DIF: the first, DIT: the first), then radix-4
  // steps of two stages each in registers (half the LDS round trips, barriers and index math of
  // two radix-2 stages, three twiddle loads instead of four; the same four products)
  const int lo_bits = DIF ? (a.L - a.t - D) : a.t;  // bits of the group index below the k digits
  auto twiddle = [&](int v, uint32_t klow, uint32_t g) -> DFr {  // omega_{2^(v+1)}^(klow * 2^lo_bits + lo)
    return ld_limbs(a.lv, (1u << v) + (klow << lo_bits) + (g & ((1u << lo_bits) - 1)));
  };
  int j = 0;
  if (D & 1) {
    const int u = a.t;  // global stage
    const int hb = DIF ? (D - 1) : 0;  // pair distance 2^hb in k
    const int v = DIF ? (a.L - u - 1) : u;  // twiddle level: omega_{2^(v+1)}
    for (uint32_t b = threadIdx.x; b < (uint32_t)(NTT_E / 2); b += NTT_T) {
      const uint32_t gl = b & (G - 1), r = b >> lgG;
      if (g0 + gl >= total_groups) continue;
      const uint32_t k = ((r >> hb) << (hb + 1)) | (r & ((1u << hb) - 1));
      const uint32_t k2 = k + (1u << hb);
      const uint32_t s0 = (k << lgG) + gl, s1 = (k2 << lgG) + gl;
      DFr x, y;
#pragma unroll
      for (int l = 0; l < 9; l++) { x.v[l] = lds[l * NTT_E + s0]; y.v[l] = lds[l * NTT_E + s1]; }
      DFr nx, ny;
      if (v == 0) {  // omega_2^0 = 1
        nx = fe_csub<FrCfg, 2>(fe_add<FrCfg>(x, y));
        ny = fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(x, y));
      } else {
        const DFr w = twiddle(v, k & ((1u << hb) - 1), g0 + gl);
        if (DIF) {
          nx = fe_csub<FrCfg, 2>(fe_add<FrCfg>(x, y));
          ny = fe_mul<FrCfg>(lw_sub<4, 1>(x, y), w);
        } else {  // lazy: no conditional subtraction inside a DIT pass (see the store)
          const DFr t = fe_mul<FrCfg>(y, w);
          nx = fe_add<FrCfg>(x, t);
          ny = fe_sub<FrCfg, 2>(x, t);
        }
      }
#pragma unroll
      for (int l = 0; l < 9; l++) { lds[l * NTT_E + s0] = nx.v[l]; lds[l * NTT_E + s1] = ny.v[l]; }
    }
    __syncthreads();
    j = 1;
  }
  for (; j < D; j += 2) {
    const int u = a.t + j;                  // first of the two global stages
    const int hb = DIF ? (D - 1 - j) : j;   // DIF: distances 2^hb, 2^(hb-1); DIT: 2^hb, 2^(hb+1)
    const int lo2 = DIF ? hb - 1 : hb;      // the two k bits are lo2 and lo2 + 1
    for (uint32_t b = threadIdx.x; b < (uint32_t)(NTT_E / 4); b += NTT_T) {
      const uint32_t gl = b & (G - 1), r = b >> lgG;
      const uint32_t g = g0 + gl;
      if (g >= total_groups) continue;
      const uint32_t k0 = ((r >> lo2) << (lo2 + 2)) | (r & ((1u << lo2) - 1));
      const uint32_t ks[4] = {k0, k0 + (1u << lo2), k0 + (2u << lo2), k0 + (3u << lo2)};
      DFr x[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t sl = (ks[q] << lgG) + gl;
#pragma unroll
        for (int l = 0; l < 9; l++) x[q].v[l] = lds[l * NTT_E + sl];
      }
      DFr y[4];
      if (DIF) {
        // stage u (distance 2^hb): (k0, k2), (k1, k3); stage u+1 (2^(hb-1)): (k0, k1), (k2, k3)
        const int v = a.L - u - 1, v2 = v - 1;
        const uint32_t m1 = (1u << hb) - 1, m2 = (1u << (hb - 1)) - 1;
        const DFr wa0 = twiddle(v, ks[0] & m1, g), wa1 = twiddle(v, ks[1] & m1, g);
        // inputs < 2r (normalised); the sums feeding y0/y1 and the differences feeding the
        // products stay limb-wise (see lw_sub), y0/y2 are carried and reduced back below 2r
        const DFr s02 = lw_add(x[0], x[2]), s13 = lw_add(x[1], x[3]);  // < 4r, limbs < 2^30
        const DFr u2 = fe_mul<FrCfg>(lw_sub<4, 1>(x[0], x[2]), wa0);   // < 2r
        const DFr u3 = fe_mul<FrCfg>(lw_sub<4, 1>(x[1], x[3]), wa1);
        y[0] = fr_qreduce(fe_add<FrCfg>(s02, s13));                  // < 8r
        y[2] = fe_csub<FrCfg, 2>(fe_add<FrCfg>(u2, u3));                // < 4r
        if (v2 == 0) {  // omega_2^0 = 1
          y[1] = fr_qreduce(lw_norm(lw_sub<8, 2>(s02, s13)));           // < 12r
          y[3] = fr_qreduce(lw_norm(lw_sub<4, 1>(u2, u3)));             // < 6r
        } else {
          const DFr wb = twiddle(v2, ks[0] & m2, g);
          y[1] = fe_mul<FrCfg>(lw_sub<8, 2>(s02, s13), wb);  // operand < 12r, limbs < 2^31.4
          y[3] = fe_mul<FrCfg>(lw_sub<4, 1>(u2, u3), wb);
        }
      } else {
        // stage u (distance 2^hb): (k0, k1), (k2, k3); stage u+1 (2^(hb+1)): (k0, k2), (k1, k3).
        // Lazy reduction: a DIT stage adds a product (< 2r) to, or subtracts it (+2r) from, a value
        // < B, so values stay < 2r(D+1) <= 22r < 2^261 in the 9 limbs, and a Montgomery product
        // of such a value with a twiddle (< r) still ends < 2r (22 r^2 < 2^261 r); the storing
        // pass reduces.  v == 0 only occurs at global stage 0, on freshly loaded values (< 2r).
        const int v = u, v2 = u + 1;
        const uint32_t m1 = (1u << hb) - 1, m2 = (2u << hb) - 1;
        // u0, u1 stay limb-wise (u1's top limb may wrap: it only reaches carried sums, whose
        // values are non-negative), u2, u3 are operands of products (limb-wise, < 26r)
        DFr a0, a1, p2, p3;
        if (v == 0) {  // omega_2^0 = 1
          a0 = fe_csub<FrCfg, 2>(fe_add<FrCfg>(x[0], x[1]));
          a1 = fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(x[0], x[1]));
          p2 = fe_csub<FrCfg, 2>(fe_add<FrCfg>(x[2], x[3]));
          p3 = fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(x[2], x[3]));
        } else {
          const DFr wa = twiddle(v, ks[0] & m1, g);
          const DFr t0 = fe_mul<FrCfg>(x[1], wa), t1 = fe_mul<FrCfg>(x[3], wa);
          a0 = lw_add(x[0], t0);
          a1 = lw_sub<2, 1>(x[0], t0);
          p2 = lw_add(x[2], t1);
          p3 = lw_sub<4, 1>(x[2], t1);
        }
        const DFr wb0 = twiddle(v2, ks[0] & m2, g), wb1 = twiddle(v2, ks[1] & m2, g);
        const DFr s0 = fe_mul<FrCfg>(p2, wb0), s1 = fe_mul<FrCfg>(p3, wb1);
        y[0] = fe_add<FrCfg>(a0, s0);
        y[2] = lw_norm(lw_sub<2, 1>(a0, s0));
        y[1] = fe_add<FrCfg>(a1, s1);
        y[3] = lw_norm(lw_sub<2, 1>(a1, s1));
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t sl = (ks[q] << lgG) + gl;
#pragma unroll
        for (int l = 0; l < 9; l++) lds[l * NTT_E + sl] = y[q].v[l];
      }
    }
    __syncthreads();
  }
  // ---- store (+ optional post-scale by natural index, + the fused epilogue)
  for (uint32_t e = threadIdx.x; e < (uint32_t)NTT_E; e += NTT_T) {
    uint32_t gl, k;
    if (lo_fast) { gl = e & (G - 1); k = e >> lgG; } else { k = e & (K - 1); gl = e >> D; }
    const uint32_t g = g0 + gl;
    if (g >= total_groups) continue;
    const uint32_t idx = DIF ? dif_index(a, g, k) : dit_index(a, g, k);
    const uint32_t slot = (k << lgG) + gl;
    DFr x;
#pragma unroll
    for (int l = 0; l < 9; l++) x.v[l] = lds[l * NTT_E + slot];
    const uint32_t nat = DIF ? brev(idx, a.L) : idx;
    if (a.post_hi) x = fe_mul<FrCfg>(x, pow_factor(a.post_lo, a.post_hi, a.post_lo_bits, nat));  // < 2r
    if (a.epi.kind == NttEpilogue::AB_MINUS_C) {  // x = c (< 22r): pa[idx] = (pa[idx] * pb[idx] - x) * k
      const DFr p = fe_mul<FrCfg>(ld_packed(a.epi.pa, idx), ld_packed(a.epi.pb, idx));
      st_packed(a.epi.pa, idx, fe_mul<FrCfg>(fe_sub<FrCfg, 32>(p, x), ld_limbs(a.epi.k, 0)));
    } else if (a.epi.kind == NttEpilogue::SCALARS) {  // canonical scalar at the natural index
      if (nat < a.epi.n_out) {
        uint32_t w8[8];
        fe_pack<FrCfg>(fe_csub<FrCfg, 1>(fe_from_mont<FrCfg>(x)), w8);  // x * 2^-261 <= r: one subtraction
        uint4* q = reinterpret_cast<uint4*>(a.epi.out + (size_t)nat * 8);
        q[0] = make_uint4(w8[0], w8[1], w8[2], w8[3]);
        q[1] = make_uint4(w8[4], w8[5], w8[6], w8[7]);
      }
    } else {
      if (!DIF && !a.post_hi) x = fr_qreduce(x);  // a lazily reduced DIT value (< 22r) -> < 2r for the packed form
      st_packed(data, idx, x);
    }
  }
}

// out[bitrev(i)] = in[i] * factor(i)   (factor optional)
__global__ void __launch_bounds__(256) k_permute(const uint32_t* in, uint32_t* out, int L, const uint32_t* lo,
                                                 const uint32_t* hi, int lo_bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1u << L)) return;
  DFr x = ld_packed(in, i);
  if (hi) x = fe_mul<FrCfg>(x, pow_factor(lo, hi, lo_bits, i));
  st_packed(out, brev(i, L), x);
}

// a[i] *= factor(i)  or a[i] *= c (constant, unpacked) when hi == nullptr.  rev_L >= 0: a holds
// 2^rev_L elements in bit-reversed order, so the factor of position i is factor(brev(i))
__global__ void __launch_bounds__(256) k_scale(uint32_t* a, uint32_t n, const uint32_t* lo, const uint32_t* hi,
                                               int lo_bits, const uint32_t* c, int rev_L) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DFr x = ld_packed(a, i);
  const DFr f = hi ? pow_factor(lo, hi, lo_bits, rev_L >= 0 ? brev(i, rev_L) : i) : ld_limbs(c, 0);
  st_packed(a, i, fe_mul<FrCfg>(x, f));
}

// unpacked table times a constant: out[j] = in[j] * k (< r), j < n  (a post-scale table k * g^(i*e)
// from the domain's g^(+-i) tables, built on the stream that uses it)
__global__ void __launch_bounds__(256) k_table_scale(uint32_t* out, const uint32_t* in, uint32_t n, FrConst k) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  DFr c;
#pragma unroll
  for (int l = 0; l < 9; l++) c.v[l] = k.v[l];
  const DFr x = fe_csub<FrCfg, 1>(fe_mul<FrCfg>(ld_limbs(in, j), c));
#pragma unroll
  for (int l = 0; l < 9; l++) out[(size_t)j * 9 + l] = x.v[l];
}

// a = a * k - b  (sub_assign of two domains whose pending constant factors differ)
__global__ void __launch_bounds__(256) k_scale_sub(uint32_t* a, const uint32_t* b, uint32_t n, FrConst k) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DFr c;
#pragma unroll
  for (int l = 0; l < 9; l++) c.v[l] = k.v[l];
  const DFr x = fe_mul<FrCfg>(ld_packed(a, i), c);
  st_packed(a, i, fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(x, ld_packed(b, i))));
}

// op 0: a *= b ; op 1: a -= b ; op 2: out = (a*b - c) * k   (H pipeline, prover.rs:221-225)
__global__ void __launch_bounds__(256) k_pointwise(uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t n,
                                                   int op, const uint32_t* k) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DFr x = ld_packed(a, i), y = ld_packed(b, i);
  DFr r;
  if (op == 0) r = fe_mul<FrCfg>(x, y);
  else if (op == 1) r = fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(x, y));
  else {
    DFr z = ld_packed(c, i);
    r = fe_mul<FrCfg>(fe_sub<FrCfg, 2>(fe_mul<FrCfg>(x, y), z), ld_limbs(k, 0));
  }
  st_packed(a, i, r);
}

// format conversion: out = in * C (C raw unpacked, 9 limbs) [* reduce to canonical]
__global__ void __launch_bounds__(256) k_fr_convert(const uint32_t* in, uint32_t* out, uint32_t n, FrConst C,
                                                    int reduce) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DFr x = ld_packed(in, i);
  DFr c;
#pragma unroll
  for (int l = 0; l < 9; l++) c.v[l] = C.v[l];
  DFr r = fe_mul<FrCfg>(x, c);
  if (reduce) r = fe_csub<FrCfg, 1>(r);  // a product is < 2r: one subtraction makes it canonical
  st_packed(out, i, r);
}

// tab[j] = lo[j & mask] * hi[j >> bits] for j < n  (builds twiddle tables on device)
__global__ void __launch_bounds__(256) k_expand_table(uint32_t* tab, uint32_t n, const uint32_t* lo,
                                                      const uint32_t* hi, int lo_bits) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  DFr x = pow_factor(lo, hi, lo_bits, j);
  x = fe_csub<FrCfg, 1>(x);
#pragma unroll
  for (int l = 0; l < 9; l++) tab[(size_t)j * 9 + l] = x.v[l];
}

// per-level twiddles from the full table: lv[2^v + x] = omega^(x * 2^(L-1-v)) (9 limbs), v < L
__global__ void __launch_bounds__(256) k_level_table(uint32_t* lv, int L, const uint32_t* tw) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e == 0 || e >= (1u << L)) return;
  const int v = 31 - __clz(e);
  const uint32_t x = e - (1u << v);
  const DFr w = ld_limbs(tw, (size_t)x << (L - 1 - v));
#pragma unroll
  for (int l = 0; l < 9; l++) lv[(size_t)e * 9 + l] = w.v[l];
}

// ------------------------------------------------------------------ host side
static inline unsigned nb(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

void launch_ntt(uint32_t* d, int L, bool dif, const uint32_t* lv, const uint32_t* post_lo, const uint32_t* post_hi,
                int post_lo_bits, hipStream_t st, const uint32_t* src, const NttEpilogue& epi) {
  if (L == 0) {  // one element: a copy, the post-scale and the epilogue
    if (src && src != d) hipMemcpyAsync(d, src, 32, hipMemcpyDeviceToDevice, st);
    if (post_hi) hipLaunchKernelGGL(k_scale, dim3(1), dim3(256), 0, st, d, 1u, post_lo, post_hi, post_lo_bits,
                                    (const uint32_t*)nullptr, -1);
    if (epi.kind == NttEpilogue::AB_MINUS_C)
      hipLaunchKernelGGL(k_pointwise, dim3(1), dim3(256), 0, st, epi.pa, epi.pb, (const uint32_t*)d, 1u, 2, epi.k);
    else if (epi.kind == NttEpilogue::SCALARS && epi.n_out)
      scalars_prepare(d, epi.out, epi.n_out, 2, 0, st);
    return;
  }
  // stages per pass: even where the total allows (a pass of odd depth runs one radix-2 stage,
  // 330 instructions per butterfly against 293 in the radix-4 steps): 2^22 = 8 + 8 + 6, not 8 + 7 + 7
  const int passes = (L + 9) / 10;
  int Ds[8];
  const int pairs = L / 2;
  for (int p = 0; p < passes; p++) Ds[p] = 2 * (pairs / passes + (p < pairs % passes ? 1 : 0));
  if (L & 1) {  // one odd pass: the shallowest one takes the extra stage
    int q = passes - 1;
    for (int p = passes - 1; p >= 0; p--)
      if (Ds[p] < Ds[q]) q = p;
    Ds[q] += 1;
  }
  int t = 0;
  for (int p = 0; p < passes; p++) {
    PassArgs a;
    a.L = L; a.t = t; a.D = Ds[p]; a.lv = lv;
    const bool last = (p == passes - 1);
    a.src = (p == 0 && src) ? src : d;
    a.post_lo = last ? post_lo : nullptr;
    a.post_hi = last ? post_hi : nullptr;
    a.post_lo_bits = post_lo_bits;
    a.epi = last ? epi : NttEpilogue();
    const size_t groups = (size_t)1 << (L - a.D);
    const size_t G = NTT_E >> a.D;
    const unsigned blocks = (unsigned)((groups + G - 1) / G);
    if (dif) hipLaunchKernelGGL(k_ntt_pass<true>, dim3(blocks), dim3(NTT_T), 0, st, d, a);
    else hipLaunchKernelGGL(k_ntt_pass<false>, dim3(blocks), dim3(NTT_T), 0, st, d, a);
    t += a.D;
  }
}

void launch_permute(const uint32_t* in, uint32_t* out, int L, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                    hipStream_t st) {
  hipLaunchKernelGGL(k_permute, dim3(nb((size_t)1 << L, 256)), dim3(256), 0, st, in, out, L, lo, hi, lo_bits);
}
void launch_scale(uint32_t* a, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits, const uint32_t* c,
                  hipStream_t st, int rev_L) {
  if (!n) return;
  hipLaunchKernelGGL(k_scale, dim3(nb(n, 256)), dim3(256), 0, st, a, (uint32_t)n, lo, hi, lo_bits, c, rev_L);
}
void launch_table_scale(uint32_t* out, const uint32_t* in, size_t n, const FrConst& k, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_table_scale, dim3(nb(n, 256)), dim3(256), 0, st, out, in, (uint32_t)n, k);
}
void launch_scale_sub(uint32_t* a, const uint32_t* b, size_t n, const FrConst& k, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_scale_sub, dim3(nb(n, 256)), dim3(256), 0, st, a, b, (uint32_t)n, k);
}
void launch_pointwise(uint32_t* a, const uint32_t* b, const uint32_t* c, size_t n, int op, const uint32_t* k,
                      hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_pointwise, dim3(nb(n, 256)), dim3(256), 0, st, a, b, c, (uint32_t)n, op, k);
}
void launch_fr_convert(const uint32_t* in, uint32_t* out, size_t n, const FrConst& C, int reduce, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_fr_convert, dim3(nb(n, 256)), dim3(256), 0, st, in, out, (uint32_t)n, C, reduce);
}
void launch_expand_table(uint32_t* tab, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                         hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_expand_table, dim3(nb(n, 256)), dim3(256), 0, st, tab, (uint32_t)n, lo, hi, lo_bits);
}
void launch_level_table(uint32_t* lv, int L, const uint32_t* tw, hipStream_t st) {
  if (L < 1) return;
  hipLaunchKernelGGL(k_level_table, dim3(nb((size_t)1 << L, 256)), dim3(256), 0, st, lv, L, tw);
}

void ntt_kernels(std::vector<KernInfo>& v) {
  v.push_back({"k_ntt_pass<DIF>", (const void*)k_ntt_pass<true>, NTT_T, 0});
  v.push_back({"k_ntt_pass<DIT>", (const void*)k_ntt_pass<false>, NTT_T, 0});
}

}  // namespace bh
