// C ABI implementation: context, bases (SRS), multiexp, EvaluationDomain,
// Parameters and the Groth16 prover core.  See include/bellman_hip.h for the
// reference interface each entry point replaces.
#include <cstdlib>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <chrono>
#include <thread>

#include "api_internal.h"
#include "dist_h.h"

using namespace bh;

namespace bh {

static thread_local hipError_t g_last_hip = hipSuccess;
void set_last_hip_error(hipError_t e) { g_last_hip = e; }

// ------------------------------------------------------------------ Fr host <-> device
static const Fr& fr_two261() {
  static Fr v = [] {
    uint64_t two[4] = {2, 0, 0, 0};
    uint64_t e[1] = {261};
    return pow_vartime(from_int<4>(two), e, 1);
  }();
  return v;
}
static const Fr& fr_two261_inv() {
  static Fr v = inv(fr_two261());
  return v;
}
static inline void split29(const uint64_t raw[4], uint32_t out[9]) {
  for (int i = 0; i < 9; i++) {
    int bit = 29 * i, w = bit >> 6, sh = bit & 63;
    uint64_t lo = raw[w] >> sh;
    if (sh > 35 && w + 1 < 4) lo |= raw[w + 1] << (64 - sh);
    out[i] = (uint32_t)(lo & 0x1fffffffu);
  }
}
void fr_to_dev_limbs(const Fr& x, uint32_t out[9]) {
  uint64_t raw[4];
  to_int(mul(x, fr_two261()), raw);
  split29(raw, out);
}
void fr_to_dev_packed(const Fr& x, uint32_t out[8]) {
  uint64_t raw[4];
  to_int(mul(x, fr_two261()), raw);
  for (int i = 0; i < 4; i++) { out[2 * i] = (uint32_t)raw[i]; out[2 * i + 1] = (uint32_t)(raw[i] >> 32); }
}
Fr fr_from_dev_packed(const uint32_t in[8]) {
  uint64_t raw[4];
  for (int i = 0; i < 4; i++) raw[i] = (uint64_t)in[2 * i] | ((uint64_t)in[2 * i + 1] << 32);
  // raw may be in [r, 2r): reduce
  if (geq_p<4>(raw)) sub_p<4>(raw);
  return mul(from_int<4>(raw), fr_two261_inv());
}

// ------------------------------------------------------------------ device point conversion
// canonical packed coordinates -> device Montgomery packed; optional on-curve check
// G1 (G1F, curve.cuh): the same in G1's representation
__global__ void __launch_bounds__(256) k_points_to_dev_g1(uint32_t* pts, size_t n, int check, uint32_t* bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  using F = G1F;
  F::T r2;
#pragma unroll
  for (int k = 0; k < F::Cf::N; k++) r2.v[k] = F::Cf::R2[k];
  F::T c[2];
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    uint32_t* w = pts + (i * 2 + k) * 12;
#pragma unroll
    for (int l = 0; l < 12; l++) nz |= w[l];
    c[k] = F::reduce(F::mul(F::unpack(w), r2));
    F::pack(c[k], w);
  }
  if (check && nz) {  // (0,0) encodes the identity (never on the curve), skip it
    const F::T four = F::add(F::add(F::one(), F::one()), F::add(F::one(), F::one()));
    const F::T lhs = F::sqr(c[1]);
    const F::T rhs = F::add(F::mul(F::sqr(c[0]), c[0]), four);
    if (!F::is_zero(F::template sub<8>(lhs, rhs))) atomicOr(bad, 1u);
  }
}

template <bool G2>
__global__ void __launch_bounds__(256) k_points_to_dev(uint32_t* pts, size_t n, int check, uint32_t* bad) {
  static_assert(G2, "G1 points: k_points_to_dev_g1");
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int NC = G2 ? 4 : 2;  // DFp coordinates per point
  DFp r2;
#pragma unroll
  for (int k = 0; k < 14; k++) r2.v[k] = FpCfg::R2[k];
  DFp c[NC];
#pragma unroll
  for (int k = 0; k < NC; k++) {
    DFp x = fe_unpack<FpCfg>(pts + (i * NC + k) * 12);
    c[k] = fe_reduce_full<FpCfg>(fe_mul<FpCfg>(x, r2));
    fe_pack<FpCfg>(c[k], pts + (i * NC + k) * 12);
  }
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < NC; k++)
#pragma unroll
    for (int l = 0; l < 14; l++) nz |= c[k].v[l];
  if (check && nz) {  // (0,0) encodes the identity (never on the curve), skip it
    DFp four = fe_add<FpCfg>(fe_add<FpCfg>(fe_one<FpCfg>(), fe_one<FpCfg>()),
                            fe_add<FpCfg>(fe_one<FpCfg>(), fe_one<FpCfg>()));
    bool ok;
    if (!G2) {
      DFp lhs = fe_sqr<FpCfg>(c[1]);
      DFp rhs = fe_add<FpCfg>(fe_mul<FpCfg>(fe_sqr<FpCfg>(c[0]), c[0]), four);
      ok = fe_is_zero<FpCfg>(fe_sub<FpCfg, 8>(lhs, rhs));
    } else {
      DFp2 x{c[0], c[1]}, y{c[2], c[3]};
      DFp2 lhs = Fp2Ops::sqr(y);
      DFp2 x3 = Fp2Ops::mul(Fp2Ops::sqr(x), x);
      DFp2 rhs{fe_add<FpCfg>(x3.c0, four), fe_add<FpCfg>(x3.c1, four)};
      DFp2 d = Fp2Ops::sub<16>(lhs, rhs);
      ok = Fp2Ops::is_zero(d);
    }
    if (!ok) atomicOr(bad, 1u);
  }
}

// Prime-order subgroup check of Parameters::read(checked) (G1Affine/G2Affine::
// from_uncompressed reject points that are not torsion-free): [r]P == O by a
// double-and-add over the bits of r in XYZZ coordinates.  Runs on the device-form points.
template <bool G2>
__global__ void __launch_bounds__(256) k_subgroup_check(const uint32_t* pts, size_t n, uint32_t* bad) {
  using C = typename std::conditional<G2, G2Ops, G1Ops>::type;
  using F = typename std::conditional<G2, Fp2Ops, G1F>::type;
  constexpr int PW = F::PACKED_WORDS;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* p = pts + i * 2 * PW;
  uint32_t nz = 0;
  for (int k = 0; k < 2 * PW; k++) nz |= p[k];
  if (!nz) return;  // the identity encoding
  typename C::A a;
  a.x = F::unpack(p);
  a.y = F::unpack(p + PW);
  // r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001, LE words
  constexpr uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                             0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  typename C::P acc = C::from_affine(a);
  for (int bit = 253; bit >= 0; bit--) {  // bit 254 is the leading one
    acc = C::dbl(acc);
    if ((R[bit >> 5] >> (bit & 31)) & 1u) acc = C::madd(acc, a);
  }
  if (!C::is_identity(acc)) atomicOr(bad, 2u);
}

// ------------------------------------------------------------------ SRS
// host affine points -> device (packed canonical words, then device conversion)
bh_status srs_upload_affine(bh_ctx* ctx, int group, const void* host_pts, size_t n, bh_srs* out) {
  out->ctx = ctx;
  out->group = group;
  out->n = n;
  out->identity_idx.clear();
  const int words = group == BH_G1 ? 24 : 48;
  std::vector<uint32_t> w((size_t)n * words);
  for (size_t i = 0; i < n; i++) {
    uint32_t* d = &w[i * words];
    if (group == BH_G1) {
      const AffinePt<Fp>& a = reinterpret_cast<const AffinePt<Fp>*>(host_pts)[i];
      if (a.infinity) { out->identity_idx.push_back(i); memset(d, 0, words * 4); continue; }
      uint64_t raw[6];
      to_int(a.x, raw); memcpy(d, raw, 48);
      to_int(a.y, raw); memcpy(d + 12, raw, 48);
    } else {
      const AffinePt<Fp2>& a = reinterpret_cast<const AffinePt<Fp2>*>(host_pts)[i];
      if (a.infinity) { out->identity_idx.push_back(i); memset(d, 0, words * 4); continue; }
      uint64_t raw[6];
      to_int(a.x.c0, raw); memcpy(d, raw, 48);
      to_int(a.x.c1, raw); memcpy(d + 12, raw, 48);
      to_int(a.y.c0, raw); memcpy(d + 24, raw, 48);
      to_int(a.y.c1, raw); memcpy(d + 36, raw, 48);
    }
  }
  BH_TRY_HIP(out->pts.alloc(std::max<size_t>(n, 1) * words * 4));
  if (n) {
    BH_TRY_HIP(hipMemcpyAsync(out->pts.p, w.data(), n * words * 4, hipMemcpyHostToDevice, ctx->stream));
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (group == BH_G1)
      hipLaunchKernelGGL(k_points_to_dev_g1, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(), n,
                         0, (uint32_t*)nullptr);
    else
      hipLaunchKernelGGL(k_points_to_dev<true>, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(), n,
                         0, (uint32_t*)nullptr);
    BH_TRY_HIP(hipGetLastError());
    BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BH_OK;
}

// parse n uncompressed encodings; returns BH_ERR_INVALID_ENCODING / BH_ERR_NOT_ON_CURVE
bh_status srs_from_bytes(bh_ctx* ctx, int group, const uint8_t* bytes, size_t n, int checked,
                                bool reject_identity, bh_srs* out) {
  const size_t pb = group == BH_G1 ? 96 : 192;
  const int words = group == BH_G1 ? 24 : 48;
  out->ctx = ctx;
  out->group = group;
  out->n = n;
  out->identity_idx.clear();
  std::vector<uint32_t> w((size_t)n * words);
  for (size_t i = 0; i < n; i++) {
    const uint8_t* b = bytes + i * pb;
    uint32_t* d = &w[i * words];
    const uint8_t flags = b[0] >> 5;
    if ((flags & 0x4) || (flags & 0x1)) return BH_ERR_INVALID_ENCODING;
    if (flags & 0x2) {
      for (size_t k = 0; k < pb; k++)
        if ((k == 0 ? (b[0] & 0x1F) : b[k]) != 0) return BH_ERR_INVALID_ENCODING;
      if (reject_identity) return BH_ERR_INVALID_ENCODING;
      out->identity_idx.push_back(i);
      memset(d, 0, words * 4);
      continue;
    }
    // each 48-byte big-endian field element -> 12 LE words, canonical check
    const int nf = group == BH_G1 ? 2 : 4;
    for (int f = 0; f < nf; f++) {
      // G2 wire order: x.c1, x.c0, y.c1, y.c0 ; device order: x.c0, x.c1, y.c0, y.c1
      int dst = group == BH_G1 ? f : (f ^ 1);
      const uint8_t* src = b + 48 * f;
      uint64_t raw[6] = {0};
      for (int k = 0; k < 48; k++) {
        uint8_t byte = src[k];
        if (f == 0 && k == 0) byte &= 0x1F;
        raw[(47 - k) / 8] |= (uint64_t)byte << (8 * ((47 - k) % 8));
      }
      if (geq_p<6>(raw)) return BH_ERR_INVALID_ENCODING;
      memcpy(d + 12 * dst, raw, 48);
    }
  }
  BH_TRY_HIP(out->pts.alloc(std::max<size_t>(n, 1) * words * 4));
  if (n) {
    DevBuf bad;
    BH_TRY_HIP(bad.alloc(4));
    BH_TRY_HIP(hipMemsetAsync(bad.p, 0, 4, ctx->stream));
    BH_TRY_HIP(hipMemcpyAsync(out->pts.p, w.data(), n * words * 4, hipMemcpyHostToDevice, ctx->stream));
    unsigned blocks = (unsigned)((n + 255) / 256);
    if (group == BH_G1)
      hipLaunchKernelGGL(k_points_to_dev_g1, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(), n,
                         checked, bad.as<uint32_t>());
    else
      hipLaunchKernelGGL(k_points_to_dev<true>, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(), n,
                         checked, bad.as<uint32_t>());
    BH_TRY_HIP(hipGetLastError());
    if (checked) {
      if (group == BH_G1)
        hipLaunchKernelGGL(k_subgroup_check<false>, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(),
                           n, bad.as<uint32_t>());
      else
        hipLaunchKernelGGL(k_subgroup_check<true>, dim3(blocks), dim3(256), 0, ctx->stream, out->pts.as<uint32_t>(),
                           n, bad.as<uint32_t>());
      BH_TRY_HIP(hipGetLastError());
    }
    uint32_t hbad = 0;
    BH_TRY_HIP(hipMemcpyAsync(&hbad, bad.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
    if (hbad & 1u) return BH_ERR_NOT_ON_CURVE;
    if (hbad & 2u) return BH_ERR_NOT_IN_SUBGROUP;
  }
  return BH_OK;
}

// ------------------------------------------------------------------ MSM glue
static inline Fp fp_from_dev_limbs(const uint32_t* limbs14) {
  // unpacked 29-bit limbs (canonical) -> packed words -> host
  uint32_t words[12] = {0};
  for (int i = 0; i < 14; i++) {
    const int bit = 29 * i;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t v = (uint64_t)limbs14[i] << sh;
    words[wi] |= (uint32_t)v;
    if (wi + 1 < 12) words[wi + 1] |= (uint32_t)(v >> 32);
  }
  return fp_from_dev_words(words);
}

// G1 (G1F: 13 balanced 30-bit digits or 14 x 29-bit limbs, R = 2^(N*BITS)): a canonical
// coordinate's limbs (C::reduce) -> packed words -> host
Fp fp_from_dev_words_g1(const uint32_t* w) {
  using Cf = G1F::Cf;
  return fp_from_dev_words_r<Cf::N * Cf::BITS>(w);
}
Fp fp_from_dev_g1(const G1F::T& x) {
  using Cf = G1F::Cf;
  uint32_t words[12] = {0};
  int64_t carry = 0;
  for (int i = 0; i < Cf::N; i++) {  // (signed) digits -> unsigned BITS-bit limbs of the value in [0, p)
    const int64_t s = (int64_t)x.v[i] + carry;
    const uint32_t limb = (uint32_t)(s & (int64_t)Cf::MASK);
    carry = s >> Cf::BITS;
    const int bit = Cf::BITS * i;
    const int wi = bit >> 5, sh = bit & 31;
    const uint64_t v = (uint64_t)limb << sh;
    words[wi] |= (uint32_t)v;
    if (wi + 1 < 12) words[wi + 1] |= (uint32_t)(v >> 32);
  }
  return fp_from_dev_words_g1(words);
}

static Jac<Fp> g1_from_xyzz(const XYZZ<G1F>& p) {
  return xyzz_to_jac(fp_from_dev_g1(p.X), fp_from_dev_g1(p.Y), fp_from_dev_g1(p.ZZ), fp_from_dev_g1(p.ZZZ));
}
// window sums -> the multiexp (Horner over the Wb windows, c doublings each; multiexp.rs:244-249),
// or, for one shared bucket window, out[0] + 2^shift * out[1] (msm_back's split reduction)
Jac<Fp> combine_g1(const XYZZ<G1F>* ws, const MsmShape& sh) {
  const int shift = reduce_split_shift(sh, false);
  if (shift >= 0) {
    Jac<Fp> z = g1_from_xyzz(ws[1]);
    for (int k = 0; k < shift; k++) z = jac_dbl(z);
    z = jac_add(g1_from_xyzz(ws[0]), z);
    if (sh.bucket_shard() && sh.bk_lo) {  // + bk_lo * (plain sum of the range's buckets)
      const uint64_t k[1] = {sh.bk_lo};
      z = jac_add(z, jac_mul(g1_from_xyzz(ws[2]), k, 1));
    }
    return z;
  }
  Jac<Fp> acc = jac_identity<Fp>();
  for (int w = sh.Wb - 1; w >= 0; w--) {
    for (int k = 0; k < sh.c; k++) acc = jac_dbl(acc);
    acc = jac_add(acc, g1_from_xyzz(ws[w]));
  }
  return acc;
}
static inline bh::Fp2 fp2_from_dev(const DFp2& v) {
  return bh::Fp2{fp_from_dev_limbs(v.c0.v), fp_from_dev_limbs(v.c1.v)};
}
static Jac<bh::Fp2> g2_from_xyzz(const XYZZ<Fp2Ops>& p) {
  return xyzz_to_jac(fp2_from_dev(p.X), fp2_from_dev(p.Y), fp2_from_dev(p.ZZ), fp2_from_dev(p.ZZZ));
}
Jac<bh::Fp2> combine_g2(const XYZZ<Fp2Ops>* ws, const MsmShape& sh) {
  const int shift = reduce_split_shift(sh, true);
  if (shift >= 0) {
    Jac<bh::Fp2> z = g2_from_xyzz(ws[1]);
    for (int k = 0; k < shift; k++) z = jac_dbl(z);
    z = jac_add(g2_from_xyzz(ws[0]), z);
    if (sh.bucket_shard() && sh.bk_lo) {  // + bk_lo * (plain sum of the range's buckets)
      const uint64_t k[1] = {sh.bk_lo};
      z = jac_add(z, jac_mul(g2_from_xyzz(ws[2]), k, 1));
    }
    return z;
  }
  Jac<bh::Fp2> acc = jac_identity<bh::Fp2>();
  for (int w = sh.Wb - 1; w >= 0; w--) {
    for (int k = 0; k < sh.c; k++) acc = jac_dbl(acc);
    acc = jac_add(acc, g2_from_xyzz(ws[w]));
  }
  return acc;
}

static MsmTiming g_no_timing;

bh_status msm_g1_device(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint32_t* d_scalars, size_t n,
                        const int32_t* d_idx, Jac<Fp>* out, float* acc_ms) {
  if (n == 0) { *out = jac_identity<Fp>(); return BH_OK; }
  MsmShape sh = msm_shape(n, ctx->window_override);
  fit_segments<G1Ops>(sh, n);
  MsmTiming tm;
  if (acc_ms) { tm.ev_acc_begin = ctx->ev[14]; tm.ev_acc_end = ctx->ev[15]; }
  BH_TRY_HIP(msm_window_sums<G1Ops>(ctx->g1ws, ctx->stream, bases->pts.as<uint32_t>(), d_scalars, n, d_idx,
                                    (uint32_t)base_offset, sh, acc_ms ? &tm : nullptr));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  if (acc_ms) { float t = 0; if (hipEventElapsedTime(&t, tm.ev_acc_begin, tm.ev_acc_end) == hipSuccess) *acc_ms += t; }
  *out = combine_g1(ctx->g1ws.host_window_sums, sh);
  return BH_OK;
}
bh_status msm_g2_device(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint32_t* d_scalars, size_t n,
                        const int32_t* d_idx, Jac<bh::Fp2>* out, float* acc_ms) {
  if (n == 0) { *out = jac_identity<bh::Fp2>(); return BH_OK; }
  MsmShape sh = msm_shape(n, ctx->window_override);
  fit_segments<G2Ops>(sh, n);
  MsmTiming tm;
  if (acc_ms) { tm.ev_acc_begin = ctx->ev[14]; tm.ev_acc_end = ctx->ev[15]; }
  BH_TRY_HIP(msm_window_sums<G2Ops>(ctx->g2ws, ctx->stream, bases->pts.as<uint32_t>(), d_scalars, n, d_idx,
                                    (uint32_t)base_offset, sh, acc_ms ? &tm : nullptr));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  if (acc_ms) { float t = 0; if (hipEventElapsedTime(&t, tm.ev_acc_begin, tm.ev_acc_end) == hipSuccess) *acc_ms += t; }
  *out = combine_g2(ctx->g2ws.host_window_sums, sh);
  return BH_OK;
}

// bellman's window rule (multiexp.rs:267-271) -- only used for error semantics
static int bellman_window(size_t n) {
  if (n < 32) return 3;
  return (int)ceil(log((double)(uint32_t)n));
}
static inline uint64_t bits_window(const uint64_t* e, int skip, int c) {
  uint64_t v = 0;
  for (int i = 0; i < c; i++) {
    int b = skip + i;
    if (b < 256 && ((e[b >> 6] >> (b & 63)) & 1)) v |= 1ull << i;
  }
  return v;
}

// Exact reference error semantics (multiexp.rs:54-85 inside multiexp_inner's window
// loop, then try_fold over the windows from the top, 244-249).
bh_status multiexp_check(const bh_srs* bases, size_t base_offset, const uint64_t* density_words, size_t n,
                         const uint64_t* exps, bool have_exps) {
  size_t set = 0;
  if (!density_words) set = n;
  else {
    for (size_t w = 0; w < n / 64; w++) set += (size_t)__builtin_popcountll(density_words[w]);
    if (n % 64) set += (size_t)__builtin_popcountll(density_words[n / 64] & ((1ull << (n % 64)) - 1ull));
  }
  const size_t avail = base_offset < bases->n ? bases->n - base_offset : 0;
  const bool eof = set > avail;
  // identity bases actually reachable
  bool any_identity = false;
  for (size_t k : bases->identity_idx)
    if (k >= base_offset && k - base_offset < set) any_identity = true;
  if (!eof && !any_identity) return BH_OK;
  if (!any_identity) return BH_ERR_UNEXPECTED_EOF;
  if (!have_exps) return BH_ERR_UNEXPECTED_IDENTITY;
  // walk entries, recording for each bellman window the first error position
  const int c = bellman_window(n);
  const int nw = (255 + c - 1) / c;  // skip in (0..255).step_by(c)
  std::vector<size_t> first_err(nw, (size_t)-1);
  std::vector<int> err_kind(nw, 0);
  size_t cursor = base_offset, eof_pos = (size_t)-1;
  size_t rank = 0;
  std::vector<char> is_id(bases->n, 0);
  for (size_t k : bases->identity_idx) is_id[k] = 1;
  for (size_t i = 0; i < n; i++) {
    bool d = density_words ? ((density_words[i >> 6] >> (i & 63)) & 1) : true;
    if (!d) continue;
    if (cursor >= bases->n) { eof_pos = i; break; }
    if (is_id[cursor]) {
      const uint64_t* e = exps + 4 * i;
      bool zero = !(e[0] | e[1] | e[2] | e[3]);
      bool one = e[0] == 1 && !(e[1] | e[2] | e[3]);
      for (int w = 0; w < nw; w++) {
        bool consumes;  // next() (not skip()) in window w
        if (zero) consumes = false;
        else if (one) consumes = (w == 0);
        else consumes = bits_window(e, w * c, c) != 0;
        if (consumes && first_err[w] == (size_t)-1) { first_err[w] = i; err_kind[w] = BH_ERR_UNEXPECTED_IDENTITY; }
      }
    }
    cursor++;
    rank++;
  }
  for (int w = nw - 1; w >= 0; w--) {
    size_t p = first_err[w];
    if (eof_pos != (size_t)-1 && (p == (size_t)-1 || eof_pos < p)) return BH_ERR_UNEXPECTED_EOF;
    if (p != (size_t)-1) return err_kind[w];
  }
  return BH_OK;
}

// ------------------------------------------------------------------ domains
static Fr fr_small(uint64_t v) { uint64_t x[4] = {v, 0, 0, 0}; return from_int<4>(x); }
static Fr fr_pow_u64(const Fr& a, uint64_t e) { return pow_vartime(a, &e, 1); }

bh_status upload_split_table(bh_ctx* ctx, DevBuf& lo, DevBuf& hi, const Fr& g, const Fr& hi_scale, int L,
                                    int lo_bits) {
  const size_t nlo = (size_t)1 << lo_bits;
  const size_t nhi = (size_t)1 << (L > lo_bits ? L - lo_bits : 0);
  std::vector<uint32_t> tl(nlo * 9), th(nhi * 9);
  Fr x = Fr::one();
  for (size_t j = 0; j < nlo; j++) { fr_to_dev_limbs(x, &tl[j * 9]); x = mul(x, g); }
  const Fr step = x;  // g^(2^lo_bits)
  Fr y = hi_scale;
  for (size_t j = 0; j < nhi; j++) { fr_to_dev_limbs(y, &th[j * 9]); y = mul(y, step); }
  BH_TRY_HIP(lo.alloc(tl.size() * 4));
  BH_TRY_HIP(hi.alloc(th.size() * 4));
  BH_TRY_HIP(hipMemcpyAsync(lo.p, tl.data(), tl.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  BH_TRY_HIP(hipMemcpyAsync(hi.p, th.data(), th.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  return BH_OK;
}

void ctx_sync_all(bh_ctx* ctx) {
  for (hipStream_t st : {ctx->h2d, ctx->stream, ctx->stream2, ctx->stream3, ctx->stream4, ctx->stream5, ctx->bg.cst,
                         ctx->bg.st})
    if (st) (void)hipStreamSynchronize(st);
  for (hipStream_t st : ctx->tstream)
    if (st) (void)hipStreamSynchronize(st);
}

bh_status ctx_domain(bh_ctx* ctx, int L, Domain** out) {
  auto it = ctx->domains.find(L);
  if (it != ctx->domains.end()) { *out = it->second.get(); return BH_OK; }
  std::unique_ptr<Domain> d(new Domain());
  d->L = L;
  const size_t m = (size_t)1 << L;
  // omega = root_of_unity^(2^(32-L))  (domain.rs:62-66)
  uint64_t rou_raw[4] = {0x3829971f439f0d2bull, 0xb63683508c2280b9ull, 0xd09b681922c813b4ull, 0x16a2a19edfe81f20ull};
  Fr omega = from_int<4>(rou_raw);
  for (int i = L; i < 32; i++) omega = sqr(omega);
  const Fr omegainv = inv(omega);
  const Fr g = fr_small(7), ginv = inv(g);
  d->minv = inv(fr_small(m));
  d->zinv = inv(sub(fr_pow_u64(g, m), Fr::one()));  // domain.rs:129-151
  // twiddles omega^j, j < m/2 (built on device from split tables)
  const int tl = L >= 1 ? L - 1 : 0;
  const int tb = (tl + 1) / 2;
  DevBuf lo, hi;
  for (int dir = 0; dir < 2; dir++) {
    bh_status s = upload_split_table(ctx, lo, hi, dir == 0 ? omega : omegainv, Fr::one(), tl, tb);
    if (s) return s;
    DevBuf& tab = dir == 0 ? d->tw_fwd : d->tw_inv;
    const size_t n = (size_t)1 << tl;
    BH_TRY_HIP(tab.alloc(n * 9 * 4));
    launch_expand_table(tab.as<uint32_t>(), n, lo.as<uint32_t>(), hi.as<uint32_t>(), tb, ctx->stream);
    DevBuf& lv = dir == 0 ? d->lv_fwd : d->lv_inv;
    BH_TRY_HIP(lv.alloc(std::max<size_t>(m, 2) * 36));
    launch_level_table(lv.as<uint32_t>(), L, tab.as<uint32_t>(), ctx->stream);
    BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  }
  d->lo_bits = (L + 1) / 2;
  bh_status s;
  if ((s = upload_split_table(ctx, d->coset_lo, d->coset_hi, g, d->minv, L, d->lo_bits))) return s;
  if ((s = upload_split_table(ctx, d->icoset_lo, d->icoset_hi, ginv, d->minv, L, d->lo_bits))) return s;
  if ((s = upload_split_table(ctx, d->gpow_lo, d->gpow_hi, g, Fr::one(), L, d->lo_bits))) return s;
  {
    DevBuf lo32;
    if ((s = upload_split_table(ctx, lo32, d->coset_hi32, g, mul(d->minv, fr_small(32)), L, d->lo_bits))) return s;
    const DevBuf* src[3][2] = {{&d->coset_lo, &d->coset_hi}, {&lo32, &d->coset_hi32}, {&d->icoset_lo, &d->icoset_hi}};
    DevBuf* dst[3] = {&d->coset_full, &d->coset32_full, &d->icoset_full};
    for (int t = 0; t < 3; t++) {
      BH_TRY_HIP(dst[t]->alloc(m * 36));
      launch_expand_table(dst[t]->as<uint32_t>(), m, src[t][0]->as<uint32_t>(), src[t][1]->as<uint32_t>(), d->lo_bits,
                          ctx->stream);
    }
    BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  }
  uint32_t cst[3 * 9];
  fr_to_dev_limbs(d->minv, cst);
  fr_to_dev_limbs(d->zinv, cst + 9);
  fr_to_dev_limbs(Fr::one(), cst + 18);
  BH_TRY_HIP(d->consts.alloc(sizeof cst));
  BH_TRY_HIP(hipMemcpy(d->consts.p, cst, sizeof cst, hipMemcpyHostToDevice));
  *out = d.get();
  ctx->domains[L] = std::move(d);
  return BH_OK;
}

static FrConst conv_const(const uint32_t (&v)[9]) {
  FrConst c;
  memcpy(c.v, v, sizeof c.v);
  return c;
}

// upload n Montgomery (bls12_381) Fr into dst (packed device form), zero-padding to `padded`
bh_status upload_fr(bh_ctx* ctx, const uint64_t* host, size_t n, size_t padded, uint32_t* dst) {
  if (padded > n) BH_TRY_HIP(hipMemsetAsync(dst + n * 8, 0, (padded - n) * 32, ctx->stream));
  if (n) {
    BH_TRY_HIP(hipMemcpyAsync(dst, host, n * 32, hipMemcpyHostToDevice, ctx->stream));
    launch_fr_convert(dst, dst, n, conv_const(FrConv::TO_DEV), 0, ctx->stream);
  }
  return BH_OK;
}
FrConst fr_to_dev_const() { return conv_const(FrConv::TO_DEV); }

HostPool& ctx_pool(bh_ctx* ctx) {
  if (!ctx->pool) {
    // memcpy workers for the staging ring: enough to outrun PCIe, few enough for a shared box
    const unsigned hc = std::thread::hardware_concurrency();
    ctx->pool.reset(new HostPool((int)std::max(1u, std::min(7u, hc ? hc - 1 : 1u))));
  }
  return *ctx->pool;
}

bh_status upload_fr_staged(bh_ctx* ctx, const uint64_t* host, size_t n, size_t padded, uint32_t* dst,
                           hipStream_t st) {
  if (padded > n) BH_TRY_HIP(hipMemsetAsync(dst + n * 8, 0, (padded - n) * 32, st));
  if (n) {
    BH_TRY_HIP(ctx->ring.copy(ctx_pool(ctx), dst, host, n * 32, st));
    launch_fr_convert(dst, dst, n, conv_const(FrConv::TO_DEV), 0, st);
    BH_TRY_HIP(hipGetLastError());
  }
  return BH_OK;
}

bh_status download_fr(bh_ctx* ctx, uint32_t* src, size_t n, uint64_t* host) {
  if (!n) return BH_OK;
  launch_fr_convert(src, src, n, conv_const(FrConv::FROM_DEV), 1, ctx->stream);
  BH_TRY_HIP(hipMemcpyAsync(host, src, n * 32, hipMemcpyDeviceToHost, ctx->stream));
  BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  return BH_OK;
}

enum FftKind { FFT, IFFT, COSET_FFT, ICOSET_FFT };

// natural -> natural transform of 2^L elements in d_a using d_tmp as scratch; result in d_a
static bh_status run_fft(bh_ctx* ctx, Domain* D, FftKind kind, uint32_t* d_a, uint32_t* d_tmp) {
  const int L = D->L;
  const uint32_t* pre_lo = nullptr;
  const uint32_t* pre_hi = nullptr;
  if (kind == COSET_FFT) { pre_lo = D->gpow_lo.as<uint32_t>(); pre_hi = D->gpow_hi.as<uint32_t>(); }
  launch_permute(d_a, d_tmp, L, pre_lo, pre_hi, D->lo_bits, ctx->stream);
  const uint32_t* tw = (kind == FFT || kind == COSET_FFT) ? D->lv_fwd.as<uint32_t>() : D->lv_inv.as<uint32_t>();
  const uint32_t* post_lo = nullptr;
  const uint32_t* post_hi = nullptr;
  int post_bits = D->lo_bits;
  if (kind == IFFT) { post_hi = D->consts.as<uint32_t>(); post_bits = -1; }
  if (kind == ICOSET_FFT) { post_lo = D->icoset_lo.as<uint32_t>(); post_hi = D->icoset_hi.as<uint32_t>(); }
  launch_ntt(d_tmp, L, false, tw, post_lo, post_hi, post_bits, ctx->stream);
  BH_TRY_HIP(hipMemcpyAsync(d_a, d_tmp, ((size_t)32) << L, hipMemcpyDeviceToDevice, ctx->stream));
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

static bh_status host_fft(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m, FftKind kind) {
  if (!ctx || !coeffs || log_m >= 32) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Domain* D;
  bh_status s = ctx_domain(ctx, (int)log_m, &D);
  if (s) return s;
  const size_t m = (size_t)1 << log_m;
  BH_TRY_HIP(ctx->staging.alloc(m * 32));
  BH_TRY_HIP(ctx->staging2.alloc(m * 32));
  // device events around the three phases (bh_last_stats [18..21): upload, transform, download ms)
  for (auto& e : ctx->fft_ev)
    if (!e) BH_TRY_HIP(hipEventCreate(&e));
  BH_TRY_HIP(hipEventRecord(ctx->fft_ev[0], ctx->stream));
  if ((s = upload_fr(ctx, coeffs, m, m, ctx->staging.as<uint32_t>()))) return s;
  BH_TRY_HIP(hipEventRecord(ctx->fft_ev[1], ctx->stream));
  if ((s = run_fft(ctx, D, kind, ctx->staging.as<uint32_t>(), ctx->staging2.as<uint32_t>()))) return s;
  BH_TRY_HIP(hipEventRecord(ctx->fft_ev[2], ctx->stream));
  if ((s = download_fr(ctx, ctx->staging.as<uint32_t>(), m, coeffs))) return s;
  BH_TRY_HIP(hipEventRecord(ctx->fft_ev[3], ctx->stream));
  BH_TRY_HIP(hipEventSynchronize(ctx->fft_ev[3]));
  for (int k = 0; k < 3; k++) {
    float t = 0;
    ctx->last_timings[18 + k] = hipEventElapsedTime(&t, ctx->fft_ev[k], ctx->fft_ev[k + 1]) == hipSuccess ? t : -1;
  }
  return BH_OK;
}

// H pipeline (prover.rs:210-231) on device-resident a|b|c (3*m packed device form, natural
// order) in d_abc; with src_abc the first passes read the inputs from there (the witness stays
// untouched, no copy).  Without hout, on return d_abc's first m entries hold the h coefficients
// in BIT-REVERSED order (device form); with hout, the last pass writes the m-1 canonical h
// scalars in natural order to hout instead (truncation + to_le_bits fused).
bh_status run_h_vector(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, const uint32_t* src_abc, int v,
                       bool raw_src) {
  const int L = D->L;
  const size_t m = (size_t)1 << L;
  // prover.rs:214-219: ifft (DIF, omega^-1) with m^-1 * g^i fused = ifft + distribute_powers(g);
  // then fft (DIT, bit-reversed -> natural) = coset_fft; c's storing pass computes
  // (a*b - c) / Z(g) into a (prover.rs:221-225: mul_assign, sub_assign, divide_by_z_on_coset)
  uint32_t* x = d_abc + (size_t)v * m * 8;
  launch_ntt(x, L, true, D->lv_inv.as<uint32_t>(), nullptr, (raw_src ? D->coset32_full : D->coset_full).as<uint32_t>(),
             POW_FULL_TABLE, st, src_abc ? src_abc + (size_t)v * m * 8 : nullptr);
  NttEpilogue e;
  if (v == 2) {
    e.kind = NttEpilogue::AB_MINUS_C;
    e.pa = d_abc;
    e.pb = d_abc + m * 8;
    e.k = D->consts.as<uint32_t>() + 9;
  }
  launch_ntt(x, L, false, D->lv_fwd.as<uint32_t>(), nullptr, nullptr, 0, st, nullptr, e);
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

bh_status run_h_final(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, uint32_t* hout) {
  const int L = D->L;
  const size_t m = (size_t)1 << L;
  // prover.rs:226: icoset_fft = ifft + distribute_powers(g^-1), fused as above (output bit-reversed)
  NttEpilogue e;
  if (hout) {
    e.kind = NttEpilogue::SCALARS;
    e.out = hout;
    e.n_out = (uint32_t)(m - 1);
  }
  launch_ntt(d_abc, L, true, D->lv_inv.as<uint32_t>(), nullptr, D->icoset_full.as<uint32_t>(), POW_FULL_TABLE, st,
             nullptr, e);
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

bh_status run_h_pipeline(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, const uint32_t* src_abc,
                         uint32_t* hout) {
  bh_status s;
  for (int v = 0; v < 3; v++)
    if ((s = run_h_vector(ctx, D, d_abc, st, src_abc, v))) return s;
  return run_h_final(ctx, D, d_abc, st, hout);
}

}  // namespace bh

// =================================================================== C ABI
extern "C" {

const char* bh_status_string(bh_status s) {
  switch (s) {
    case BH_OK: return "ok";
    case BH_ERR_UNEXPECTED_IDENTITY: return "encountered an identity element in the CRS";
    case BH_ERR_UNEXPECTED_EOF: return "I/O error: expected more bases from source";
    case BH_ERR_POLY_DEGREE_TOO_LARGE: return "polynomial degree is too large";
    case BH_ERR_DENSITY_SIZE_MISMATCH: return "density query size differs from the number of exponents";
    case BH_ERR_UNCONSTRAINED_VARIABLE: return "auxiliary variable was unconstrained";
    case BH_ERR_INVALID_ARGUMENT: return "invalid argument";
    case BH_ERR_INVALID_ENCODING: return "invalid point encoding";
    case BH_ERR_NOT_IN_SUBGROUP: return "point is not in the prime-order subgroup";
    case BH_ERR_SCRATCH_LIMIT: return "a kernel's scratch would exceed the device's scratch limit";
    case BH_ERR_NOT_ON_CURVE: return "point not on curve";
    case BH_ERR_OUT_OF_MEMORY: return "device out of memory";
    case BH_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

int bh_version(void) { return 1; }

// The prover keeps 12 streams in flight (accumulations, sorts, H, small multiexps and one
// reduction tail per large multiexp).  HIP maps streams onto GPU_MAX_HW_QUEUES hardware
// queues (4 by default); streams sharing a queue serialise behind each other's work: with 4,
// a reduction tail waits behind another multiexp's tail, and the sort and H streams behind
// tails (measured in a kernel trace: queue ids shared by streams 6/7, 4/9, 5/8).  Raise the
// value to 16 when it is lower (BH_KEEP_HW_QUEUES=1 keeps the environment's value); this runs
// when the library is loaded, before the runtime reads it at its first HIP call.
// A value the caller set explicitly below 16 is still raised (the GPU box exports 4), but never
// silently: the override is reported once on stderr (include/bellman_hip.h documents the rule;
// the bench line records the environment's value and the effective one).
__attribute__((constructor)) static void bh_hw_queues() {
  const char* cur = getenv("GPU_MAX_HW_QUEUES");
  const char* keep = getenv("BH_KEEP_HW_QUEUES");
  if (keep && keep[0] == '1') return;
  if (!cur || atoi(cur) < 16) {
    setenv("GPU_MAX_HW_QUEUES", "16", 1);
    if (cur)
      fprintf(stderr, "bellman_hip: GPU_MAX_HW_QUEUES=%s raised to 16 for this process (the prover's concurrent "
                      "streams need their own hardware queues; BH_KEEP_HW_QUEUES=1 keeps %s)\n", cur, cur);
  }
}

static std::atomic<int> g_masked_ctxs[64];  // live CU-masked contexts per device (0 or 1)
static std::atomic<int> g_live_ctxs[64];    // live contexts per device (scratch report)
}  // extern "C"
namespace bh {
int live_contexts(int device) { return device >= 0 && device < 64 ? g_live_ctxs[device].load() : 0; }
}  // namespace bh
extern "C" {
static void release_mask(bh_ctx* c) {  // (every path that deletes a created context)
  if (c->cu_masked) g_masked_ctxs[c->device].fetch_sub(1);
  c->cu_masked = false;
  if (c->counted) g_live_ctxs[c->device].fetch_sub(1);
  c->counted = false;
}

bh_status bh_ctx_create(int device, bh_ctx** out) {
  if (!out) return BH_ERR_INVALID_ARGUMENT;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return BH_ERR_HIP;
  BH_TRY_HIP(hipSetDevice(device));
  bh_ctx* c = new bh_ctx();
  c->device = device;
  if (device < 64) {
    g_live_ctxs[device]++;
    c->counted = true;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking) != hipSuccess) {
    release_mask(c); delete c;
    return BH_ERR_HIP;
  }
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) { release_mask(c); delete c; return BH_ERR_HIP; }
  // Every stream of a proof at high priority: side streams (sorts, H, reduction tails), the main
  // stream (the G1 accumulations) too -- with the G2 accumulation on a high-priority stream, a G1
  // workgroup lost every dispatch race for the register room beside a G2 wave to the sorts' and
  // H's (round-5 rehearsal: N = 8 10.09-10.11 -> 9.61-9.66 ms per rank, N = 2 31.4-31.5 ->
  // 31.0-31.1, N = 1 within noise; profiles/r05_ab_sched_N1_2_8.txt).  Accumulation streams below H
  // and the sorts let H finish ~2 ms earlier in bh_prove but made it 1 ms slower, and the resident
  // proof too (profiles/r06_ab_acc_priority_dropin.txt).  And so must the host -> device copy
  // stream be: with every compute queue at high priority, a default-priority queue's packets (the
  // copies' completion markers the staging ring waits on) went unprocessed while the accumulations
  // kept dispatching -- the drop-in's b and c landed at 33 and 45 ms instead of 7 and 10.
  const int side = prio_hi;
  (void)prio_lo;
  (void)hipStreamDestroy(c->stream);
  (void)hipStreamDestroy(c->h2d);
  if (hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c->h2d, hipStreamNonBlocking, prio_hi) != hipSuccess) {
    release_mask(c); delete c;
    return BH_ERR_HIP;
  }
  if (hipStreamCreateWithPriority(&c->stream2, hipStreamNonBlocking, side) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream3, hipStreamNonBlocking, side) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream4, hipStreamNonBlocking, side) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream5, hipStreamNonBlocking, side) != hipSuccess) {
    release_mask(c); delete c;
    return BH_ERR_HIP;
  }
  // The reduction tails run on a quarter of the CUs (every 4th, a CU mask): their waves are
  // latency-bound chains of point additions that would otherwise hold SIMD slots of the
  // accumulations on every CU (same-box A/B at 2^22: -0.5 to -0.8 ms per proof with 64 of 256
  // CUs; 32 or 96 were no better).
  // A CU-masked stream takes a hardware queue of its own: only the first live context of a
  // device masks (virtual ranks and extra lanes are further contexts; 8 of them with 8 masked
  // tail queues each oversubscribed the queues and one rank never ran -- a hang).
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  c->cu_masked = device >= 0 && device < 64 && g_masked_ctxs[device].fetch_add(1) == 0;
  if (!c->cu_masked && device >= 0 && device < 64) g_masked_ctxs[device].fetch_sub(1);
  // 1 created, 0 not masked, -1 error; k: the CUs the stream gets
  auto masked = [&](hipStream_t* st, int k) -> int {
    if (!c->cu_masked) return 0;
    if (k <= 0 || ncu <= 0 || k >= ncu) return 0;
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    const int step = ncu / k;
    for (int i = 0, got = 0; i < ncu && got < k; i++)
      if (i % step == step - 1) { mask[(size_t)i / 32] |= 1u << (i % 32); got++; }
    return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data()) == hipSuccess ? 1 : -1;
  };
  for (auto& t : c->tstream) {
    const int r = masked(&t, ncu / 4);
    if (r < 0 || (r == 0 && hipStreamCreateWithPriority(&t, hipStreamNonBlocking, side) != hipSuccess)) {
      release_mask(c); delete c;
      return BH_ERR_HIP;
    }
  }
  // (Masking the sorts, the replicated H or the distributed H -- c->stream4d, half the CUs in round
  // 3 -- was measured and removed: with every prover stream at high priority the unmasked streams
  // win, e.g. N = 8 9.61-9.66 against 10.09-10.11 ms per rank with the distributed H on half the
  // CUs, profiles/r05_ab_sched_N1_2_8.txt.)
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) { release_mask(c); delete c; return BH_ERR_HIP; }
  for (auto& e : c->jev)
    if (hipEventCreate(&e) != hipSuccess) { release_mask(c); delete c; return BH_ERR_HIP; }
  if (hipHostMalloc(&c->host_out1, 8 * 128 * sizeof(XYZZ<G1F>), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&c->host_out2, 2 * 128 * sizeof(XYZZ<Fp2Ops>), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&c->host_counts, 32 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&c->host_spans, 8 * MAX_SPAN_BLOCKS * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
    release_mask(c); delete c;
    return BH_ERR_OUT_OF_MEMORY;
  }
  *out = c;
  return BH_OK;
}

// A context that borrows every stream of `primary` (bh_prove_batch's pipelined lanes): its own
// workspaces, events and pinned buffers, so a second proof can be enqueued while the first
// one's tails run, and no hardware queue more -- the streams' order is the pipeline.
__attribute__((visibility("hidden"))) bh_status ctx_create_lane(bh_ctx* primary, bh_ctx** out) {
  bh_ctx* c = new bh_ctx();
  c->device = primary->device;
  c->borrowed_streams = true;
  c->stream = primary->stream;
  c->stream2 = primary->stream2;
  c->stream3 = primary->stream3;
  c->stream4 = primary->stream4;
  c->stream5 = primary->stream5;
  c->h2d = primary->h2d;
  for (int q = 0; q < bh_ctx::TAIL_STREAMS; q++) c->tstream[q] = primary->tstream[q];
  c->tables = primary->tables;
  c->window_override = primary->window_override;
  bool ok = true;
  for (auto& e : c->ev) ok = ok && hipEventCreate(&e) == hipSuccess;
  for (auto& e : c->jev) ok = ok && hipEventCreate(&e) == hipSuccess;
  ok = ok && hipHostMalloc(&c->host_out1, 8 * 128 * sizeof(XYZZ<G1F>), hipHostMallocDefault) == hipSuccess &&
       hipHostMalloc(&c->host_out2, 2 * 128 * sizeof(XYZZ<Fp2Ops>), hipHostMallocDefault) == hipSuccess &&
       hipHostMalloc(&c->host_counts, 32 * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess &&
       hipHostMalloc(&c->host_spans, 8 * MAX_SPAN_BLOCKS * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess;
  if (!ok) {
    bh_ctx_destroy(c);
    return BH_ERR_OUT_OF_MEMORY;
  }
  *out = c;
  return BH_OK;
}

bh_status bh_ctx_destroy(bh_ctx* ctx) {
  if (!ctx) return BH_OK;
  for (bh_ctx* v : ctx->vranks) bh_ctx_destroy(v);
  ctx->vranks.clear();
  for (bh_ctx* v : ctx->lanes) bh_ctx_destroy(v);
  ctx->lanes.clear();
  (void)hipSetDevice(ctx->device);
  {  // the EvaluationDomain uploader: finish the queued copies, then stop
    {
      std::lock_guard<std::mutex> lk(ctx->dup.mu);
      ctx->dup.stop = true;
    }
    ctx->dup.cv.notify_all();
    if (ctx->dup.th.joinable()) ctx->dup.th.join();
  }
  {  // bh_compute_h_scalars producers still uploading: their deferred multiexps enqueue first
    std::unique_lock<std::mutex> lk(ctx->bg.count_mu);
    ctx->bg.cv.wait(lk, [&] { return ctx->bg.active == 0; });
  }
  ctx_sync_all(ctx);  // nothing may still read the workspaces released below (jobs' too)
  bh_ctx_release_jobs(ctx);
  for (auto& e : ctx->fft_ev)
    if (e) (void)hipEventDestroy(e);
  ctx->bg.ring.release();  // (waits for its slots' copies on bg.cst)
  if (ctx->bg.st) (void)hipStreamDestroy(ctx->bg.st);
  if (ctx->bg.cst) (void)hipStreamDestroy(ctx->bg.cst);
  for (auto& e : ctx->bg.vec)
    if (e) (void)hipEventDestroy(e);
  ctx->bg.pool.reset();
  ctx->bg.abc.release();
  if (ctx->h2d) (void)hipStreamSynchronize(ctx->h2d);
  ctx->ring.release();
  ctx->pool.reset();
  delete ctx->dropin;
  ctx->dropin = nullptr;
  ctx->g1ws.release();
  ctx->g2ws.release();
  for (auto& w : ctx->pw1) w.release();
  for (auto& w : ctx->pw2) w.release();
  ctx->domains.clear();
  ctx->evdom_pool.clear();
  for (auto& e : ctx->ev) if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->jev) if (e) (void)hipEventDestroy(e);
  if (ctx->host_out1) (void)hipHostFree(ctx->host_out1);
  if (ctx->host_out2) (void)hipHostFree(ctx->host_out2);
  if (ctx->host_counts) (void)hipHostFree(ctx->host_counts);
  if (ctx->host_spans) (void)hipHostFree(ctx->host_spans);
  if (!ctx->borrowed_streams) {
    (void)hipStreamDestroy(ctx->stream);
    if (ctx->h2d) (void)hipStreamDestroy(ctx->h2d);
    (void)hipStreamDestroy(ctx->stream2);
    (void)hipStreamDestroy(ctx->stream3);
    (void)hipStreamDestroy(ctx->stream4);
    if (ctx->stream5) (void)hipStreamDestroy(ctx->stream5);
    for (auto& t : ctx->tstream) (void)hipStreamDestroy(t);
  }
  const int dev = ctx->device;
  release_mask(ctx);
  delete ctx->dist;
  delete ctx;
  // the last context of the device gone: the pooled scalar buffers (up to 2 GiB) go with it
  // (vectors still alive return theirs to the pool later, kept until the next drain or exit)
  if (bh::live_contexts(dev) == 0) scalar_pool_drain(dev);
  return BH_OK;
}

bh_status bh_ctx_reserve(bh_ctx* ctx, size_t max_msm_len, uint32_t max_log_domain) {
  if (!ctx) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  if (max_msm_len) {
    BH_TRY_HIP(ctx->g1ws.reserve(max_msm_len));
    BH_TRY_HIP(ctx->g2ws.reserve(max_msm_len));
  }
  size_t n = std::max(max_msm_len, (size_t)1 << max_log_domain);
  BH_TRY_HIP(ctx->staging.alloc(n * 32));
  BH_TRY_HIP(ctx->staging2.alloc(n * 32));
  BH_TRY_HIP(ctx->idx.alloc(n * 4));
  BH_TRY_HIP(ctx->dtmp.alloc((n / 64 + 2) * 4));
  BH_TRY_HIP(ctx->dscan.alloc(scan_scratch_words(n / 64 + 2) * 4 + 64));
  BH_TRY_HIP(ctx->hbuf.alloc(((size_t)1 << max_log_domain) * 32));
  if (max_log_domain) {
    Domain* D;
    bh_status s = ctx_domain(ctx, (int)max_log_domain, &D);
    if (s) return s;
  }
  return BH_OK;
}

bh_status bh_ctx_set_tables(bh_ctx* ctx, int enable) {
  if (!ctx || (enable != 0 && enable != 1)) return BH_ERR_INVALID_ARGUMENT;
  ctx->tables = enable;
  return BH_OK;
}

bh_status bh_ctx_set_window(bh_ctx* ctx, int c) {
  if (!ctx || c < 0 || c > 20 || c == 1) return BH_ERR_INVALID_ARGUMENT;
  ctx->window_override = c;
  return BH_OK;
}

// ---------------------------------------------------------------- SRS
bh_status bh_srs_upload(bh_ctx* ctx, int group, const uint8_t* bytes, size_t n, int checked, bh_srs** out) {
  if (!ctx || !out || (group != BH_G1 && group != BH_G2) || (n && !bytes)) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  bh_srs* s = new bh_srs();
  bh_status st = srs_from_bytes(ctx, group, bytes, n, checked, false, s);
  if (st) { delete s; return st; }
  *out = s;
  return BH_OK;
}

bh_status bh_srs_free(bh_srs* srs) {
  delete srs;
  return BH_OK;
}
size_t bh_srs_len(const bh_srs* srs) { return srs ? srs->n : 0; }

bh_status bh_srs_get(const bh_srs* srs, size_t i, uint8_t* out) {
  if (!srs || !out || i >= srs->n) return BH_ERR_INVALID_ARGUMENT;
  const int words = srs->group == BH_G1 ? 24 : 48;
  uint32_t w[48];
  BH_TRY_HIP(hipMemcpy(w, srs->pts.as<uint32_t>() + i * words, words * 4, hipMemcpyDeviceToHost));
  bool inf = std::find(srs->identity_idx.begin(), srs->identity_idx.end(), i) != srs->identity_idx.end();
  if (srs->group == BH_G1) {
    AffinePt<Fp> a{fp_from_dev_words_g1(w), fp_from_dev_words_g1(w + 12), inf};
    g1_to_uncompressed(a, out);
  } else {
    AffinePt<bh::Fp2> a{bh::Fp2{fp_from_dev_words(w), fp_from_dev_words(w + 12)},
                        bh::Fp2{fp_from_dev_words(w + 24), fp_from_dev_words(w + 36)}, inf};
    g2_to_uncompressed(a, out);
  }
  return BH_OK;
}

// ---------------------------------------------------------------- multiexp
bh_status bh_multiexp(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint64_t* density_words,
                      size_t density_len, const uint64_t* exponents, size_t n, int scalar_format, uint8_t* out) {
  if (!ctx || !bases || !out || (n && !exponents)) return BH_ERR_INVALID_ARGUMENT;
  if (scalar_format != BH_SCALARS_CANONICAL && scalar_format != BH_SCALARS_MONTGOMERY) return BH_ERR_INVALID_ARGUMENT;
  if (density_words && density_len != n) return BH_ERR_DENSITY_SIZE_MISMATCH;
  if (n > 0x7fffffffull) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  if (bh_status sc = scratch_check(ctx)) return sc;  // rather than an abort inside the runtime
  // error semantics first (needs canonical exponents only when identity bases are reachable)
  std::vector<uint64_t> canon;
  const uint64_t* ex_c = exponents;
  if (scalar_format == BH_SCALARS_MONTGOMERY && !bases->identity_idx.empty()) {
    canon.resize(n * 4);
    for (size_t i = 0; i < n; i++) {
      Fr x;
      memcpy(x.v, exponents + 4 * i, 32);
      fr_to_canonical(x, &canon[4 * i]);
    }
    ex_c = canon.data();
  }
  bh_status st = multiexp_check(bases, base_offset, density_words, n, ex_c, true);
  if (st) return st;
  BH_TRY_HIP(ctx->staging.alloc(std::max<size_t>(n, 1) * 32));
  BH_TRY_HIP(ctx->staging2.alloc(std::max<size_t>(n, 1) * 32));
  uint32_t* d_sc = ctx->staging2.as<uint32_t>();
  if (n) {
    BH_TRY_HIP(hipMemcpyAsync(ctx->staging.p, exponents, n * 32, hipMemcpyHostToDevice, ctx->stream));
    BH_TRY_HIP(scalars_prepare(ctx->staging.as<uint32_t>(), d_sc, n, scalar_format == BH_SCALARS_MONTGOMERY ? 1 : 0,
                               0, ctx->stream));
  }
  const int32_t* d_idx = nullptr;
  DevBuf dwords;
  if (density_words && n) {
    const size_t nw = (n + 63) / 64;
    BH_TRY_HIP(dwords.alloc(nw * 8));
    BH_TRY_HIP(ctx->idx.alloc(n * 4));
    BH_TRY_HIP(ctx->dtmp.alloc((nw + 1) * 4));
    BH_TRY_HIP(ctx->dscan.alloc(scan_scratch_words(nw + 1) * 4 + 64));
    BH_TRY_HIP(hipMemcpyAsync(dwords.p, density_words, nw * 8, hipMemcpyHostToDevice, ctx->stream));
    BH_TRY_HIP(density_index(dwords.as<uint64_t>(), n, (uint32_t)base_offset, ctx->idx.as<int32_t>(),
                             ctx->dtmp.as<uint32_t>(), ctx->dscan.as<uint32_t>(), ctx->stream));
    d_idx = ctx->idx.as<int32_t>();
  }
  if (bases->group == BH_G1) {
    Jac<Fp> r;
    if ((st = msm_g1_device(ctx, bases, base_offset, d_sc, n, d_idx, &r, nullptr))) return st;
    g1_to_uncompressed(jac_to_affine(r), out);
  } else {
    Jac<bh::Fp2> r;
    if ((st = msm_g2_device(ctx, bases, base_offset, d_sc, n, d_idx, &r, nullptr))) return st;
    g2_to_uncompressed(jac_to_affine(r), out);
  }
  return BH_OK;
}

// ---------------------------------------------------------------- EvaluationDomain
bh_status bh_domain_size(size_t len, size_t* m, uint32_t* log_m) {
  size_t mm = 1;
  uint32_t e = 0;
  while (mm < len) {
    mm *= 2;
    e++;
    if (e >= 32) return BH_ERR_POLY_DEGREE_TOO_LARGE;  // domain.rs:51-60 (S = 32)
  }
  if (m) *m = mm;
  if (log_m) *log_m = e;
  return BH_OK;
}

bh_status bh_fft(bh_ctx* ctx, uint64_t* a, uint32_t log_m) { return host_fft(ctx, a, log_m, FFT); }
bh_status bh_ifft(bh_ctx* ctx, uint64_t* a, uint32_t log_m) { return host_fft(ctx, a, log_m, IFFT); }
bh_status bh_coset_fft(bh_ctx* ctx, uint64_t* a, uint32_t log_m) { return host_fft(ctx, a, log_m, COSET_FFT); }
bh_status bh_icoset_fft(bh_ctx* ctx, uint64_t* a, uint32_t log_m) { return host_fft(ctx, a, log_m, ICOSET_FFT); }

bh_status bh_distribute_powers(bh_ctx* ctx, uint64_t* coeffs, size_t len, const uint64_t g_mont[4]) {
  if (!ctx || (len && !coeffs) || !g_mont) return BH_ERR_INVALID_ARGUMENT;
  if (!len) return BH_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  int L = 0;
  while (((size_t)1 << L) < len) L++;
  Fr g;
  memcpy(g.v, g_mont, 32);
  DevBuf lo, hi;
  const int lo_bits = (L + 1) / 2;
  bh_status s = upload_split_table(ctx, lo, hi, g, Fr::one(), L, lo_bits);
  if (s) return s;
  BH_TRY_HIP(ctx->staging.alloc(len * 32));
  if ((s = upload_fr(ctx, coeffs, len, len, ctx->staging.as<uint32_t>()))) return s;
  launch_scale(ctx->staging.as<uint32_t>(), len, lo.as<uint32_t>(), hi.as<uint32_t>(), lo_bits, nullptr, ctx->stream);
  return download_fr(ctx, ctx->staging.as<uint32_t>(), len, coeffs);
}

bh_status bh_divide_by_z_on_coset(bh_ctx* ctx, uint64_t* coeffs, uint32_t log_m) {
  if (!ctx || !coeffs || log_m >= 32) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Domain* D;
  bh_status s = ctx_domain(ctx, (int)log_m, &D);
  if (s) return s;
  const size_t m = (size_t)1 << log_m;
  BH_TRY_HIP(ctx->staging.alloc(m * 32));
  if ((s = upload_fr(ctx, coeffs, m, m, ctx->staging.as<uint32_t>()))) return s;
  launch_scale(ctx->staging.as<uint32_t>(), m, nullptr, nullptr, 0, D->consts.as<uint32_t>() + 9, ctx->stream);
  return download_fr(ctx, ctx->staging.as<uint32_t>(), m, coeffs);
}

static bh_status host_pointwise(bh_ctx* ctx, uint64_t* a, const uint64_t* b, size_t len, int op) {
  if (!ctx || (len && (!a || !b))) return BH_ERR_INVALID_ARGUMENT;
  if (!len) return BH_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  BH_TRY_HIP(ctx->staging.alloc(len * 32));
  BH_TRY_HIP(ctx->staging2.alloc(len * 32));
  bh_status s;
  if ((s = upload_fr(ctx, a, len, len, ctx->staging.as<uint32_t>()))) return s;
  if ((s = upload_fr(ctx, b, len, len, ctx->staging2.as<uint32_t>()))) return s;
  launch_pointwise(ctx->staging.as<uint32_t>(), ctx->staging2.as<uint32_t>(), nullptr, len, op, nullptr, ctx->stream);
  return download_fr(ctx, ctx->staging.as<uint32_t>(), len, a);
}
bh_status bh_mul_assign(bh_ctx* ctx, uint64_t* a, const uint64_t* b, size_t len) {
  return host_pointwise(ctx, a, b, len, 0);
}
bh_status bh_sub_assign(bh_ctx* ctx, uint64_t* a, const uint64_t* b, size_t len) {
  return host_pointwise(ctx, a, b, len, 1);
}

// ---- the multiexp seam on device-resident data (include/bellman_hip.h)
bh_status bh_params_vector(const bh_params* p, int which, const bh_srs** out) {
  if (!p || !out) return BH_ERR_INVALID_ARGUMENT;
  switch (which) {
    case BH_VEC_H: *out = &p->h; return BH_OK;
    case BH_VEC_L: *out = &p->l; return BH_OK;
    case BH_VEC_A: *out = &p->a; return BH_OK;
    case BH_VEC_B_G1: *out = &p->b_g1; return BH_OK;
    case BH_VEC_B_G2: *out = &p->b_g2; return BH_OK;
    default: return BH_ERR_INVALID_ARGUMENT;
  }
}

namespace {
struct ScalarPool {
  std::mutex mu;
  std::multimap<size_t, void*> bufs;  // bytes -> device pointer
  size_t held = 0;
};
ScalarPool g_scalar_pool[64];
constexpr size_t SCALAR_POOL_CAP = (size_t)2 << 30;  // per device
}  // namespace

void* scalar_pool_take(int device, size_t bytes, size_t* got) {
  if (device < 0 || device >= 64) return nullptr;
  ScalarPool& pl = g_scalar_pool[device];
  std::lock_guard<std::mutex> lk(pl.mu);
  auto it = pl.bufs.lower_bound(bytes);
  if (it == pl.bufs.end() || it->first > bytes + bytes / 4) return nullptr;  // (no gross over-size)
  void* p = it->second;
  *got = it->first;
  pl.held -= it->first;
  pl.bufs.erase(it);
  return p;
}

void scalar_pool_give(int device, void* p, size_t bytes) {
  if (device >= 0 && device < 64) {
    ScalarPool& pl = g_scalar_pool[device];
    std::lock_guard<std::mutex> lk(pl.mu);
    if (pl.held + bytes <= SCALAR_POOL_CAP) {
      pl.bufs.emplace(bytes, p);
      pl.held += bytes;
      return;
    }
  }
  (void)hipSetDevice(device);
  (void)hipFree(p);
}

void scalar_pool_drain(int device) {
  if (device < 0 || device >= 64) return;
  ScalarPool& pl = g_scalar_pool[device];
  std::lock_guard<std::mutex> lk(pl.mu);
  (void)hipSetDevice(device);
  for (auto& kv : pl.bufs) (void)hipFree(kv.second);
  pl.bufs.clear();
  pl.held = 0;
}

bh_status new_scalar_buf(bh_ctx* ctx, size_t n, std::shared_ptr<bh_scalar_buf>* out) {
  static std::atomic<uint64_t> next_id{1};
  auto buf = std::make_shared<bh_scalar_buf>();
  buf->device = ctx->device;
  buf->owner = ctx;
  buf->id = next_id.fetch_add(1);
  const size_t bytes = std::max<size_t>(n, 1) * 32;
  size_t got = 0;
  if (void* p = scalar_pool_take(ctx->device, bytes, &got)) {
    buf->d.p = p;
    buf->d.bytes = got;
  } else {
    BH_TRY_HIP(buf->d.alloc(bytes));
  }
  BH_TRY_HIP(hipEventCreateWithFlags(&buf->ready, hipEventDisableTiming));
  *out = std::move(buf);
  return BH_OK;
}

bh_status bh_scalars_upload(bh_ctx* ctx, const uint64_t* exponents, size_t n, int scalar_format, bh_scalars** out) {
  if (!ctx || !out || (n && !exponents)) return BH_ERR_INVALID_ARGUMENT;
  if (scalar_format != BH_SCALARS_CANONICAL && scalar_format != BH_SCALARS_MONTGOMERY) return BH_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  std::shared_ptr<bh_scalar_buf> buf;
  bh_status s = new_scalar_buf(ctx, n, &buf);
  if (s) return s;
  // on the copy stream (never behind compute); bh_compute_h_scalars' producer pauses its own
  // upload meanwhile, so these vectors (read by the first sorts) land first
  if (n) {
    ctx->bg.fg_uploads++;
    hipError_t e = ctx->ring.copy(ctx_pool(ctx), buf->d.p, exponents, n * 32, ctx->h2d);
    ctx->bg.fg_uploads--;
    BH_TRY_HIP(e);
    BH_TRY_HIP(scalars_prepare(buf->d.as<uint32_t>(), buf->d.as<uint32_t>(), n,
                               scalar_format == BH_SCALARS_MONTGOMERY ? 1 : 0, 0, ctx->h2d));
  }
  BH_TRY_HIP(hipEventRecord(buf->ready, ctx->h2d));
  *out = new bh_scalars{n, std::move(buf)};
  return BH_OK;
}

size_t bh_scalars_len(const bh_scalars* s) { return s ? s->n : 0; }

bh_status bh_scalars_free(bh_scalars* s) {
  if (s && s->buf) s->buf->wait_enqueued();  // a producer has read the caller's host buffers
  delete s;  // the device vector lives on while a submitted multiexp still reads it
  return BH_OK;
}

}  // extern "C"

namespace bh {
// the background copy machinery (caller holds ctx->bg.mu): streams, pinned ring, memcpy workers
bh_status bg_init(bh_ctx* ctx) {
  auto& bg = ctx->bg;
  if (bg.st) return BH_OK;
  // high priority, like the prover's H stream: its passes must not starve beside the
  // accumulations (the multiexp on h sorts only after them)
  int lo = 0, hi = 0;
  BH_TRY_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  BH_TRY_HIP(hipStreamCreateWithPriority(&bg.st, hipStreamNonBlocking, hi));
  BH_TRY_HIP(hipStreamCreateWithPriority(&bg.cst, hipStreamNonBlocking, hi));  // (as ctx->h2d)
  for (auto& e : bg.vec) BH_TRY_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  BH_TRY_HIP(bg.ring.init());
  bg.pool.reset(new HostPool(3));
  return BH_OK;
}

// dst (device) <- src (pageable host) on bg.cst, in 16 MB pieces (one ring slot), paused while a
// bh_scalars_upload streams (the assignments feed the first sorts; H is needed last).  Returns
// once the host buffer has been read.
bh_status bg_copy(bh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  auto& bg = ctx->bg;
  const size_t piece = (size_t)16 << 20;
  for (size_t off = 0; off < bytes; off += piece) {
    while (bg.fg_uploads.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
    BH_TRY_HIP(bg.ring.copy(*bg.pool, reinterpret_cast<uint8_t*>(dst) + off,
                            reinterpret_cast<const uint8_t*>(src) + off, std::min(piece, bytes - off), bg.cst));
  }
  return BH_OK;
}
}  // namespace bh

extern "C" {

bh_status bh_compute_h_scalars(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c, size_t nc,
                               bh_scalars** h_out) {
  if (!ctx || (nc && (!a || !b || !c)) || !h_out) return BH_ERR_INVALID_ARGUMENT;
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(nc, &m, &L);
  if (s) return s;
  Domain* D;
  std::shared_ptr<bh_scalar_buf> buf;
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    BH_TRY_HIP(hipSetDevice(ctx->device));
    if ((s = ctx_domain(ctx, (int)L, &D))) return s;  // built here: the domain map is ctx->mu's
    if ((s = new_scalar_buf(ctx, m - 1, &buf))) return s;
  }
  buf->enqueued = false;
  {
    std::lock_guard<std::mutex> lk(ctx->bg.count_mu);
    ctx->bg.active++;
  }
  // The producer holds no reference to the vector (its destructor joins the producer); the
  // caller's a, b, c stay borrowed until the upload has read them (bh_scalars_sync)
  bh_scalar_buf* raw = buf.get();
  const auto t_call = std::chrono::steady_clock::now();
  raw->producer = std::thread([ctx, raw, a, b, c, nc, m, D, t_call] {
    auto since = [t_call] {
      return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
    };
    auto run = [&]() -> bh_status {
      auto& bg = ctx->bg;
      std::lock_guard<std::mutex> lk(bg.mu);
      BH_TRY_HIP(hipSetDevice(ctx->device));
      bh_status bs = bg_init(ctx);
      if (bs) return bs;
      // a|b|c: the copies (bg.cst) start after the previous producer's H (bg.st) is done with it;
      // each vector's transforms (bg.st) start as soon as its own copy has landed
      BH_TRY_HIP(bg.abc.alloc(3 * m * 32));
      BH_TRY_HIP(hipEventRecord(bg.vec[3], bg.st));
      BH_TRY_HIP(hipStreamWaitEvent(bg.cst, bg.vec[3], 0));
      uint32_t* abc = bg.abc.as<uint32_t>();
      const uint64_t* src[3] = {a, b, c};
      // BH_HOST_TIMING: the producer's stages on stderr (ms since the call)
      static const bool timing = getenv("BH_HOST_TIMING") != nullptr;
      const auto t0 = std::chrono::steady_clock::now();
      auto stamp = [&](const char* what, int v) {
        if (timing)
          fprintf(stderr, "h producer: %s %d at %.2f ms\n", what, v,
                  std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      };
      for (int v = 0; v < 3; v++) {
        uint32_t* dst = abc + (size_t)v * m * 8;
        if (m > nc) BH_TRY_HIP(hipMemsetAsync(dst + nc * 8, 0, (m - nc) * 32, bg.cst));
        if (nc) {
          if ((bs = bg_copy(ctx, dst, src[v], nc * 32))) return bs;
          stamp("uploaded", v);
        }
        raw->stamps[v] = since();
        BH_TRY_HIP(hipEventRecord(bg.vec[v], bg.cst));
        BH_TRY_HIP(hipStreamWaitEvent(bg.st, bg.vec[v], 0));
        if (nc) launch_fr_convert(dst, dst, nc, fr_to_dev_const(), 0, bg.st);
        bh_status hs = run_h_vector(ctx, D, abc, bg.st, nullptr, v);
        if (hs) return hs;
      }
      stamp("H enqueued", 3);
      // the last pass writes h as canonical scalars, natural order, truncated to m-1 (prover.rs:227-231)
      bh_status hs = run_h_final(ctx, D, abc, bg.st, raw->d.as<uint32_t>());
      if (hs) return hs;
      raw->stamps[3] = since();
      BH_TRY_HIP(hipEventRecord(raw->ready, bg.st));
      return BH_OK;
    };
    const bh_status st = run();
    if (st) {  // nothing waits for `ready`: make it a completed event
      (void)hipEventRecord(raw->ready, nullptr);
    }
    {
      std::lock_guard<std::mutex> lk(raw->mu);
      raw->status = st;
      for (auto& f : raw->deferred) f(st);
      raw->stamps[5] = (double)raw->deferred.size();
      raw->deferred.clear();
      raw->stamps[4] = since();
      raw->enqueued = true;
    }
    raw->cv.notify_all();
    {
      std::lock_guard<std::mutex> lk(ctx->bg.count_mu);
      ctx->bg.active--;
    }
    ctx->bg.cv.notify_all();
  });
  *h_out = new bh_scalars{m - 1, std::move(buf)};
  return BH_OK;
}

bh_status bh_scalars_stamps(bh_scalars* s, double out[6]) {
  if (!s || !s->buf || !out) return BH_ERR_INVALID_ARGUMENT;
  s->buf->wait_enqueued();
  memcpy(out, s->buf->stamps, sizeof(s->buf->stamps));
  return BH_OK;
}

bh_status bh_scalars_sync(bh_scalars* s) {
  if (!s || !s->buf) return BH_ERR_INVALID_ARGUMENT;
  s->buf->wait_enqueued();
  return s->buf->status;
}

bh_status bh_compute_h(bh_ctx* ctx, const uint64_t* a, const uint64_t* b, const uint64_t* c, size_t nc,
                       uint64_t* h_out, size_t* h_len) {
  if (!ctx || (nc && (!a || !b || !c)) || !h_out) return BH_ERR_INVALID_ARGUMENT;
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(nc, &m, &L);
  if (s) return s;
  std::lock_guard<std::mutex> lk(ctx->mu);
  BH_TRY_HIP(hipSetDevice(ctx->device));
  Domain* D;
  if ((s = ctx_domain(ctx, (int)L, &D))) return s;
  BH_TRY_HIP(ctx->staging.alloc(3 * m * 32));
  BH_TRY_HIP(ctx->staging2.alloc(m * 32));
  uint32_t* abc = ctx->staging.as<uint32_t>();
  if ((s = upload_fr(ctx, a, nc, m, abc))) return s;
  if ((s = upload_fr(ctx, b, nc, m, abc + m * 8))) return s;
  if ((s = upload_fr(ctx, c, nc, m, abc + 2 * m * 8))) return s;
  if ((s = run_h_pipeline(ctx, D, abc, ctx->stream))) return s;
  // bit-reversed -> natural
  launch_permute(abc, ctx->staging2.as<uint32_t>(), (int)L, nullptr, nullptr, 0, ctx->stream);
  if ((s = download_fr(ctx, ctx->staging2.as<uint32_t>(), m - 1, h_out))) return s;
  if (h_len) *h_len = m - 1;
  return BH_OK;
}

}  // extern "C"
