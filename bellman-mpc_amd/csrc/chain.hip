// Native synthetic workload: the "MiMC chain" circuit (the reference's MiMCDemo,
// mimc_mod.rs:40-130, with R rounds and seeded constants) synthesized by a C++
// mirror of the R1CS API (lib.rs:207-623) into
//   * a ProvingAssignment (prover.rs:55-156)   -> bh_chain_witness
//   * a KeypairAssembly   (generator.rs:44-156) -> bh_chain_params, which runs
//     the classic CRS algorithm (generator.rs:310-572, without the fork's MPC
//     asserts) with device fixed-base scalar multiplication (crs.hip).
// Constants / preimage come from splitmix64 (seed, seed+1) exactly as
// oracle/circuits.py:fr_stream, so proofs are comparable with the oracle.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <memory>
#include <thread>
#include <vector>

#include "api_internal.h"
#include "crs.h"

using namespace bh;

namespace {

// ---------------------------------------------------------------- R1CS mirror (lib.rs)
struct Var {
  bool input;
  uint32_t index;
};
struct Term {
  Var v;
  Fr coeff;
};
struct LC {  // LinearCombination (lib.rs:240-350)
  Term t[4];
  int n = 0;
  LC& add(Var v, const Fr& c) { t[n++] = Term{v, c}; return *this; }
};

inline uint64_t splitmix64(uint64_t& st) {
  st += 0x9E3779B97F4A7C15ull;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// oracle/circuits.py fr_stream: 4 words little-endian, reduced mod r
std::vector<Fr> fr_stream(uint64_t seed, size_t count) {
  std::vector<Fr> out(count);
  uint64_t st = seed;
  for (size_t i = 0; i < count; i++) {
    uint64_t w[4];
    for (int k = 0; k < 4; k++) w[k] = splitmix64(st);
    // reduce a 256-bit value mod r (< 2^256 < 3r): subtract r at most twice
    while (geq_p<4>(w)) sub_p<4>(w);
    out[i] = fr_from_canonical(w);
  }
  return out;
}

// prover.rs:55-156
struct ProvingAssignmentN {
  std::vector<uint64_t> a_aux_density, b_input_density, b_aux_density;  // bit words
  size_t n_aux_bits = 0, n_in_bits = 0;
  std::vector<Fr> a, b, c, inputs, aux;
  static void push_bit(std::vector<uint64_t>& w, size_t n) { if ((n & 63) == 0) w.push_back(0); }
  static void set_bit(std::vector<uint64_t>& w, size_t i) { w[i >> 6] |= 1ull << (i & 63); }
  Var alloc(const Fr& v) {
    aux.push_back(v);
    push_bit(a_aux_density, n_aux_bits);
    push_bit(b_aux_density, n_aux_bits);
    n_aux_bits++;
    return Var{false, (uint32_t)(aux.size() - 1)};
  }
  Var alloc_input(const Fr& v) {
    inputs.push_back(v);
    push_bit(b_input_density, n_in_bits);
    n_in_bits++;
    return Var{true, (uint32_t)(inputs.size() - 1)};
  }
  Fr eval(const LC& lc, std::vector<uint64_t>* in_d, std::vector<uint64_t>* aux_d) {  // prover.rs:19-53
    Fr acc = Fr::zero();
    for (int i = 0; i < lc.n; i++) {
      const Term& t = lc.t[i];
      Fr v;
      if (t.v.input) { v = inputs[t.v.index]; if (in_d) set_bit(*in_d, t.v.index); }
      else { v = aux[t.v.index]; if (aux_d) set_bit(*aux_d, t.v.index); }
      if (t.coeff != Fr::one()) v = mul(v, t.coeff);
      acc = add(acc, v);
    }
    return acc;
  }
  void enforce(const LC& la, const LC& lb, const LC& lc) {
    a.push_back(eval(la, nullptr, &a_aux_density));
    b.push_back(eval(lb, &b_input_density, &b_aux_density));
    c.push_back(eval(lc, nullptr, nullptr));
  }
};

// generator.rs:44-156 (term lists per variable: (coeff, constraint))
struct KeypairAssemblyN {
  struct Entry { Fr coeff; uint32_t row; };
  size_t num_constraints = 0;
  std::vector<std::vector<Entry>> at_in, bt_in, ct_in, at_aux, bt_aux, ct_aux;
  Var alloc(const Fr&) {
    at_aux.emplace_back(); bt_aux.emplace_back(); ct_aux.emplace_back();
    return Var{false, (uint32_t)(at_aux.size() - 1)};
  }
  Var alloc_input(const Fr&) {
    at_in.emplace_back(); bt_in.emplace_back(); ct_in.emplace_back();
    return Var{true, (uint32_t)(at_in.size() - 1)};
  }
  void put(const LC& l, std::vector<std::vector<Entry>>& in, std::vector<std::vector<Entry>>& ax) {
    for (int i = 0; i < l.n; i++)
      (l.t[i].v.input ? in : ax)[l.t[i].v.index].push_back(Entry{l.t[i].coeff, (uint32_t)num_constraints});
  }
  void enforce(const LC& la, const LC& lb, const LC& lc) {
    put(la, at_in, at_aux);
    put(lb, bt_in, bt_aux);
    put(lc, ct_in, ct_aux);
    num_constraints++;
  }
};

// MiMCDemo::synthesize (mimc_mod.rs:50-129) with `rounds` rounds, then the
// input constraints x*0 = 0 (prover.rs:198-204 / generator.rs:276-282).
template <class CS>
void synthesize_chain(CS& cs, const std::vector<Fr>& consts, const Fr& xl0, const Fr& xr0) {
  const Var one = cs.alloc_input(Fr::one());  // alloc_input("one")
  Fr xl_v = xl0, xr_v = xr0;
  Var xl = cs.alloc(xl_v);
  Var xr = cs.alloc(xr_v);
  const Fr fone = Fr::one();
  const Fr mone = neg(Fr::one());
  const size_t R = consts.size();
  for (size_t i = 0; i < R; i++) {
    const Fr& ci = consts[i];
    const Fr t = add(xl_v, ci);
    const Fr tmp_v = sqr(t);
    const Var tmp = cs.alloc(tmp_v);
    LC A, B, C;
    A.add(xl, fone).add(one, ci);
    B.add(xl, fone).add(one, ci);
    C.add(tmp, fone);
    cs.enforce(A, B, C);
    const Fr new_xl_v = add(mul(t, tmp_v), xr_v);
    const Var new_xl = (i == R - 1) ? cs.alloc_input(new_xl_v) : cs.alloc(new_xl_v);
    LC A2, B2, C2;
    A2.add(tmp, fone);
    B2.add(xl, fone).add(one, ci);
    C2.add(new_xl, fone).add(xr, mone);
    cs.enforce(A2, B2, C2);
    xr = xl; xr_v = xl_v;
    xl = new_xl; xl_v = new_xl_v;
  }
}

template <class CS>
void finish_inputs(CS& cs, size_t num_inputs) {
  for (size_t i = 0; i < num_inputs; i++) {
    LC A, B, C;
    A.add(Var{true, (uint32_t)i}, Fr::one());
    cs.enforce(A, B, C);
  }
}

// host precomputed window table T[w][d-1] = d * 2^(8w) * G  (32 x 255 affine)
template <class T>
std::vector<AffinePt<T>> fixed_base_table(const Jac<T>& gen) {
  std::vector<Jac<T>> jac(32 * 255);
  Jac<T> base = gen;
  for (int w = 0; w < 32; w++) {
    Jac<T> acc = base;
    for (int d = 1; d <= 255; d++) {
      jac[w * 255 + d - 1] = acc;
      acc = jac_add(acc, base);
    }
    for (int k = 0; k < 8; k++) base = jac_dbl(base);
  }
  // batch normalisation (Montgomery's trick)
  std::vector<T> pre(jac.size());
  T accz = tone<T>();
  for (size_t i = 0; i < jac.size(); i++) { pre[i] = accz; accz = mul(accz, jac[i].Z); }
  T inv_all = inv(accz);
  std::vector<AffinePt<T>> out(jac.size());
  for (size_t i = jac.size(); i-- > 0;) {
    T zi = mul(inv_all, pre[i]);
    inv_all = mul(inv_all, jac[i].Z);
    T zi2 = sqr(zi);
    out[i].x = mul(jac[i].X, zi2);
    out[i].y = mul(jac[i].Y, mul(zi2, zi));
    out[i].infinity = false;
  }
  return out;
}

static const uint64_t G1X[6] = {0xfb3af00adb22c6bbull, 0x6c55e83ff97a1aefull, 0xa14e3a3f171bac58ull,
                                0xc3688c4f9774b905ull, 0x2695638c4fa9ac0full, 0x17f1d3a73197d794ull};
static const uint64_t G1Y[6] = {0x0caa232946c5e7e1ull, 0xd03cc744a2888ae4ull, 0x00db18cb2c04b3edull,
                                0xfcf5e095d5d00af6ull, 0xa09e30ed741d8ae4ull, 0x08b3f481e3aaa0f1ull};
static const uint64_t G2X0[6] = {0xd48056c8c121bdb8ull, 0x0bac0326a805bbefull, 0xb4510b647ae3d177ull,
                                 0xc6e47ad4fa403b02ull, 0x260805272dc51051ull, 0x024aa2b2f08f0a91ull};
static const uint64_t G2X1[6] = {0xe5ac7d055d042b7eull, 0x334cf11213945d57ull, 0xb5da61bbdc7f5049ull,
                                 0x596bd0d09920b61aull, 0x7dacd3a088274f65ull, 0x13e02b6052719f60ull};
static const uint64_t G2Y0[6] = {0xe193548608b82801ull, 0x923ac9cc3baca289ull, 0x6d429a695160d12cull,
                                 0xadfd9baa8cbdd3a7ull, 0x8cc9cdc6da2e351aull, 0x0ce5d527727d6e11ull};
static const uint64_t G2Y1[6] = {0xaaa9075ff05f79beull, 0x3f370d275cec1da1ull, 0x267492ab572e99abull,
                                 0xcb3e287e85a763afull, 0x32acd2b02bc28b99ull, 0x0606c4a02ea734ccull};

Jac<Fp> g1_gen() { return Jac<Fp>{from_int<6>(G1X), from_int<6>(G1Y), Fp::one()}; }
Jac<bh::Fp2> g2_gen() {
  return Jac<bh::Fp2>{bh::Fp2{from_int<6>(G2X0), from_int<6>(G2X1)}, bh::Fp2{from_int<6>(G2Y0), from_int<6>(G2Y1)},
                      bh::Fp2::one()};
}

void canonical_words(const Fr& x, uint32_t* w8) {
  uint64_t raw[4];
  fr_to_canonical(x, raw);
  for (int i = 0; i < 4; i++) { w8[2 * i] = (uint32_t)raw[i]; w8[2 * i + 1] = (uint32_t)(raw[i] >> 32); }
}

// scalars (canonical, host) -> packed affine points in `out` (device) via the GPU
template <class C, class T>
bh_status fixed_base_to_srs(bh_ctx* ctx, const std::vector<AffinePt<T>>& table, const std::vector<Fr>& scalars,
                            int group, bh_srs* out) {
  const size_t n = scalars.size();
  out->ctx = ctx;
  out->group = group;
  out->n = n;
  out->identity_idx.clear();
  const int words = group == BH_G1 ? 24 : 48;
  BH_TRY_HIP(out->pts.alloc(std::max<size_t>(n, 1) * words * 4));
  if (!n) return BH_OK;
  bh_srs tab;
  bh_status s = srs_upload_affine(ctx, group, table.data(), table.size(), &tab);
  if (s) return s;
  const size_t chunk = std::min<size_t>(n, (size_t)1 << 21);
  DevBuf d_sc, d_xyzz, d_scr;
  BH_TRY_HIP(d_sc.alloc(chunk * 32));
  BH_TRY_HIP(d_xyzz.alloc(chunk * sizeof(typename C::P)));
  BH_TRY_HIP(d_scr.alloc(chunk * sizeof(typename C::P) / 4 + 64));
  std::vector<uint32_t> hs(chunk * 8);
  for (size_t base = 0; base < n; base += chunk) {
    const size_t k = std::min(chunk, n - base);
    for (size_t i = 0; i < k; i++) canonical_words(scalars[base + i], &hs[i * 8]);
    BH_TRY_HIP(hipMemcpyAsync(d_sc.p, hs.data(), k * 32, hipMemcpyHostToDevice, ctx->stream));
    BH_TRY_HIP(fixed_base_batch<C>(tab.pts.as<uint32_t>(), d_sc.as<uint32_t>(), k, d_xyzz.p, d_scr.p,
                                   out->pts.as<uint32_t>() + base * words, ctx->stream));
    BH_TRY_HIP(hipStreamSynchronize(ctx->stream));
  }
  return BH_OK;
}

}  // namespace

// ---------------------------------------------------------------- fused chain synthesis
// MiMCDemo::synthesize (mimc_mod.rs:50-129) fused with the ProvingAssignment it feeds
// (prover.rs:55-156) for this circuit: only the recurrence xl' = (xl + c)^3 + xr is serial (the
// witness); every assignment, linear-combination value and density bit is a function of it, so
// after the serial pass the rows are written by several threads.  The output is byte-identical
// to the generic mirror above (the same canonical Montgomery values: add/sub/mul all reduce
// fully), which BH_CHAIN_GENERIC=1 selects (tests/test_chain_synthesis.py compares the two).
//   aux:    [xl0, xr0, tmp_0, xl_1, tmp_1, xl_2, ..., tmp_{R-1}]        (2R + 1)
//   inputs: [one, xl_R]                                                    (2)
//   row 2i:   a = b = t_i = xl_i + c_i,  c = tmp_i = t_i^2                 (A = xl + one*c_i, C = tmp)
//   row 2i+1: a = tmp_i,  b = t_i,  c = xl_{i+1} - xr_i                    (A = tmp, C = new_xl - xr)
//   rows 2R, 2R+1: a = inputs[j], b = c = 0                                (prover.rs:198-204)
//   a_aux density: every aux but xr0; b_aux: xl0 and xl_1..xl_{R-1}; b_input: one
struct ChainRows {
  Fr* a; Fr* b; Fr* c; Fr* inputs; Fr* aux;
  uint64_t* a_aux_d; uint64_t* b_in_d; uint64_t* b_aux_d;
};

static bool chain_generic() {
  static const bool v = [] {
    const char* e = getenv("BH_CHAIN_GENERIC");
    return e && e[0] == '1';
  }();
  return v;
}

static void parallel_for(size_t n, const std::function<void(size_t, size_t)>& body) {
  const unsigned hc = std::thread::hardware_concurrency();
  const size_t T = std::max<size_t>(1, std::min<size_t>({(size_t)(hc ? hc : 1), (size_t)16, n / 65536 + 1}));
  if (T == 1) { body(0, n); return; }
  std::vector<std::thread> th;
  for (size_t k = 0; k < T; k++) th.emplace_back([&, k] { body(n * k / T, n * (k + 1) / T); });
  for (auto& t : th) t.join();
}

// fr_stream (same values) with the splitmix64 stream seeked per element -- the state after k
// draws is seed + k * 0x9E3779B97F4A7C15 -- so the constants are drawn by several threads
static std::vector<Fr> fr_stream_par(uint64_t seed, size_t count) {
  std::vector<Fr> out(count);
  parallel_for(count, [&](size_t lo, size_t hi) {
    uint64_t st = seed + (uint64_t)(4 * lo) * 0x9E3779B97F4A7C15ull;
    for (size_t i = lo; i < hi; i++) {
      uint64_t w[4];
      for (int k = 0; k < 4; k++) w[k] = splitmix64(st);
      while (geq_p<4>(w)) sub_p<4>(w);
      out[i] = fr_from_canonical(w);
    }
  });
  return out;
}

static void chain_fused(size_t R, uint64_t seed, uint64_t preimage_seed, const ChainRows& o) {
  const auto t0 = std::chrono::steady_clock::now();
  const std::vector<Fr> consts = fr_stream_par(seed, R);
  const std::vector<Fr> pre = fr_stream(preimage_seed, 2);
  const auto t1 = std::chrono::steady_clock::now();
  // serial pass: the witness.  xl[i] for i <= R, t and tmp per round (aux holds tmp/xl in place)
  // uninitialised (Fr is trivially constructible): the pages are first touched by the writers
  std::unique_ptr<Fr[]> xl(new Fr[R + 1]), t(new Fr[R]);
  xl[0] = pre[0];
  Fr xr = pre[1];
  for (size_t i = 0; i < R; i++) {
    t[i] = add(xl[i], consts[i]);
    const Fr tmp = sqr(t[i]);
    o.aux[2 + 2 * i] = tmp;
    xl[i + 1] = add(mul(t[i], tmp), xr);
    xr = xl[i];
  }
  const auto t2 = std::chrono::steady_clock::now();
  if (getenv("BH_HOST_TIMING"))
    fprintf(stderr, "chain synthesis: constants %.1f ms, recurrence %.1f ms\n",
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(t2 - t1).count());
  // rows, assignments and densities in parallel
  const size_t na = 2 * R + 1, nw = (na + 63) / 64;
  o.aux[0] = pre[0];
  o.aux[1] = pre[1];
  o.inputs[0] = Fr::one();
  o.inputs[1] = xl[R];
  parallel_for(R, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) {
      const Fr& tmp = o.aux[2 + 2 * i];
      if (i + 1 < R) o.aux[3 + 2 * i] = xl[i + 1];
      const Fr& xri = i ? xl[i - 1] : pre[1];
      o.a[2 * i] = t[i]; o.b[2 * i] = t[i]; o.c[2 * i] = tmp;
      o.a[2 * i + 1] = tmp; o.b[2 * i + 1] = t[i]; o.c[2 * i + 1] = sub(xl[i + 1], xri);
    }
  });
  for (int j = 0; j < 2; j++) {
    o.a[2 * R + j] = o.inputs[j];
    o.b[2 * R + j] = Fr::zero();
    o.c[2 * R + j] = Fr::zero();
  }
  parallel_for(nw, [&](size_t lo, size_t hi) {
    for (size_t w = lo; w < hi; w++) {
      uint64_t am = ~0ull, bm = 0;
      for (int k = 0; k < 64; k++) {
        const size_t idx = w * 64 + (size_t)k;
        if (idx >= na) { am &= ~(1ull << k); continue; }
        if (idx == 1) am &= ~(1ull << k);                                   // xr0 is in no A
        if (idx == 0 || ((idx & 1) && idx >= 3)) bm |= 1ull << k;           // xl0, xl_1..xl_{R-1}
      }
      o.a_aux_d[w] = am;
      o.b_aux_d[w] = bm;
    }
  });
  o.b_in_d[0] = 1;  // one appears in every B
}

extern "C" {

bh_status bh_chain_witness(bh_ctx* ctx, size_t rounds, uint64_t seed, bh_witness** out) {
  return bh_chain_witness_preimage(ctx, rounds, seed, seed + 1, out);
}

bh_status bh_chain_witness_preimage(bh_ctx* ctx, size_t rounds, uint64_t seed, uint64_t preimage_seed,
                                    bh_witness** out) {
  if (!ctx || !out || rounds == 0) return BH_ERR_INVALID_ARGUMENT;
  if (!chain_generic()) {
    const size_t nc = 2 * rounds + 2, na = 2 * rounds + 1, nw = (na + 63) / 64;
    std::unique_ptr<Fr[]> a(new Fr[nc]), b(new Fr[nc]), c(new Fr[nc]), in(new Fr[2]), aux(new Fr[na]);
    std::vector<uint64_t> ad(nw), bd(nw), bi(1);
    const auto t0 = std::chrono::steady_clock::now();
    chain_fused(rounds, seed, preimage_seed, ChainRows{a.get(), b.get(), c.get(), in.get(), aux.get(),
                                                       ad.data(), bi.data(), bd.data()});
    const auto t1 = std::chrono::steady_clock::now();
    const bh_status st = bh_witness_upload(ctx, a[0].v, b[0].v, c[0].v, nc, in[0].v, 2, aux[0].v, na, ad.data(),
                                           bi.data(), bd.data(), out);
    if (getenv("BH_HOST_TIMING")) {
      auto ms = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
        return std::chrono::duration<double, std::milli>(y - x).count();
      };
      fprintf(stderr, "chain witness: synthesis %.1f ms, upload %.1f ms\n", ms(t0, t1),
              ms(t1, std::chrono::steady_clock::now()));
    }
    return st;
  }
  const std::vector<Fr> consts = fr_stream(seed, rounds);
  const std::vector<Fr> pre = fr_stream(preimage_seed, 2);
  ProvingAssignmentN cs;
  const size_t nc = 2 * rounds + 2;
  cs.a.reserve(nc); cs.b.reserve(nc); cs.c.reserve(nc);
  cs.aux.reserve(2 * rounds + 1);
  synthesize_chain(cs, consts, pre[0], pre[1]);
  finish_inputs(cs, cs.inputs.size());
  static_assert(sizeof(Fr) == 32, "Fr layout");
  return bh_witness_upload(ctx, cs.a[0].v, cs.b[0].v, cs.c[0].v, cs.a.size(), cs.inputs[0].v, cs.inputs.size(),
                           cs.aux[0].v, cs.aux.size(), cs.a_aux_density.data(), cs.b_input_density.data(),
                           cs.b_aux_density.data(), out);
}

bh_status bh_chain_sizes(size_t rounds, size_t out[3]) {
  if (!out || rounds == 0) return BH_ERR_INVALID_ARGUMENT;
  out[0] = 2 * rounds + 2;  // constraints: 2 per round + the 2 input constraints (prover.rs:198-204)
  out[1] = 2;               // inputs: one, image
  out[2] = 2 * rounds + 1;  // aux: xl, xr and one per round
  return BH_OK;
}

bh_status bh_chain_assignment(size_t rounds, uint64_t seed, uint64_t preimage_seed, uint64_t* a, uint64_t* b,
                              uint64_t* c, uint64_t* inputs, uint64_t* aux, uint64_t* a_aux_density,
                              uint64_t* b_input_density, uint64_t* b_aux_density) {
  size_t sz[3];
  bh_status st = bh_chain_sizes(rounds, sz);
  if (st) return st;
  if (!a || !b || !c || !inputs || !aux || !a_aux_density || !b_input_density || !b_aux_density)
    return BH_ERR_INVALID_ARGUMENT;
  if (!chain_generic()) {
    static_assert(sizeof(Fr) == 32, "Fr layout");
    chain_fused(rounds, seed, preimage_seed,
                ChainRows{reinterpret_cast<Fr*>(a), reinterpret_cast<Fr*>(b), reinterpret_cast<Fr*>(c),
                          reinterpret_cast<Fr*>(inputs), reinterpret_cast<Fr*>(aux), a_aux_density,
                          b_input_density, b_aux_density});
    return BH_OK;
  }
  const std::vector<Fr> consts = fr_stream(seed, rounds);
  const std::vector<Fr> pre = fr_stream(preimage_seed, 2);
  ProvingAssignmentN cs;
  cs.a.reserve(sz[0]); cs.b.reserve(sz[0]); cs.c.reserve(sz[0]);
  cs.aux.reserve(sz[2]);
  synthesize_chain(cs, consts, pre[0], pre[1]);
  finish_inputs(cs, cs.inputs.size());
  if (cs.a.size() != sz[0] || cs.inputs.size() != sz[1] || cs.aux.size() != sz[2]) return BH_ERR_INVALID_ARGUMENT;
  memcpy(a, cs.a.data(), sz[0] * 32);
  memcpy(b, cs.b.data(), sz[0] * 32);
  memcpy(c, cs.c.data(), sz[0] * 32);
  memcpy(inputs, cs.inputs.data(), sz[1] * 32);
  memcpy(aux, cs.aux.data(), sz[2] * 32);
  memcpy(a_aux_density, cs.a_aux_density.data(), (sz[2] + 63) / 64 * 8);
  memcpy(b_input_density, cs.b_input_density.data(), (sz[1] + 63) / 64 * 8);
  memcpy(b_aux_density, cs.b_aux_density.data(), (sz[2] + 63) / 64 * 8);
  return BH_OK;
}

bh_status bh_chain_params(bh_ctx* ctx, size_t rounds, uint64_t seed, uint64_t alpha_u, uint64_t beta_u,
                          uint64_t gamma_u, uint64_t delta_u, uint64_t tau_u, bh_params** out) {
  if (!ctx || !out || rounds == 0) return BH_ERR_INVALID_ARGUMENT;
  auto small = [](uint64_t v) { uint64_t w[4] = {v, 0, 0, 0}; return fr_from_canonical(w); };
  const Fr alpha = small(alpha_u), beta = small(beta_u), gamma = small(gamma_u), delta = small(delta_u),
           tau = small(tau_u);
  if (gamma.is_zero() || delta.is_zero()) return BH_ERR_UNEXPECTED_IDENTITY;  // generator.rs:330-345
  const std::vector<Fr> consts = fr_stream(seed, rounds);
  KeypairAssemblyN asm_;
  synthesize_chain(asm_, consts, Fr::zero(), Fr::zero());
  finish_inputs(asm_, asm_.at_in.size());
  size_t m;
  uint32_t L;
  bh_status s = bh_domain_size(asm_.num_constraints, &m, &L);
  if (s) return s;
  std::unique_ptr<bh_params> p(new bh_params());
  p->ctx = ctx;
  const Fr gamma_inv = inv(gamma), delta_inv = inv(delta);
  // powers of tau, z(tau) (generator.rs:349-372)
  std::vector<Fr> powers(m);
  Fr cur = Fr::one();
  for (size_t i = 0; i < m; i++) { powers[i] = cur; cur = mul(cur, tau); }
  const Fr zt = sub(cur, Fr::one());  // tau^m - 1
  const Fr hcoeff = mul(zt, delta_inv);
  std::vector<Fr> hsc(m - 1);
  for (size_t i = 0; i + 1 < m; i++) hsc[i] = mul(powers[i], hcoeff);
  // Lagrange coefficients: ifft of the powers of tau on the device (generator.rs:400-401)
  s = bh_ifft(ctx, powers[0].v, L);
  if (s) return s;
  const std::vector<Fr>& lag = powers;
  auto eval_at = [&](const std::vector<KeypairAssemblyN::Entry>& es) {
    Fr acc = Fr::zero();
    for (const auto& e : es) acc = add(acc, mul(lag[e.row], e.coeff));
    return acc;
  };
  // eval() of generator.rs:411-510 for inputs (ext = ic, / gamma) and aux (ext = l, / delta)
  std::vector<Fr> a_sc, b_sc, ic_sc, l_sc;
  const size_t ni = asm_.at_in.size(), na = asm_.at_aux.size();
  auto run = [&](const std::vector<std::vector<KeypairAssemblyN::Entry>>& at,
                 const std::vector<std::vector<KeypairAssemblyN::Entry>>& bt,
                 const std::vector<std::vector<KeypairAssemblyN::Entry>>& ct, const Fr& inv_, std::vector<Fr>& ext) {
    for (size_t j = 0; j < at.size(); j++) {
      const Fr u = eval_at(at[j]), v = eval_at(bt[j]), w = eval_at(ct[j]);
      if (!u.is_zero()) a_sc.push_back(u);   // identities are filtered (generator.rs:614-632)
      if (!v.is_zero()) b_sc.push_back(v);
      ext.push_back(mul(add(add(mul(u, beta), mul(v, alpha)), w), inv_));
    }
  };
  run(asm_.at_in, asm_.bt_in, asm_.ct_in, gamma_inv, ic_sc);
  run(asm_.at_aux, asm_.bt_aux, asm_.ct_aux, delta_inv, l_sc);
  for (const Fr& e : l_sc)
    if (e.is_zero()) return BH_ERR_UNCONSTRAINED_VARIABLE;  // generator.rs:582-586
  (void)ni; (void)na;
  // device fixed-base multiplications
  const Jac<Fp> g1 = g1_gen();
  const Jac<bh::Fp2> g2 = g2_gen();
  const auto t1 = fixed_base_table<Fp>(g1);
  const auto t2 = fixed_base_table<bh::Fp2>(g2);
  {
    std::lock_guard<std::mutex> lk(ctx->mu);
    BH_TRY_HIP(hipSetDevice(ctx->device));
    if ((s = fixed_base_to_srs<G1Ops>(ctx, t1, hsc, BH_G1, &p->h))) return s;
    if ((s = fixed_base_to_srs<G1Ops>(ctx, t1, l_sc, BH_G1, &p->l))) return s;
    if ((s = fixed_base_to_srs<G1Ops>(ctx, t1, a_sc, BH_G1, &p->a))) return s;
    if ((s = fixed_base_to_srs<G1Ops>(ctx, t1, b_sc, BH_G1, &p->b_g1))) return s;
    if ((s = fixed_base_to_srs<G2Ops>(ctx, t2, b_sc, BH_G2, &p->b_g2))) return s;
  }
  // ic and the verifying key on the host (ni points)
  auto g1mul = [&](const Fr& k) { uint64_t c[4]; fr_to_canonical(k, c); return jac_to_affine(jac_mul(g1, c, 4)); };
  auto g2mul = [&](const Fr& k) { uint64_t c[4]; fr_to_canonical(k, c); return jac_to_affine(jac_mul(g2, c, 4)); };
  for (const Fr& e : ic_sc) p->ic.push_back(g1mul(e));
  p->alpha_g1 = g1mul(alpha);
  p->beta_g1 = g1mul(beta);
  p->beta_g2 = g2mul(beta);
  p->gamma_g2 = g2mul(gamma);
  p->delta_g1 = g1mul(delta);
  p->delta_g2 = g2mul(delta);
  *out = p.release();
  return BH_OK;
}

}  // extern "C"
