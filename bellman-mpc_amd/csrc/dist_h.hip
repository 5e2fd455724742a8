// Distributed H pipeline: see dist_h.h for the data distribution.  Restates, split over N
// ranks, the H block of create_proof (reference src/groth16/prover.rs:210-231):
//   a, b, c: ifft, coset_fft (domain.rs:81-99, 101-125); a*b - c; divide_by_z_on_coset
//   (domain.rs:139-151); icoset_fft.
//
// Index algebra (m = N*M, omega of order m, n = N*j + r, k = M*t + q):
//   inverse  X[M t + q] = sum_r w_N^(-r t) * w^(-r q) * Y_r[q],  Y_r = iNTT_M(x[N j + r])
//   forward  V[N j + r] = NTT_M over q of  w^(q r) * sum_t w_N^(t r) * v[M t + q]
// so each transform is a local M-point NTT (existing LDS passes), an all-to-all of C = M/N
// element chunks and, per q, an N-point DFT with the w^(+-q r) twiddles, done in registers.
#include "dist_h.h"
#include "ntt_common.cuh"

namespace bh {

struct DistArgs {
  uint32_t M, C, rank, m_minus_1;
  const uint32_t* tw_fwd;  // omega^j, j < m/2 (domain of size m, unpacked)
  const uint32_t* tw_inv;
  const uint32_t* sc_lo;   // power table over the global index k (g^k m^-1 or g^-k m^-1): split, or
  const uint32_t* sc_hi;   // full in sc_hi (sc_bits = POW_FULL_TABLE, pow_factor)
  int sc_bits;
  uint32_t wN[16][9], wNinv[16][9];  // w_N^k, w_N^-k (device Montgomery limbs)
};

template <int N>
__device__ __forceinline__ DFr wconst(const uint32_t (&w)[16][9], int k) {
  DFr r;
#pragma unroll
  for (int l = 0; l < 9; l++) r.v[l] = w[k][l];
  return r;
}

// X[k] = sum_j x[j] w^(j k), natural order in and out (radix-2 DIT, fully unrolled)
template <int N>
__device__ __forceinline__ void small_dft(DFr (&x)[N], const uint32_t (&w)[16][9]) {
  constexpr int LOG = N == 2 ? 1 : N == 4 ? 2 : N == 8 ? 3 : 4;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const int j = (int)(__builtin_bitreverse32((uint32_t)i) >> (32 - LOG));
    if (i < j) {
      DFr t = x[i];
      x[i] = x[j];
      x[j] = t;
    }
  }
#pragma unroll
  for (int h = 1; h < N; h <<= 1) {
    const int step = N / (2 * h);
#pragma unroll
    for (int s = 0; s < N; s += 2 * h) {
#pragma unroll
      for (int jj = 0; jj < h; jj++) {
        const DFr t = jj == 0 ? x[s + jj + h] : fe_mul<FrCfg>(x[s + jj + h], wconst<N>(w, jj * step));
        const DFr u = x[s + jj];
        x[s + jj] = fe_csub<FrCfg, 2>(fe_add<FrCfg>(u, t));
        x[s + jj + h] = fe_csub<FrCfg, 2>(fe_sub<FrCfg, 2>(u, t));
      }
    }
  }
}

// x[r] *= s^r for r < N
template <int N>
__device__ __forceinline__ void geometric(DFr (&x)[N], const DFr& s) {
  DFr p = s;
#pragma unroll
  for (int r = 1; r < N; r++) {
    x[r] = fe_mul<FrCfg>(x[r], p);
    if (r + 1 < N) p = fe_mul<FrCfg>(p, s);
  }
}

// out[vec*M + brev(j)] = full[vec*m + N*j + r]: this rank's residue class, bit-reversed for DIT
__global__ void __launch_bounds__(256) k_gather_class(const uint32_t* full, uint32_t* out, uint32_t M, int Lm,
                                                      uint32_t N, uint32_t r, uint32_t nvec, size_t m) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)nvec * M) return;
  const uint32_t vec = (uint32_t)(gid / M), j = (uint32_t)(gid % M);
  const uint4* src = reinterpret_cast<const uint4*>(full + ((size_t)vec * m + (size_t)N * j + r) * 8);
  uint4* dst = reinterpret_cast<uint4*>(out + ((size_t)vec * M + brev(j, Lm)) * 8);
  dst[0] = src[0];
  dst[1] = src[1];
}

// after exchange 1: received Y_r[q] (r = source rank) for q in this rank's chunk.
// inverse N-DFT over r (with w^(-r q)), scale g^k m^-1 (ifft + distribute_powers), forward
// N-DFT over t (with w^(q r')) -> out[vec*M + r'*C + u], row r' bound for rank r'.
template <int N>
__global__ void __launch_bounds__(256) k_dist_mid(const uint32_t* recv, uint32_t* out, DistArgs a, uint32_t nvec) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nvec * a.C) return;
  const uint32_t vec = gid / a.C, u = gid % a.C;
  const uint32_t q = a.rank * a.C + u;
  const size_t base = (size_t)vec * a.M + u;
  DFr x[N];
#pragma unroll
  for (int r = 0; r < N; r++) x[r] = ld_packed(recv, base + (size_t)r * a.C);
  geometric<N>(x, ld_limbs(a.tw_inv, q));
  small_dft<N>(x, a.wNinv);
#pragma unroll
  for (int t = 0; t < N; t++) x[t] = fe_mul<FrCfg>(x[t], pow_factor(a.sc_lo, a.sc_hi, a.sc_bits, t * a.M + q));
  small_dft<N>(x, a.wN);
  geometric<N>(x, ld_limbs(a.tw_fwd, q));
#pragma unroll
  for (int r = 0; r < N; r++) st_packed(out, base + (size_t)r * a.C, x[r]);
}

// after exchange 3: inverse N-DFT over r, scale g^-k m^-1 (icoset), canonical scalars of
// h[M t + q] at hbuf[t*C + u], their global index (-1 for k = m-1: truncation, prover.rs:227)
template <int N>
__global__ void __launch_bounds__(256) k_dist_final(const uint32_t* recv, uint32_t* hbuf, int32_t* hidx,
                                                    DistArgs a) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= a.C) return;
  const uint32_t q = a.rank * a.C + u;
  DFr x[N];
#pragma unroll
  for (int r = 0; r < N; r++) x[r] = ld_packed(recv, u + (size_t)r * a.C);
  geometric<N>(x, ld_limbs(a.tw_inv, q));
  small_dft<N>(x, a.wNinv);
#pragma unroll
  for (int t = 0; t < N; t++) {
    const uint32_t k = t * a.M + q;
    DFr v = fe_mul<FrCfg>(x[t], pow_factor(a.sc_lo, a.sc_hi, a.sc_bits, k));
    v = fe_csub<FrCfg, 1>(fe_from_mont<FrCfg>(v));  // <= r: one subtraction
    uint32_t w[8];
    fe_pack<FrCfg>(v, w);
    uint4* p = reinterpret_cast<uint4*>(hbuf + ((size_t)t * a.C + u) * 8);
    p[0] = make_uint4(w[0], w[1], w[2], w[3]);
    p[1] = make_uint4(w[4], w[5], w[6], w[7]);
    hidx[(size_t)t * a.C + u] = k == a.m_minus_1 ? -1 : (int32_t)k;
  }
}

// ------------------------------------------------------------------ host side
static int log2i(int n) {
  int l = 0;
  while ((1 << l) < n) l++;
  return l;
}

bool dist_h_eligible(int N, int L) {
  if (N < 2 || N > 16 || (N & (N - 1))) return false;
  return L >= 2 * log2i(N) + 1;
}

bh_status dist_h_init(bh_ctx* ctx, DistH& d, int N, int rank, int L) {
  if (!dist_h_eligible(N, L) || rank < 0 || rank >= N) return BH_ERR_INVALID_ARGUMENT;
  d.N = N;
  d.rank = rank;
  d.L = L;
  d.Lm = L - log2i(N);
  d.M = (size_t)1 << d.Lm;
  d.C = d.M / N;
  BH_TRY_HIP(d.work.alloc(3 * d.M * 32));
  BH_TRY_HIP(d.recv.alloc(3 * d.M * 32));
  BH_TRY_HIP(d.hbuf.alloc(d.M * 32));
  BH_TRY_HIP(d.hidx.alloc(d.M * 4));
  Domain *D, *Dm;
  bh_status s;
  if ((s = ctx_domain(ctx, L, &D)) || (s = ctx_domain(ctx, d.Lm, &Dm))) return s;
  return BH_OK;
}

static bh_status make_args(bh_ctx* ctx, const DistH& d, bool icoset, DistArgs* a) {
  Domain* D;
  bh_status s = ctx_domain(ctx, d.L, &D);
  if (s) return s;
  a->M = (uint32_t)d.M;
  a->C = (uint32_t)d.C;
  a->rank = (uint32_t)d.rank;
  a->m_minus_1 = (uint32_t)(((size_t)1 << d.L) - 1);
  a->tw_fwd = D->tw_fwd.as<uint32_t>();
  a->tw_inv = D->tw_inv.as<uint32_t>();
  // the factors g^(+-k) m^-1 over the global index k: the domain's full tables (one load per element)
  a->sc_lo = nullptr;
  a->sc_hi = icoset ? D->icoset_full.as<uint32_t>() : D->coset_full.as<uint32_t>();
  a->sc_bits = POW_FULL_TABLE;
  // w_N = root_of_unity^(2^(32 - log N))  (the same root as domain.rs:62-66, of order N)
  uint64_t rou_raw[4] = {0x3829971f439f0d2bull, 0xb63683508c2280b9ull, 0xd09b681922c813b4ull, 0x16a2a19edfe81f20ull};
  Fr w = from_int<4>(rou_raw);
  for (int i = log2i(d.N); i < 32; i++) w = sqr(w);
  const Fr winv = inv(w);
  Fr p = Fr::one(), pi = Fr::one();
  for (int k = 0; k < 16; k++) {
    fr_to_dev_limbs(p, a->wN[k]);
    fr_to_dev_limbs(pi, a->wNinv[k]);
    p = mul(p, w);
    pi = mul(pi, winv);
  }
  return BH_OK;
}

static inline unsigned blocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

bh_status dist_h_phase1(bh_ctx* ctx, DistH& d, const uint32_t* abc_full, hipStream_t st) {
  Domain* Dm;
  bh_status s = ctx_domain(ctx, d.Lm, &Dm);
  if (s) return s;
  const size_t m = (size_t)1 << d.L;
  hipLaunchKernelGGL(k_gather_class, dim3(blocks(3 * d.M, 256)), dim3(256), 0, st, abc_full, d.work.as<uint32_t>(),
                     (uint32_t)d.M, d.Lm, (uint32_t)d.N, (uint32_t)d.rank, 3u, m);
  // Y_r = iNTT_M of the residue class: DIT (bit-reversed in, natural out), omega_M^-1
  for (int v = 0; v < 3; v++)
    launch_ntt(d.work.as<uint32_t>() + v * d.M * 8, d.Lm, false, Dm->lv_inv.as<uint32_t>(), nullptr, nullptr, 0, st);
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

template <int N>
static void launch_mid(const DistH& d, const DistArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_dist_mid<N>, dim3(blocks(3 * d.C, 256)), dim3(256), 0, st, d.recv.as<uint32_t>(),
                     d.work.as<uint32_t>(), a, 3u);
}
template <int N>
static void launch_final(const DistH& d, const DistArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_dist_final<N>, dim3(blocks(d.C, 256)), dim3(256), 0, st, d.work.as<uint32_t>(),
                     d.hbuf.as<uint32_t>(), d.hidx.as<int32_t>(), a);
}

bh_status dist_h_phase2(bh_ctx* ctx, DistH& d, hipStream_t st) {
  DistArgs a;
  bh_status s = make_args(ctx, d, false, &a);
  if (s) return s;
  switch (d.N) {
    case 2: launch_mid<2>(d, a, st); break;
    case 4: launch_mid<4>(d, a, st); break;
    case 8: launch_mid<8>(d, a, st); break;
    case 16: launch_mid<16>(d, a, st); break;
    default: return BH_ERR_INVALID_ARGUMENT;
  }
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

bh_status dist_h_phase3(bh_ctx* ctx, DistH& d, hipStream_t st) {
  Domain *D, *Dm;
  bh_status s;
  if ((s = ctx_domain(ctx, d.L, &D)) || (s = ctx_domain(ctx, d.Lm, &Dm))) return s;
  uint32_t* a = d.recv.as<uint32_t>();
  uint32_t* b = a + d.M * 8;
  uint32_t* c = b + d.M * 8;
  // coset_fft's local M-point NTTs: DIF (natural q in, bit-reversed j out), omega_M
  for (uint32_t* x : {a, b, c}) launch_ntt(x, d.Lm, true, Dm->lv_fwd.as<uint32_t>(), nullptr, nullptr, 0, st);
  // a*b - c, divide_by_z_on_coset (order-agnostic: the three vectors share the layout)
  launch_pointwise(a, b, c, d.M, 2, D->consts.as<uint32_t>() + 9, st);
  // icoset_fft's local iNTT_M: DIT (bit-reversed j in, natural q out), omega_M^-1
  launch_ntt(a, d.Lm, false, Dm->lv_inv.as<uint32_t>(), nullptr, nullptr, 0, st);
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

bh_status dist_h_final(bh_ctx* ctx, DistH& d, hipStream_t st) {
  DistArgs a;
  bh_status s = make_args(ctx, d, true, &a);
  if (s) return s;
  switch (d.N) {
    case 2: launch_final<2>(d, a, st); break;
    case 4: launch_final<4>(d, a, st); break;
    case 8: launch_final<8>(d, a, st); break;
    case 16: launch_final<16>(d, a, st); break;
    default: return BH_ERR_INVALID_ARGUMENT;
  }
  BH_TRY_HIP(hipGetLastError());
  return BH_OK;
}

bh_status dist_h_run(bh_ctx* ctx, DistH& d, const uint32_t* abc_full, const HExchange& ex, hipStream_t st) {
  bh_status s;
  if ((s = dist_h_phase1(ctx, d, abc_full, st))) return s;
  if ((s = ex(d.work.as<uint32_t>(), d.recv.as<uint32_t>(), 3, st))) return s;
  if ((s = dist_h_phase2(ctx, d, st))) return s;
  if ((s = ex(d.work.as<uint32_t>(), d.recv.as<uint32_t>(), 3, st))) return s;
  if ((s = dist_h_phase3(ctx, d, st))) return s;
  if ((s = ex(d.recv.as<uint32_t>(), d.work.as<uint32_t>(), 1, st))) return s;
  return dist_h_final(ctx, d, st);
}

void dist_kernels(std::vector<KernInfo>& v) {
  v.push_back({"k_dist_mid<2>", (const void*)k_dist_mid<2>, 256, 0});
  v.push_back({"k_dist_mid<4>", (const void*)k_dist_mid<4>, 256, 0});
  v.push_back({"k_dist_mid<8>", (const void*)k_dist_mid<8>, 256, 0});
  v.push_back({"k_dist_mid<16>", (const void*)k_dist_mid<16>, 256, 0});
  v.push_back({"k_dist_final<2>", (const void*)k_dist_final<2>, 256, 0});
  v.push_back({"k_dist_final<4>", (const void*)k_dist_final<4>, 256, 0});
  v.push_back({"k_dist_final<8>", (const void*)k_dist_final<8>, 256, 0});
  v.push_back({"k_dist_final<16>", (const void*)k_dist_final<16>, 256, 0});
}

}  // namespace bh
