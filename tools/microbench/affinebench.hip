// Microbenchmark for the round-4 lever DESIGN.md section 8 names: G1 additions in affine
// coordinates with a per-thread Montgomery batch inversion, against the XYZZ mixed addition the
// accumulation uses now (same run, same random operand pool).
//
// Per thread: K pairs (P_k, Q_k) gathered from a 4096-point pool (L2-resident, like
// curvebench), d_k = x2 - x1, prefix products of the d_k kept in a per-thread scratch column in
// HBM, ONE Fermat inversion (a^(p-2), 380 squarings + the set bits of p-2 as products), then
// back-substitution: 1/d_k, lambda = (y2 - y1)/d_k, x3 = lambda^2 - x1 - x2,
// y3 = lambda (x1 - x3) - y1.  5M + 1S per addition plus the inversion's share (~570 products / K).
// Operands are random residues, not curve points: a throughput measurement only.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 affinebench.hip -o affinebench
#include "../../bellman-mpc_amd/csrc/curve.cuh"
#include <stdio.h>
#include <vector>

using T = DFp;

struct Exp {
  uint32_t w[12];  // p - 2, little-endian 32-bit words
};

__device__ __forceinline__ T fe_inv(const T& a, const Exp& e) {
  T r = fe_one<FpCfg>();
  for (int wi = 11; wi >= 0; wi--) {
    const uint32_t word = e.w[wi];
    for (int b = 31; b >= 0; b--) {
      r = fe_sqr<FpCfg>(r);
      if ((word >> b) & 1u) r = fe_mul<FpCfg>(r, a);
    }
  }
  return r;
}

template <int K>
__global__ void __launch_bounds__(256, 2) kaffine(const uint32_t* pts, T* scratch, uint32_t* out, Exp e, int reps) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int nthr = gridDim.x * blockDim.x;
  uint32_t chk = 0;
  for (int r = 0; r < reps; r++) {
    auto ld = [&](int k, int which, T& x, T& y) {
      const uint32_t* src = pts + 24 * ((t * 7 + k * 13 + which * 1031 + r * 17) & 4095);
      x = fe_unpack<FpCfg>(src);
      y = fe_unpack<FpCfg>(src + 12);
    };
    T acc = fe_one<FpCfg>();
    for (int k = 0; k < K; k++) {
      T x1, y1, x2, y2;
      ld(k, 0, x1, y1);
      ld(k, 1, x2, y2);
      scratch[(size_t)k * nthr + t] = acc;  // coalesced: column k of all threads
      acc = fe_mul<FpCfg>(acc, fe_sub<FpCfg, 2>(x2, x1));
    }
    T inv = fe_inv(acc, e);
    for (int k = K - 1; k >= 0; k--) {
      T x1, y1, x2, y2;
      ld(k, 0, x1, y1);
      ld(k, 1, x2, y2);
      const T d = fe_sub<FpCfg, 2>(x2, x1);
      const T dinv = fe_mul<FpCfg>(inv, scratch[(size_t)k * nthr + t]);
      inv = fe_mul<FpCfg>(inv, d);
      const T lam = fe_mul<FpCfg>(fe_sub<FpCfg, 2>(y2, y1), dinv);
      const T x3 = fe_sub<FpCfg, 4>(fe_sqr<FpCfg>(lam), fe_add<FpCfg>(x1, x2));
      const T y3 = fe_sub<FpCfg, 2>(fe_mul<FpCfg>(lam, fe_sub<FpCfg, 8>(x1, x3)), y1);
      chk ^= x3.v[0] ^ y3.v[1];
    }
  }
  out[t] = chk;
}

// the accumulation's XYZZ mixed addition over the same pool (one bucket per thread)
__global__ void __launch_bounds__(256, 2) kmadd(const uint32_t* pts, uint32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  G1Ops::P acc = G1Ops::identity();
  for (int i = 0; i < iters; i++) {
    const uint32_t* src = pts + 24 * ((t * 7 + i * 13) & 4095);
    G1Ops::A a;
    a.x = fe_unpack<FpCfg>(src);
    a.y = fe_unpack<FpCfg>(src + 12);
    acc = G1Ops::madd(acc, a);
  }
  out[t] = acc.X.v[0] ^ acc.Y.v[1] ^ acc.ZZ.v[2];
}

int main() {
  const int blocks = 256 * 8, threads = 256;
  const long nthr = (long)blocks * threads;
  uint32_t *pts, *out;
  T* scratch;
  (void)hipMalloc(&pts, 4096 * 24 * 4);
  (void)hipMalloc(&out, nthr * 4);
  (void)hipMalloc(&scratch, (size_t)1024 * nthr * sizeof(T));
  {  // random residues below 2^380
    std::vector<uint32_t> h(4096 * 24);
    uint64_t x = 88172645463325252ull;
    for (size_t i = 0; i < h.size(); i++) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      h[i] = (uint32_t)x;
      if (i % 12 == 11) h[i] &= 0x0fffffffu;
    }
    (void)hipMemcpy(pts, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  }
  Exp e;  // p - 2 from the 29-bit limbs
  {
    unsigned __int128 acc = 0;
    int bits = 0, wi = 0;
    for (int i = 0; i < 14; i++) {
      acc |= (unsigned __int128)FpCfg::P[i] << bits;
      bits += 29;
      while (bits >= 32 && wi < 12) { e.w[wi++] = (uint32_t)acc; acc >>= 32; bits -= 32; }
    }
    while (wi < 12) { e.w[wi++] = (uint32_t)acc; acc >>= 32; }
    e.w[0] -= 2;  // p is odd and > 2: no borrow
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms;
  for (int rep = 0; rep < 2; rep++) {
    kmadd<<<blocks, threads>>>(pts, out, 8);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    kmadd<<<blocks, threads>>>(pts, out, 256);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("XYZZ madd: %.3f G add/s (%.2f ms)\n", nthr * 256.0 / (ms * 1e6), ms);
#define RUNK(K, REPS)                                                                                  \
  kaffine<K><<<blocks, threads>>>(pts, scratch, out, e, 1);                                           \
  (void)hipDeviceSynchronize();                                                                        \
  (void)hipEventRecord(e0);                                                                            \
  kaffine<K><<<blocks, threads>>>(pts, scratch, out, e, REPS);                                        \
  (void)hipEventRecord(e1);                                                                            \
  (void)hipEventSynchronize(e1);                                                                       \
  (void)hipEventElapsedTime(&ms, e0, e1);                                                              \
  printf("batch-affine K=%d: %.3f G add/s (%.2f ms)\n", K, nthr * (double)K * REPS / (ms * 1e6), ms);
    RUNK(32, 8) RUNK(64, 4) RUNK(128, 2) RUNK(256, 1) RUNK(512, 1) RUNK(1024, 1)
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
