// Microbenchmark + cross-check: G1 (BLS12-381 Fp) arithmetic in 14 x 29-bit limbs (FIPS, one
// interleaved scan, R = 2^406) against 13 x 30-bit limbs (separated product / reduction scans,
// R = 2^390).  Part 1 runs the same sequence of field operations and XYZZ mixed additions in
// both representations from canonical inputs and compares the canonical outputs word for word;
// part 2 times chains of mixed additions (curvebench's shape) and of plain products.
#include "../../bellman-mpc_amd/csrc/curve.cuh"
#include "fp_variants.cuh"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

using G1_29 = CurveOps<FpOps>;
using G1_30 = CurveOps<Fp30Ops>;
using G1_30s = CurveOps<Fp30sOps>;

template <class F>
__device__ typename F::T to_mont(const uint32_t* w) {
  using Cfg = typename F::Cf;
  typename F::T x = F::unpack(w), r2;
#pragma unroll
  for (int i = 0; i < Cfg::N; i++) r2.v[i] = Cfg::R2[i];
  return F::mul(x, r2);
}
template <class F>
__device__ void from_mont(const typename F::T& x, uint32_t* w) {
  using Cfg = typename F::Cf;
  typename F::T one = F::zero();
  one.v[0] = 1;
  F::pack(F::reduce(F::mul(x, one)), w);
}

// per thread: 8 canonical field elements in, 12 words x 7 results out
template <class C, class F>
__global__ void kcheck(const uint32_t* in, uint32_t* out, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t* w = in + (size_t)t * 8 * 12;
  typename F::T e[8];
  for (int i = 0; i < 8; i++) e[i] = to_mont<F>(w + 12 * i);
  uint32_t* o = out + (size_t)t * 7 * 12;
  from_mont<F>(F::mul(e[0], e[1]), o);
  from_mont<F>(F::sqr(e[2]), o + 12);
  from_mont<F>(F::template mul_sub<4>(e[3], e[4], e[5], e[6]), o + 24);
  // a chain of mixed additions of the affine points (e0,e1), (e2,e3), ... onto (e4, e5)
  typename C::P acc = C::identity();
  for (int r = 0; r < 5; r++)
    for (int i = 0; i < 4; i++) {
      typename C::A a;
      a.x = e[(2 * i + r) & 7];
      a.y = e[(2 * i + 1 + 3 * r) & 7];
      acc = C::madd(acc, a);
    }
  const typename C::P q = C::dbl(acc);
  from_mont<F>(q.X, o + 36);
  from_mont<F>(q.Y, o + 48);
  from_mont<F>(q.ZZ, o + 60);
  from_mont<F>(q.ZZZ, o + 72);
}

template <class C, class F, int W>
__global__ void __launch_bounds__(256, W) kmadd(const uint32_t* pts, uint32_t* out, int iters) {
  constexpr int PW = F::PACKED_WORDS;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  typename C::P acc = C::identity();
  for (int i = 0; i < iters; i++) {
    const uint32_t* src = pts + 2 * PW * ((t * 7 + i * 13) & 4095);
    typename C::A a;
    a.x = F::unpack(src);
    a.y = F::unpack(src + PW);
    acc = C::madd(acc, a);
  }
  acc = C::reduce(acc);
  F::pack(acc.X, out + 2 * PW * t);
}

template <class F>
__global__ void __launch_bounds__(256, 2) kmul(const uint32_t* x, uint32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  typename F::T a = F::unpack(x + (t & 1023) * 12), b = F::unpack(x + ((t + 1) & 1023) * 12);
  typename F::T c = F::unpack(x + ((t + 2) & 1023) * 12), d = F::unpack(x + ((t + 3) & 1023) * 12);
  for (int i = 0; i < iters; i++) {
    a = F::mul(a, b);
    c = F::mul(c, d);
  }
  F::pack(F::add(a, c), out + (size_t)t * 12);  // out holds >= 12 words per thread
}

static const char* P_HEX = "1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab";

int main() {
  // canonical inputs < p: random 381-bit words with the top word masked below p's
  const int n = 1 << 14;
  uint32_t* h_in = (uint32_t*)malloc((size_t)n * 8 * 12 * 4);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < (size_t)n * 8 * 12; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    h_in[i] = (uint32_t)s;
    if (i % 12 == 11) h_in[i] &= 0x19ffffffu;  // < p's top word 0x1a0111ea
  }
  uint32_t *d_in, *o29, *o30, *o30s;
  hipMalloc(&d_in, (size_t)n * 8 * 12 * 4);
  hipMalloc(&o29, (size_t)n * 7 * 12 * 4);
  hipMalloc(&o30, (size_t)n * 7 * 12 * 4);
  hipMalloc(&o30s, (size_t)n * 7 * 12 * 4);
  hipMemcpy(d_in, h_in, (size_t)n * 8 * 12 * 4, hipMemcpyHostToDevice);
  kcheck<G1_29, FpOps><<<n / 256, 256>>>(d_in, o29, n);
  kcheck<G1_30, Fp30Ops><<<n / 256, 256>>>(d_in, o30, n);
  kcheck<G1_30s, Fp30sOps><<<n / 256, 256>>>(d_in, o30s, n);
  hipDeviceSynchronize();
  uint32_t* a = (uint32_t*)malloc((size_t)n * 7 * 12 * 4);
  uint32_t* b = (uint32_t*)malloc((size_t)n * 7 * 12 * 4);
  hipMemcpy(a, o29, (size_t)n * 7 * 12 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b, o30, (size_t)n * 7 * 12 * 4, hipMemcpyDeviceToHost);
  long bad = 0;
  for (size_t i = 0; i < (size_t)n * 7 * 12; i++) bad += a[i] != b[i];
  printf("cross-check (%d threads x 7 results, 29-bit vs 30-bit limbs): %ld differing words\n", n, bad);
  hipMemcpy(b, o30s, (size_t)n * 7 * 12 * 4, hipMemcpyDeviceToHost);
  long bad_s = 0;
  for (size_t i = 0; i < (size_t)n * 7 * 12; i++) bad_s += a[i] != b[i];
  printf("cross-check (29-bit vs 30-bit balanced digits): %ld differing words\n", bad_s);
  bad += bad_s;
  (void)P_HEX;

  uint32_t *pts, *out;
  hipMalloc(&pts, 4096 * 48 * 4);
  hipMalloc(&out, (size_t)(1 << 21) * 48 * 4);  // >= 48 words per thread of the 2^20-thread grids
  hipMemcpy(pts, d_in, 4096 * 24 * 4, hipMemcpyDeviceToDevice);  // canonical values as bases
  hipMemcpy(pts + 4096 * 24, d_in, 4096 * 24 * 4, hipMemcpyDeviceToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 16, threads = 256, iters = 64;
  const long nthr = (long)blocks * threads;
  float ms;
#define RUN(C, F, W, name)                                                                                  \
  kmadd<C, F, W><<<blocks, threads>>>(pts, out, 4);                                                         \
  hipDeviceSynchronize();                                                                                   \
  hipEventRecord(e0);                                                                                       \
  kmadd<C, F, W><<<blocks, threads>>>(pts, out, iters);                                                     \
  hipEventRecord(e1);                                                                                       \
  hipEventSynchronize(e1);                                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                                         \
  printf("%s W=%d: %.2f G madd/s (%.2f ms)\n", name, W, nthr* iters / (ms * 1e6), ms);
#define RUNMUL(F, name)                                                                                     \
  hipEventRecord(e0);                                                                                       \
  kmul<F><<<blocks, threads>>>(pts, out, 256);                                                                   \
  hipEventRecord(e1);                                                                                       \
  hipEventSynchronize(e1);                                                                                  \
  hipEventElapsedTime(&ms, e0, e1);                                                                         \
  printf("%s: %.1f G Fp-mul/s (%.2f ms)\n", name, nthr * 256 * 2 / (ms * 1e6), ms);
  for (int r = 0; r < 2; r++) {
    RUN(G1_29, FpOps, 1, "G1 14x29") RUN(G1_29, FpOps, 2, "G1 14x29")
    RUN(G1_30, Fp30Ops, 1, "G1 13x30") RUN(G1_30, Fp30Ops, 2, "G1 13x30")
    RUN(G1_30s, Fp30sOps, 1, "G1 13x30s") RUN(G1_30s, Fp30sOps, 2, "G1 13x30s")
    RUNMUL(FpOps, "mul 14x29") RUNMUL(Fp30Ops, "mul 13x30") RUNMUL(Fp30sOps, "mul 13x30s")
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return bad == 0 ? 0 : 1;
}
