// Microbenchmark: XYZZ mixed-addition throughput with part of the bucket accumulator resident
// in LDS instead of registers (one word plane per coordinate word, 256 lanes apart: conflict
// free).  Question: does shortening the accumulator's register live ranges (G2: 112 registers
// for X, Y, ZZ, ZZZ; the kernel spills 48 VGPRs to scratch on top of 256 AGPRs) buy more than
// the LDS round trips cost?  Variants: base (all in registers), zl (ZZ, ZZZ in LDS), all (X, Y,
// ZZ, ZZZ in LDS).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 curvebench_lds.hip
#include "../../bellman-mpc_amd/csrc/curve.cuh"
#include <stdio.h>

template <class T>
__device__ __forceinline__ T lds_ld(const uint32_t* p) {
  T t;
  uint32_t* w = reinterpret_cast<uint32_t*>(&t);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) w[i] = p[i * 256];
  return t;
}
template <class T>
__device__ __forceinline__ void lds_st(uint32_t* p, const T& t) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&t);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); i++) p[i * 256] = w[i];
  asm volatile("" ::: "memory");
}

// madd with coordinates where MASK bit k (X=1, Y=2, ZZ=4, ZZZ=8) lives in LDS
template <class C, int MASK>
__device__ __forceinline__ void madd_lds(typename C::P& r, uint32_t* lds, const typename C::A& a) {
  using F = typename std::conditional<std::is_same<C, G1Ops>::value, FpOps, Fp2Ops>::type;
  using T = typename F::T;
  constexpr int NW = sizeof(T) / 4;
  uint32_t* pX = lds;
  uint32_t* pY = lds + NW * 256;
  uint32_t* pZZ = lds + 2 * NW * 256;
  uint32_t* pZZZ = lds + 3 * NW * 256;
  auto X = [&]() { return (MASK & 1) ? lds_ld<T>(pX) : r.X; };
  auto Y = [&]() { return (MASK & 2) ? lds_ld<T>(pY) : r.Y; };
  auto ZZ = [&]() { return (MASK & 4) ? lds_ld<T>(pZZ) : r.ZZ; };
  auto ZZZ = [&]() { return (MASK & 8) ? lds_ld<T>(pZZZ) : r.ZZZ; };
  auto put = [&](int bit, T& reg, uint32_t* p, const T& v) {
    if (MASK & bit) lds_st<T>(p, v);
    else reg = v;
  };
  const T zz = ZZ();
  if (F::is_zero(zz)) {
    put(1, r.X, pX, a.x); put(2, r.Y, pY, a.y); put(4, r.ZZ, pZZ, F::one()); put(8, r.ZZZ, pZZZ, F::one());
    return;
  }
  T U2 = F::mul(a.x, zz);
  T S2 = F::mul(a.y, ZZZ());
  T Pd = F::template sub<C::KX>(U2, X());
  T R = F::template sub<C::KY>(S2, Y());
  if (F::is_zero(Pd)) {  // random distinct bases: never taken (throughput bench)
    put(4, r.ZZ, pZZ, F::zero());
    return;
  }
  T PP = F::sqr(Pd);
  T PPP = F::mul(Pd, PP);
  T Q = F::mul(X(), PP);
  T X3 = F::template sub<C::K1>(F::sqr(R), F::add(PPP, F::add(Q, Q)));
  T Y3 = F::template mul_sub<C::KY>(R, F::template sub<C::K2>(Q, X3), Y(), PPP);
  put(1, r.X, pX, X3);
  put(2, r.Y, pY, Y3);
  put(4, r.ZZ, pZZ, F::mul(ZZ(), PP));
  put(8, r.ZZZ, pZZZ, F::mul(ZZZ(), PPP));
}

template <class C, int W, int MASK>
__global__ void __launch_bounds__(256, W) kmadd(const uint32_t* pts, uint32_t* out, int iters) {
  using F = typename std::conditional<std::is_same<C, G1Ops>::value, FpOps, Fp2Ops>::type;
  constexpr int PW = F::PACKED_WORDS;
  constexpr int NW = sizeof(typename F::T) / 4;
  constexpr int NL = MASK > 0 ? 4 : 0;
  __shared__ uint32_t lds[NL ? NL * NW * 256 : 1];
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  typename C::P acc = C::identity();
  uint32_t* my = lds + threadIdx.x;
  if (MASK > 0) {
    if (MASK & 1) lds_st(my, acc.X);
    if (MASK & 2) lds_st(my + NW * 256, acc.Y);
    if (MASK & 4) lds_st(my + 2 * NW * 256, acc.ZZ);
    if (MASK & 8) lds_st(my + 3 * NW * 256, acc.ZZZ);
  }
  for (int i = 0; i < iters; i++) {
    const uint32_t* src = pts + 2 * PW * ((t * 7 + i * 13) & 4095);
    typename C::A a;
    a.x = F::unpack(src);
    a.y = F::unpack(src + PW);
    if (MASK < 0) acc = C::madd(acc, a);  // the library's madd (exceptional doubling inlined)
    else madd_lds<C, (MASK < 0 ? 0 : MASK)>(acc, my, a);
  }
  if (MASK > 0 && (MASK & 1)) acc.X = lds_ld<typename F::T>(my);
  acc = C::reduce(acc);
  F::pack(acc.X, out + 2 * PW * t);
}

int main() {
  uint32_t *pts, *out;
  (void)hipMalloc(&pts, 4096 * 48 * 4);
  (void)hipMalloc(&out, (size_t)(1 << 21) * 48 * 4);
  {  // distinct pseudo-random bases (values < 2^380, not on the curve: throughput only)
    static uint32_t h[4096 * 48];
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < 4096 * 48; i++) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      h[i] = (uint32_t)x;
      if (i % 12 == 11) h[i] &= 0x0fffffffu;
    }
    (void)hipMemcpy(pts, h, sizeof(h), hipMemcpyHostToDevice);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int threads = 256, iters = 64;
  float ms;
#define RUN(C, W, M, name)                                                                        \
  {                                                                                               \
    const int blocks = 256 * W * 4;                                                               \
    const long nthr = (long)blocks * threads;                                                     \
    kmadd<C, W, M><<<blocks, threads>>>(pts, out, 4);                                             \
    (void)hipDeviceSynchronize();                                                                 \
    (void)hipEventRecord(e0);                                                                     \
    kmadd<C, W, M><<<blocks, threads>>>(pts, out, iters);                                         \
    (void)hipEventRecord(e1);                                                                     \
    (void)hipEventSynchronize(e1);                                                                \
    (void)hipEventElapsedTime(&ms, e0, e1);                                                       \
    printf("%s W=%d lds_mask=%d: %.3f G madd/s (%.2f ms)\n", name, W, M, nthr * iters / (ms * 1e6), ms); \
  }
  for (int r = 0; r < 2; r++) {
    RUN(G1Ops, 2, -1, "G1") RUN(G1Ops, 2, 0, "G1") RUN(G1Ops, 2, 12, "G1") RUN(G1Ops, 3, 12, "G1")
    RUN(G1Ops, 3, 15, "G1")
    RUN(G2Ops, 1, -1, "G2") RUN(G2Ops, 1, 0, "G2") RUN(G2Ops, 1, 12, "G2") RUN(G2Ops, 1, 15, "G2")
    RUN(G2Ops, 1, 4, "G2") RUN(G2Ops, 2, 15, "G2")
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
