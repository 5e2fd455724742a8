// Microbenchmark: the library's Montgomery product (field.cuh fe_mul: the compiler starts each
// column on a fresh v_mad_u64_u32 chain and merges it with the carried accumulator, one 64-bit add
// per column) against the same product written as ONE dependent chain of inline-asm mads seeded
// with the carry (no merges; the hazard recogniser puts an s_nop 0 after each asm mad, and the
// chain is latency-bound per wave).  Throughput in G products/s at 2 and 4 waves per SIMD, for Fr
// (9 limbs) and Fp (14 limbs).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../bellman-mpc_amd/csrc chainbench.hip -o chainbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "field.cuh"

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);            \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint64_t mad_asm(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, sc;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint64_t mad_asm_s(uint32_t a, uint32_t b_uniform, uint64_t c) {
  uint64_t r, sc;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(sc) : "v"(a), "s"(b_uniform), "v"(c));
  return r;
}

// fe_mul with every column one dependent chain: carry-seeded, products in order, m*p last
template <class C>
__device__ __forceinline__ Fe<C> fe_mul_chain(const Fe<C>& a, const Fe<C>& b) {
  constexpr int N = C::N;
  constexpr bool P0_ONE = C::P[0] == 1u;
  Fe<C> r;
  uint32_t m[N];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * N - 1; k++) {
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); i++) acc = mad_asm(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = (k < N ? 0 : k - N + 1); i < (k < N ? k : N); i++) acc = mad_asm_s(m[i], C::P[k - i], acc);
    if (k < N) {
      m[k] = ((uint32_t)acc * C::INV) & C::MASK;
      if (P0_ONE) {
        acc = (acc + C::MASK) >> C::BITS;
        continue;
      }
      acc = mad_asm_s(m[k], C::P[0], acc);
    } else {
      r.v[k - N] = (uint32_t)acc & C::MASK;
    }
    acc >>= C::BITS;
  }
  r.v[N - 1] = (uint32_t)acc;
  return r;
}

template <class C, bool CHAIN, int W>
__global__ void __launch_bounds__(256, W) kmul(uint32_t* x, int iters) {
  constexpr int N = C::N;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  Fe<C> a, b, c, d;
  for (int i = 0; i < N; i++) {
    a.v[i] = x[(t * N + i) & 4095] & C::MASK;
    b.v[i] = x[i] & C::MASK;
    c.v[i] = a.v[i] ^ 0x1234;
    d.v[i] = b.v[i] ^ 0x777;
  }
  a.v[N - 1] &= 0xffff;
  c.v[N - 1] &= 0xffff;
  for (int it = 0; it < iters; it++) {
    if (CHAIN) {
      a = fe_mul_chain<C>(a, b);
      c = fe_mul_chain<C>(c, d);
    } else {
      a = fe_mul<C>(a, b);
      c = fe_mul<C>(c, d);
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < N; i++) s ^= a.v[i] ^ c.v[i];
  x[4096 + t] = s;
}

template <class C, bool CHAIN, int W>
static int run(const char* name, uint32_t* dx, int cus) {
  const int blocks = cus * W * 8;  // a 256-thread block is one wave per SIMD: W blocks per CU resident, 8 rounds
  const int iters = 2000;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kmul<C, CHAIN, W>), dim3(blocks), dim3(256), 0, 0, dx, 50);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((kmul<C, CHAIN, W>), dim3(blocks), dim3(256), 0, 0, dx, iters);
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double muls = 2.0 * iters * blocks * 256.0;
  printf("%-24s W=%d blocks=%d  %.3f ms  %.2f G mul/s\n", name, W, blocks, ms, muls / ms / 1e6);
  return 0;
}

int main() {
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* dx;
  CHK(hipMalloc(&dx, (4096 + (1 << 22)) * 4));
  uint32_t* hx = (uint32_t*)malloc(4096 * 4);
  for (int i = 0; i < 4096; i++) hx[i] = 0x9e3779b9u * (i + 1);
  CHK(hipMemcpy(dx, hx, 4096 * 4, hipMemcpyHostToDevice));
  int e = 0;
  {  // the chain form computes the same products
    const int nb = cus * 8, nt = nb * 256;
    uint32_t* o1 = (uint32_t*)malloc(nt * 4);
    uint32_t* o2 = (uint32_t*)malloc(nt * 4);
    hipLaunchKernelGGL((kmul<FpCfg, false, 2>), dim3(nb), dim3(256), 0, 0, dx, 7);
    CHK(hipMemcpy(o1, dx + 4096, nt * 4, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((kmul<FpCfg, true, 2>), dim3(nb), dim3(256), 0, 0, dx, 7);
    CHK(hipMemcpy(o2, dx + 4096, nt * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < nt; i++) bad += o1[i] != o2[i];
    hipLaunchKernelGGL((kmul<FrCfg, false, 2>), dim3(nb), dim3(256), 0, 0, dx, 7);
    CHK(hipMemcpy(o1, dx + 4096, nt * 4, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((kmul<FrCfg, true, 2>), dim3(nb), dim3(256), 0, 0, dx, 7);
    CHK(hipMemcpy(o2, dx + 4096, nt * 4, hipMemcpyDeviceToHost));
    for (int i = 0; i < nt; i++) bad += o1[i] != o2[i];
    printf("chain == fe_mul: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
    free(o1);
    free(o2);
  }
  e |= run<FrCfg, false, 2>("Fr fe_mul (compiler)", dx, cus);
  e |= run<FrCfg, true, 2>("Fr one chain (asm)", dx, cus);
  e |= run<FrCfg, false, 4>("Fr fe_mul (compiler)", dx, cus);
  e |= run<FrCfg, true, 4>("Fr one chain (asm)", dx, cus);
  e |= run<FpCfg, false, 2>("Fp fe_mul (compiler)", dx, cus);
  e |= run<FpCfg, true, 2>("Fp one chain (asm)", dx, cus);
  e |= run<FpCfg, false, 1>("Fp fe_mul (compiler)", dx, cus);
  e |= run<FpCfg, true, 1>("Fp one chain (asm)", dx, cus);
  CHK(hipFree(dx));
  return e;
}
