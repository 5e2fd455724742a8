// Host G1/G2 scalar-multiplication cost of host_arith.h (proof assembly: 6 G1 + 1 G2).
// g++ -O3 -std=c++17 -Ibellman-mpc_amd/csrc tools/microbench/host_scalar_mul.cpp -o /tmp/hsm
#include "host_arith.h"
#include <chrono>
#include <cstdio>
using namespace bh;
int main() {
  uint64_t k[4] = {0x1234567890abcdefULL, 0xfedcba0987654321ULL, 0x0f0f0f0f0f0f0f0fULL, 0x0123456789abcdefULL};
  Jac<Fp> g = jac_identity<Fp>();
  g.X = Fp::one(); g.Y = add(Fp::one(), Fp::one()); g.Z = Fp::one();
  Jac<Fp2> g2 = jac_identity<Fp2>();
  g2.X = Fp2::one(); g2.Y = add(Fp2::one(), Fp2::one()); g2.Z = Fp2::one();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 20; i++) g = jac_mul(g, k, 4);
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < 20; i++) g2 = jac_mul(g2, k, 4);
  auto t2 = std::chrono::steady_clock::now();
  printf("G1 mul %.3f ms  G2 mul %.3f ms\n", std::chrono::duration<double, std::milli>(t1 - t0).count() / 20,
         std::chrono::duration<double, std::milli>(t2 - t1).count() / 20);
  return (int)(g.X.is_zero() + g2.X.is_zero());
}
