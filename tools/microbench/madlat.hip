// Microbenchmark: v_mad_u64_u32 rate by the number of independent accumulation chains per
// thread (K) and the waves per SIMD (W).  A product-scanning Montgomery column is ONE dependent
// chain (acc += a_i * b_j), so K = 1 at the kernel's occupancy prices its mads if issue is
// latency-bound; madbench.hip's K = 8 gives the issue-rate peak.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int K, int W>
__global__ void __launch_bounds__(256, W) kmad(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[K];
  uint64_t acc[K];
  for (int k = 0; k < K; k++) { a[k] = in[(t + k) & 1023] | 1u; acc[k] = k; }
  uint32_t b = in[t & 1023];
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8 / K; r++) {
#pragma unroll
      for (int k = 0; k < K; k++) acc[k] = (uint64_t)a[k] * (b + r) + acc[k];
    }
    b += (uint32_t)acc[i % K];
  }
  uint64_t s = 0;
  for (int k = 0; k < K; k++) s ^= acc[k];
  out[t] = s;
}
template <int K, int W>
void run(const uint32_t* in, uint64_t* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * W, threads = 256, iters = 8192;  // W blocks of 4 waves per CU = W waves per SIMD
  kmad<K, W><<<blocks, threads>>>(in, out, 16);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  kmad<K, W><<<blocks, threads>>>(in, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double mads = (double)blocks * threads * iters * 8;
  printf("chains K=%d waves/SIMD W=%d: %.2f T mads/s (%.3f ms)\n", K, W, mads / (ms * 1e9), ms);
}
int main() {
  uint32_t* in;
  uint64_t* out;
  (void)hipMalloc(&in, 4096);
  (void)hipMalloc(&out, (size_t)(1 << 24) * 8);
  (void)hipMemset(in, 0x37, 4096);
  for (int rep = 0; rep < 2; rep++) {
    run<1, 1>(in, out); run<2, 1>(in, out); run<4, 1>(in, out); run<8, 1>(in, out);
    run<1, 2>(in, out); run<2, 2>(in, out); run<4, 2>(in, out); run<8, 2>(in, out);
    run<1, 4>(in, out); run<2, 4>(in, out); run<4, 4>(in, out);
  }
  return 0;
}
