// Peak v_mad_u64_u32 throughput on gfx950: every thread runs 8 independent 64-bit
// multiply-accumulate chains (acc_k = a_k * b + acc_k), so the measured rate is the
// issue rate, not the latency.  Reported in T mads/s; the integer-ALU roofline of
// bench.py prices the Montgomery arithmetic against it.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void __launch_bounds__(256) kmad(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[8];
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) { a[k] = in[(t + k) & 1023] | 1u; acc[k] = k; }
  uint32_t b = in[t & 1023];
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (uint64_t)a[k] * b + acc[k];
    b += (uint32_t)acc[i & 7];
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[t] = s;
}
int main() {
  uint32_t* in; uint64_t* out;
  (void)hipMalloc(&in, 4096); (void)hipMalloc(&out, (size_t)(1 << 24) * 8);
  (void)hipMemset(in, 0x37, 4096);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int blocks = 256 * 32, threads = 256, iters = 4096;
  kmad<<<blocks, threads>>>(in, out, 16); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  kmad<<<blocks, threads>>>(in, out, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double mads = (double)blocks * threads * iters * 8;
  printf("v_mad_u64_u32: %.2f T/s (%.2f ms)\n", mads / (ms * 1e9), ms);
  return 0;
}
