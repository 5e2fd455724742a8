// FP64 FMA issue rate against v_mad_u64_u32 on gfx950 (same kernel shape as madbench.hip: 8
// independent chains per thread, so the rate is issue-bound): the question is whether limb
// products done as exact double-precision FMAs (52-bit limbs, hi/lo by two FMAs) could beat the
// 29-bit integer mads of field.cuh.  Prints T ops/s for both, back to back, ~0.3 s each.
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

__global__ void __launch_bounds__(256) kfma(const double* in, double* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double a[8], acc[8];
  for (int k = 0; k < 8; k++) { a[k] = in[(t + k) & 511] * 0.999; acc[k] = k; }
  double b = in[t & 511];
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = __builtin_fma(a[k], b, acc[k]);
    b = __builtin_fma(b, 0.9999999, 1e-9);
  }
  double s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[t] = s;
}

int main() {
  uint32_t* in;
  uint64_t* out;
  double *din, *dout;
  (void)hipMalloc(&in, 4096);
  (void)hipMalloc(&out, (size_t)(1 << 24) * 8);
  (void)hipMalloc(&din, 4096);
  (void)hipMalloc(&dout, (size_t)(1 << 24) * 8);
  (void)hipMemset(in, 0x37, 4096);
  double h[512];
  for (int i = 0; i < 512; i++) h[i] = 1.0 + i * 1e-6;
  (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256 * 32, threads = 256, iters = 8192;
  for (int rep = 0; rep < 2; rep++) {
    kmad<<<blocks, threads>>>(in, out, 16);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    kmad<<<blocks, threads>>>(in, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)blocks * threads * iters * 8;
    printf("v_mad_u64_u32: %.2f T/s (%.2f ms)\n", ops / (ms * 1e9), ms);
    kfma<<<blocks, threads>>>(din, dout, 16);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    kfma<<<blocks, threads>>>(din, dout, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("v_fma_f64:     %.2f T/s (%.2f ms)\n", ops / (ms * 1e9), ms);
  }
  return 0;
}
