#include <hip/hip_runtime.h>
#include <stdio.h>
template <int MODE>
__global__ void __launch_bounds__(256) k(const uint32_t* in, uint64_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a[8]; uint64_t acc[8];
  for (int j = 0; j < 8; j++) { a[j] = in[(t + j) & 1023] | 1u; acc[j] = j; }
  uint32_t b = in[t & 1023];
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (MODE == 0) acc[j] = (uint64_t)a[j] * b + acc[j];                    // v_mad_u64_u32
      else if (MODE == 1) a[j] = a[j] * b + (uint32_t)j;                      // v_mul_lo + add (v_mad_u32_u24? no: mul_lo)
      else if (MODE == 2) { uint64_t p = (uint64_t)a[j] * b; a[j] = (uint32_t)p ^ (uint32_t)j; }  // low half via mad_u64
      else if (MODE == 3) acc[j] = acc[j] - ((uint64_t)a[j] << 3) + b;       // 64-bit sub + add (co/cndmask chains)
      else { a[j] = ((a[j] + b) & 0x1fffffffu) + (a[j] >> 29); }             // 32-bit limb add, mask, shift
    }
    b += (MODE == 0) ? (uint32_t)acc[i & 7] : a[i & 7];
  }
  uint64_t s = 0;
  for (int j = 0; j < 8; j++) s ^= acc[j] ^ a[j];
  out[t] = s;
}
int main() {
  uint32_t* in; uint64_t* out;
  (void)hipMalloc(&in, 4096); (void)hipMalloc(&out, (size_t)(1 << 24) * 8);
  (void)hipMemset(in, 0x37, 4096);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int blocks = 256 * 32, threads = 256, iters = 4096;
  for (int mode = 0; mode < 5; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      if (mode == 0) k<0><<<blocks, threads>>>(in, out, iters);
      else if (mode == 1) k<1><<<blocks, threads>>>(in, out, iters);
      else if (mode == 2) k<2><<<blocks, threads>>>(in, out, iters);
      else if (mode == 3) k<3><<<blocks, threads>>>(in, out, iters);
      else k<4><<<blocks, threads>>>(in, out, iters);
      (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("mode %d (%s): %.2f T ops/s\n", mode, mode == 0 ? "mad_u64_u32" : mode == 1 ? "mul_lo_u32+add" : mode == 2 ? "mad_u64 low half" : mode == 3 ? "u64 sub+add (C ops)" : "u32 add+mask+shift (C ops)", (double)blocks * threads * iters * 8 / (ms * 1e9));
    }
  }
  return 0;
}
