// Microbenchmark: Fp (BLS12-381 base field) Montgomery multiplication throughput
// on gfx950 for two limb layouts, plus raw v_mad_u64_u32 issue rate.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "consts.h"
#define CHK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__device__ __forceinline__ void mul32(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int N=12; uint32_t t[N+2];
  #pragma unroll
  for (int i=0;i<N+2;i++) t[i]=0;
  #pragma unroll
  for (int i=0;i<N;i++) {
    uint64_t C = 0;
    #pragma unroll
    for (int j=0;j<N;j++) { uint64_t s = (uint64_t)a[j]*b[i] + t[j] + C; t[j]=(uint32_t)s; C=s>>32; }
    uint64_t s = (uint64_t)t[N] + C; t[N]=(uint32_t)s; t[N+1]=(uint32_t)(s>>32);
    uint32_t m = t[0]*INV32;
    s = (uint64_t)m*P32[0] + t[0]; C = s>>32;
    #pragma unroll
    for (int j=1;j<N;j++) { s=(uint64_t)m*P32[j]+t[j]+C; t[j-1]=(uint32_t)s; C=s>>32; }
    s=(uint64_t)t[N]+C; t[N-1]=(uint32_t)s; t[N]=t[N+1]+(uint32_t)(s>>32);
  }
  #pragma unroll
  for (int i=0;i<N;i++) r[i]=t[i];
}
__device__ __forceinline__ void mul29(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  const int N=14; const uint32_t MASK=0x1fffffffu; uint32_t m[N]; uint64_t acc=0;
  #pragma unroll
  for (int k=0;k<2*N-1;k++) {
    #pragma unroll
    for (int i=(k<N?0:k-N+1); i<=(k<N?k:N-1); i++) acc += (uint64_t)a[i]*b[k-i];
    #pragma unroll
    for (int i=(k<N?0:k-N+1); i<(k<N?k:N); i++) acc += (uint64_t)m[i]*P29[k-i];
    if (k<N) { m[k]=((uint32_t)acc*INV29)&MASK; acc += (uint64_t)m[k]*P29[0]; }
    else r[k-N]=(uint32_t)acc&MASK;
    acc >>= 29;
  }
  r[N-1]=(uint32_t)acc;
}
template<int V>
__global__ void __launch_bounds__(256) kmul(uint32_t* x, int iters) {
  constexpr int N = V==0 ? 12 : 14;
  uint32_t a[N], b[N], c[N], d[N];
  int t = blockIdx.x*blockDim.x+threadIdx.x;
  for (int i=0;i<N;i++){a[i]=x[(t*N+i)&4095]&0xfffffff; b[i]=x[i]&0xfffffff; c[i]=a[i]^0x1234; d[i]=b[i]^0x777;}
  for (int it=0; it<iters; it++) {
    if (V==0) { mul32(a,a,b); mul32(c,c,d); } else { mul29(a,a,b); mul29(c,c,d); }
  }
  uint32_t s=0; for (int i=0;i<N;i++) s ^= a[i]^c[i];
  x[4096+t] = s;
}
__global__ void kmad(uint32_t* x, int iters) {
  int t = blockIdx.x*blockDim.x+threadIdx.x;
  uint64_t acc[8]; uint32_t a = x[t&4095], b = x[(t+1)&4095];
  for (int i=0;i<8;i++) acc[i]=i;
  for (int it=0; it<iters; it++) {
    #pragma unroll
    for (int i=0;i<8;i++) acc[i] += (uint64_t)(a+i)*b;
    a ^= (uint32_t)acc[0];
  }
  uint64_t s=0; for (int i=0;i<8;i++) s^=acc[i];
  x[4096+t]=(uint32_t)s;
}
int main() {
  uint32_t* x; CHK(hipMalloc(&x, (4096+(1<<24))*4)); CHK(hipMemset(x, 7, (4096+(1<<24))*4));
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int blocks = 256*8*4, threads=256; long nthr = (long)blocks*threads;
  for (int rep=0; rep<2; rep++) {
    int iters=64; float ms;
    hipEventRecord(e0); kmul<0><<<blocks,threads>>>(x,iters); hipEventRecord(e1); CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms,e0,e1); printf("mul32 CIOS : %.1f G Fp-mul/s (%.2f ms)\n", nthr*iters*2/(ms*1e6), ms);
    hipEventRecord(e0); kmul<1><<<blocks,threads>>>(x,iters); hipEventRecord(e1); CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms,e0,e1); printf("mul29 FIPS : %.1f G Fp-mul/s (%.2f ms)\n", nthr*iters*2/(ms*1e6), ms);
    iters=4096;
    hipEventRecord(e0); kmad<<<blocks,threads>>>(x,iters); hipEventRecord(e1); CHK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms,e0,e1); printf("v_mad_u64_u32: %.1f T/s (%.2f ms)\n", nthr*iters*8/(ms*1e9), ms);
  }
  return 0;
}
