// Device helpers shared by the NTT family (ntt.hip) and the distributed H pipeline
// (dist_h.hip): packed DFr loads/stores, unpacked table entries, bit reversal and the
// split power tables factor(i) = lo[i & mask] * hi[i >> lo_bits].
#pragma once
#include "field.cuh"
#include "ntt.h"

namespace bh {

__device__ __forceinline__ DFr ld_packed(const uint32_t* a, size_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(a + i * 8);
  uint4 x = p[0], y = p[1];
  uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  return fe_unpack<FrCfg>(w);
}
__device__ __forceinline__ void st_packed(uint32_t* a, size_t i, const DFr& v) {
  uint32_t w[8];
  fe_pack<FrCfg>(v, w);
  uint4* p = reinterpret_cast<uint4*>(a + i * 8);
  p[0] = make_uint4(w[0], w[1], w[2], w[3]);
  p[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
__device__ __forceinline__ DFr ld_limbs(const uint32_t* t, size_t i) {  // unpacked table entry (9 words)
  DFr r;
#pragma unroll
  for (int k = 0; k < 9; k++) r.v[k] = t[i * 9 + k];
  return r;
}
__device__ __forceinline__ uint32_t brev(uint32_t x, int bits) {
  return bits ? (__builtin_bitreverse32(x) >> (32 - bits)) : 0u;
}
// factor(i) = lo[i & (2^lo_bits-1)] * hi[i >> lo_bits]   (tables unpacked)
// lo_bits = POW_FULL_TABLE (ntt.h): hi[i] (a full table); other lo_bits < 0: constant factor hi[0]
__device__ __forceinline__ DFr pow_factor(const uint32_t* lo, const uint32_t* hi, int lo_bits, uint32_t i) {
  if (lo_bits == POW_FULL_TABLE) return ld_limbs(hi, i);
  if (lo_bits < 0) return ld_limbs(hi, 0);
  return fe_mul<FrCfg>(ld_limbs(lo, i & ((1u << lo_bits) - 1u)), ld_limbs(hi, i >> lo_bits));
}

}  // namespace bh
