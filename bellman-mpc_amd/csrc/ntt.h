// Host interface of the device NTT family (ntt.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "field.cuh"

namespace bh {

struct FrConst {
  uint32_t v[9];  // raw 29-bit limbs
};

// In-place transform of 2^L packed Fr (device Montgomery, < 2r).
// dif=true: natural -> bit-reversed; dif=false: bit-reversed -> natural.
// tw: unpacked table omega^j, j < 2^(L-1).  post_lo/hi (optional): the stored
// element with natural index i is multiplied by lo[i & mask] * hi[i >> lo_bits].
void launch_ntt(uint32_t* d, int L, bool dif, const uint32_t* tw, const uint32_t* post_lo, const uint32_t* post_hi,
                int post_lo_bits, hipStream_t st);
void launch_permute(const uint32_t* in, uint32_t* out, int L, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                    hipStream_t st);
void launch_scale(uint32_t* a, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits, const uint32_t* c,
                  hipStream_t st);
// op 0: a *= b ; 1: a -= b ; 2: a = (a*b - c) * k
void launch_pointwise(uint32_t* a, const uint32_t* b, const uint32_t* c, size_t n, int op, const uint32_t* k,
                      hipStream_t st);
void launch_fr_convert(const uint32_t* in, uint32_t* out, size_t n, const FrConst& C, int reduce, hipStream_t st);
void launch_expand_table(uint32_t* tab, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                         hipStream_t st);

}  // namespace bh
