// Host interface of the device NTT family (ntt.hip).
#pragma once
#include "kinfo.h"
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "field.cuh"

namespace bh {

constexpr int POW_FULL_TABLE = -2;
  // post_lo_bits / pow_factor: a full m-entry table in hi

struct FrConst {
  uint32_t v[9];  // raw 29-bit limbs
};

// What the storing (last) pass of a transform writes, fused into it:
//   STORE      : the transform, in place (d)
//   AB_MINUS_C : the transform is c (natural order): pa[i] = (pa[i] * pb[i] - c[i]) * k[0]
//                (prover.rs:221-225: a*b - c, divide_by_z_on_coset), c itself is not stored
//   SCALARS    : out[nat] = canonical scalar of element nat for nat < n_out (prover.rs:227-231:
//                truncate to m-1 and to_le_bits, natural order), the transform is not stored
struct NttEpilogue {
  enum Kind { STORE = 0, AB_MINUS_C = 1, SCALARS = 2 };
  int kind = STORE;
  uint32_t* pa = nullptr;
  const uint32_t* pb = nullptr;
  const uint32_t* k = nullptr;  // unpacked constant (9 limbs)
  uint32_t* out = nullptr;
  uint32_t n_out = 0;
};

// Transform of 2^L packed Fr (device Montgomery, < 2r) into d; the first pass reads src
// (default: d, in place).  dif=true: natural -> bit-reversed; dif=false: bit-reversed -> natural.
// lv: per-level twiddles (9 limbs each) lv[2^v + x] = omega_{2^(v+1)}^x (launch_level_table).
// post_lo/hi (optional): the stored element with natural index i is multiplied by
// lo[i & mask] * hi[i >> lo_bits], or by hi[i] with post_lo_bits = POW_FULL_TABLE (one product
// per element instead of two; the H block's coset / icoset factors, Domain::*_full).
void launch_ntt(uint32_t* d, int L, bool dif, const uint32_t* lv, const uint32_t* post_lo, const uint32_t* post_hi,
                int post_lo_bits, hipStream_t st, const uint32_t* src = nullptr,
                const NttEpilogue& epi = NttEpilogue());
// lv (2^L entries of 9 limbs) from the unpacked full table tw (omega^j, j < 2^(L-1))
void launch_level_table(uint32_t* lv, int L, const uint32_t* tw, hipStream_t st);
void launch_permute(const uint32_t* in, uint32_t* out, int L, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                    hipStream_t st);
// a[i] *= lo[i & mask] * hi[i >> lo_bits] (or the constant c when hi is null); rev_L >= 0: a is
// in bit-reversed order (2^rev_L elements) and position i takes the factor of index brev(i)
void launch_scale(uint32_t* a, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits, const uint32_t* c,
                  hipStream_t st, int rev_L = -1);
// out[j] = in[j] * k for unpacked (9-limb) table entries, reduced below r
void launch_table_scale(uint32_t* out, const uint32_t* in, size_t n, const FrConst& k, hipStream_t st);
// a = a * k - b (packed)
void launch_scale_sub(uint32_t* a, const uint32_t* b, size_t n, const FrConst& k, hipStream_t st);
// op 0: a *= b ; 1: a -= b ; 2: a = (a*b - c) * k
void launch_pointwise(uint32_t* a, const uint32_t* b, const uint32_t* c, size_t n, int op, const uint32_t* k,
                      hipStream_t st);
void launch_fr_convert(const uint32_t* in, uint32_t* out, size_t n, const FrConst& C, int reduce, hipStream_t st);
void launch_expand_table(uint32_t* tab, size_t n, const uint32_t* lo, const uint32_t* hi, int lo_bits,
                         hipStream_t st);
// the NTT unit's kernels (scratch budget, scratch.cpp)
void ntt_kernels(std::vector<KernInfo>& v);

}  // namespace bh
