// Device self-tests of field arithmetic whose correctness rests on hand-derived bounds
// (tests/test_gpu_selftest.py; not part of the public ABI, declared in api_internal.h).
//
// fe2_mul_sub_kara (field.cuh; Fp2Ops::mul_sub_lazy, the G2 mixed addition's Y3 = R (Q - X3) - Y1
// PPP under one Montgomery reduction per half) keeps signed Karatsuba column sums in a biased
// unsigned 64-bit accumulator: the bias and the +p fix-up of a negative top limb are argued from
// operand values < 2^386 with normalised 29-bit limbs.  This kernel evaluates it, and the same
// a*b - c*d as two full Fp2 products and a subtraction (the path it replaced), on caller-chosen
// operands -- the test drives both at the stated maxima and where the result is negative before
// the fix-up, against host big integers.
#include "api_internal.h"

namespace {
__global__ void __launch_bounds__(64) k_selftest_fp2_mul_sub(const uint32_t* in, uint32_t* out, uint32_t n) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  constexpr int N = FpCfg::N;
  auto ld = [&](int k) {
    DFp x;
#pragma unroll
    for (int l = 0; l < N; l++) x.v[l] = in[((size_t)t * 8 + k) * N + l];
    return x;
  };
  const DFp2 a{ld(0), ld(1)}, b{ld(2), ld(3)}, c{ld(4), ld(5)}, d{ld(6), ld(7)};
  const DFp2 lazy = Fp2Ops::mul_sub_lazy(a, b, c, d);
  const DFp2 two = Fp2Ops::sub<2>(Fp2Ops::mul(a, b), Fp2Ops::mul(c, d));
  const DFp* r[4] = {&lazy.c0, &lazy.c1, &two.c0, &two.c1};
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int l = 0; l < N; l++) out[((size_t)t * 4 + k) * N + l] = r[k]->v[l];
}
}  // namespace

// n cases of 8 Fp operands (a0, a1, b0, b1, c0, c1, d0, d1; 14 raw 29-bit limbs each) ->
// 4 Fp results per case (lazy c0, c1; two-product c0, c1), raw limbs
extern "C" bh_status bh_selftest_fp2_mul_sub(int device, const uint32_t* in, size_t n, uint32_t* out) {
  if ((n && (!in || !out)) || n > (1u << 20)) return BH_ERR_INVALID_ARGUMENT;
  if (!n) return BH_OK;
  BH_TRY_HIP(hipSetDevice(device));
  const size_t in_b = n * 8 * FpCfg::N * 4, out_b = n * 4 * FpCfg::N * 4;
  bh::DevBuf din, dout;
  BH_TRY_HIP(din.alloc(in_b));
  BH_TRY_HIP(dout.alloc(out_b));
  BH_TRY_HIP(hipMemcpy(din.p, in, in_b, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_selftest_fp2_mul_sub, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, nullptr,
                     din.as<uint32_t>(), dout.as<uint32_t>(), (uint32_t)n);
  BH_TRY_HIP(hipGetLastError());
  BH_TRY_HIP(hipMemcpy(out, dout.p, out_b, hipMemcpyDeviceToHost));
  return BH_OK;
}
