// G2 instantiation of the batch-affine bucket accumulation (msm_aff.cuh): Fp2 coordinates
// (column-wise Karatsuba products, as in the G2 XYZZ accumulation), one Fp inversion of the norm
// per thread.  Level 0 reads the G2 window-table records (raw limbs in 64-word lines), the others
// the level records (raw limbs, 56 words).
#define BH_FP2_KARATSUBA 1
#include "msm_aff.cuh"

namespace bh {

namespace {
template <bool PK>
__global__ void __launch_bounds__(256) k_aff_fwd_g2(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                                    const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt,
                                                    uint32_t K, uint32_t* pre, uint32_t* prod) {
  aff::aff_fwd<aff::G2A, PK>(entries, src, rec, in_off, out_off, nbt, K, pre, prod);
}
// one wave per SIMD (the LDS prefetch of two records takes 96-112 KB per workgroup): the whole
// register file, AGPRs included
template <bool PK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_aff_bwd_g2(const uint32_t* entries, const uint32_t* src, uint32_t rec, const uint32_t* in_off,
             const uint32_t* out_off, uint32_t nbt, uint32_t K, const uint32_t* pre, const uint32_t* prod,
             uint32_t* dst) {
  __shared__ uint4 lds[4 * 2 * (PK ? aff::G2A::Q_PK : aff::G2A::Q_RAW) * 64];
  aff::aff_bwd<aff::G2A, PK>(entries, src, rec, in_off, out_off, nbt, K, pre, prod, dst, lds);
}
}  // namespace

AffinePlan affine_plan_g2(size_t Emax, size_t nbt, int halves) {
  static const size_t resident = aff::resident_of((const void*)k_aff_bwd_g2<false>);
  return affine_plan(Emax, nbt, halves, resident, true);
}

hipError_t affine_levels_g2(MsmWorkspace<G2Ops>& ws, hipStream_t st, const uint32_t* d_bases, uint32_t rec,
                            const AffinePlan& pl, size_t nbt, const uint32_t** final_pts) {
  return aff::levels_run<aff::G2A>(ws, st, d_bases, rec, pl, nbt, k_aff_fwd_g2<true>, k_aff_bwd_g2<true>,
                                   k_aff_fwd_g2<false>, k_aff_bwd_g2<false>, final_pts);
}

void aff_kernels_g2(std::vector<KernInfo>& v) {
  v.push_back({"k_aff_fwd_g2<packed>", (const void*)k_aff_fwd_g2<true>, 256, 0});
  v.push_back({"k_aff_bwd_g2<packed>", (const void*)k_aff_bwd_g2<true>, 256, 0});
  v.push_back({"k_aff_fwd_g2", (const void*)k_aff_fwd_g2<false>, 256, 0});
  v.push_back({"k_aff_bwd_g2", (const void*)k_aff_bwd_g2<false>, 256, 0});
}

}  // namespace bh
