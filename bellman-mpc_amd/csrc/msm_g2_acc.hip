// G2Ops instantiation of the device MSM, part 1: workspace, digit sort and the bucket
// accumulation kernels (see msm_impl.cuh).  The accumulation's Fp2 products use the column-wise
// Karatsuba form (field.cuh); every kernel of this unit is emitted here only.
#define BH_FP2_KARATSUBA 1
#include "msm_impl.cuh"

namespace bh {
template struct MsmWorkspace<G2Ops>;
template void fit_segments<G2Ops>(MsmShape&, size_t);
template void fit_segments_E<G2Ops>(MsmShape&, size_t);
template hipError_t msm_sort<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, size_t, const int32_t*,
                                     uint32_t, const MsmShape&);
template hipError_t msm_accumulate<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, size_t, const MsmShape&,
                                           MsmTiming*);
template void msm_acc_kernels<G2Ops>(std::vector<KernInfo>&);
}  // namespace bh
