// G1Ops instantiation of the device MSM, part 1: workspace, digit sort and the bucket
// accumulation kernels (see msm_impl.cuh).
#include "msm_impl.cuh"

namespace bh {
template struct MsmWorkspace<G1Ops>;
template void fit_segments<G1Ops>(MsmShape&, size_t);
template void fit_segments_E<G1Ops>(MsmShape&, size_t);
template hipError_t msm_sort<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, size_t, const int32_t*,
                                     uint32_t, const MsmShape&);
template hipError_t msm_accumulate<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, size_t, const MsmShape&,
                                           MsmTiming*);
template void msm_acc_kernels<G1Ops>(std::vector<KernInfo>&);
}  // namespace bh
