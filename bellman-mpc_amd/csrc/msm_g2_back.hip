// G2Ops instantiation of the device MSM, part 2: continuation fix-up, bucket reduction
// and window sums (see msm_impl.cuh).
#include "msm_impl.cuh"

namespace bh {
// instantiated in msm_g2_acc.hip (the accumulation kernels compile there, in parallel)
extern template struct MsmWorkspace<G2Ops>;
extern template void fit_segments<G2Ops>(MsmShape&, size_t);
extern template void fit_segments_E<G2Ops>(MsmShape&, size_t);
extern template hipError_t msm_sort<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, size_t, const int32_t*,
                                            uint32_t, const MsmShape&);
extern template hipError_t msm_accumulate<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, size_t,
                                                  const MsmShape&, MsmTiming*);

template hipError_t msm_window_sums<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, const uint32_t*, size_t,
                                         const int32_t*, uint32_t, const MsmShape&, MsmTiming*);
template hipError_t msm_front<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, const uint32_t*, const uint32_t*, size_t,
                                   const int32_t*, uint32_t, const MsmShape&, MsmTiming*);
template hipError_t msm_back<G2Ops>(MsmWorkspace<G2Ops>&, hipStream_t, size_t, const MsmShape&, typename G2Ops::P*, int, hipEvent_t, const uint32_t*);
template void msm_back_kernels<G2Ops>(std::vector<KernInfo>&);
}  // namespace bh
