// G1Ops instantiation of the device MSM, part 2: continuation fix-up, bucket reduction
// and window sums (see msm_impl.cuh).
#include "msm_impl.cuh"

namespace bh {
// instantiated in msm_g1_acc.hip (the accumulation kernels compile there, in parallel)
extern template struct MsmWorkspace<G1Ops>;
extern template void fit_segments<G1Ops>(MsmShape&, size_t);
extern template void fit_segments_E<G1Ops>(MsmShape&, size_t);
extern template hipError_t msm_sort<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, size_t, const int32_t*,
                                            uint32_t, const MsmShape&);
extern template hipError_t msm_accumulate<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, size_t,
                                                  const MsmShape&, MsmTiming*);

template hipError_t msm_window_sums<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, const uint32_t*, size_t,
                                         const int32_t*, uint32_t, const MsmShape&, MsmTiming*);
template hipError_t msm_front<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, const uint32_t*, const uint32_t*, size_t,
                                   const int32_t*, uint32_t, const MsmShape&, MsmTiming*);
template hipError_t msm_back<G1Ops>(MsmWorkspace<G1Ops>&, hipStream_t, size_t, const MsmShape&, typename G1Ops::P*, int, hipEvent_t, const uint32_t*);
template void msm_back_kernels<G1Ops>(std::vector<KernInfo>&);

// resident threads per CU of the G1 bucket reduction at its launch shape (msm_back: 256-thread
// blocks, one point of LDS per thread)
size_t reduce_blocks_resident_per_cu_g1() {
  int blocks = 1;
  const int BT = (int)reduce_block_max(false);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, (const void*)k_reduce_blocks<G1Ops>, BT,
                                                   BT * sizeof(typename G1Ops::P)) != hipSuccess ||
      blocks < 1)
    blocks = 1;
  return (size_t)blocks * BT;
}
}  // namespace bh
