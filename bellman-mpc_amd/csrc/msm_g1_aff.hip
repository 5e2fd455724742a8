// G1 instantiation of the batch-affine bucket accumulation (msm_aff.cuh), the shared AffineBufs
// and the level plan.
#include "msm_aff.cuh"

namespace bh {

namespace {
// the forward kernel at four waves per SIMD (128 VGPRs): its gathers hide behind occupancy
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_aff_fwd_g1(const uint32_t* entries, const uint32_t* src, uint32_t rec, const uint32_t* in_off,
             const uint32_t* out_off, uint32_t nbt, uint32_t K, uint32_t* pre, uint32_t* prod) {
  aff::aff_fwd<aff::G1A, false>(entries, src, rec, in_off, out_off, nbt, K, pre, prod);
}
__global__ void __launch_bounds__(256) k_aff_bwd_g1(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                                    const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt,
                                                    uint32_t K, const uint32_t* pre, const uint32_t* prod,
                                                    uint32_t* dst) {
  __shared__ uint4 lds[4 * 2 * aff::G1A::Q_RAW * 64];
  aff::aff_bwd<aff::G1A, false>(entries, src, rec, in_off, out_off, nbt, K, pre, prod, dst, lds);
}
}  // namespace

hipError_t AffineBufs::reserve(size_t pts0, size_t pts1, size_t pre_bytes) {  // (mu held)
  hipError_t e;
  const size_t want[2] = {pts0, pts1};
  for (int i = 0; i < 2; i++) {
    if (want[i] <= cap_pts[i]) continue;
    if (pts[i]) (void)hipFree(pts[i]);
    pts[i] = nullptr;
    cap_pts[i] = 0;
    if ((e = hipMalloc(&pts[i], want[i])) != hipSuccess) return e;
    cap_pts[i] = want[i];
  }
  if (pre_bytes > cap_pre) {
    if (pre) (void)hipFree(pre);
    pre = nullptr;
    cap_pre = 0;
    if ((e = hipMalloc(&pre, pre_bytes)) != hipSuccess) return e;
    cap_pre = pre_bytes;
  }
  return hipSuccess;
}

void AffineBufs::release() {
  for (int i = 0; i < 2; i++) {
    if (pts[i]) (void)hipFree(pts[i]);
    pts[i] = nullptr;
    cap_pts[i] = 0;
  }
  if (pre) (void)hipFree(pre);
  pre = nullptr;
  cap_pre = 0;
}

AffinePlan affine_plan(size_t Emax, size_t nbt, int halves, size_t resident, bool g2) {
  AffinePlan pl;
  const bool on = aff::env_int(g2 ? "BH_AFFINE_G2" : "BH_AFFINE_G1", aff::env_int("BH_AFFINE", 0)) != 0;
  const int rounds = std::max(1, aff::env_int("BH_AFF_ROUNDS", 2));
  const int kmin = std::max(1, aff::env_int("BH_AFF_KMIN", 16));
  const int lmax = std::min(AFF_LMAX, std::max(0, aff::env_int("BH_AFF_LEVELS", AFF_LMAX)));
  const size_t min_e = (size_t)std::max(1, aff::env_int("BH_AFF_MIN_E", 1 << 18));
  pl.Eb[0] = Emax;
  if (!on || halves || Emax < min_e) return pl;
  const size_t T = (size_t)rounds * resident;
  for (int l = 0; l < lmax; l++) {
    const size_t Eo = (pl.Eb[l] + nbt) / 2 + 1;  // >= sum_b ceil(c_b / 2)
    const size_t K = (Eo + T - 1) / T;
    if (K < (size_t)kmin) break;
    pl.K[l] = (uint32_t)K;
    pl.blocks[l] = (uint32_t)((Eo + K * 256 - 1) / (K * 256));
    pl.Eb[l + 1] = Eo;
    pl.levels = l + 1;
  }
  return pl;
}

AffinePlan affine_plan_g1(size_t Emax, size_t nbt, int halves) {
  static const size_t resident = aff::resident_of((const void*)k_aff_bwd_g1);
  return affine_plan(Emax, nbt, halves, resident, false);
}

hipError_t affine_levels_g1(MsmWorkspace<G1Ops>& ws, hipStream_t st, const uint32_t* d_bases, uint32_t rec,
                            const AffinePlan& pl, size_t nbt, const uint32_t** final_pts) {
  return aff::levels_run<aff::G1A>(ws, st, d_bases, rec, pl, nbt, k_aff_fwd_g1, k_aff_bwd_g1, k_aff_fwd_g1,
                                   k_aff_bwd_g1, final_pts);
}

void aff_kernels_g1(std::vector<KernInfo>& v) {
  v.push_back({"k_aff_fwd_g1", (const void*)k_aff_fwd_g1, 256, 0});
  v.push_back({"k_aff_bwd_g1", (const void*)k_aff_bwd_g1, 256, 0});
}

}  // namespace bh
