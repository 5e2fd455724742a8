// Scratch (private segment) budget of the library's kernels against the device's scratch limit.
//
// A kernel that spills keeps its private segment in scratch memory, which the runtime (ROCr)
// provisions per hardware queue for the waves a dispatch can have in flight: bytes/lane x 64
// lanes x waves.  The amount is shared by every queue of the device
// (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX); a dispatch whose need cannot be met fails inside the
// runtime with HSA_STATUS_ERROR_OUT_OF_RESOURCES and aborts the process -- the round-2 failure of
// k_reduce_window<G2> (2 648 B/lane at the time).  Here each kernel's private-segment size
// (hipFuncGetAttributes) and occupancy give its worst per-queue need; times the queues one context
// can run such kernels on at once, it is compared with the limit before a proof or multiexp is
// enqueued, which then returns BH_ERR_SCRATCH_LIMIT instead of reaching the abort.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "api_internal.h"
#include "dist_h.h"

namespace bh {

namespace {

struct AgentQuery {
  uint32_t bdf = 0, domain = 0;
  bool found = false;
  uint64_t limit_max = 0, limit_cur = 0;
};

hsa_status_t visit_agent(hsa_agent_t a, void* p) {
  AgentQuery* q = static_cast<AgentQuery*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, dom = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  if (bdf != q->bdf || dom != q->domain) return HSA_STATUS_SUCCESS;
  q->found = true;
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX, &q->limit_max);
  (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT, &q->limit_cur);
  return HSA_STATUS_INFO_BREAK;
}

}  // namespace

// out: [0] device scratch limit (bytes, shared by all queues; 0 = unknown), [1] current per-queue
// threshold, [2] worst bytes/lane, [3] its per-queue need at the scratch-slot bound (bytes),
// [4] queues counted, [5] the context's total need, [6] fits (1/0), [7] kernels checked, [8] the
// worst kernel's per-queue need at its occupancy, [9] live contexts on the device now (the limit is
// shared by all of them: [5] x [9] bounds a device full of such contexts running at once).
// Scope of the decision [6]: ONE context's queues.  Further contexts of the device -- a batch's
// lanes (which borrow their primary's streams: no queue more) and the one-device rehearsal's
// virtual ranks (which prove one after another) -- are counted in [9], refreshed on every call,
// but not in [6]: callers that run several contexts' proofs concurrently on one device must
// budget [5] x [9] themselves (bh_scratch_report exposes both).
bh_status scratch_report(bh_ctx* ctx, uint64_t out[10], std::string* worst) {
  static std::mutex mu;  // (computed once per context, by whichever thread asks first)
  std::lock_guard<std::mutex> lk(mu);
  if (ctx->scratch_done) {
    ctx->scratch_rep[9] = (uint64_t)std::max(1, live_contexts(ctx->device));
    memcpy(out, ctx->scratch_rep, sizeof(ctx->scratch_rep));
    if (worst) *worst = ctx->scratch_worst;
    return BH_OK;
  }
  BH_TRY_HIP(hipSetDevice(ctx->device));
  hipDeviceProp_t prop;
  BH_TRY_HIP(hipGetDeviceProperties(&prop, ctx->device));
  AgentQuery q;
  q.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
  q.domain = (uint32_t)prop.pciDomainID;
  if (hsa_init() == HSA_STATUS_SUCCESS) {
    (void)hsa_iterate_agents(visit_agent, &q);
    (void)hsa_shut_down();
  }
  std::vector<KernInfo> ks;
  msm_acc_kernels<G1Ops>(ks);
  msm_acc_kernels<G2Ops>(ks);
  msm_back_kernels<G1Ops>(ks);
  msm_back_kernels<G2Ops>(ks);
  ntt_kernels(ks);
  dist_kernels(ks);
  const uint64_t cus = (uint64_t)std::max(prop.multiProcessorCount, 1);
  const uint64_t slots_per_cu = 32;  // KFD max_slots_scratch_cu (profiles/r03_kfd_queue_props.txt)
  // per queue: at the scratch-slot bound (what the runtime may reserve for a large dispatch:
  // 32 waves per CU) and at the kernel's occupancy (the waves resident at once)
  uint64_t worst_need = 0, worst_lane = 0, worst_resident = 0;
  std::string wname = "-";
  for (const KernInfo& k : ks) {
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, k.fn) != hipSuccess) continue;
    const uint64_t lane = (uint64_t)a.localSizeBytes;
    if (!lane) continue;
    int blocks = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k.fn, k.block, k.lds) != hipSuccess || blocks < 1)
      blocks = 1;
    const uint64_t waves_cu = std::min<uint64_t>(slots_per_cu, (uint64_t)blocks * ((k.block + 63) / 64));
    const uint64_t per_lane = (lane + 15) / 16 * 16;
    const uint64_t need = per_lane * 64 * slots_per_cu * cus;
    if (need > worst_need) {
      worst_need = need;
      worst_lane = lane;
      worst_resident = per_lane * 64 * waves_cu * cus;
      wname = k.name;
    }
  }
  // queues of one context that run spilling kernels concurrently: the reduction tails, the small
  // multiexps' stream and the (distributed) H stream
  const uint64_t queues = (uint64_t)bh_ctx::TAIL_STREAMS + 2;
  const uint64_t total = worst_need * queues;
  const bool fits = q.limit_max == 0 || total <= q.limit_max;
  ctx->scratch_rep[0] = q.limit_max;
  ctx->scratch_rep[1] = q.limit_cur;
  ctx->scratch_rep[2] = worst_lane;
  ctx->scratch_rep[3] = worst_need;
  ctx->scratch_rep[4] = queues;
  ctx->scratch_rep[5] = total;
  ctx->scratch_rep[6] = fits ? 1 : 0;
  ctx->scratch_rep[7] = ks.size();
  ctx->scratch_rep[8] = worst_resident;
  ctx->scratch_rep[9] = (uint64_t)std::max(1, live_contexts(ctx->device));
  ctx->scratch_worst = wname;
  ctx->scratch_done = true;
  memcpy(out, ctx->scratch_rep, sizeof(ctx->scratch_rep));
  if (worst) *worst = wname;
  return BH_OK;
}

bh_status scratch_check(bh_ctx* ctx) {
  uint64_t r[10];
  bh_status s = scratch_report(ctx, r, nullptr);
  if (s) return s;
  return r[6] ? BH_OK : BH_ERR_SCRATCH_LIMIT;
}

}  // namespace bh

extern "C" bh_status bh_scratch_report(bh_ctx* ctx, uint64_t* out, size_t n, char* worst_kernel, size_t cap) {
  if (!ctx || (!out && n)) return BH_ERR_INVALID_ARGUMENT;
  uint64_t r[10];
  std::string w;
  bh_status s = bh::scratch_report(ctx, r, &w);
  if (s) return s;
  for (size_t i = 0; i < n && i < 10; i++) out[i] = r[i];
  if (worst_kernel && cap) {
    const size_t m = std::min(cap - 1, w.size());
    memcpy(worst_kernel, w.data(), m);
    worst_kernel[m] = 0;
  }
  return BH_OK;
}
