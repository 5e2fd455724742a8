// Internal types shared by the C ABI implementation files.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/bellman_hip.h"
#include "host_arith.h"
#include "msm.h"
#include "ntt.h"
#include "staging.h"

namespace bh {

#define BH_TRY_HIP(expr)                                  \
  do {                                                    \
    hipError_t _e = (expr);                               \
    if (_e != hipSuccess) {                               \
      bh::set_last_hip_error(_e);                         \
      return (_e == hipErrorOutOfMemory) ? BH_ERR_OUT_OF_MEMORY : BH_ERR_HIP; \
    }                                                     \
  } while (0)

void set_last_hip_error(hipError_t e);

// device buffer owning wrapper
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t b) {
    if (b <= bytes && p) return hipSuccess;
    if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
    hipError_t e = hipMalloc(&p, b ? b : 16);
    if (e == hipSuccess) bytes = b;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// NTT domain tables for one log size (device, unpacked 9-limb entries)
struct Domain {
  int L = -1;
  DevBuf tw_fwd, tw_inv;                  // omega^j, omega^-j, j < m/2
  DevBuf lv_fwd, lv_inv;                  // per-level twiddles, 9 limbs each (launch_level_table)
  DevBuf coset_lo, coset_hi;              // g^i split tables, hi folded with m^-1   (ifft -> coset)
  DevBuf coset_hi32;                      // the same hi table times 32: the ifft of bls12_381-Montgomery
                                          // input (R = 2^256) read as device values (R = 2^261)
  DevBuf icoset_lo, icoset_hi;            // g^-i split, hi folded with m^-1        (icoset)
  DevBuf gpow_lo, gpow_hi;                // g^i (no m^-1)                           (coset_fft input)
  // the H block's post-scale factors as full m-entry tables (coset, coset x 32, icoset: 36 B per
  // entry, 453 MB at 2^22): one product per element in the storing pass instead of two
  DevBuf coset_full, coset32_full, icoset_full;
  DevBuf consts;                          // [0] m^-1, [1] 1/Z(g), [2] one
  int lo_bits = 0;
  Fr minv, zinv;
};

// a device-resident EvaluationDomain's buffers (evaldomain.hip): coefficients, permute scratch,
// post-scale table, and the event after the last work that read them on ctx->stream; a freed
// domain's set is pooled by its context for the next one (no hipFree / hipMalloc per call)
struct EvdomBufs {
  DevBuf buf, tmp, post;
  hipEvent_t idle = nullptr, landed = nullptr;  // landed: the last upload into buf (bg.cst)
  EvdomBufs() = default;
  EvdomBufs(const EvdomBufs&) = delete;
  EvdomBufs& operator=(const EvdomBufs&) = delete;
  ~EvdomBufs() {
    if (idle) (void)hipEventDestroy(idle);
    if (landed) (void)hipEventDestroy(landed);
  }
};

struct bh_ctx_impl;
struct DistH;
}  // namespace bh

struct bh_job_slot;  // jobs.hip: one in-flight async multiexp's stream, workspace and buffers
struct bh_job;
// jobs.hip: the async multiexps' recycled slots and the jobs not yet waited for.  Shared by the
// context and every outstanding job, so it outlives bh_ctx_destroy: a job of a destroyed
// context is detached (its wait reports an error and touches nothing of the context).
struct bh_job_registry {
  std::mutex mu;
  bool alive = true;                       // false once the context is destroyed
  std::vector<bh_job_slot*> all_slots, free_slots;
  std::vector<bh_job*> pending;            // submitted, not yet waited for
  // recent digit sorts, by what determines them (jobs.hip: a job with the same scalars, density
  // map, base offset and digit geometry copies the sorted entries instead of sorting again, as
  // bh_prove does for b_g1_aux / b_g2_aux); valid while the slot has not been taken again
  struct SortRec {
    uint64_t scalars_id = 0;  // bh_scalar_buf::id (never reused)
    uint64_t dens_hash = 0;
    size_t n = 0, base_offset = 0;
    int c = 0, W = 0, NB = 0, Wb = 0, pre = 0;
    bh_job_slot* slot = nullptr;
    int group = 0;
    uint64_t use = 0;
  };
  std::vector<SortRec> sorts;
};

struct bh_srs {
  bh_ctx* ctx = nullptr;
  int group = BH_G1;
  size_t n = 0;
  bh::DevBuf pts;                    // packed affine, device Montgomery
  std::vector<size_t> identity_idx;  // indices of points at infinity (rejected by next())
  // prover window table (built lazily, see prepare_tables in prover.hip) over the bases
  // [win_lo, win_hi) -- a shard's slice or the whole vector:
  // win[(i - win_lo)*win_W + w] = 2^(win_c*w) * P_i, packed affine, one record per win_rec words
  // (shared: an asynchronous multiexp reading the table holds it until its wait, so a rebuild
  // never frees or overwrites a table under a job in flight; win_mu guards the fields for those
  // readers, the prover reads them under its Parameters lock)
  std::shared_ptr<bh::DevBuf> win = std::make_shared<bh::DevBuf>();
  mutable std::mutex win_mu;
  int win_c = 0, win_W = 0, win_rec = 0;  // win_rec: u32 words per record (128-B aligned)
  size_t win_lo = 0, win_hi = 0;
  // the table addressed by GLOBAL base index (entries encode i*W + w): the allocation shifted
  // back by win_lo records (only indices in [win_lo, win_hi) are ever formed)
  const uint32_t* win_global() const {
    return reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(win->p) -
                                             (uintptr_t)win_lo * (uintptr_t)win_W * (uintptr_t)win_rec * 4u);
  }
  bool win_covers(int c, size_t lo, size_t hi) const { return win_c == c && win_c && win_lo <= lo && hi <= win_hi; }
  // the last table request that could not be met (HBM short): not retried every proof
  int skip_c = 0;
  size_t skip_lo = 0, skip_hi = 0;
};

struct bh_params {
  bh_ctx* ctx = nullptr;
  // window tables and h shares: built under an exclusive lock, read by proofs under a shared
  // one (several contexts of one device may prove with one Parameters)
  std::shared_mutex mu;
  // VerifyingKey (host form)
  bh::AffinePt<bh::Fp> alpha_g1, beta_g1, delta_g1;
  bh::AffinePt<bh::Fp2> beta_g2, gamma_g2, delta_g2;
  std::vector<bh::AffinePt<bh::Fp>> ic;
  bh_srs h, l, a, b_g1, b_g2;
  // h bases of one rank's distributed-H share (dist_h.h: h[M*t + q], q in the rank's chunk),
  // gathered into share order so that a shard-sized window table covers them; key (N, rank, L)
  std::map<std::tuple<int, int, int>, std::unique_ptr<bh_srs>> h_shares;
  // host copies of the leading bases of a, b_g1, b_g2 (the public inputs' bases), read back from
  // the device on first use for the host input multiexps: under head_mu, only ever grown, and
  // each proof copies the points it needs out while holding it (prover.hip host_input_msms)
  std::mutex head_mu;
  std::vector<bh::AffinePt<bh::Fp>> h_a_head, h_b1_head;
  std::vector<bh::AffinePt<bh::Fp2>> h_b2_head;
};

constexpr size_t TABLE_MIN_USED = (size_t)1 << 16;  // smaller multiexps use plain windows

// A device-resident scalar vector (bh_scalars_upload, bh_compute_h_scalars): canonical packed
// Fr (8 LE u32 each), shared by every multiexp submitted on it; `ready` is recorded once the
// producing stream has written it (submits order their streams after it).
// bh_compute_h_scalars produces it from a host thread (`producer`: the a, b, c upload and the H
// passes): until that thread has enqueued its work (`enqueued`), `ready` is not recorded yet, so
// multiexps submitted meanwhile park their own enqueue in `deferred`, which the producer runs,
// under mu, right after recording `ready` (argument: the producer's status).
// Device buffers of finished scalar vectors, kept per device for the next vector of the same size
// (api.hip): a vector's hipFree would wait for the whole device, and a caller that drops one while
// another proof's multiexps run (a seam caller's Arcs) would hold every HIP call of the process
// behind them.  take: a buffer of at least `bytes` or null; give: keeps it (bounded) or frees it.
extern "C" void* scalar_pool_take(int device, size_t bytes, size_t* got);
// selftest.hip (tests/test_gpu_selftest.py): fe2_mul_sub_kara and the two-product form on
// caller-chosen operands
extern "C" bh_status bh_selftest_fp2_mul_sub(int device, const uint32_t* in, size_t n, uint32_t* out);
struct bh_scalar_buf;
// a device scalar vector of n canonical scalars (pooled), its ready event created
extern "C" bh_status new_scalar_buf(bh_ctx* ctx, size_t n, std::shared_ptr<bh_scalar_buf>* out);
extern "C" void scalar_pool_give(int device, void* p, size_t bytes);
extern "C" void scalar_pool_drain(int device);  // frees every pooled buffer of the device

struct bh_scalar_buf {
  bh::DevBuf d;
  uint64_t id = 0;  // unique per vector (jobs' sort sharing is keyed on it, not on d's address)
  // the context whose producer thread (if any) makes it: only that context may park deferred
  // enqueues on it (its teardown waits for its producers, which run them)
  const bh_ctx* owner = nullptr;
  hipEvent_t ready = nullptr;
  int device = 0;
  std::mutex mu;
  std::condition_variable cv;
  bool enqueued = true;
  bh_status status = BH_OK;
  // bh_compute_h_scalars' producer, ms since the call: [0..3) a, b, c copies enqueued, [3] H enqueued,
  // [4] deferred multiexps enqueued, [5] submits deferred behind it
  double stamps[6] = {-1, -1, -1, -1, -1, 0};
  std::vector<std::function<void(bh_status)>> deferred;
  std::thread producer;
  void wait_enqueued() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return enqueued; });
  }
  ~bh_scalar_buf() {
    if (producer.joinable()) producer.join();
    if (ready) {
      (void)hipSetDevice(device);
      (void)hipEventSynchronize(ready);
      (void)hipEventDestroy(ready);
    }
    // Invariant for the pool (no device sync here): nothing in flight still reads this buffer.
    // The producer's H wrote it behind `ready` (synchronised above), and every multiexp that read
    // it holds this shared buffer until its wait has host-synchronised the work (jobs.hip).
    if (d.p) scalar_pool_give(device, d.p, d.bytes);
    d.p = nullptr;
    d.bytes = 0;
  }
};
struct bh_scalars {
  size_t n = 0;
  std::shared_ptr<bh_scalar_buf> buf;
};

struct bh_witness {
  bh_ctx* ctx = nullptr;
  size_t num_constraints = 0, m = 0, num_inputs = 0, num_aux = 0;
  int log_m = 0;
  bh::DevBuf abc;          // 3 * m packed device-Montgomery Fr (a | b | c), zero padded
  bh::DevBuf inputs, aux;  // canonical packed scalars
  bh::DevBuf dens;         // a_aux | b_input | b_aux density words
  size_t a_aux_words = 0, b_in_words = 0, b_aux_words = 0;
  std::vector<uint64_t> a_aux_density, b_input_density, b_aux_density;  // host copies (EOF checks)
  size_t a_aux_total = 0, b_in_total = 0, b_aux_total = 0;
  // set bits before word k of each density map (k = 0..words): base index of a scalar shard
  std::vector<size_t> a_aux_prefix, b_aux_prefix;
  // the density index maps (a_aux | b_input | b_aux: base index or -1 per scalar), built once at
  // bh_witness_upload: a function of the density words only (the prover builds them per proof for
  // bh_prove's per-call witness)
  bh::DevBuf idx3;
  bool idx_ready = false;
  // raw = true: abc/inputs/aux hold the caller's bls12_381 Montgomery words, not yet converted
  // (bh_prove's asynchronous upload; the prover converts on its own streams)
  bool raw = false;
  // the public inputs as canonical scalars on the host too (4 LE u64 each): the input
  // multiexps of a proof are a handful of terms and run on a host thread (prover.hip)
  std::vector<uint64_t> h_inputs;
};

struct bh_ctx {
  int device = 0;
  bool cu_masked = false;  // its tail streams are CU-masked (the first live context of a device)
  bool borrowed_streams = false;  // a pipelined batch lane: the streams are its primary's (ctx_create_lane)
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // prover: the multiexps' reduction tails (high priority)
  hipStream_t stream3 = nullptr;  // prover: density maps and the multiexps' sorts (high priority)
  hipStream_t stream4 = nullptr;  // prover: H pipeline
  hipStream_t stream5 = nullptr;  // prover: the second G1 accumulation lane
  // prover: reduction-tail streams (high priority, CU-masked on the first context of a device).
  // A proof has at most 5 large multiexps unless the public inputs number in the thousands;
  // more tails share these round robin.  Kept small for the device's hardware-queue budget
  // (24 CP queues per MI355X, DESIGN.md section 5: a CU-masked stream owns a queue).
  static constexpr int TAIL_STREAMS = 5;
  hipStream_t tstream[TAIL_STREAMS] = {};
  bh::DistH* dist = nullptr;       // prover: this rank's distributed-H state (bh_prove_witness_partial_comm)
  int window_override = 0;
  int tables = 1;  // 1: the prover builds and uses SRS window tables (bh_ctx_set_tables)
  // contexts of this device running ranks of one proof side by side (the virtual ranks of
  // bh_prove_witness_partials_local): bucket shards weigh their workspaces by it
  int co_ranks = 1;
  bh::MsmWorkspace<G1Ops> g1ws;
  bh::MsmWorkspace<G2Ops> g2ws;
  // one workspace per prover multiexp (result slot order), so that sorts, accumulations and
  // tails of different multiexps never share buffers (about 1 GB each at 2^22 points)
  bh::MsmWorkspace<G1Ops> pw1[6];
  bh::MsmWorkspace<G2Ops> pw2[2];
  XYZZ<G1F>* host_out1 = nullptr;     // pinned, 8 jobs x 128 windows (c >= 2)
  XYZZ<Fp2Ops>* host_out2 = nullptr;  // pinned, 2 jobs x 128 windows
  hipEvent_t jev[48] = {};
  std::map<int, std::unique_ptr<bh::Domain>> domains;
  bh::DevBuf staging;     // generic host->device staging (scalars, polynomials)
  bh::DevBuf staging2;
  bh::DevBuf idx;         // density index map
  bh::DevBuf dtmp;        // density scan tmp
  bh::DevBuf dscan;       // scan scratch
  bh::DevBuf dscan2;      // scan scratch of derived (compacted) sorts
  bh::DevBuf hbuf;        // H pipeline scratch (h scalars canonical)
  bh::DevBuf idx3;        // density index maps of a_aux | b_input | b_aux
  hipEvent_t ev[16] = {};
  double last_timings[24] = {};  // bh_last_timings [0,10) + bh_last_stats extras
  hipEvent_t fft_ev[4] = {};     // bh_fft & co.: upload / transform / download boundaries
  uint32_t* host_counts = nullptr;  // pinned: [0,16) entries (= mixed additions) of each prover multiexp
  uint32_t* host_spans = nullptr;   // pinned: MAX_SPAN_BLOCKS per-workgroup max_span words per prover multiexp
  bh::DevBuf dspan;                 // device words for max_span (the same layout)
  std::vector<bh_ctx*> vranks;      // bh_prove_witness_partials_local: the virtual ranks' contexts
  std::vector<bh_ctx*> lanes;       // bh_prove_batch: the lanes' contexts
  // host -> device staging of caller buffers (bh_prove, bh_witness_upload): H2D copy stream,
  // pinned ring, memcpy threads; dropin = the device witness bh_prove reuses call after call
  hipStream_t h2d = nullptr;
  bh::H2DRing ring;
  std::unique_ptr<bh::HostPool> pool;
  bh_witness* dropin = nullptr;
  // bh_compute_h_scalars' producer threads: their own copy stream, pinned ring, memcpy workers and
  // a|b|c buffer (under bg.mu, one producer at a time), so that an upload in flight never holds
  // mu; bh_ctx_destroy waits for bg_active == 0
  struct Background {
    std::mutex mu;
    hipStream_t st = nullptr;   // the H transforms
    hipStream_t cst = nullptr;  // the a, b, c copies
    hipEvent_t vec[4] = {};     // a, b, c landed; [3] the previous producer's H done
    bh::H2DRing ring;
    std::unique_ptr<bh::HostPool> pool;
    bh::DevBuf abc;
    std::atomic<int> fg_uploads{0};  // bh_scalars_upload copies in flight (the producer pauses)
    std::mutex count_mu;
    std::condition_variable cv;
    int active = 0;
  } bg;
  // device-resident EvaluationDomains (evaldomain.hip): one thread uploads their coefficients in
  // call order through the bg copy machinery (under bg.mu), so an ifft can run while the next
  // domain is still streaming in; bh_ctx_destroy drains and joins it
  struct DomainUploads {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    std::thread th;
    bool stop = false;
  } dup;
  std::vector<std::unique_ptr<bh::EvdomBufs>> evdom_pool;  // freed domains' buffers (under mu)
  // bh_multiexp_submit / _wait (jobs.hip): recycled per-job resources under their own lock (a
  // submit never waits behind a proof holding mu)
  std::shared_ptr<bh_job_registry> jobs = std::make_shared<bh_job_registry>();
  std::mutex mu;
  // scratch budget (scratch.cpp), computed once: see bh_scratch_report
  bool scratch_done = false;
  bool counted = false;  // in api.hip's live-context count of its device
  uint64_t scratch_rep[10] = {};
  std::string scratch_worst;
};

void bh_ctx_release_jobs(bh_ctx* ctx);
extern "C" bh_status ctx_create_lane(bh_ctx* primary, bh_ctx** out);  // (defined in api.hip's C block; not exported in the header)

namespace bh {
bh_status ctx_domain(bh_ctx* ctx, int L, Domain** out);
// background copies (caller holds ctx->bg.mu): create the bg streams / ring once; copy pageable
// host bytes to the device on bg.cst (returns once the host buffer has been read)
bh_status bg_init(bh_ctx* ctx);
// split power tables g^i = lo[i & mask] * hi[i >> lo_bits] (hi scaled by hi_scale), uploaded on
// ctx->stream and synchronised (caller holds ctx->mu)
bh_status upload_split_table(bh_ctx* ctx, DevBuf& lo, DevBuf& hi, const Fr& g, const Fr& hi_scale, int L,
                             int lo_bits);
bh_status bg_copy(bh_ctx* ctx, void* dst, const void* src, size_t bytes);
// wait for every stream of the context (error paths, teardown)
void ctx_sync_all(bh_ctx* ctx);
// host <-> device Fr helpers
void fr_to_dev_limbs(const Fr& x, uint32_t out[9]);
void fr_to_dev_packed(const Fr& x, uint32_t out[8]);
Fr fr_from_dev_packed(const uint32_t in[8]);
// G1 device coordinates (C::reduce output, G1F's limb or balanced-digit form; packed words) -> host
Fp fp_from_dev_g1(const G1F::T& x);
Fp fp_from_dev_words_g1(const uint32_t* w);
// combine per-window sums (host Horner, multiexp.rs:244-249)
Jac<Fp> combine_g1(const XYZZ<G1F>* ws, const MsmShape& sh);
Jac<Fp2> combine_g2(const XYZZ<Fp2Ops>* ws, const MsmShape& sh);
// run one MSM whose scalars/index map are already on the device; returns result on host
bh_status msm_g1_device(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint32_t* d_scalars, size_t n,
                        const int32_t* d_idx, Jac<Fp>* out, float* acc_ms);
bh_status msm_g2_device(bh_ctx* ctx, const bh_srs* bases, size_t base_offset, const uint32_t* d_scalars, size_t n,
                        const int32_t* d_idx, Jac<Fp2>* out, float* acc_ms);
bh_status upload_fr(bh_ctx* ctx, const uint64_t* host, size_t n, size_t padded, uint32_t* dst);
// the same through the context's pinned staging ring, enqueued on st (caller holds ctx->mu)
bh_status upload_fr_staged(bh_ctx* ctx, const uint64_t* host, size_t n, size_t padded, uint32_t* dst, hipStream_t st);
bh::HostPool& ctx_pool(bh_ctx* ctx);
// bls12_381 Montgomery (R = 2^256) -> device Montgomery (R = 2^261) multiplier for launch_fr_convert
FrConst fr_to_dev_const();
bh_status download_fr(bh_ctx* ctx, uint32_t* src, size_t n, uint64_t* host);
bh_status run_h_pipeline(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, const uint32_t* src_abc = nullptr,
                         uint32_t* hout = nullptr);
// the same in stages, so that each vector's transforms can be enqueued as its upload lands:
// run_h_vector(v) for v = 0, 1, 2 in order (v = 2 folds (a*b - c)/Z into a), then run_h_final
// raw_src: src_abc holds bls12_381 Montgomery words (read in place, the factor 2^5 between the
// two Montgomery radices folded into the ifft's storing-pass scale); its padding must be zero
bh_status run_h_vector(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, const uint32_t* src_abc, int v,
                       bool raw_src = false);
bh_status run_h_final(bh_ctx* ctx, Domain* D, uint32_t* d_abc, hipStream_t st, uint32_t* hout);
bh_status srs_from_bytes(bh_ctx* ctx, int group, const uint8_t* bytes, size_t n, int checked, bool reject_identity,
                         bh_srs* out);
// reference-exact error semantics of multiexp (EOF / identity), host side
bh_status multiexp_check(const bh_srs* bases, size_t base_offset, const uint64_t* density_words, size_t n,
                         const uint64_t* exps_canonical, bool need_exps);
bh_status srs_upload_affine(bh_ctx* ctx, int group, const void* host_affine_g1_or_g2, size_t n, bh_srs* out);
// The all-to-all step of the distributed H pipeline: for each of nvec vectors of M = N*C
// packed-Fr elements, chunk p of send goes to rank p, which stores it as chunk `this rank` of
// recv; stream-ordered on st.  Over RCCL (comm.cpp) or, to run the identical prover code with N
// virtual ranks on one device, by device copies between threads (prover.hip).
struct Exchanger {
  virtual ~Exchanger() {}
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual bh_status exchange(const uint32_t* send, uint32_t* recv, size_t C, size_t M, int nvec, hipStream_t st) = 0;
};
std::unique_ptr<Exchanger> rccl_exchanger(bh_comm* c);
// smallest rank count that uses the distributed H pipeline (2)
size_t dist_h_min_ranks();
// the scratch budget check (scratch.cpp): BH_ERR_SCRATCH_LIMIT when the worst spilling kernel's
// per-queue scratch times the context's queues exceeds the device's scratch limit (thread-safe;
// computed once per context)
bh_status scratch_report(bh_ctx* ctx, uint64_t out[10], std::string* worst);
// live contexts of a device (api.hip)
int live_contexts(int device);
bh_status scratch_check(bh_ctx* ctx);
int comm_rank(const bh_comm* c);
int comm_size(const bh_comm* c);
}  // namespace bh
