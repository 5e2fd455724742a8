// Host interface of the device Pippenger MSM (msm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>

#include "curve.cuh"
#include "kinfo.h"

namespace bh {

// Window-table record of a G1 base (one 128-byte line): the affine x and y as 14 + 14 raw 29-bit
// device limbs (canonical values), so the accumulation reads its operands without unpacking.
// Plain base vectors stay packed (2 x 12 words); G2 table records are packed in 64 words.
constexpr uint32_t G1_TABLE_REC = 32;

struct MsmShape {
  int c;    // window bits
  int W;    // digit windows = ceil(256 / c) (signed digits need one spare bit)
  int NB;   // buckets per bucket window = 2^(c-1)
  int L;    // buckets per running-sum thread
  int S;    // sorted entries per accumulation thread
  int Wb;   // bucket windows: W, or 1 with a window table (all windows share the buckets)
  int pre;  // 1: bases are a window table T[i*W + w] = 2^(c*w) * P_i (entry = i*W + w)
  int rec;  // u32 words per base record (0: packed affine, 2 x PACKED_WORDS; see G1_TABLE_REC)
  // Bucket shard (Wb == 1 only; bk_hi > bk_lo): only the digits whose bucket lies in
  // [bk_lo, bk_hi) are sorted, accumulated and reduced -- one rank's part of a multiexp split
  // across ranks by bucket range (every rank reads all scalars, the ranks' parts sum to the
  // multiexp).  Both bounds are multiples of BUCKET_SHARD_GRANULE; the device returns three points
  // (reduce_split_shift below).  0, 0: every bucket.
  uint32_t bk_lo = 0, bk_hi = 0;
  bool bucket_shard() const { return bk_hi > bk_lo; }
  uint32_t red_lo() const { return bucket_shard() ? bk_lo : 0u; }
  uint32_t red_nb() const { return bucket_shard() ? bk_hi - bk_lo : (uint32_t)NB; }
};
// a bucket shard's bounds are multiples of this: every partition of the digit sort (<= 128
// buckets at the table window sizes) lies in one rank's range, and the range is a whole number
// of k_reduce_blocks blocks (L * BT divides it: L <= 4 for G1's 256 threads, <= 8 for G2's 128)
constexpr uint32_t BUCKET_SHARD_GRANULE = 1024;
MsmShape msm_shape(size_t n, int c_override);
// shape for a window table: c from the cost model n*ceil(256/c) + ~6.5 * 2^(c-1)
int msm_table_c(size_t n);
MsmShape msm_shape_table(size_t n, int c);

// Bucket-reduction geometry (msm_back): L buckets per level-1 thread, blocks of
// reduce_block_threads() threads.  With a single bucket window (Wb == 1) the device returns
// two points and the host finishes the window: out[0] + 2^reduce_split_shift() * out[1]
// (the shift's doublings are a serial chain: cheaper on the host than on one device thread).
uint32_t reduce_block_max(bool g2);  // 256 (G1) / 128 (G2) threads (64 and 128 were slower)
// (for a bucket range of nbr buckets, L per thread)
inline uint32_t reduce_threads_for(uint32_t nbr, uint32_t L, bool g2) {
  const uint32_t T = nbr / L, bmax = reduce_block_max(g2);
  return T < bmax ? T : bmax;
}
inline uint32_t reduce_block_threads(const MsmShape& sh, bool g2) {
  return reduce_threads_for((uint32_t)sh.NB, (uint32_t)sh.L, g2);
}
inline int reduce_lg2(uint32_t x) {
  int r = 0;
  while ((1u << r) < x) r++;
  return r;
}
inline int reduce_shift_for(uint32_t nbr, uint32_t L, bool g2) {
  return reduce_lg2(L) + reduce_lg2(reduce_threads_for(nbr, L, g2));
}
inline int reduce_split_shift(const MsmShape& sh, bool g2) {
  return sh.Wb == 1 ? reduce_shift_for(sh.red_nb(), (uint32_t)sh.L, g2) : -1;
}
// A bucket shard's device result is out[0] + 2^reduce_split_shift * out[1] + bk_lo * out[2]
// (combine_g1 / combine_g2; out[2] = the plain sum of the range's buckets, each of which holds
// digit bk_lo more than its position in the range).
// Level-2 geometry of the bucket reduction over nblk level-1 blocks: BT2 threads (a power of two)
// of Lb blocks each (a power of two), BT2 * Lb >= nblk (blocks past nblk read as identities)
inline void reduce_level2(uint32_t nblk, bool g2, uint32_t* BT2, uint32_t* Lb) {
  const uint32_t bmax = g2 ? 128u : 256u;
  uint32_t lb = 1;
  while ((size_t)bmax * lb < nblk) lb <<= 1;
  uint32_t t = 1;
  while ((size_t)t * lb < nblk) t <<= 1;
  *BT2 = t;
  *Lb = lb;
}

struct MsmTiming {
  hipEvent_t ev_acc_begin = nullptr, ev_acc_end = nullptr;  // bracket k_accumulate_dev
};

// G2 window-table record: raw-limb x, y (4 x 14 limbs, 56 words) in a 256-B line
constexpr uint32_t G2_TABLE_REC = 64;

template <class C>
struct MsmWorkspace {
  size_t cap_n = 0, cap_E = 0, cap_nbt = 0, cap_segs = 0, cap_T = 0;
  uint32_t *entries = nullptr, *counts = nullptr, *offsets = nullptr, *cursor = nullptr, *scan_scratch = nullptr,
           *cont_bucket = nullptr, *tilecounts = nullptr, *tscan = nullptr;
  uint2* recs = nullptr;
  size_t cap_tc = 0;
  typename C::P *bucket_sums = nullptr, *conts = nullptr, *seg_weighted = nullptr, *seg_sum = nullptr,
                *window_sums = nullptr;
  typename C::P* host_window_sums = nullptr;  // pinned, W entries after the stream completes
  static size_t bytes_needed(size_t n);
  hipError_t reserve(size_t n_max);                         // every automatic shape up to n_max
  hipError_t reserve_shape(size_t n, const MsmShape& sh);    // grow (never shrink) for one shape
  hipError_t grow(size_t E, size_t nbt, size_t segs, size_t T);
  void release();
};

// Enqueue an MSM on `st`; on completion ws.host_window_sums[0..Wb) hold the
// canonical XYZZ sum of every window (device Montgomery form).
// d_scalars: n canonical scalars (8 LE u32 words each); d_idx: per-scalar base
// index (-1 = density bit clear) or nullptr for idx = base_offset + i.
template <class C>
hipError_t msm_window_sums(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, const uint32_t* d_scalars,
                           size_t n, const int32_t* d_idx, uint32_t base_offset, const MsmShape& sh,
                           MsmTiming* timing);

// The same MSM split in two stream-ordered halves: front = digit sort + bucket
// accumulation, back = bucket reduction + window sums -> host_out (pinned, Wb entries).
// set sh.S for curve C's accumulation kernel on the current device (see msm_impl.cuh)
template <class C>
void fit_segments(MsmShape& sh, size_t n);
template <class C>
void fit_segments_E(MsmShape& sh, size_t E);  // the same for E expected entries
// The entries fit_segments sizes a multiexp's segments for: n * W for n scalars and W windows,
// not used * W (`used` = the density set's scalars).  So a half-density multiexp (b_g1_aux,
// b_g2_aux) gets segments for twice its entries, i.e. half its rounds (1.5 at 3 rounds): alone its
// last round is half empty (G2 17.2 against 13.4 ms), but in the overlapped proof that is 1.1 ms
// per 2^22 proof faster than sizing it for its own entries (profiles/r05_ab_seg_used.txt).
size_t seg_entries(size_t n, size_t used, int W);
template <class C>
hipError_t msm_sort(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_scalars, size_t n, const int32_t* d_idx,
                    uint32_t base_offset, const MsmShape& sh);
template <class C>
hipError_t msm_accumulate(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, size_t n, const MsmShape& sh,
                          MsmTiming* timing);
template <class C>
hipError_t msm_front(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, const uint32_t* d_scalars,
                     size_t n, const int32_t* d_idx, uint32_t base_offset, const MsmShape& sh, MsmTiming* timing);
// max_span: the largest number of continuation partials of one bucket (max_span() below)
// when known, so that only the continuation-tree levels that can do work are launched;
// -1: every level a bucket could need
// d_span_words (with max_span = -1): max_span()'s device words for this multiexp -- the kernels
// read the longest span themselves (fold in the reduction up to 8 segments, else k_cont_seq),
// so the host need not wait for the sort before enqueueing the tail
template <class C>
hipError_t msm_back(MsmWorkspace<C>& ws, hipStream_t st, size_t n, const MsmShape& sh, typename C::P* host_out,
                    int max_span = -1, hipEvent_t acc_done = nullptr, const uint32_t* d_span_words = nullptr);

size_t scan_scratch_words(size_t n);
// the kernels each MSM unit emits (scratch budget, scratch.cpp)
template <class C>
void msm_acc_kernels(std::vector<KernInfo>& v);
template <class C>
void msm_back_kernels(std::vector<KernInfo>& v);
size_t reduce_blocks_resident_per_cu_g1();  // (msm_g1_back.hip)
// max over buckets of (last segment - first segment) for segment length S: the
// continuation-tree depth msm_back needs.  Each of max_span_blocks(nbt) workgroups writes its
// own maximum to d_words[b] and the (pinned) h_words receive them, stream-ordered; the host takes
// the max (max_span_host).  No zero-initialised word, so no fill kernel ahead of it: on a side
// stream beside a whole-GPU accumulation every extra dispatch waits for a free slot.
constexpr uint32_t MAX_SPAN_BLOCKS = 256;
inline uint32_t max_span_blocks(size_t nbt) {
  const size_t g = (nbt + 255) / 256;
  return (uint32_t)(g < 1 ? 1 : (g > MAX_SPAN_BLOCKS ? MAX_SPAN_BLOCKS : g));
}
inline uint32_t max_span_host(const uint32_t* h_words, size_t nbt) {
  uint32_t m = 0;
  for (uint32_t b = 0, g = max_span_blocks(nbt); b < g; b++) m = h_words[b] > m ? h_words[b] : m;
  return m;
}
hipError_t max_span(const uint32_t* counts, const uint32_t* offsets, size_t nbt, uint32_t S, uint32_t* d_words,
                    uint32_t* h_words, hipStream_t st);
void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, uint32_t* scratch, hipStream_t st);
hipError_t scalars_prepare(const uint32_t* d_in, uint32_t* d_out, size_t n, int mode, int log_perm, hipStream_t st);
hipError_t density_index(const uint64_t* d_words, size_t n, uint32_t base_offset, int32_t* d_idx, uint32_t* d_tmp,
                         uint32_t* d_scan_scratch, hipStream_t st);

}  // namespace bh

namespace bh {
// LDS radix-partition sort of the (window, bucket) entries; fills entries, counts[0..nbt),
// offsets[0..nbt] (offsets[nbt] = E)
size_t sort_tilecount_words(const MsmShape& sh, size_t n);
// sorted entries of a sparser density map over the same scalars/digits, by stable compaction of
// an already sorted source (src_off: the source's base offset; idx: the target's shard-relative
// base-index map, -1 = absent).  pos: Emax+1 words scratch; scan_scratch: derive_scratch_words.
size_t derive_scratch_words(size_t Emax);
// [b0, b1]: the buckets whose offsets the source sort set (a bucket shard's range; 0, 0: all)
hipError_t derive_sorted(const uint32_t* src_entries, const uint32_t* src_offsets, size_t nbt, size_t Emax, int pre,
                         uint32_t W, uint32_t src_off, const int32_t* idx, uint32_t* pos, uint32_t* scan_scratch,
                         uint32_t* dst_entries, uint32_t* dst_counts, uint32_t* dst_offsets, hipStream_t st,
                         size_t b0 = 0, size_t b1 = 0);
hipError_t sort_entries(const uint32_t* d_scalars, size_t n, const int32_t* d_idx, uint32_t base_offset,
                        const MsmShape& sh, uint32_t* tilecounts, uint32_t* tscan_scratch, uint2* recs,
                        uint32_t* entries, uint32_t* counts, uint32_t* offsets, hipStream_t st);
}  // namespace bh
