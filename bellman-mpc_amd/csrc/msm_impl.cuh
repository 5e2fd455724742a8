// Curve-generic MSM kernels and host driver (included once per curve by
// msm_g1.hip / msm_g2.hip so the two instantiations compile in parallel).
#pragma once
#include <cstdlib>

#include "msm.h"
#include <algorithm>


namespace bh {

static inline unsigned msm_blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

// ----------------------------------------------------------------- accumulate
template <class C>
__device__ __forceinline__ void store_point(typename C::P* dst, const typename C::P& p) {
  constexpr int WORDS = sizeof(typename C::P) / 16;
  const uint4* s = reinterpret_cast<const uint4*>(&p);
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < WORDS; k++) d[k] = s[k];
}
template <class C>
__device__ __forceinline__ typename C::P load_point(const typename C::P* src) {
  typename C::P p;
  constexpr int WORDS = sizeof(typename C::P) / 16;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint4* d = reinterpret_cast<uint4*>(&p);
#pragma unroll
  for (int k = 0; k < WORDS; k++) d[k] = s[k];
  return p;
}

// largest b in [0, nb) with offsets[b] <= pos  (offsets has nb+1 entries, offsets[nb] > pos)
__device__ __forceinline__ uint32_t find_bucket(const uint32_t* offsets, uint32_t nb, uint32_t pos) {
  uint32_t lo = 0, hi = nb;  // invariant offsets[lo] <= pos < offsets[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= pos) lo = mid;
    else hi = mid;
  }
  return lo;
}

// full sum of bucket gb: own partial + the (tree-reduced) continuation partials,
// which k_cont_tree has folded into conts[s_first + 1]
template <class C>
__device__ __forceinline__ typename C::P bucket_value(uint32_t gb, const uint32_t* counts, const uint32_t* offsets,
                                                      const typename C::P* bucket_sums, const typename C::P* conts,
                                                      uint32_t S) {
  const uint32_t cnt = counts[gb];
  if (cnt == 0) return C::identity();
  typename C::P v = load_point<C>(&bucket_sums[gb]);
  const uint32_t off = offsets[gb];
  const uint32_t s_first = off / S, s_last = (off + cnt - 1) / S;
  if (s_last > s_first) v = C::add(v, load_point<C>(&conts[s_first + 1]));
  return v;
}

// Level `stride` = F^k of an F-ary tree over each bucket's continuation partials
// conts[s_first+1 .. s_last]: node j (j = s - s_first - 1, a multiple of F*stride) adds the
// partials at j + i*stride, i = 1..F-1 (F-1 serial additions per level instead of one per
// level of the binary tree).  After the levels with stride < span, conts[s_first+1] holds the sum.
template <class C, int F>
__global__ void __launch_bounds__(256) k_cont_treeF(const uint32_t* cont_bucket, const uint32_t* counts,
                                                    const uint32_t* offsets, uint32_t nbt, uint32_t S,
                                                    uint32_t stride, uint32_t b_lo, uint32_t b_hi,
                                                    typename C::P* conts) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t E = offsets[nbt];
  if ((size_t)s * S >= E) return;
  const uint32_t b = cont_bucket[s];
  if (b == 0xffffffffu || b < b_lo || b >= b_hi) return;  // buckets [b_lo, b_hi) only
  const uint32_t off = offsets[b];
  const uint32_t s_first = off / S;
  const uint32_t ncont = (off + counts[b] - 1) / S - s_first;
  const uint32_t j = s - s_first - 1;
  if (j % (stride * F) != 0 || j + stride >= ncont) return;
  typename C::P acc = load_point<C>(&conts[s]);
  for (int i = 1; i < F; i++)
    if (j + i * stride < ncont) acc = C::add(acc, load_point<C>(&conts[s + i * stride]));
  store_point<C>(&conts[s], acc);
}

// longest span folded by the Q-thread kernel below; longer ones take the 4-ary tree.  The
// tree's levels are full-grid launches: beside a running accumulation they cost more than a
// sequential fold of ~16 partials (N = 8 rehearsal at 2^22: 13.4 ms per rank with 4, 10.7 ms
// with 24).
inline size_t cont_seq_max() { return 64; }

// Max over the g per-workgroup words k_max_span wrote (msm_common.hip): the longest bucket span,
// read by every workgroup of the kernels below when the host has not read it (device-decided
// tails: no host wait between a multiexp's sort and the enqueue of its tail).  Block-uniform.
__device__ __forceinline__ uint32_t block_span(const uint32_t* words, uint32_t g) {
  __shared__ uint32_t red[4];
  uint32_t m = 0;
  for (uint32_t i = threadIdx.x; i < g; i += blockDim.x) m = max(m, words[i]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = red[0];
  for (uint32_t w = 1; w < (blockDim.x + 63) / 64; w++) m = max(m, red[w]);
  __syncthreads();  // (red is reused by the next call)
  return m;
}

// The same fold for buckets spanning at most cont_seq_max() segments, Q threads per bucket:
// thread q of bucket b sums the partials i = q, q+Q, q+2Q, ... of conts[s_first+1 ..
// s_last], then the Q sums meet in LDS (log2(Q) more additions), so a bucket spanning 16
// segments costs 4 + 2 serial additions instead of 15.  The tails are VALU-bound chains
// on a small fraction of the SIMDs: serial depth is their latency.
// span_words != null (device-decided): the whole grid returns when the longest span is at most
// fold_span (k_reduce_blocks folds those), and otherwise folds every bucket spanning at most
// seq_max segments; longer ones are k_cont_long's (a serial chain over thousands of partials
// would be the tail's latency: a witness full of ones puts most entries in one bucket).
template <class C, int Q>
__global__ void __launch_bounds__(256) k_cont_seq(const uint32_t* counts, const uint32_t* offsets, uint32_t b0,
                                                  uint32_t nbr, uint32_t S, typename C::P* conts,
                                                  const uint32_t* span_words, uint32_t span_g, uint32_t fold_span,
                                                  uint32_t seq_max) {
  extern __shared__ uint4 lds_raw[];
  typename C::P* lds = reinterpret_cast<typename C::P*>(lds_raw);
  if (span_words && block_span(span_words, span_g) <= fold_span) return;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t b = b0 + gid / Q, q = gid % Q;  // buckets [b0, b0 + nbr)
  uint32_t s_first = 0, ncont = 0;
  if (gid / Q < nbr) {
    const uint32_t cnt = counts[b];
    if (cnt) {
      const uint32_t off = offsets[b];
      s_first = off / S;
      ncont = (off + cnt - 1) / S - s_first;  // partials conts[s_first+1 .. s_first+ncont]
      if (span_words && ncont > seq_max) ncont = 0;  // k_cont_long's
    }
  }
  typename C::P acc = C::identity();
  if (ncont >= 2)
    for (uint32_t i = q; i < ncont; i += Q) acc = C::add(acc, load_point<C>(&conts[s_first + 1 + i]));
  store_point<C>(&lds[threadIdx.x], acc);
  __syncthreads();
  for (uint32_t h = Q / 2; h > 0; h >>= 1) {
    if (q < h && ncont >= 2) {
      acc = C::add(acc, load_point<C>(&lds[threadIdx.x + h]));
      store_point<C>(&lds[threadIdx.x], acc);
    }
    __syncthreads();
  }
  if (q == 0 && ncont >= 2) store_point<C>(&conts[s_first + 1], acc);
}

// Device-decided tails, buckets spanning more than seq_max segments (rare: a bucket holding a
// large share of the entries): one workgroup per such bucket, its threads summing strided
// partials, then an LDS tree, into conts[s_first+1].  A grid-stride pass over the buckets finds
// them; the whole grid returns at once when the longest span is at most seq_max.
template <class C>
__global__ void __launch_bounds__(256) k_cont_long(const uint32_t* counts, const uint32_t* offsets, uint32_t b0,
                                                   uint32_t nbr, uint32_t S, typename C::P* conts,
                                                   const uint32_t* span_words, uint32_t span_g, uint32_t seq_max) {
  extern __shared__ uint4 lds_raw[];
  typename C::P* lds = reinterpret_cast<typename C::P*>(lds_raw);
  __shared__ uint32_t list[256];
  __shared__ uint32_t nlist;
  if (block_span(span_words, span_g) <= seq_max) return;
  const uint32_t tid = threadIdx.x, BT = blockDim.x;
  for (uint32_t base = blockIdx.x * BT; base < nbr; base += gridDim.x * BT) {
    if (tid == 0) nlist = 0;
    __syncthreads();
    if (base + tid < nbr) {
      const uint32_t b = b0 + base + tid, cnt = counts[b];
      if (cnt) {
        const uint32_t off = offsets[b];
        if ((off + cnt - 1) / S - off / S > seq_max) list[atomicAdd(&nlist, 1u)] = b;
      }
    }
    __syncthreads();
    const uint32_t nl = nlist;
    for (uint32_t li = 0; li < nl; li++) {
      const uint32_t b = list[li], off = offsets[b];
      const uint32_t s_first = off / S, ncont = (off + counts[b] - 1) / S - s_first;
      // ceil(ncont / BT) strided steps, then log2(BT) tree steps: one addition call site (a G2
      // addition inlined twice doubles the unit's compile time)
      const uint32_t nit = (ncont + BT - 1) / BT;
      uint32_t lg = 0;
      while ((1u << lg) < BT) lg++;
      typename C::P acc = C::identity();
      for (uint32_t st = 0; st < nit + lg; st++) {
        typename C::P x;
        bool act;
        if (st < nit) {
          const uint32_t i = st * BT + tid;
          act = i < ncont;
          if (act) x = load_point<C>(&conts[s_first + 1 + i]);
        } else {
          if (st == nit) store_point<C>(&lds[tid], acc);
          __syncthreads();
          const uint32_t h = BT >> (st - nit + 1);
          act = tid < h;
          if (act) x = load_point<C>(&lds[tid + h]);
        }
        if (act) acc = C::add(acc, x);
        if (st >= nit) {
          __syncthreads();
          if (act) store_point<C>(&lds[tid], acc);
        }
      }
      if (tid == 0) store_point<C>(&conts[s_first + 1], acc);
      __syncthreads();
    }
  }
}

// ---- Bucket reduction: window total  sum_{b < NB} (b+1) * B_b  (bucket b holds digit b+1;
// multiexp.rs:225-235 computes it as one serial running sum per window).  Here it is a
// two-level summation by parts with no scalar multiplications of partial sums:
//   thread t of block `blk` (t = blk*BT + i) owns buckets [t*L, t*L + L):
//     R_t = sum_k B,  A_t = sum_k (k+1) B          (2L additions, the running-sum idiom)
//   then  sum_b (b+1) B_b = sum_t A_t + L * sum_t t R_t,  and inside a block
//     sum_i (t0 + i) R = t0 * S_blk + sum_i V_i,   V_i = sum_{j > i} R_j (LDS suffix scan)
//   so block blk emits Y_blk = sum_i (A_i + L*V_i) and S_blk = sum_i R_i, and
//     window total = sum_blk Y_blk + (L*BT) * sum_blk blk * S_blk,
//   the same shape one level up (k_reduce_window, one block per window).
// Work ~ (2 + (log2 BT + log2 L) / L) additions per bucket; serial depth 2L + 2 log2 BT + log2 L.
//
// Each kernel is written as short programs of point operations with ONE addition and one
// doubling call site (operands chosen per step): a G2 addition is ~20 000 instructions, and
// every inlined copy would cost minutes of compile time.

template <class C>
__device__ __forceinline__ typename C::P dbl_times(typename C::P v, int k) {
  for (int j = 0; j < k; j++) v = C::dbl(v);
  return v;
}

// Block epilogue shared by both levels (lds: blockDim points, 2 * blockDim with split).  v = this thread's value:
//   suffix scan over the block; V = sum_{j > i} v_j (exclusive suffix);
//   x = base + 2^lg1 * V;
//   compose (lg2 >= 0): x = extra + 2^lg2 * x, then the block sum of x;
//   split   (lg2 <  0): the block sums of x and of extra side by side (two interleaved trees).
// Thread 0 ends with lds[0] = sum x, lds[BT] = sum extra (split), *s_blk = sum v.
template <class C>
__device__ __forceinline__ void block_epilogue(typename C::P v, const typename C::P& base, int lg1,
                                               const typename C::P& extra, int lg2, bool split, typename C::P* lds,
                                               typename C::P* s_blk) {
  const uint32_t i = threadIdx.x, BT = blockDim.x;
  int lgBT = 0;
  while ((1u << lgBT) < BT) lgBT++;
  const int n_final = lg2 >= 0 ? 2 : 1;
  store_point<C>(&lds[i], v);
  __syncthreads();
  const int steps = 2 * lgBT + n_final;
  for (int st = 0; st < steps; st++) {
    typename C::P a = v, b;
    bool act;
    uint32_t dst = i;
    if (st < lgBT) {  // suffix scan: v += v[i + 2^st]
      const uint32_t d = 1u << st;
      act = i + d < BT;
      if (act) b = load_point<C>(&lds[i + d]);
    } else if (st < lgBT + n_final) {  // x = base + 2^lg1 V, then x = extra + 2^lg2 x
      const bool first = st == lgBT;
      if (first) {
        b = i + 1 < BT ? load_point<C>(&lds[i + 1]) : C::identity();
        if (i == 0) *s_blk = load_point<C>(&lds[0]);
      } else {
        b = v;
      }
      b = dbl_times<C>(b, first ? lg1 : lg2);
      a = first ? base : extra;
      act = true;
    } else {  // tree level with half size h: x-part on threads [0, h), extra-part on [h, 2h)
      const uint32_t h = BT >> (st - lgBT - n_final + 1);
      act = split ? i < 2 * h : i < h;
      if (act) {
        dst = i < h ? i : BT + (i - h);
        a = load_point<C>(&lds[dst]);
        b = load_point<C>(&lds[dst + h]);
      }
    }
    __syncthreads();
    if (act) {
      v = C::add(a, b);
      store_point<C>(&lds[dst], v);
    }
    if (split && st == lgBT + n_final - 1) store_point<C>(&lds[BT + i], extra);
    __syncthreads();
  }
}

// Level 1: grid = Wb * nblk blocks of BT threads (T = NB / L = nblk * BT); block
// (w, blk) writes Y[w*nblk + blk] and S[w*nblk + blk].  A bucket spanning accumulation
// segments s_first .. s_last has continuation partials conts[s_first+1 .. s_last]; with fold
// they are all added here (short spans), else k_cont_seq / k_cont_treeF has already folded
// them into conts[s_first+1].
template <class C>
__global__ void __launch_bounds__(256) k_reduce_blocks(const uint32_t* counts, const uint32_t* offsets,
                                                       const typename C::P* bucket_sums, const typename C::P* conts,
                                                       uint32_t S, uint32_t b0, uint32_t NB, uint32_t L, int lgL,
                                                       uint32_t nblk, int fold, typename C::P* Y, typename C::P* Ssum,
                                                       const uint32_t* span_words, uint32_t span_g, uint32_t fold_span) {
  extern __shared__ uint4 lds_raw[];
  typename C::P* lds = reinterpret_cast<typename C::P*>(lds_raw);
  if (span_words) fold = block_span(span_words, span_g) <= fold_span ? 1 : 0;  // device-decided
  const uint32_t i = threadIdx.x;
  const uint32_t w = blockIdx.x / nblk, blk = blockIdx.x % nblk;
  const uint32_t gb0 = b0 + w * NB + (blk * blockDim.x + i) * L;
  // G2 (448-byte points, one wave per SIMD): the running total `acc` waits in this thread's LDS
  // slot (free until the epilogue) instead of registers, which the compiler otherwise spills
  // to scratch (KB per lane)
  constexpr bool acc_lds = sizeof(typename C::P) > 256;
  typename C::P run = C::identity(), acc = C::identity(), bk = C::identity();
  if (acc_lds) store_point<C>(&lds[i], acc);
  // per bucket k = L-1 .. 0:  bk = partial (+ each continuation partial);  run += bk;  acc += run
  int k = (int)L - 1;
  uint32_t op = 0, c_next = 0, c_end = 0;  // op 0: load, 1: continuation, 2: run, 3: acc
  while (k >= 0) {
    typename C::P a, b;
    if (op == 0) {
      const uint32_t gb = gb0 + (uint32_t)k, cnt = counts[gb];
      bk = C::identity();
      c_next = c_end = 0;
      if (cnt) {
        bk = load_point<C>(&bucket_sums[gb]);
        const uint32_t off = offsets[gb];
        const uint32_t s_first = off / S, s_last = (off + cnt - 1) / S;
        c_next = s_first + 1;
        c_end = s_last > s_first ? (fold ? s_last + 1 : s_first + 2) : c_next;
      }
      op = c_next < c_end ? 1 : 2;
      continue;
    }
    if (op == 1) { a = bk; b = load_point<C>(&conts[c_next]); }
    else if (op == 2) { a = run; b = bk; }
    else { a = acc_lds ? load_point<C>(&lds[i]) : acc; b = run; }
    const typename C::P r = C::add(a, b);
    if (op == 1) {
      bk = r;
      if (++c_next == c_end) op = 2;
    } else if (op == 2) {
      run = r;
      op = 3;
    } else {
      if (acc_lds) store_point<C>(&lds[i], r);
      else acc = r;
      op = 0;
      k--;
    }
  }
  if (acc_lds) acc = load_point<C>(&lds[i]);
  __syncthreads();  // every thread has its acc back before the epilogue reuses the slots
  typename C::P s_blk;
  block_epilogue<C>(run, acc, lgL, acc, -1, false, lds, &s_blk);
  if (i == 0) {
    store_point<C>(&Y[blockIdx.x], load_point<C>(&lds[0]));
    store_point<C>(&Ssum[blockIdx.x], s_blk);
  }
}

// Level 2: one block of BT2 threads per window over its nblk = BT2 * Lb (Y, S) pairs:
//   sum_blk Y + M * sum_blk blk * S,  M = 2^lgM = L * BT (level 1's block size)
// thread j owns blocks [j*Lb, j*Lb + Lb): P_j = sum Y, A'_j = sum_k k S, R'_j = sum_k S, and
//   sum_blk blk S = sum_j (A'_j + Lb * V'_j),  V'_j = sum_{j' > j} R'_j'
// -> out[w] = the window total (canonical coordinates); split (one window): out[0] = sum P,
// out[1] = sum_blk blk * S, out[2] = sum_blk S, and the host adds 2^lgM * out[1]
// (reduce_split_shift; out[2] is the plain bucket sum a bucket range's offset multiplies).
template <class C>
__global__ void __launch_bounds__(256) k_reduce_window(const typename C::P* Y, const typename C::P* Ssum,
                                                       uint32_t nblk, uint32_t Lb, int lgLb, int lgM, int split,
                                                       typename C::P* out) {
  extern __shared__ uint4 lds_raw[];
  typename C::P* lds = reinterpret_cast<typename C::P*>(lds_raw);
  const uint32_t i = threadIdx.x, w = blockIdx.x;
  const size_t base = (size_t)w * nblk + (size_t)i * Lb;
  typename C::P run = C::identity(), acc = C::identity(), p = C::identity();
  // per block k = Lb-1 .. 0:  acc += run;  run += S_k;  p += Y_k  (blocks past nblk: identities,
  // reduce_level2)
  for (uint32_t it = 0; it < 3 * Lb; it++) {
    const uint32_t k = Lb - 1 - it / 3, op = it % 3;
    const bool in = i * Lb + k < nblk;
    typename C::P a, b;
    if (op == 0) { a = acc; b = run; }
    else if (op == 1) { a = run; b = in ? load_point<C>(&Ssum[base + k]) : C::identity(); }
    else { a = p; b = in ? load_point<C>(&Y[base + k]) : C::identity(); }
    const typename C::P r = C::add(a, b);
    if (op == 0) acc = r;
    else if (op == 1) run = r;
    else p = r;
  }
  typename C::P s_all;
  block_epilogue<C>(run, acc, lgLb, p, split ? -1 : lgM, split != 0, lds, &s_all);
  if (i == 0) {
    if (split) {
      out[0] = C::reduce(load_point<C>(&lds[blockDim.x]));
      out[1] = C::reduce(load_point<C>(&lds[0]));
      out[2] = C::reduce(s_all);
    } else {
      out[w] = C::reduce(load_point<C>(&lds[0]));
    }
  }
}

// The G2 segment loop of k_accumulate_pf.  A G2 mixed addition held whole in registers needs
// the accumulator (4 Fp2 = 112 words), the base (56) and madd-2008-s's temporaries at once: the
// allocator parked ~3 600 values per addition in AGPRs (v_accvgpr_read/write, a fifth of the
// loop's VALU instructions).  Here the accumulator's ZZ and ZZZ live in LDS between additions
// (component-major uint4 rows, one lane per column: conflict-free), the formula is ordered so
// that every input dies at its last use (ZZ3 = ZZ1*PP right after PP, ZZZ3 = ZZZ1*PPP right after
// PPP, y2 read after x2's product), and the next base's prefetch is issued once y2 is read.  The
// exceptional cases run through the same instruction stream (a separate doubling routine inlined
// in the loop took the kernel back to 512 registers with scratch spills; out of line it needs a
// call stack: scratch in the hot kernel).  Identity is a register flag.
// Bounds as CurveOps::madd (MB = 2: X < 10p, Y < 4p, ZZ, ZZZ < 2p).
#define G2_SB() __builtin_amdgcn_sched_barrier(0)
// DIRECT: no LDS prefetch slots (pre unused): each coordinate of the base is loaded from `bases`
// when it is needed, and the other wave of the SIMD covers the latency (two waves per SIMD: 57 KB
// of LDS per 256-thread block instead of 114).
template <class F, int NW, int NQ, bool ZZ_LDS, bool DIRECT = false, class Issue>
__device__ __forceinline__ void accumulate_lds(uint4 (*pre)[64], int lane, int nq, bool limbs,
                                               const uint32_t* entries, const uint32_t* offsets, uint32_t start,
                                               uint32_t end, uint32_t pos0, uint32_t seg, uint32_t b, uint32_t next,
                                               bool started_here, uint32_t e_cur, uint32_t e_next, Issue& issue,
                                               XYZZ<F>* bucket_sums, XYZZ<F>* conts,
                                               const uint32_t* bases = nullptr, uint32_t rec = 0) {
  using T = typename F::T;
  using Cv = CurveOps<F>;
  // rows of VW-word vectors, one column per thread: uint4 rows for G2 (7 per coordinate), uint2
  // for G1 (7: 14 words)
  constexpr int VW = (NW % 4 == 0) ? 4 : 2;
  constexpr int RH = NW / VW;
  using V = typename std::conditional<VW == 4, uint4, uint2>::type;
  // ZZZ always in LDS; ZZ too when ZZ_LDS (else a register, as X and Y)
  __shared__ V zzz_s[RH][256];
  __shared__ V zz_s[ZZ_LDS ? RH : 1][256];
  T ZZr = F::zero();
  const int t = threadIdx.x;
  auto put_rows = [&](V (*arr)[256], const T& v) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
    for (int q = 0; q < RH; q++) {
      V w;
      uint32_t* d = reinterpret_cast<uint32_t*>(&w);
#pragma unroll
      for (int k = 0; k < VW; k++) d[k] = s[VW * q + k];
      arr[q][t] = w;
    }
  };
  auto get_rows = [&](V (*arr)[256]) {
    T v;
    uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int q = 0; q < RH; q++) {
      const V w = arr[q][t];
      const uint32_t* s = reinterpret_cast<const uint32_t*>(&w);
#pragma unroll
      for (int k = 0; k < VW; k++) d[VW * q + k] = s[k];
    }
    return v;
  };
  auto put_zz = [&](const T& v) {
    if constexpr (ZZ_LDS) put_rows(zz_s, v);
    else ZZr = v;
  };
  auto get_zz = [&]() {
    if constexpr (ZZ_LDS) return get_rows(zz_s);
    else return ZZr;
  };
  // coordinate `half` (0 = x, 1 = y) of the base in this lane's prefetch slot
  auto base_coord = [&](int half) {
    T v;
    if constexpr (DIRECT) {
      const uint4* src = reinterpret_cast<const uint4*>(bases + (size_t)(e_cur & 0x7fffffffu) * rec);
      uint32_t* d = reinterpret_cast<uint32_t*>(&v);
      if (limbs) {
#pragma unroll
        for (int q = 0; q < NW / 4; q++) {
          const uint4 u = src[half * (NW / 4) + q];
          d[4 * q] = u.x; d[4 * q + 1] = u.y; d[4 * q + 2] = u.z; d[4 * q + 3] = u.w;
        }
      } else {
        constexpr int PQ = F::PACKED_WORDS / 4;
        uint32_t w[F::PACKED_WORDS];
#pragma unroll
        for (int q = 0; q < PQ; q++) {
          const uint4 u = src[half * PQ + q];
          w[4 * q] = u.x; w[4 * q + 1] = u.y; w[4 * q + 2] = u.z; w[4 * q + 3] = u.w;
        }
        v = F::unpack(w);
      }
      return v;
    }
    if (limbs) {  // raw limbs: words [half*NW, half*NW + NW) of the record
      uint32_t* d = reinterpret_cast<uint32_t*>(&v);
      if constexpr (NW % 4 == 0) {  // G2: pieces [half*NW/4, half*NW/4 + NW/4)
#pragma unroll
        for (int q = 0; q < NW / 4; q++) {
          const uint4 u = pre[half * (NW / 4) + q][lane];
          d[4 * q] = u.x; d[4 * q + 1] = u.y; d[4 * q + 2] = u.z; d[4 * q + 3] = u.w;
        }
      } else {  // G1: x = words 0..13 (pieces 0-3), y = words 14..27 (pieces 3-6)
        uint32_t w[2 * NW + 4];
#pragma unroll
        for (int q = 0; q < (2 * NW + 3) / 4; q++) {
          if (q < (half * NW) / 4 || q > (half * NW + NW - 1) / 4) continue;
          const uint4 u = pre[q][lane];
          w[4 * q] = u.x; w[4 * q + 1] = u.y; w[4 * q + 2] = u.z; w[4 * q + 3] = u.w;
        }
#pragma unroll
        for (int k = 0; k < NW; k++) d[k] = w[half * NW + k];
      }
    } else {  // packed: PACKED_WORDS words = PACKED_WORDS / 4 pieces per coordinate
      constexpr int PQ = F::PACKED_WORDS / 4;
      uint32_t w[F::PACKED_WORDS];
#pragma unroll
      for (int q = 0; q < PQ; q++) {
        const uint4 u = pre[half * PQ + q][lane];
        w[4 * q] = u.x; w[4 * q + 1] = u.y; w[4 * q + 2] = u.z; w[4 * q + 3] = u.w;
      }
      v = F::unpack(w);
    }
    return v;
  };
  // y of base j (negated for a negative digit), then base j+1's prefetch into the same slot
  auto take_y = [&](uint32_t j) {
    T y = base_coord(1);
    if (e_cur & 0x80000000u) y = F::template sub<1>(F::zero(), y);
    if constexpr (!DIRECT) __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS slot is read before it is refilled
    if (j + 1 < end) {
      if constexpr (!DIRECT) issue(e_next);
      e_cur = e_next;
      e_next = (j + 2 < end) ? (entries ? entries[j + 2] : j + 2) : 0u;
    }
    return y;
  };
  T X = F::zero(), Y = F::zero();
  bool ident = true;
  auto flush = [&](XYZZ<F>* dst) {
    XYZZ<F> p;
    if (ident) {
      p = Cv::identity();
    } else {
      p.X = X; p.Y = Y; p.ZZ = get_zz(); p.ZZZ = get_rows(zzz_s);
    }
    store_point<Cv>(dst, p);
  };
  for (uint32_t j = start; j < end; j++) {
    if (j == next) {
      flush(started_here ? &bucket_sums[b] : &conts[seg]);
      b++;
      while (offsets[b + 1] <= j) b++;
      next = offsets[b + 1];
      started_here = true;
      ident = true;
    }
    if constexpr (!DIRECT) __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0): base j has landed in LDS
    const T x2 = base_coord(0);
    if (ident) {
      Y = take_y(j);
      X = x2;
      put_zz(F::one());
      put_rows(zzz_s, F::one());
      ident = false;
      continue;
    }
    // (scheduling barriers between the products: interleaving two Fp2 products' working sets
    // is what overflows the register file)
    const T ZZ1 = get_zz();
    T Pd = F::template sub<Cv::KX>(F::mul(x2, ZZ1), X);  // U2 - X1 < 18p
    G2_SB();
    const T y2 = take_y(j);
    T R = F::template sub<Cv::KY>(F::mul(y2, get_rows(zzz_s)), Y);  // S2 - Y1 < 6p
    G2_SB();
    // P = +-a (rare): P == -a gives the identity; P == a takes this instruction stream as
    // dbl-2008-s of P (Pd := 2 Y1 < 8p, R := 3 X1^2 < 6p, no PPP term in X3), as G1's unified madd
    bool twice = false, neg = false;
    if (F::is_zero(Pd)) {
      twice = F::is_zero(R);
      neg = !twice;
      if (twice) {
        Pd = F::add(Y, Y);
        const T xx = F::sqr(X);
        R = F::add(F::add(xx, xx), xx);
      }
    }
    G2_SB();
    const T PP = F::sqr(Pd);
    G2_SB();
    put_zz(F::mul(ZZ1, PP));  // ZZ3
    G2_SB();
    const T PPP = F::mul(Pd, PP);
    G2_SB();
    put_rows(zzz_s, F::mul(get_rows(zzz_s), PPP));  // ZZZ3
    G2_SB();
    const T Q = F::mul(X, PP);
    G2_SB();
    const T Q2 = F::add(Q, Q);
    const T X3 = F::template sub<Cv::K1>(F::sqr(R), twice ? Q2 : F::add(PPP, Q2));
    G2_SB();
    if constexpr (std::is_same<F, Fp2Ops>::value) {
      // one reduction per half for both Karatsuba products (fe2_mul_sub_kara): R < 6p,
      // Q - X3 + 16p < 18p, Y < 4p, PPP < 2p, all < 2^386 with normalised limbs; Y3 < 2p
      // (round 5: two products and a subtraction before, 14 761 against 14 038 VALU lane-
      // instructions per madd; checked at the operand maxima by tests/test_gpu_selftest.py)
      Y = F::mul_sub_lazy(R, F::template sub<Cv::K2>(Q, X3), Y, PPP);
    } else {  // one reduction for both products (fe_mul2)
      Y = F::template mul_sub<Cv::KY>(R, F::template sub<Cv::K2>(Q, X3), Y, PPP);
    }
    X = X3;
    if (neg) ident = true;
    G2_SB();
  }
  flush(started_here ? &bucket_sums[b] : &conts[seg]);
}

// Bucket accumulation: thread `seg` adds the bases of sorted entries [seg*S, seg*S + S) into
// their buckets (XYZZ mixed additions), storing a bucket's sum when the bucket ends inside the
// segment, or its continuation partial (conts[seg]) when the bucket started in an earlier
// segment.  The next entry's affine base is prefetched global -> LDS by
// global_load_lds_dwordx4 (no VGPR cost) while the current mixed addition runs: each wave
// owns NQ x 64 x 16 B of LDS, lane l's base occupying slot l of each of the NQ rows.
// Only the entries of buckets [b_lo, b_hi) (a bucket shard's range); a segment cut by the range
// keeps the continuation bookkeeping of the whole segment.
// (A register-load variant without the prefetch measured slower and was removed.)
template <class C>
__global__ void __launch_bounds__(256) k_accumulate_pf(const uint32_t* entries, const uint32_t* offsets, uint32_t nbt,
                                                       const uint32_t* bases, uint32_t rec, uint32_t S,
                                                       uint32_t b_lo, uint32_t b_hi, typename C::P* bucket_sums,
                                                       typename C::P* conts, uint32_t* cont_bucket) {
  using F = typename std::conditional<std::is_same<C, G1Ops>::value, G1F, Fp2Ops>::type;
  constexpr int PW = F::PACKED_WORDS;
  constexpr bool G1 = std::is_same<C, G1Ops>::value;
  constexpr int NW = sizeof(typename F::T) / 4;    // raw limb words per coordinate (G1: 14)
  constexpr int NQ = NW / 2;                       // 16-byte pieces per raw-limb base (G1 7, G2 14)
  // Window-table records hold raw limbs (G1_TABLE_REC 7 pieces, G2_TABLE_REC 14: no unpacking); plain
  // vectors are packed (6 / 12 pieces)
  const bool limbs = G1 ? rec == G1_TABLE_REC : rec == G2_TABLE_REC;
  const int nq = limbs ? NQ : 2 * PW / 4;
  __shared__ uint4 pre[4][NQ][64];
  const uint32_t E_lo = offsets[b_lo], E_hi = offsets[b_hi];
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pos0 = seg * S;
  const uint32_t start = max(pos0, E_lo);
  if (pos0 >= E_hi || start >= pos0 + S) return;
  const uint32_t end = min(pos0 + S, E_hi);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto issue = [&](uint32_t e) {
    const uint32_t* src = bases + (size_t)(e & 0x7fffffffu) * rec;
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (q < nq)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 4 * q),
                                         (__attribute__((address_space(3))) void*)&pre[wv][q][0], 16, 0, 0);
  };
  auto entry = [&](uint32_t j) { return entries ? entries[j] : j; };
  uint32_t e_cur = entry(start);
  issue(e_cur);
  uint32_t e_next = (start + 1 < end) ? entry(start + 1) : 0u;
  // (searched within [b_lo, b_hi]: a bucket shard's sort leaves the other buckets' offsets unset)
  uint32_t b = b_lo + find_bucket(offsets + b_lo, b_hi - b_lo, start);
  uint32_t next = offsets[b + 1];
  bool started_here = offsets[b] >= pos0;
  if (start == pos0) cont_bucket[seg] = started_here ? 0xffffffffu : b;
  if constexpr (!G1) {
    accumulate_lds<F, NW, NQ, true>(pre[wv], lane, nq, limbs, entries, offsets, start, end, pos0, seg, b, next,
                                    started_here, e_cur, e_next, issue, bucket_sums, conts);
    return;
  }
  // (G1 through the same loop with ZZZ, or ZZ and ZZZ, in LDS: no faster, removed in round 6)
  typename C::P acc = C::identity();
  for (uint32_t j = start; j < end; j++) {
    if (j == next) {
      if (started_here) store_point<C>(&bucket_sums[b], acc);
      else store_point<C>(&conts[seg], acc);
      b++;
      while (offsets[b + 1] <= j) b++;
      next = offsets[b + 1];
      started_here = true;
      acc = C::identity();
    }
    __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0): base j has landed in LDS
    uint32_t w[4 * NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      if (q < nq) {
        const uint4 v = pre[wv][q][lane];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      }
    }
    typename C::A a;
    if (limbs) {
#pragma unroll
      for (int k = 0; k < NW; k++) {
        reinterpret_cast<uint32_t*>(&a.x)[k] = w[k];
        reinterpret_cast<uint32_t*>(&a.y)[k] = w[NW + k];
      }
    } else {
      a.x = F::unpack(w);
      a.y = F::unpack(w + PW);
    }
    if (e_cur & 0x80000000u) a = C::neg_affine(a);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS slot is read before it is refilled
    if (j + 1 < end) {
      issue(e_next);
      e_cur = e_next;
      e_next = (j + 2 < end) ? entry(j + 2) : 0u;
    }
    acc = C::madd(acc, a);
  }
  if (started_here) store_point<C>(&bucket_sums[b], acc);
  else store_point<C>(&conts[seg], acc);
}

// G2 accumulation without LDS prefetch slots (accumulate_lds<DIRECT>): 57 KB of LDS per block and
// at most 256 registers, so two waves per SIMD.  Same segments, bookkeeping and results as
// k_accumulate_pf<G2> (BH_G2_DIRECT=1 selects it: A/B).
template <class C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_accumulate_g2d(const uint32_t* entries, const uint32_t* offsets, uint32_t nbt, const uint32_t* bases, uint32_t rec,
                 uint32_t S, uint32_t b_lo, uint32_t b_hi, typename C::P* bucket_sums, typename C::P* conts,
                 uint32_t* cont_bucket) {
  using F = Fp2Ops;
  constexpr int NW = sizeof(typename F::T) / 4;
  const bool limbs = rec == G2_TABLE_REC;
  const uint32_t E_lo = offsets[b_lo], E_hi = offsets[b_hi];
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t pos0 = seg * S;
  const uint32_t start = max(pos0, E_lo);
  if (pos0 >= E_hi || start >= pos0 + S) return;
  const uint32_t end = min(pos0 + S, E_hi);
  auto entry = [&](uint32_t j) { return entries ? entries[j] : j; };
  const uint32_t e_cur = entry(start);
  const uint32_t e_next = (start + 1 < end) ? entry(start + 1) : 0u;
  const uint32_t b = b_lo + find_bucket(offsets + b_lo, b_hi - b_lo, start);
  const uint32_t next = offsets[b + 1];
  const bool started_here = offsets[b] >= pos0;
  if (start == pos0) cont_bucket[seg] = started_here ? 0xffffffffu : b;
  auto no_issue = [](uint32_t) {};
  accumulate_lds<F, NW, NW / 2, true, true>(nullptr, 0, 0, limbs, entries, offsets, start, end, pos0, seg, b, next,
                                           started_here, e_cur, e_next, no_issue, bucket_sums, conts, bases, rec);
}

// Segment length S so that the accumulation grid is exactly ROUNDS full waves of
// resident workgroups (occupancy from the compiled kernel, CUs from the device): a
// partial last round would leave most of the chip idle for its whole duration.
// BH_G2_DIRECT=1 (A/B): the G2 accumulation without LDS prefetch slots, two waves per SIMD
inline bool g2_direct() {
  static const bool v = [] {
    const char* e = getenv("BH_G2_DIRECT");
    return e && e[0] == '1';
  }();
  return v;
}
template <class C>
const void* accumulate_kernel() {
  if constexpr (!std::is_same<C, G1Ops>::value)
    if (g2_direct()) return (const void*)k_accumulate_g2d<C>;
  return (const void*)k_accumulate_pf<C>;
}

template <class C>
void fit_segments_E(MsmShape& sh, size_t E);
template <class C>
void fit_segments(MsmShape& sh, size_t n) {
  fit_segments_E<C>(sh, n * (size_t)sh.W);
}
template <class C>
void fit_segments_E(MsmShape& sh, size_t E) {
  static const size_t conc = [] {
    int dev = 0, cus = 256, blocks = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* k = accumulate_kernel<C>();
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, 0) != hipSuccess || blocks < 1) blocks = 1;
    return (size_t)cus * (size_t)blocks * 256;
  }();
  // 3 rounds (round 5; 4 before): same-box 2^22 bench 53.2-53.4 ms per proof against 54.6 with 4,
  // 53.4-53.9 with 2, 58.5-59.4 with 1, and the rehearsal faster at N = 1, 2 and 8 too
  // (profiles/r05_ab_acc_rounds.txt): fewer segments are fewer continuation partials and bucket
  // stores, and with the G2 and G1 accumulations sharing the SIMDs a third round balances the
  // finish well enough.  Round 6: 2, 1.5, 4 and 6 rounds (G1, G2 or both) no better at N = 1, 4
  // and 8 or for bh_prove (profiles/r06_ab_acc_rounds.txt).  Segments of at least 8 entries
  // (shorter ones multiply the continuation partials and the per-segment bucket search).
  constexpr size_t ROUNDS = 3, MIN_S = 8;
  const size_t slots = std::max<size_t>(ROUNDS * conc / 256 * 256, 256);
  size_t S = (E + slots - 1) / slots;
  sh.S = (int)std::min<size_t>(std::max<size_t>(S, MIN_S), (size_t)1 << 16);
}

template <class C>
size_t MsmWorkspace<C>::bytes_needed(size_t n) {
  MsmShape sh = msm_shape(n, 0);
  size_t E = n * (size_t)sh.W;
  size_t nbt = (size_t)sh.Wb * sh.NB;
  size_t segs = (E + sh.S - 1) / sh.S + 1;
  size_t T = (size_t)sh.Wb * (sh.NB / sh.L);
  return E * 4 + nbt * 4 * 3 + 16 + nbt * sizeof(typename C::P) + segs * sizeof(typename C::P) +
         2 * T * sizeof(typename C::P) + n * 4;
}

template <class C>
hipError_t MsmWorkspace<C>::grow(size_t E, size_t nbt, size_t segs, size_t T) {
  hipError_t err;
  if (E > cap_E) {
    if (entries) hipFree(entries);
    if (recs) hipFree(recs);
    entries = nullptr;
    recs = nullptr;
    if ((err = hipMalloc(&entries, std::max<size_t>(E, 1) * 4)) != hipSuccess) return err;
    if ((err = hipMalloc(&recs, std::max<size_t>(E, 1) * 8)) != hipSuccess) return err;
    cap_E = E;
  }
  if (nbt > cap_nbt) {
    if (counts) hipFree(counts);
    if (offsets) hipFree(offsets);
    if (cursor) hipFree(cursor);
    if (scan_scratch) hipFree(scan_scratch);
    if (bucket_sums) hipFree(bucket_sums);
    counts = offsets = cursor = scan_scratch = nullptr;
    bucket_sums = nullptr;
    if ((err = hipMalloc(&counts, (nbt + 1) * 4)) != hipSuccess) return err;
    if ((err = hipMalloc(&offsets, (nbt + 1) * 4)) != hipSuccess) return err;
    if ((err = hipMalloc(&cursor, (nbt + 1) * 4)) != hipSuccess) return err;
    if ((err = hipMalloc(&scan_scratch, scan_scratch_words(nbt + 1) * 4 + 64)) != hipSuccess) return err;
    if ((err = hipMalloc(&bucket_sums, nbt * sizeof(typename C::P))) != hipSuccess) return err;
    cap_nbt = nbt;
  }
  if (segs > cap_segs) {
    if (conts) hipFree(conts);
    if (cont_bucket) hipFree(cont_bucket);
    conts = nullptr;
    cont_bucket = nullptr;
    if ((err = hipMalloc(&conts, segs * sizeof(typename C::P))) != hipSuccess) return err;
    if ((err = hipMalloc(&cont_bucket, segs * 4)) != hipSuccess) return err;
    cap_segs = segs;
  }
  if (T > cap_T) {
    if (seg_weighted) hipFree(seg_weighted);
    if (seg_sum) hipFree(seg_sum);
    seg_weighted = seg_sum = nullptr;
    if ((err = hipMalloc(&seg_weighted, T * sizeof(typename C::P))) != hipSuccess) return err;
    if ((err = hipMalloc(&seg_sum, T * sizeof(typename C::P))) != hipSuccess) return err;
    cap_T = T;
  }
  if (!window_sums) {
    if ((err = hipMalloc(&window_sums, 256 * sizeof(typename C::P))) != hipSuccess) return err;
    if ((err = hipHostMalloc(&host_window_sums, 256 * sizeof(typename C::P), hipHostMallocDefault)) != hipSuccess)
      return err;
  }
  return hipSuccess;
}

template <class C>
hipError_t MsmWorkspace<C>::reserve_shape(size_t n, const MsmShape& sh) {
  const size_t E = n * (size_t)sh.W;
  const size_t nbt = (size_t)sh.Wb * sh.NB;
  const size_t segs = (E + sh.S - 1) / sh.S + 1;
  const size_t T = (size_t)sh.Wb * (sh.NB / sh.L);
  const size_t tc = sort_tilecount_words(sh, n);
  if (tc > cap_tc) {
    if (tilecounts) hipFree(tilecounts);
    if (tscan) hipFree(tscan);
    tilecounts = tscan = nullptr;
    hipError_t err;
    if ((err = hipMalloc(&tilecounts, tc * 4)) != hipSuccess) return err;
    if ((err = hipMalloc(&tscan, scan_scratch_words(tc) * 4 + 64)) != hipSuccess) return err;
    cap_tc = tc;
  }
  return grow(E, nbt, segs, T);
}

// size for every automatic shape up to n_max
template <class C>
hipError_t MsmWorkspace<C>::reserve(size_t n_max) {
  for (size_t n = 1;; n <<= 1) {
    size_t nn = std::min(n, n_max);
    hipError_t e = reserve_shape(nn, msm_shape(nn, 0));
    if (e != hipSuccess) return e;
    if (nn == n_max) break;
  }
  if (n_max > cap_n) cap_n = n_max;
  return hipSuccess;
}

template <class C>
void MsmWorkspace<C>::release() {
  if (entries) hipFree(entries);
  if (recs) hipFree(recs);
  if (tilecounts) hipFree(tilecounts);
  if (tscan) hipFree(tscan);
  recs = nullptr;
  tilecounts = tscan = nullptr;
  cap_tc = 0;
  if (counts) hipFree(counts);
  if (offsets) hipFree(offsets);
  if (cursor) hipFree(cursor);
  if (scan_scratch) hipFree(scan_scratch);
  if (bucket_sums) hipFree(bucket_sums);
  if (conts) hipFree(conts);
  if (cont_bucket) hipFree(cont_bucket);
  cont_bucket = nullptr;
  if (seg_weighted) hipFree(seg_weighted);
  if (seg_sum) hipFree(seg_sum);
  if (window_sums) hipFree(window_sums);
  if (host_window_sums) hipHostFree(host_window_sums);
  entries = counts = offsets = cursor = scan_scratch = nullptr;
  bucket_sums = conts = seg_weighted = seg_sum = window_sums = nullptr;
  host_window_sums = nullptr;
  cap_n = cap_E = cap_nbt = cap_segs = cap_T = 0;
}

// Front half: sort the digits and accumulate the buckets (stream `st`).
template <class C>
hipError_t msm_sort(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_scalars, size_t n, const int32_t* d_idx,
                    uint32_t base_offset, const MsmShape& sh) {
  hipError_t e = ws.reserve_shape(n, sh);
  if (e != hipSuccess) return e;
  sort_entries(d_scalars, n, d_idx, base_offset, sh, ws.tilecounts, ws.tscan, ws.recs, ws.entries, ws.counts,
               ws.offsets, st);
  return hipGetLastError();
}

// bucket accumulation over the sorted entries
template <class C>
hipError_t msm_accumulate(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, size_t n, const MsmShape& sh,
                          MsmTiming* timing) {
  const size_t nbt = (size_t)sh.Wb * sh.NB;
  if (n > 0) {
    const size_t Emax = n * (size_t)sh.W;
    const size_t segs = (Emax + sh.S - 1) / sh.S;
    uint32_t launch_range_first = 0, launch_range_end = 0;
    if (timing && timing->ev_acc_begin) hipEventRecord(timing->ev_acc_begin, st);
    using F = typename std::conditional<std::is_same<C, G1Ops>::value, G1F, Fp2Ops>::type;
    const uint32_t rec = sh.rec ? (uint32_t)sh.rec : 2u * F::PACKED_WORDS;
    if (sh.bucket_shard()) {  // only the shard's buckets are sorted (their offsets alone are set)
      launch_range_first = sh.bk_lo;
      launch_range_end = sh.bk_hi;
    }
    auto launch = [&](uint32_t lo, uint32_t hi) {
      if constexpr (!std::is_same<C, G1Ops>::value) {
        if (g2_direct()) {
          hipLaunchKernelGGL(k_accumulate_g2d<C>, dim3(msm_blocks_for(segs, 256)), dim3(256), 0, st, ws.entries,
                             ws.offsets, (uint32_t)nbt, d_bases, rec, (uint32_t)sh.S, lo, hi, ws.bucket_sums,
                             ws.conts, ws.cont_bucket);
          return;
        }
      }
      hipLaunchKernelGGL(k_accumulate_pf<C>, dim3(msm_blocks_for(segs, 256)), dim3(256), 0, st, ws.entries,
                         ws.offsets, (uint32_t)nbt, d_bases, rec, (uint32_t)sh.S, lo, hi, ws.bucket_sums, ws.conts,
                         ws.cont_bucket);
    };
    if (sh.bucket_shard()) launch(launch_range_first, launch_range_end);
    else launch(0u, (uint32_t)nbt);
    if (timing && timing->ev_acc_end) hipEventRecord(timing->ev_acc_end, st);
  }
  return hipGetLastError();
}

// Front half of one multiexp: sort + accumulation, stream-ordered on st.
template <class C>
hipError_t msm_front(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, const uint32_t* d_scalars,
                     size_t n, const int32_t* d_idx, uint32_t base_offset, const MsmShape& sh, MsmTiming* timing) {
  hipError_t e = msm_sort<C>(ws, st, d_scalars, n, d_idx, base_offset, sh);
  if (e != hipSuccess) return e;
  return msm_accumulate<C>(ws, st, d_bases, n, sh, timing);
}

// Reduction of the buckets [b0, b0 + nbr) of each of Wb windows (window stride NB): continuation
// fix-up, then the two-level summation by parts into out[] (Wb totals, or 3 points when split).
struct SpanSrc {  // device-decided tails: k_max_span's words (null: the host decided)
  const uint32_t* words = nullptr;
  uint32_t g = 0, fold_span = 0, seq_max = 0;
};

// The sorted view the accumulation left for the reduction: the sort's counts/offsets and the
// shape's S.
struct AccView {
  const uint32_t *counts, *offsets;
  uint32_t S;
  size_t E;  // upper bound of the accumulated records
  const uint32_t* span_words;  // (null: the sort's, passed to msm_back)
};
template <class C>
AccView acc_view(const MsmWorkspace<C>& ws, size_t n, const MsmShape& sh) {
  return AccView{ws.counts, ws.offsets, (uint32_t)sh.S, n * (size_t)sh.W, nullptr};
}

template <class C>
static void reduce_range(MsmWorkspace<C>& ws, const AccView& v, hipStream_t st, const MsmShape& sh, size_t segs,
                         size_t span, bool fold, bool seq, uint32_t b0, uint32_t nbr, uint32_t L, uint32_t y_off,
                         typename C::P* out, const SpanSrc& dev = SpanSrc()) {
  constexpr bool G2 = sizeof(typename C::P) > 256;
  const size_t nb_all = (size_t)sh.Wb * nbr;
  const size_t nbt = (size_t)sh.Wb * sh.NB;
  if (dev.words || (!fold && seq)) {
    constexpr int Q = 4;
    constexpr uint32_t B = G2 ? 128 : 256;  // LDS: B points
    if (dev.words || span >= 2)
      hipLaunchKernelGGL((k_cont_seq<C, Q>), dim3(msm_blocks_for(nb_all * Q, B)), dim3(B), B * sizeof(typename C::P),
                         st, v.counts, v.offsets, b0, (uint32_t)nb_all, v.S, ws.conts, dev.words, dev.g,
                         dev.fold_span, dev.seq_max);
    // device-decided spans beyond seq_max: one workgroup per such bucket (returns at once when
    // there is none)
    if (dev.words)
      hipLaunchKernelGGL((k_cont_long<C>), dim3(std::min<unsigned>(msm_blocks_for(nb_all, B), 256u)), dim3(B),
                         B * sizeof(typename C::P), st, v.counts, v.offsets, b0, (uint32_t)nb_all, v.S, ws.conts,
                         dev.words, dev.g, dev.seq_max);
  } else if (!fold) {
    for (size_t stride = 1; stride < span; stride *= 4)
      hipLaunchKernelGGL((k_cont_treeF<C, 4>), dim3(msm_blocks_for(segs, 256)), dim3(256), 0, st, ws.cont_bucket,
                         v.counts, v.offsets, (uint32_t)nbt, v.S, (uint32_t)stride, b0, (uint32_t)(b0 + nb_all),
                         ws.conts);
  }
  // two-level summation by parts (k_reduce_blocks, k_reduce_window): Y/S per level-1 block
  // in seg_weighted / seg_sum (from y_off), the totals in out
  const uint32_t T = nbr / L;
  const uint32_t BT = reduce_threads_for(nbr, L, G2);
  const uint32_t nblk = T / BT;
  uint32_t BT2, Lb;
  reduce_level2(nblk, G2, &BT2, &Lb);
  const int split = sh.Wb == 1 ? 1 : 0;
  hipLaunchKernelGGL(k_reduce_blocks<C>, dim3((unsigned)(sh.Wb * nblk)), dim3(BT), BT * sizeof(typename C::P), st,
                     v.counts, v.offsets, ws.bucket_sums, ws.conts, v.S, b0, (uint32_t)sh.NB, L, reduce_lg2(L), nblk,
                     fold ? 1 : 0, ws.seg_weighted + y_off, ws.seg_sum + y_off, dev.words, dev.g, dev.fold_span);
  hipLaunchKernelGGL(k_reduce_window<C>, dim3((unsigned)sh.Wb), dim3(BT2), 2 * BT2 * sizeof(typename C::P), st,
                     ws.seg_weighted + y_off, ws.seg_sum + y_off, nblk, Lb, reduce_lg2(Lb),
                     reduce_lg2(L) + reduce_lg2(BT), split, out);
}

// Back half: continuation fix-up, summation by parts and the per-window sums, copied to host_out
// (Wb entries; 2 for one shared window, 3 for a bucket shard).
template <class C>
hipError_t msm_back(MsmWorkspace<C>& ws, hipStream_t st, size_t n, const MsmShape& sh, typename C::P* host_out,
                    int max_span, hipEvent_t acc_done, const uint32_t* d_span_words) {
  // continuation partials: a bucket spanning up to REDUCE_FOLD_SPAN segments has them added
  // by its reduction thread (no extra launch); longer spans (known from the sort) are folded
  // first -- Q threads per bucket, or log-depth 4-ary tree levels
  constexpr size_t REDUCE_FOLD_SPAN = 8;
  const AccView v = acc_view<C>(ws, n, sh);
  const size_t segs = (v.E + v.S - 1) / v.S;
  const size_t span = max_span >= 0 ? (size_t)max_span : segs;
  const bool fold = max_span >= 0 && span <= REDUCE_FOLD_SPAN;
  const bool seq = max_span >= 0 && span <= cont_seq_max();
  SpanSrc dev;
  if (max_span < 0 && d_span_words) {  // device-decided: fold up to REDUCE_FOLD_SPAN, else k_cont_seq
    dev.words = d_span_words;
    dev.g = max_span_blocks((size_t)sh.Wb * sh.red_nb());  // (sort_job's k_max_span range)
    dev.fold_span = (uint32_t)REDUCE_FOLD_SPAN;
    dev.seq_max = (uint32_t)cont_seq_max();
  }
  (void)acc_done;  // (stream order: the caller's st already follows the accumulation)
  reduce_range<C>(ws, v, st, sh, segs, span, fold, seq, sh.red_lo(), sh.red_nb(), (uint32_t)sh.L, 0, ws.window_sums,
                  dev);
  const int outs = sh.bucket_shard() ? 3 : (sh.Wb == 1 ? 2 : sh.Wb);
  hipMemcpyAsync(host_out, ws.window_sums, outs * sizeof(typename C::P), hipMemcpyDeviceToHost, st);
  return hipGetLastError();
}

template <class C>
void msm_acc_kernels(std::vector<KernInfo>& v) {
  v.push_back({std::is_same<C, G1Ops>::value ? "k_accumulate_pf<G1>" : "k_accumulate_pf<G2>",
               (const void*)k_accumulate_pf<C>, 256, 0});
  if constexpr (!std::is_same<C, G1Ops>::value)
    v.push_back({"k_accumulate_g2d", (const void*)k_accumulate_g2d<C>, 256, 0});
}
template <class C>
void msm_back_kernels(std::vector<KernInfo>& v) {
  constexpr bool G2 = sizeof(typename C::P) > 256;
  const size_t P = sizeof(typename C::P);
  const int B = G2 ? 128 : 256, BT = (int)reduce_block_max(G2);
  v.push_back({G2 ? "k_reduce_blocks<G2>" : "k_reduce_blocks<G1>", (const void*)k_reduce_blocks<C>, BT, BT * P});
  v.push_back({G2 ? "k_reduce_window<G2>" : "k_reduce_window<G1>", (const void*)k_reduce_window<C>, BT,
               2 * BT * P});
  v.push_back({G2 ? "k_cont_seq<G2>" : "k_cont_seq<G1>", (const void*)k_cont_seq<C, 4>, B, B * P});
  v.push_back({G2 ? "k_cont_long<G2>" : "k_cont_long<G1>", (const void*)k_cont_long<C>, B, B * P});
  v.push_back({G2 ? "k_cont_treeF<G2>" : "k_cont_treeF<G1>", (const void*)k_cont_treeF<C, 4>, 256, 0});
}

template <class C>
hipError_t msm_window_sums(MsmWorkspace<C>& ws, hipStream_t st, const uint32_t* d_bases, const uint32_t* d_scalars,
                           size_t n, const int32_t* d_idx, uint32_t base_offset, const MsmShape& sh,
                           MsmTiming* timing) {
  hipError_t e = msm_front<C>(ws, st, d_bases, d_scalars, n, d_idx, base_offset, sh, timing);
  if (e != hipSuccess) return e;
  e = ws.reserve_shape(n, sh);
  if (e != hipSuccess) return e;
  return msm_back<C>(ws, st, n, sh, ws.host_window_sums);
}

}  // namespace bh
