// Pippenger multi-scalar multiplication on gfx950 -- the device replacement for
// multiexp::multiexp / multiexp_inner (reference src/multiexp.rs:159-281).
//
// The reference walks all n (scalar, density) pairs once per c-bit window,
// adds each base into bucket[digit-1] (multiexp.rs:191-223), then sums the
// buckets by parts (229-233) and Horner-combines the windows (244-249).
// Here the same sum is computed as a data-parallel pipeline:
//
//   k_hist      one thread per scalar: signed c-bit digits (|d| <= 2^(c-1)),
//               histogram of (window, |d|) bucket sizes      [global atomics]
//   scan        exclusive scan of the histogram -> bucket offsets
//   k_scatter   one thread per scalar: place (base index | sign) into its
//               bucket's slice of the entry array (counting sort)
//   k_accumulate one thread per fixed-size SEGMENT of S sorted entries:
//               mixed XYZZ additions of the gathered affine bases; perfectly
//               load balanced whatever the digit distribution.  Partial sums
//               of buckets that straddle segments go to a per-segment slot.
//   k_bucket_reduce one thread per L consecutive buckets: running sums
//               (summation by parts) -> (sum_t, weighted_t)
//   k_seg_combine  weighted_t + (t*L)*sum_t
//   k_sum_groups   per-window sum of the segment results, a 4-ary tree of launches
// The host then performs the W-window Horner step (multiexp.rs:244-249).
//
// Semantics of the reference Source (multiexp.rs:45-86) are reproduced by the
// caller: bases are consumed only where the density bit is set (the index map
// built by k_density_index), EOF / identity errors are detected on the host.
#include "msm.h"

#include <algorithm>

namespace bh {

static inline unsigned blocks_for(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }


// ----------------------------------------------------------------- scans
// exclusive scan of uint32 (in place allowed), recursive over tiles of 1024
// dn (optional): a device word bounding the scan to its first *dn + 1 elements (tiles past it
// exit; their sums read 0), for scans sized by a device-side count (derive_sorted)
__device__ __forceinline__ size_t scan_len(size_t n, const uint32_t* dn) {
  return dn ? min(n, (size_t)*dn + 1) : n;
}
__global__ void __launch_bounds__(256) k_scan_tile(const uint32_t* in, uint32_t* out, uint32_t* tile_sums, size_t n,
                                                   const uint32_t* dn) {
  __shared__ uint32_t s[256];
  n = scan_len(n, dn);
  if ((size_t)blockIdx.x * 1024 >= n) {
    if (threadIdx.x == 0 && tile_sums) tile_sums[blockIdx.x] = 0;
    return;
  }
  const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
  uint32_t v[4];
  uint32_t local = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    v[i] = (base + i < n) ? in[base + i] : 0u;
    local += v[i];
  }
  s[threadIdx.x] = local;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t t = (threadIdx.x >= (unsigned)off) ? s[threadIdx.x - off] : 0u;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - local;  // exclusive prefix of this thread
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 255 && tile_sums) tile_sums[blockIdx.x] = s[255];
}

__global__ void k_scan_add(uint32_t* out, const uint32_t* tile_prefix, size_t n, const uint32_t* dn) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < scan_len(n, dn)) out[i] += tile_prefix[i >> 10];
}

// scratch must hold scan_scratch_words(n) words
size_t scan_scratch_words(size_t n) {
  size_t tiles = (n + 1023) / 1024;
  if (tiles <= 1) return 1;
  return tiles + scan_scratch_words(tiles);
}

static void exclusive_scan_b(const uint32_t* in, uint32_t* out, size_t n, uint32_t* scratch, hipStream_t st,
                             const uint32_t* dn) {
  size_t tiles = (n + 1023) / 1024;
  if (tiles == 0) return;
  if (tiles == 1) {
    hipLaunchKernelGGL(k_scan_tile, dim3(1), dim3(256), 0, st, in, out, (uint32_t*)nullptr, n, dn);
    return;
  }
  uint32_t* sums = scratch;
  hipLaunchKernelGGL(k_scan_tile, dim3((unsigned)tiles), dim3(256), 0, st, in, out, sums, n, dn);
  exclusive_scan_b(sums, sums, tiles, scratch + tiles, st, nullptr);  // (the tile sums past dn are 0)
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, sums, n, dn);
}

void exclusive_scan(const uint32_t* in, uint32_t* out, size_t n, uint32_t* scratch, hipStream_t st) {
  exclusive_scan_b(in, out, n, scratch, st, nullptr);
}

// ----------------------------------------------------------------- scalars
// mode 0: canonical LE words; 1: bls12_381 Montgomery (R=2^256); 2: device Montgomery (R=2^261)
// Optional gather through a bit-reversal permutation of length 2^log_perm
__global__ void __launch_bounds__(256) k_scalars_prepare(const uint32_t* in, uint32_t* out, size_t n, int mode,
                                                          int log_perm) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  size_t src = i;
  if (log_perm > 0) src = __builtin_bitreverse32((uint32_t)i) >> (32 - log_perm);
  const uint4* p = reinterpret_cast<const uint4*>(in + src * 8);
  uint4 a = p[0], b = p[1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  if (mode == 0) {
    // canonical words are Scalar::to_le_bits of a field element (< r); a caller's word >= r
    // (< 2^256 < 3r) is reduced: the reference's multiexp walks all 256 bits, and
    // (k mod r) * P = k * P for every point of the prime-order group, so the result is the same
    constexpr uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                               0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
    for (int it = 0; it < 2; it++) {
      bool ge = true;
      for (int k = 7; k >= 0; k--) {
        if (w[k] != R[k]) { ge = w[k] > R[k]; break; }
      }
      if (!ge) break;
      uint32_t borrow = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint64_t d = (uint64_t)w[k] - R[k] - borrow;
        w[k] = (uint32_t)d;
        borrow = (uint32_t)(d >> 63);
      }
    }
  } else {
    DFr x = fe_unpack<FrCfg>(w);
    DFr r;
    if (mode == 1) {
      DFr k = fe_zero<FrCfg>();
      k.v[0] = 32u;  // x*32*2^-261 = x*2^-256
      r = fe_csub<FrCfg, 1>(fe_mul<FrCfg>(x, k));  // < r + 1: one subtraction
    } else {
      r = fe_csub<FrCfg, 1>(fe_from_mont<FrCfg>(x));  // x*2^-261 <= r
    }
    fe_pack<FrCfg>(r, w);
  }
  uint4* q = reinterpret_cast<uint4*>(out + i * 8);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// ----------------------------------------------------------------- density
__global__ void k_density_popc(const uint64_t* words, size_t nwords, uint32_t* popc) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwords) popc[i] = (uint32_t)__popcll(words[i]);
}

// idx[i] = base_offset + #set bits before i  (if bit i set) else -1
__global__ void k_density_index(const uint64_t* words, const uint32_t* word_prefix, size_t n, uint32_t base_offset,
                                int32_t* idx) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t w = words[i >> 6];
  const int bit = (int)(i & 63);
  if ((w >> bit) & 1ull) {
    const uint64_t below = bit ? (w & ((1ull << bit) - 1ull)) : 0ull;
    idx[i] = (int32_t)(base_offset + word_prefix[i >> 6] + (uint32_t)__popcll(below));
  } else {
    idx[i] = -1;
  }
}

// ----------------------------------------------------------------- digits
struct DigitCfg {
  int c, W, NB, pre;
};

// bucket id and entry of digit d of window w for base `base`
__device__ __forceinline__ uint32_t digit_bucket(const DigitCfg& cfg, int w, int d) {
  const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;
  return cfg.pre ? b : (uint32_t)w * cfg.NB + b;
}
__device__ __forceinline__ uint32_t digit_entry(const DigitCfg& cfg, uint32_t base, int w, int d) {
  const uint32_t e = cfg.pre ? base * (uint32_t)cfg.W + (uint32_t)w : base;
  return e | (d < 0 ? 0x80000000u : 0u);
}

// signed digit of window w; returns digit in [-2^(c-1), 2^(c-1)], updates carry
__device__ __forceinline__ int digit_at(const uint32_t* s, int w, int c, uint32_t& carry) {
  const int bit = w * c;
  const int wi = bit >> 5, sh = bit & 31;
  uint64_t lo = (wi < 8) ? s[wi] : 0u;
  uint64_t hi = (wi + 1 < 8) ? s[wi + 1] : 0u;
  uint32_t raw = (uint32_t)((((hi << 32) | lo) >> sh) & ((1ull << c) - 1ull));
  uint32_t d = raw + carry;
  const uint32_t half = 1u << (c - 1);
  if (d > half) {
    carry = 1;
    return (int)d - (int)(1u << c);
  }
  carry = 0;
  return (int)d;
}

__device__ __forceinline__ void load_scalar(const uint32_t* scalars, size_t i, uint32_t* s) {
  const uint4* p = reinterpret_cast<const uint4*>(scalars + i * 8);
  uint4 a = p[0], b = p[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
  s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

// Window choice: c ~ log2(n) - 6, clamped to [4, 16], preferring the c in
// {c-1, c, c+1} whose top window is fullest (a nearly empty top window piles
// every scalar into a handful of giant buckets).  Segment length S keeps about
// 2^18 accumulation threads in flight.  Results never depend on either choice.
// minimum bucket-reduction threads: a small bucket set's tail is latency-bound
static constexpr size_t REDUCE_T_MIN = 16384;

MsmShape msm_shape(size_t n, int c_override) {
  MsmShape sh;
  int c = c_override;
  if (c <= 0) {
    int lg = 0;
    while (((size_t)1 << (lg + 1)) <= n) lg++;
    int c0 = std::max(4, std::min(16, lg - 6));
    int best = c0, best_fill = -1;
    for (int cc = std::max(4, c0 - 1); cc <= std::min(16, c0 + 1); cc++) {
      const int W = (256 + cc - 1) / cc;
      const int top = 256 - (W - 1) * cc;  // bits in the top window
      const int fill = top * 16 / cc;      // 0..16
      if (fill > best_fill || (fill == best_fill && cc == c0)) { best = cc; best_fill = fill; }
    }
    c = best;
  }
  sh.c = c;
  sh.W = (256 + c - 1) / c;
  sh.NB = 1 << (c - 1);
  // buckets per reduction thread (msm_back): up to 8 (~3 additions per bucket; 16 would do less
  // work, but its longer-lived waves cost the overlapped accumulations more: +2 ms per 2^22
  // proof in a same-box A/B), fewer when that leaves under 16384 threads (a small bucket set's
  // tail is latency-bound: a shard's G2 tail at 2^15 buckets took 5.8 ms beside the
  // accumulations with L = 8, 4096 threads)
  sh.L = std::min<int>(8, sh.NB);
  while (sh.L > 1 && (size_t)sh.W * (size_t)(sh.NB / sh.L) < REDUCE_T_MIN) sh.L >>= 1;
  size_t E = n * (size_t)sh.W;
  int S = 16;
  while (S < 256 && E / (size_t)(2 * S) >= ((size_t)1 << 18)) S <<= 1;
  sh.S = S;
  sh.Wb = sh.W;
  sh.pre = 0;
  sh.rec = 0;
  return sh;
}

// With a window table every digit window adds into one shared set of 2^(c-1) buckets, so
// the accumulation costs n*ceil(256/c) mixed additions and the reduction ~6.5 * 2^(c-1)
// mixed-addition equivalents, independent of W.  The reduction does ~3 full additions per bucket
// (msm_back), but beside the accumulations its latency-bound waves cost about twice their
// instructions: measured at 2^20 points, c = 16 beats c = 20 by 0.5 ms per proof (a weight of
// 3.6 picked c = 20 there); c = 20 stays the choice at 2^22.
// Only window sizes whose top window holds >= 10 real scalar bits: with shared buckets a
// nearly empty top window (e.g. c = 17: the 16th window only takes the carry; c = 18: 3 bits)
// pours up to n/2 entries into a handful of small-digit buckets, whose continuation partials
// then need the log-depth tree (msm_back).  For 255-bit scalars: c = 16, 20, 22, 24.
uint32_t reduce_block_max(bool g2) { return g2 ? 128u : 256u; }

// Entries the accumulation grid is sized for: n * W, the query's full length even where a density
// map leaves about half of it (b_g1_aux, b_g2_aux).  Sized for the used entries, b_g2_aux alone is
// 13.4 against 17.2 ms, but the overlapped 2^22 proof is 1.1-1.3 ms slower: the longer segments
// leave room beside it for the G1 accumulations (profiles/r05_ab_seg_used.txt).
size_t seg_entries(size_t n, size_t used, int W) {
  (void)used;
  return std::max<size_t>(n, 1) * (size_t)std::max(W, 1);
}

int msm_table_c(size_t n) {
  int best = 16;
  double best_cost = 1e300;
  for (int c = 8; c <= 24; c++) {
    const int W = (256 + c - 1) / c;
    if (255 - (W - 1) * c < 10) continue;
    const double cost = (double)n * W + 6.5 * (double)((size_t)1 << (c - 1));
    if (cost < best_cost) { best_cost = cost; best = c; }
  }
  return best;
}

MsmShape msm_shape_table(size_t n, int c) {
  MsmShape sh = msm_shape(n, c);
  sh.Wb = 1;
  sh.pre = 1;
  // one shared bucket window: the reduction's thread count is NB / L
  while (sh.L > 1 && (size_t)(sh.NB / sh.L) < REDUCE_T_MIN) sh.L >>= 1;
  return sh;
}

// ----------------------------------------------------------------- LDS radix partition sort
// Entries are keyed by the global bucket id gb = w*NB + |d|-1 (< nbt).  Pass 1 counts,
// per tile of PT_TILE scalars, how many entries fall in each coarse partition
// p = gb >> lo_bits (<= 4096 partitions, LDS histogram); a scan turns the
// partition-major counts into offsets; pass 3 scatters (entry, gb & lo_mask)
// records with LDS cursors; pass 4 (one workgroup per partition) sorts its
// records by the low bits with an LDS counting sort and writes the final entry
// array plus counts[gb] / offsets[gb] for every bucket of the partition.
static constexpr int PT_TILE = 4096;  // scalars per tile

// [plo, phi): the partitions a bucket shard keeps (MsmShape::bk_lo); digits outside are skipped by
// both passes, so the scan leaves their partitions empty and k_part_sort writes zero counts there
__global__ void __launch_bounds__(256) k_part_count(const uint32_t* scalars, size_t n, const int32_t* idx,
                                                    DigitCfg cfg, int lo_bits, uint32_t P, uint32_t ntiles,
                                                    uint32_t plo, uint32_t phi, uint32_t* tilecounts) {
  extern __shared__ uint32_t hist[];
  for (uint32_t i = threadIdx.x; i < P; i += 256) hist[i] = 0;
  __syncthreads();
  const size_t s0 = (size_t)blockIdx.x * PT_TILE;
  const size_t s1 = min(s0 + PT_TILE, n);
  for (size_t s = s0 + threadIdx.x; s < s1; s += 256) {
    if (idx && idx[s] < 0) continue;
    uint32_t sc[8];
    load_scalar(scalars, s, sc);
    uint32_t carry = 0;
    for (int w = 0; w < cfg.W; w++) {
      const int d = digit_at(sc, w, cfg.c, carry);
      if (d != 0) {
        const uint32_t p = digit_bucket(cfg, w, d) >> lo_bits;
        if (p - plo < phi - plo) atomicAdd(&hist[p], 1u);
      }
    }
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < P; p += 256) tilecounts[(size_t)p * ntiles + blockIdx.x] = hist[p];
  // the scan's extra last word (its output is the total): zeroed here rather than by a fill
  if (blockIdx.x == 0 && threadIdx.x == 0) tilecounts[(size_t)P * ntiles] = 0;
}

__global__ void __launch_bounds__(256) k_part_scatter(const uint32_t* scalars, size_t n, const int32_t* idx,
                                                      uint32_t base_offset, DigitCfg cfg, int lo_bits, uint32_t P,
                                                      uint32_t ntiles, uint32_t plo, uint32_t phi,
                                                      const uint32_t* offs, uint2* recs) {
  extern __shared__ uint32_t cur[];
  for (uint32_t p = threadIdx.x; p < P; p += 256) cur[p] = offs[(size_t)p * ntiles + blockIdx.x];
  __syncthreads();
  const uint32_t lo_mask = (1u << lo_bits) - 1u;
  const size_t s0 = (size_t)blockIdx.x * PT_TILE;
  const size_t s1 = min(s0 + PT_TILE, n);
  for (size_t s = s0 + threadIdx.x; s < s1; s += 256) {
    uint32_t base;
    if (idx) {
      const int32_t v = idx[s];
      if (v < 0) continue;
      base = (uint32_t)v;
    } else {
      base = base_offset + (uint32_t)s;
    }
    uint32_t sc[8];
    load_scalar(scalars, s, sc);
    uint32_t carry = 0;
    for (int w = 0; w < cfg.W; w++) {
      const int d = digit_at(sc, w, cfg.c, carry);
      if (d != 0) {
        const uint32_t gb = digit_bucket(cfg, w, d);
        if ((gb >> lo_bits) - plo >= phi - plo) continue;
        const uint32_t pos = atomicAdd(&cur[gb >> lo_bits], 1u);
        recs[pos] = make_uint2(digit_entry(cfg, base, w, d), gb & lo_mask);
      }
    }
  }
}

// one workgroup per partition; bins = 2^lo_bits <= 4096
// (partitions p0 .. P-1 of the grid; a bucket shard sorts only its own and passes its end as P,
// and its last partition also writes offsets[nbt], the shard's entry count)
__global__ void __launch_bounds__(256) k_part_sort(const uint2* recs, const uint32_t* offs, uint32_t ntiles,
                                                   uint32_t P, int lo_bits, uint32_t nbt, uint32_t* entries,
                                                   uint32_t* counts, uint32_t* offsets, uint32_t p0) {
  __shared__ uint32_t bins[4096];
  __shared__ uint32_t part[256];
  const uint32_t p = p0 + blockIdx.x;
  const uint32_t nb = 1u << lo_bits;
  const uint32_t start = offs[(size_t)p * ntiles];
  const uint32_t end = offs[(size_t)(p + 1) * ntiles];  // offs has P*ntiles+1 entries
  for (uint32_t i = threadIdx.x; i < nb; i += 256) bins[i] = 0;
  __syncthreads();
  for (uint32_t j = start + threadIdx.x; j < end; j += 256) atomicAdd(&bins[recs[j].y], 1u);
  __syncthreads();
  // exclusive scan of bins: each thread owns a contiguous run of nb/256 (or 1) bins
  const uint32_t per = (nb + 255) / 256;
  const uint32_t b0 = threadIdx.x * per;
  uint32_t local = 0;
  for (uint32_t k = 0; k < per; k++) if (b0 + k < nb) local += bins[b0 + k];
  part[threadIdx.x] = local;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t t = (threadIdx.x >= (unsigned)off) ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = start + part[threadIdx.x] - local;
  for (uint32_t k = 0; k < per; k++) {
    const uint32_t b = b0 + k;
    if (b >= nb) break;
    const uint32_t cnt = bins[b];
    const uint32_t gb = (p << lo_bits) + b;
    if (gb < nbt) { counts[gb] = cnt; offsets[gb] = run; }
    bins[b] = run;  // becomes the write cursor
    run += cnt;
  }
  if (p == P - 1 && threadIdx.x == 0) {
    offsets[nbt] = end;
    if (((size_t)P << lo_bits) < nbt) offsets[P << lo_bits] = end;  // a shard's end bucket
  }
  __syncthreads();
  for (uint32_t j = start + threadIdx.x; j < end; j += 256) {
    const uint2 r = recs[j];
    const uint32_t pos = atomicAdd(&bins[r.y], 1u);
    entries[pos] = r.x;
  }
}

// ----------------------------------------------------------------- derived sorts
// A multiexp over the same scalars and digit geometry as an already sorted one, but a
// sparser density map (a_aux, b_aux against l: prover.rs:259-307 all take the aux assignment),
// has the same bucket order: its sorted entries are the source's with every entry whose
// scalar is absent dropped and the base index remapped -- a stable compaction.
__device__ __forceinline__ bool derive_keep(uint32_t e, int pre, uint32_t W, uint32_t src_off, const int32_t* idx,
                                            uint32_t* out_entry) {
  const uint32_t v = e & 0x7fffffffu;
  const uint32_t base = pre ? v / W : v;
  const int32_t nb = idx[base - src_off];
  if (nb < 0) return false;
  *out_entry = ((pre ? (uint32_t)nb * W + (v - base * W) : (uint32_t)nb)) | (e & 0x80000000u);
  return true;
}

__global__ void __launch_bounds__(256) k_derive_mark(const uint32_t* src_entries, const uint32_t* src_E, size_t Emax,
                                                     int pre, uint32_t W, uint32_t src_off, const int32_t* idx,
                                                     uint32_t* mark) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t E = *src_E;
  if (j > Emax || j > E) return;  // (the scan reads marks 0 .. src_E only)
  uint32_t ne;
  mark[j] = (j < E && derive_keep(src_entries[j], pre, W, src_off, idx, &ne)) ? 1u : 0u;
}

__global__ void __launch_bounds__(256) k_derive_write(const uint32_t* src_entries, const uint32_t* src_E, int pre,
                                                      uint32_t W, uint32_t src_off, const int32_t* idx,
                                                      const uint32_t* pos, uint32_t* dst_entries) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= *src_E) return;
  uint32_t ne;
  if (derive_keep(src_entries[j], pre, W, src_off, idx, &ne)) dst_entries[pos[j]] = ne;
}

// buckets [b0, b1] (b1 <= nbt; a bucket shard's range, whose offsets alone are set), and
// dst_offsets[nbt] = the derived entry count
__global__ void __launch_bounds__(256) k_derive_offsets(const uint32_t* src_offsets, size_t nbt, size_t b0, size_t b1,
                                                        const uint32_t* pos, uint32_t* dst_offsets,
                                                        uint32_t* dst_counts) {
  const size_t b = b0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > b1) return;
  const uint32_t o = pos[src_offsets[b]];
  dst_offsets[b] = o;
  if (b < b1) dst_counts[b] = pos[src_offsets[b + 1]] - o;
  if (b == b1 && b1 < nbt) dst_offsets[nbt] = o;
}

size_t derive_scratch_words(size_t Emax) { return scan_scratch_words(Emax + 1) + 64; }

hipError_t derive_sorted(const uint32_t* src_entries, const uint32_t* src_offsets, size_t nbt, size_t Emax, int pre,
                         uint32_t W, uint32_t src_off, const int32_t* idx, uint32_t* pos, uint32_t* scan_scratch,
                         uint32_t* dst_entries, uint32_t* dst_counts, uint32_t* dst_offsets, hipStream_t st,
                         size_t b0, size_t b1) {
  if (b1 == 0 || b1 > nbt) b1 = nbt;
  const uint32_t* src_E = src_offsets + nbt;
  hipLaunchKernelGGL(k_derive_mark, dim3(blocks_for(Emax + 1, 256)), dim3(256), 0, st, src_entries, src_E, Emax, pre, W,
                     src_off, idx, pos);
  // positions 0 .. src_E only: with a bucket shard the source holds ~1/N of the Emax records
  exclusive_scan_b(pos, pos, Emax + 1, scan_scratch, st, src_E);
  hipLaunchKernelGGL(k_derive_write, dim3(blocks_for(Emax, 256)), dim3(256), 0, st, src_entries, src_E, pre, W, src_off,
                     idx, pos, dst_entries);
  hipLaunchKernelGGL(k_derive_offsets, dim3(blocks_for(b1 - b0 + 1, 256)), dim3(256), 0, st, src_offsets, nbt, b0, b1,
                     pos, dst_offsets, dst_counts);
  return hipGetLastError();
}

void sort_geometry(const MsmShape& sh, size_t n, int* lo_bits, uint32_t* P, uint32_t* ntiles) {
  const size_t nbt = (size_t)sh.Wb * sh.NB;
  int bits = 0;
  while (((size_t)1 << bits) < nbt) bits++;
  int lo = bits > 12 ? bits - 12 : 0;
  *lo_bits = lo;
  *P = (uint32_t)((nbt + ((size_t)1 << lo) - 1) >> lo);
  *ntiles = (uint32_t)std::max<size_t>(1, (n + PT_TILE - 1) / PT_TILE);
}

size_t sort_tilecount_words(const MsmShape& sh, size_t n) {
  int lo;
  uint32_t P, nt;
  sort_geometry(sh, n, &lo, &P, &nt);
  return (size_t)P * nt + 1;
}

// counts/offsets (nbt+1 words) and the sorted entry array for one MSM
hipError_t sort_entries(const uint32_t* d_scalars, size_t n, const int32_t* d_idx, uint32_t base_offset,
                        const MsmShape& sh, uint32_t* tilecounts, uint32_t* tscan_scratch, uint2* recs,
                        uint32_t* entries, uint32_t* counts, uint32_t* offsets, hipStream_t st) {
  const size_t nbt = (size_t)sh.Wb * sh.NB;
  DigitCfg cfg{sh.c, sh.W, sh.NB, sh.pre};
  int lo;
  uint32_t P, nt;
  sort_geometry(sh, n, &lo, &P, &nt);
  const size_t tw = (size_t)P * nt + 1;
  if (n == 0) {
    hipMemsetAsync(counts, 0, (nbt + 1) * 4, st);
    hipMemsetAsync(offsets, 0, (nbt + 1) * 4, st);
    return hipGetLastError();
  }
  // a bucket shard keeps the partitions of [bk_lo, bk_hi) (multiples of BUCKET_SHARD_GRANULE, so
  // of the partition width 2^lo)
  const uint32_t plo = sh.bucket_shard() ? sh.bk_lo >> lo : 0u;
  const uint32_t phi = sh.bucket_shard() ? sh.bk_hi >> lo : P;
  hipLaunchKernelGGL(k_part_count, dim3(nt), dim3(256), P * 4, st, d_scalars, n, d_idx, cfg, lo, P, nt, plo, phi,
                     tilecounts);
  // a shard scans only its partitions' slice of the partition-major tile counts (the word after
  // the slice is the next partition's first count, 0, or the extra last word): 1/N of the scan
  if (sh.bucket_shard())
    exclusive_scan(tilecounts + (size_t)plo * nt, tilecounts + (size_t)plo * nt, (size_t)(phi - plo) * nt + 1,
                   tscan_scratch, st);
  else
    exclusive_scan(tilecounts, tilecounts, tw, tscan_scratch, st);
  hipLaunchKernelGGL(k_part_scatter, dim3(nt), dim3(256), P * 4, st, d_scalars, n, d_idx, base_offset, cfg, lo, P,
                     nt, plo, phi, tilecounts, recs);
  hipLaunchKernelGGL(k_part_sort, dim3(phi - plo), dim3(256), 0, st, recs, tilecounts, nt, phi, lo, (uint32_t)nbt,
                     entries, counts, offsets, plo);
  return hipGetLastError();
}

// ----------------------------------------------------------------- helpers used by the API layer
hipError_t scalars_prepare(const uint32_t* d_in, uint32_t* d_out, size_t n, int mode, int log_perm, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scalars_prepare, dim3(blocks_for(n, 256)), dim3(256), 0, st, d_in, d_out, n, mode, log_perm);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_max_span(const uint32_t* counts, const uint32_t* offsets, size_t nbt,
                                                  uint32_t S, uint32_t* out) {
  uint32_t m = 0;
  for (size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x; b < nbt; b += (size_t)gridDim.x * blockDim.x) {
    const uint32_t cnt = counts[b];
    if (cnt) {
      const uint32_t off = offsets[b];
      m = max(m, (off + cnt - 1) / S - off / S);
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d));
  __shared__ uint32_t wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = max(max(wm[0], wm[1]), max(wm[2], wm[3]));  // every block writes
}

hipError_t max_span(const uint32_t* counts, const uint32_t* offsets, size_t nbt, uint32_t S, uint32_t* d_words,
                    uint32_t* h_words, hipStream_t st) {
  const unsigned g = max_span_blocks(nbt);
  hipLaunchKernelGGL(k_max_span, dim3(g), dim3(256), 0, st, counts, offsets, nbt, S, d_words);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && h_words) e = hipMemcpyAsync(h_words, d_words, g * 4, hipMemcpyDeviceToHost, st);
  return e;
}

hipError_t density_index(const uint64_t* d_words, size_t n, uint32_t base_offset, int32_t* d_idx, uint32_t* d_tmp,
                         uint32_t* d_scan_scratch, hipStream_t st) {
  const size_t nwords = (n + 63) / 64;
  if (nwords == 0) return hipSuccess;
  hipLaunchKernelGGL(k_density_popc, dim3(blocks_for(nwords, 256)), dim3(256), 0, st, d_words, nwords, d_tmp);
  exclusive_scan(d_tmp, d_tmp, nwords, d_scan_scratch, st);
  hipLaunchKernelGGL(k_density_index, dim3(blocks_for(n, 256)), dim3(256), 0, st, d_words, d_tmp, n, base_offset,
                     d_idx);
  return hipGetLastError();
}

}  // namespace bh
