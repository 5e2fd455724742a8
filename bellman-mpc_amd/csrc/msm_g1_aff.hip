// Batch-affine bucket accumulation for G1 (msm.h: AffinePlan) -- the first part of the device
// replacement for the bucket loop of multiexp_inner (reference src/multiexp.rs:191-223:
// buckets[digit - 1].add_assign_mixed(base) for every (scalar, base) pair of a window).
//
// The sorted entries of one bucket are summed as a tree instead of a chain: level l adds entries
// (2j, 2j+1) of every bucket into record j of level l+1 (an odd last entry is carried over), so a
// level's additions are all independent.  In affine coordinates an addition needs
// lambda = (y1 - y0) / (x1 - x0); a thread takes K consecutive output records of a level, builds
// the prefix products of their denominators (one product each, kept in a coalesced scratch column
// in HBM), inverts the total once (safegcd.h) and walks back: 1/d_k = inv * prefix_(k-1),
// inv *= d_k.  Per addition that is 3 products for the shared inversion and 2M + 1S for the
// point: 6 field products against the XYZZ mixed addition's 10 (8M + 2S, k_accumulate_pf),
// plus the inversion's share, ~20 000 / K instructions.
//
// Exceptional pairs keep the group law exact, as in bls12_381's complete formulas: x0 = x1 with
// y0 = y1 doubles (lambda = 3 x0^2 / 2 y0, the denominator joins the batch like any other),
// y0 = -y1 gives the point at infinity (a record with AFF_IDENT set: carried, never inverted).
//
// Level 0 reads the window-table records through the sorted entries (base index | sign << 31),
// the others read the previous level's records in order.  Values stay below 2p between levels.
#include "msm.h"
#include "safegcd.h"

#include <algorithm>
#include <cstdlib>

namespace bh {

namespace {

using F = FpCfg;
constexpr int NW = F::N;  // 14 limbs per coordinate

// slot classes, kept in bits 30-31 of the top limb word of the slot's prefix product (< 2^5 for
// values below 2p)
enum : uint32_t { AC_COPY = 0, AC_ADD = 1, AC_DBL = 2, AC_IDENT = 3 };

__device__ __forceinline__ DFp fp_inv_mont(const DFp& a) {
  const DFp c = fe_reduce_full<F>(a);
  int32_t s[SG_NL];
  sg_from29(c.v, s);
  sg_inverse(s);
  DFp y, r3;
  sg_to29(s, y.v);
#pragma unroll
  for (int i = 0; i < NW; i++) r3.v[i] = FpInvCfg::R3[i];
  return fe_mul<F>(y, r3);  // (aR)^-1 * R^3 * R^-1 = a^-1 R
}

struct RecRef {
  const uint32_t* p;
  bool neg;
};

__device__ __forceinline__ RecRef rec_at(const uint32_t* entries, const uint32_t* src, uint32_t rec, uint32_t i) {
  if (entries) {
    const uint32_t e = entries[i];
    return RecRef{src + (size_t)(e & 0x7fffffffu) * rec, (e >> 31) != 0};
  }
  return RecRef{src + (size_t)i * rec, false};
}

// x: words 0..13 (16 loaded); identity flag in word 13
__device__ __forceinline__ void load_x(const RecRef& r, DFp& x, bool& ident) {
  const uint4* q = reinterpret_cast<const uint4*>(r.p);
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4 v = q[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
  ident = (w[13] & AFF_IDENT) != 0;
#pragma unroll
  for (int i = 0; i < NW; i++) x.v[i] = w[i];
}

__device__ __forceinline__ void load_xy(const RecRef& r, DFp& x, DFp& y, bool& ident) {
  const uint4* q = reinterpret_cast<const uint4*>(r.p);
  uint32_t w[28];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint4 v = q[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
  ident = (w[13] & AFF_IDENT) != 0;
#pragma unroll
  for (int i = 0; i < NW; i++) {
    x.v[i] = w[i];
    y.v[i] = w[NW + i];
  }
  if (r.neg) y = fe_sub<F, 1>(fe_zero<F>(), y);  // p - y, in (0, p]
}

__device__ __forceinline__ void store_rec(uint32_t* dst, const DFp& x, const DFp& y, bool ident) {
  uint32_t w[28];
#pragma unroll
  for (int i = 0; i < NW; i++) {
    w[i] = ident ? 0u : x.v[i];
    w[NW + i] = ident ? 0u : y.v[i];
  }
  if (ident) w[13] = AFF_IDENT;
  uint4* q = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < 7; k++) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// largest b in [0, nb) with offsets[b] <= pos (offsets[nb] > pos)
__device__ __forceinline__ uint32_t find_bucket_aff(const uint32_t* offsets, uint32_t nb, uint32_t pos) {
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] <= pos) lo = mid;
    else hi = mid;
  }
  return lo;
}

// x < 6p -> < 2p
__device__ __forceinline__ DFp below2p(const DFp& x) { return fe_csub<F, 2>(fe_csub<F, 4>(x)); }

// A level runs as two kernels over the same thread -> slot map.  Thread t owns output records
// [t*K, t*K + K) of the level (bucket b's records at out_off[b] .. out_off[b+1]); record j of
// bucket b is the sum of input records in_off[b] + 2j and + 2j + 1 (when present).  A thread's
// slots therefore cover one contiguous range of the level's input: cursors walk it with the
// current bucket's bounds in registers (memory is read only when a bucket ends), so no slot
// waits on a chain of dependent loads.
//  * k_aff_fwd (few registers, four waves per SIMD): classifies each slot, stores the prefix
//    products of the denominators (scratch planes, word (k*14 + limb)*T + t, the slot class in the
//    top bits) and the thread's total (prod planes, word limb*T + t); entries two slots ahead and
//    the x coordinates one slot ahead are in flight during the current slot's product.
//  * k_aff_bwd: inverts the total, then walks the slots backwards with the previous slot's two
//    records prefetched global -> LDS (global_load_lds, no VGPR cost) and its entries one further
//    slot ahead, during the current slot's ~3 000 instructions (as k_accumulate_pf does).

// forward cursor: i = the current slot's first input, iend = its bucket's end
struct FCur {
  uint32_t b, i, iend;
  __device__ __forceinline__ void init(uint32_t o, const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt) {
    b = find_bucket_aff(out_off, nbt, o);
    i = in_off[b] + 2 * (o - out_off[b]);
    iend = in_off[b + 1];
  }
  __device__ __forceinline__ bool has1() const { return i + 1 < iend; }
  __device__ __forceinline__ void next(const uint32_t* in_off) {  // (only while a next slot exists)
    i += has1() ? 2u : 1u;
    while (i == iend) iend = in_off[++b + 1];  // the next non-empty bucket starts at i
  }
};

// backward cursor: i = the current slot's first input, ibeg / iend = its bucket's bounds
struct BCur {
  uint32_t b, i, ibeg, iend;
  __device__ __forceinline__ void init(uint32_t o, const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt) {
    b = find_bucket_aff(out_off, nbt, o);
    ibeg = in_off[b];
    iend = in_off[b + 1];
    i = ibeg + 2 * (o - out_off[b]);
  }
  __device__ __forceinline__ bool has1() const { return i + 1 < iend; }
  __device__ __forceinline__ void prev(const uint32_t* in_off) {  // (only while a previous slot exists)
    if (i > ibeg) {
      i -= 2;
      return;
    }
    iend = ibeg;
    do ibeg = in_off[--b]; while (ibeg == iend);  // the previous non-empty bucket ends at iend
    i = ibeg + 2 * ((iend - ibeg - 1) / 2);        // its last slot (a lone record when odd)
  }
};

// the entries of a slot (level 0) or its record indices (entries == null)
struct SlotE {
  uint32_t e0, e1;
  bool has1;
};
__device__ __forceinline__ SlotE slot_entries(const uint32_t* entries, uint32_t i, bool has1) {
  SlotE s;
  s.has1 = has1;
  if (entries) {
    s.e0 = entries[i];
    s.e1 = has1 ? entries[i + 1] : s.e0;
  } else {
    s.e0 = i;
    s.e1 = has1 ? i + 1 : i;
  }
  return s;
}
__device__ __forceinline__ RecRef rec_of(const uint32_t* src, uint32_t rec, uint32_t e) {
  return RecRef{src + (size_t)(e & 0x7fffffffu) * rec, (e >> 31) != 0};
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_aff_fwd(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                                 const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt,
                                                 uint32_t K, uint32_t* pre, uint32_t* prod) {
  const uint32_t T = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t Eo = out_off[nbt];
  const uint32_t o0 = t * K;
  if (o0 >= Eo) return;
  const uint32_t o1 = min(o0 + K, Eo);
  FCur cur;
  cur.init(o0, in_off, out_off, nbt);
  // pipeline: slot o's x in registers, slot o+1's entries, the cursor at slot o+2
  SlotE se = slot_entries(entries, cur.i, cur.has1());
  if (o0 + 1 < o1) cur.next(in_off);
  SlotE sn = se;
  if (o0 + 1 < o1) sn = slot_entries(entries, cur.i, cur.has1());
  if (o0 + 2 < o1) cur.next(in_off);
  DFp cx0, cx1;
  bool cid0, cid1;
  load_x(rec_of(src, rec, se.e0), cx0, cid0);
  load_x(rec_of(src, rec, se.e1), cx1, cid1);
  DFp acc = fe_one<F>();
  for (uint32_t o = o0; o < o1; o++) {
    DFp nx0, nx1;
    bool nid0 = false, nid1 = false;
    SlotE snn = sn;
    if (o + 1 < o1) {  // slot o+1's x, slot o+2's entries
      load_x(rec_of(src, rec, sn.e0), nx0, nid0);
      load_x(rec_of(src, rec, sn.e1), nx1, nid1);
      if (o + 2 < o1) {
        snn = slot_entries(entries, cur.i, cur.has1());
        if (o + 3 < o1) cur.next(in_off);
      }
    }
    uint32_t cls = AC_COPY;
    DFp d;
    if (se.has1 && !cid0 && !cid1) {
      d = fe_sub<F, 2>(cx1, cx0);  // < 4p
      cls = AC_ADD;
      if (fe_is_zero<F>(d)) {  // rare: P0 = +-P1
        DFp x0, y0, x1, y1;
        bool i0_, i1_;
        load_xy(rec_of(src, rec, se.e0), x0, y0, i0_);
        load_xy(rec_of(src, rec, se.e1), x1, y1, i1_);
        if (fe_is_zero<F>(fe_sub<F, 2>(y1, y0))) {
          cls = AC_DBL;
          d = fe_add<F>(y0, y0);  // 2 y0 < 4p, never 0 (no point of order 2)
        } else {
          cls = AC_IDENT;
        }
      }
    }
    const uint32_t k = o - o0;
    uint32_t* pk = pre + (size_t)k * NW * T + t;
#pragma unroll
    for (int l = 0; l < NW; l++) pk[(size_t)l * T] = l == NW - 1 ? (acc.v[l] | (cls << 30)) : acc.v[l];
    if (cls == AC_ADD || cls == AC_DBL) acc = fe_mul<F>(acc, d);
    se = sn;
    sn = snn;
    cx0 = nx0;
    cx1 = nx1;
    cid0 = nid0;
    cid1 = nid1;
  }
#pragma unroll
  for (int l = 0; l < NW; l++) prod[(size_t)l * T + t] = acc.v[l];
}

__global__ void __launch_bounds__(256) k_aff_bwd(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                                 const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt,
                                                 uint32_t K, const uint32_t* pre, const uint32_t* prod,
                                                 uint32_t* dst) {
  __shared__ uint4 lds[4][14][64];  // per wave: record 0 in pieces 0..6, record 1 in 7..13
  const uint32_t T = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t Eo = out_off[nbt];
  const uint32_t o0 = t * K;
  if (o0 >= Eo) return;
  const uint32_t o1 = min(o0 + K, Eo);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto issue = [&](const SlotE& s) {
    const uint32_t* p0 = src + (size_t)(s.e0 & 0x7fffffffu) * rec;
    const uint32_t* p1 = src + (size_t)(s.e1 & 0x7fffffffu) * rec;
#pragma unroll
    for (int q = 0; q < 7; q++)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p0 + 4 * q),
                                       (__attribute__((address_space(3))) void*)&lds[wv][q][0], 16, 0, 0);
    if (s.has1) {
#pragma unroll
      for (int q = 0; q < 7; q++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p1 + 4 * q),
                                         (__attribute__((address_space(3))) void*)&lds[wv][7 + q][0], 16, 0, 0);
    }
  };
  auto load_pre = [&](uint32_t o, DFp& pf) {
    const uint32_t* pk = pre + (size_t)(o - o0) * NW * T + t;
#pragma unroll
    for (int l = 0; l < NW; l++) pf.v[l] = pk[(size_t)l * T];
  };
  DFp inv;
#pragma unroll
  for (int l = 0; l < NW; l++) inv.v[l] = prod[(size_t)l * T + t];
  inv = fp_inv_mont(inv);
  // pipeline: slot o's records in LDS and its prefix in pfn, slot o-1's entries, cursor at o-2
  BCur cur;
  uint32_t o = o1 - 1;
  cur.init(o, in_off, out_off, nbt);
  SlotE se = slot_entries(entries, cur.i, cur.has1());
  SlotE sp = se;
  if (o > o0) {
    cur.prev(in_off);
    sp = slot_entries(entries, cur.i, cur.has1());
    if (o - 1 > o0) cur.prev(in_off);
  }
  issue(se);
  DFp pfn;
  load_pre(o, pfn);
  for (;;) {
    __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0): slot o's records are in LDS, its prefix in pfn
    uint32_t w0[28], w1[28];
#pragma unroll
    for (int q = 0; q < 7; q++) {
      const uint4 v0 = lds[wv][q][lane], v1 = lds[wv][7 + q][lane];
      w0[4 * q] = v0.x; w0[4 * q + 1] = v0.y; w0[4 * q + 2] = v0.z; w0[4 * q + 3] = v0.w;
      w1[4 * q] = v1.x; w1[4 * q + 1] = v1.y; w1[4 * q + 2] = v1.z; w1[4 * q + 3] = v1.w;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): read before the slots are refilled
    const SlotE cs = se;
    DFp pf = pfn;
    if (o > o0) {  // slot o-1's records and prefix, slot o-2's entries: in flight during slot o
      issue(sp);
      load_pre(o - 1, pfn);
      se = sp;
      if (o - 1 > o0) {
        sp = slot_entries(entries, cur.i, cur.has1());
        if (o - 2 > o0) cur.prev(in_off);
      }
    }
    const uint32_t cls = pf.v[NW - 1] >> 30;
    pf.v[NW - 1] &= F::MASK;
    DFp x0, y0, x1, y1;
#pragma unroll
    for (int i = 0; i < NW; i++) {
      x0.v[i] = w0[i];
      y0.v[i] = w0[NW + i];
      x1.v[i] = w1[i];
      y1.v[i] = w1[NW + i];
    }
    const bool id0 = (w0[NW - 1] & AFF_IDENT) != 0;
    const bool id1 = !cs.has1 || (w1[NW - 1] & AFF_IDENT) != 0;
    if (cs.e0 >> 31) y0 = fe_sub<F, 1>(fe_zero<F>(), y0);  // p - y, in (0, p]
    if (cs.has1 && (cs.e1 >> 31)) y1 = fe_sub<F, 1>(fe_zero<F>(), y1);
    DFp xo, yo;
    bool ido = false;
    if (cls == AC_COPY) {
      // a lone record, or a pair with the point at infinity in it: the other one (or infinity)
      const bool take1 = cs.has1 && id0;
      xo = take1 ? x1 : x0;
      yo = take1 ? y1 : y0;
      ido = take1 ? id1 : id0;
    } else if (cls == AC_IDENT) {
      ido = true;
    } else {
      const bool dbl = cls == AC_DBL;
      const DFp d = dbl ? fe_add<F>(y0, y0) : fe_sub<F, 2>(x1, x0);
      const DFp dinv = fe_mul<F>(inv, pf);
      inv = fe_mul<F>(inv, d);
      DFp num;
      if (dbl) {
        const DFp xx = fe_sqr<F>(x0);
        num = fe_add<F>(fe_add<F>(xx, xx), xx);  // 3 x0^2 < 6p
      } else {
        num = fe_sub<F, 2>(y1, y0);  // < 4p
      }
      const DFp lam = fe_mul<F>(num, dinv);  // < 2p
      const DFp sx = dbl ? fe_add<F>(x0, x0) : fe_add<F>(x0, x1);  // < 4p
      xo = below2p(fe_sub<F, 4>(fe_sqr<F>(lam), sx));
      yo = below2p(fe_sub<F, 2>(fe_mul<F>(lam, fe_sub<F, 2>(x0, xo)), y0));
    }
    store_rec(dst + (size_t)o * G1_AFF_REC, xo, yo, ido);
    if (o == o0) break;
    o--;
  }
}

// per-level record counts ceil(count / 2^l) (l = 1..L; word nbt of each = 0 for the scan) and the
// last level's counts
__global__ void __launch_bounds__(256) k_aff_counts(const uint32_t* counts, uint32_t nbt, int L, uint32_t* lv,
                                                    uint32_t* last) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nbt) return;
  const uint32_t c = b < nbt ? counts[b] : 0u;
  for (int l = 1; l <= L; l++) {
    const uint32_t v = (uint32_t)(((uint64_t)c + (1ull << l) - 1) >> l);
    lv[(size_t)(l - 1) * (nbt + 1) + b] = v;
    if (l == L) last[b] = v;
  }
}

// resident threads of the level kernel on this device (occupancy x CUs)
size_t affine_resident() {
  static const size_t v = [] {
    int dev = 0, cus = 256, blocks = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, (const void*)k_aff_bwd, 256, 0) != hipSuccess ||
        blocks < 1)
      blocks = 1;
    return (size_t)cus * (size_t)blocks * 256;
  }();
  return v;
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
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

// BH_AFFINE=0 turns the levels off (A/B); BH_AFF_ROUNDS (2): resident rounds of threads per
// level; BH_AFF_KMIN (16): the smallest K a level is run with; BH_AFF_LEVELS: at most this many;
// BH_AFF_MIN_E (2^18): fewer entries take the XYZZ accumulation alone.  Read on every call (tests
// set them around one multiexp); the accumulation and its reduction are enqueued under one setting.
AffinePlan affine_plan_g1(size_t Emax, size_t nbt, int halves) {
  AffinePlan pl;
  const bool on = env_int("BH_AFFINE", 0) != 0;
  const int rounds = std::max(1, env_int("BH_AFF_ROUNDS", 2));
  const int kmin = std::max(1, env_int("BH_AFF_KMIN", 16));
  const int lmax = std::min(AFF_LMAX, std::max(0, env_int("BH_AFF_LEVELS", AFF_LMAX)));
  const size_t min_e = (size_t)std::max(1, env_int("BH_AFF_MIN_E", 1 << 18));
  pl.Eb[0] = Emax;
  if (!on || halves || Emax < min_e) return pl;
  const size_t T = (size_t)rounds * affine_resident();
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

hipError_t affine_reserve_g1(MsmWorkspace<G1Ops>& ws, size_t nbt) {
  if (nbt <= ws.cap_anbt && ws.aoff) return hipSuccess;
  for (uint32_t** p : {&ws.aoff, &ws.acnt, &ws.ascan, &ws.aspan}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  ws.cap_anbt = 0;
  hipError_t e;
  if ((e = hipMalloc(&ws.aoff, (size_t)AFF_LMAX * (nbt + 1) * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&ws.acnt, (nbt + 1) * 4)) != hipSuccess) return e;
  if ((e = hipMalloc(&ws.ascan, scan_scratch_words(nbt + 1) * 4 + 64)) != hipSuccess) return e;
  if ((e = hipMalloc(&ws.aspan, MAX_SPAN_BLOCKS * 4)) != hipSuccess) return e;
  ws.cap_anbt = nbt;
  return hipSuccess;
}

hipError_t affine_levels_g1(MsmWorkspace<G1Ops>& ws, hipStream_t st, const uint32_t* d_bases, uint32_t rec,
                            const AffinePlan& pl, size_t nbt, const uint32_t** final_pts) {
  *final_pts = nullptr;
  if (pl.levels == 0) return hipSuccess;
  hipError_t e;
  if ((e = affine_reserve_g1(ws, nbt)) != hipSuccess) return e;
  size_t pre_words = 0;
  for (int l = 0; l < pl.levels; l++)
    pre_words = std::max(pre_words, (size_t)(pl.K[l] + 1) * NW * (size_t)pl.blocks[l] * 256);  // + the totals
  const size_t rb = (size_t)G1_AFF_REC * 4;
  if ((e = ws.aff->reserve(pl.Eb[1] * rb, pl.levels > 1 ? pl.Eb[2] * rb : 16, pre_words * 4)) != hipSuccess) return e;
  const unsigned cb = (unsigned)((nbt + 1 + 255) / 256);
  hipLaunchKernelGGL(k_aff_counts, dim3(cb), dim3(256), 0, st, ws.counts, (uint32_t)nbt, pl.levels, ws.aoff, ws.acnt);
  for (int l = 0; l < pl.levels; l++) {
    uint32_t* off = ws.aoff + (size_t)l * (nbt + 1);
    exclusive_scan(off, off, nbt + 1, ws.ascan, st);
  }
  const uint32_t* src = d_bases;
  const uint32_t* ent = ws.entries;
  const uint32_t* in_off = ws.offsets;
  uint32_t r = rec;
  for (int l = 0; l < pl.levels; l++) {
    uint32_t* dst = reinterpret_cast<uint32_t*>(ws.aff->pts[l & 1]);
    const uint32_t* out_off = ws.aoff + (size_t)l * (nbt + 1);
    uint32_t* pre = reinterpret_cast<uint32_t*>(ws.aff->pre);
    uint32_t* prod = pre + (size_t)pl.K[l] * NW * pl.blocks[l] * 256;
    hipLaunchKernelGGL(k_aff_fwd, dim3(pl.blocks[l]), dim3(256), 0, st, ent, src, r, in_off, out_off, (uint32_t)nbt,
                       pl.K[l], pre, prod);
    hipLaunchKernelGGL(k_aff_bwd, dim3(pl.blocks[l]), dim3(256), 0, st, ent, src, r, in_off, out_off, (uint32_t)nbt,
                       pl.K[l], (const uint32_t*)pre, (const uint32_t*)prod, dst);
    src = dst;
    ent = nullptr;
    in_off = out_off;
    r = G1_AFF_REC;
  }
  *final_pts = src;
  // the last level's longest bucket span (segments of pl.S), read by the reduction tail
  if ((e = max_span(ws.acnt, ws.aoff + (size_t)(pl.levels - 1) * (nbt + 1), nbt, (uint32_t)pl.S, ws.aspan, nullptr,
                    st)) != hipSuccess)
    return e;
  return hipGetLastError();
}

}  // namespace bh
