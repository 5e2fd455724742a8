// Batch-affine bucket accumulation (msm.h: AffinePlan), group-generic; instantiated for G1 in
// msm_g1_aff.hip and for G2 in msm_g2_aff.hip.  It is the first part of the device replacement for
// the bucket loop of multiexp_inner (reference src/multiexp.rs:191-223:
// buckets[digit - 1].add_assign_mixed(base) for every (scalar, base) pair of a window).
//
// The sorted entries of one bucket are summed as a tree instead of a chain: level l adds entries
// (2j, 2j+1) of every bucket into record j of level l+1 (an odd last entry is carried over), so a
// level's additions are all independent.  In affine coordinates an addition needs
// lambda = (y1 - y0) / (x1 - x0); a thread takes K consecutive output records of a level, builds
// the prefix products of their denominators (one product each, kept in coalesced scratch planes
// in HBM), inverts the total once (safegcd.h) and walks back: 1/d_k = inv * prefix_(k-1),
// inv *= d_k.  Per addition that is 3 products for the shared inversion and 2M + 1S for the
// point: 6 field products against the XYZZ mixed addition's ~10 (8M + 2S, k_accumulate_pf),
// plus the inversion's share, ~30 000 / K instructions (G2: products in Fp2, one Fp inversion of
// the norm per thread).
//
// Exceptional pairs keep the group law exact, as in bls12_381's complete formulas: x0 = x1 with
// y0 = y1 doubles (lambda = 3 x0^2 / 2 y0, the denominator joins the batch like any other),
// y0 = -y1 gives the point at infinity (a record with AFF_IDENT set: carried, never inverted).
//
// Level 0 reads the window-table records through the sorted entries (base index | sign << 31),
// the others read the previous level's records in order.  Values stay below 2p between levels.
#pragma once
#include <algorithm>
#include <cstdlib>

#include "msm.h"
#include "safegcd.h"

namespace bh {
namespace aff {

using FC = FpCfg;

__device__ __forceinline__ DFp fp_inv_mont(const DFp& a) {
  const DFp c = fe_reduce_full<FC>(a);
  int32_t s[SG_NL];
  sg_from29(c.v, s);
  sg_inverse(s);
  DFp y, r3;
  sg_to29(s, y.v);
#pragma unroll
  for (int i = 0; i < FC::N; i++) r3.v[i] = FpInvCfg::R3[i];
  return fe_mul<FC>(y, r3);  // (aR)^-1 * R^3 * R^-1 = a^-1 R
}

__device__ __forceinline__ DFp fp_below2p(const DFp& x) { return fe_csub<FC, 2>(fe_csub<FC, 4>(x)); }  // < 6p -> < 2p

// ---- group adapters: coordinate type, its operations, and the record formats
// raw record (a level's): x then y as raw 29-bit limbs (G1: 14 + 14 words, G2: 28 + 28);
// table record: raw limbs as a level record, in a 32-word (G1) / 64-word (G2) line.  The
// point-at-infinity flag is word 13 (x's first coordinate's top limb) in both.
struct G1A {
  using T = DFp;
  static constexpr int NC = 14;               // words per coordinate (raw)
  static constexpr uint32_t REC = G1_AFF_REC;  // words per level record
  static constexpr int Q_RAW = 7, XQ_RAW = 4;  // 16-byte pieces: record, its x (+ 2 words)
  static constexpr int Q_PK = 7, XQ_PK = 4;    // table records (raw limbs too)
  static constexpr bool TABLE_PACKED = false;
  static BH_DEV T mul(const T& a, const T& b) { return fe_mul<FC>(a, b); }
  static BH_DEV T sqr(const T& a) { return fe_sqr<FC>(a); }
  static BH_DEV T add(const T& a, const T& b) { return fe_add<FC>(a, b); }
  template <uint32_t K> static BH_DEV T sub(const T& a, const T& b) { return fe_sub<FC, K>(a, b); }
  static BH_DEV bool is_zero(const T& a) { return fe_is_zero<FC>(a); }
  static BH_DEV T one() { return fe_one<FC>(); }
  static BH_DEV T neg(const T& a) { return fe_sub<FC, 1>(fe_zero<FC>(), a); }  // p - a, a canonical
  static BH_DEV T below2p(const T& a) { return fp_below2p(a); }
  static BH_DEV T inv(const T& a) { return fp_inv_mont(a); }
  static BH_DEV void coord(const uint32_t* w, bool packed, T& x) {  // (packed is never set for G1)
#pragma unroll
    for (int i = 0; i < NC; i++) x.v[i] = w[i];
  }
};

struct G2A {
  using T = DFp2;
  static constexpr int NC = 28;
  static constexpr uint32_t REC = G2_AFF_REC;
  static constexpr int Q_RAW = 14, XQ_RAW = 7;
  static constexpr int Q_PK = 14, XQ_PK = 7;  // table records (raw limbs too)
  static constexpr bool TABLE_PACKED = false;
  static BH_DEV T mul(const T& a, const T& b) { return Fp2Ops::mul(a, b); }
  static BH_DEV T sqr(const T& a) { return Fp2Ops::sqr(a); }
  static BH_DEV T add(const T& a, const T& b) { return Fp2Ops::add(a, b); }
  template <uint32_t K> static BH_DEV T sub(const T& a, const T& b) { return Fp2Ops::sub<K>(a, b); }
  static BH_DEV bool is_zero(const T& a) { return Fp2Ops::is_zero(a); }
  static BH_DEV T one() { return Fp2Ops::one(); }
  static BH_DEV T neg(const T& a) { return T{fe_sub<FC, 1>(fe_zero<FC>(), a.c0), fe_sub<FC, 1>(fe_zero<FC>(), a.c1)}; }
  static BH_DEV T below2p(const T& a) { return T{fp_below2p(a.c0), fp_below2p(a.c1)}; }
  // (a0 + a1 u)^-1 = (a0 - a1 u) / (a0^2 + a1^2): one Fp inversion of the norm
  static BH_DEV T inv(const T& a) {
    const DFp ni = fp_inv_mont(fe_add<FC>(fe_sqr<FC>(a.c0), fe_sqr<FC>(a.c1)));
    return T{fe_mul<FC>(a.c0, ni), fe_sub<FC, 2>(fe_zero<FC>(), fe_mul<FC>(a.c1, ni))};
  }
  static BH_DEV void coord(const uint32_t* w, bool packed, T& x) {
    if (packed) {
      x.c0 = fe_unpack<FC>(w);
      x.c1 = fe_unpack<FC>(w + 12);
    } else {
#pragma unroll
      for (int i = 0; i < 14; i++) {
        x.c0.v[i] = w[i];
        x.c1.v[i] = w[14 + i];
      }
    }
  }
};

template <class A>
BH_DEV uint32_t& word(typename A::T& x, int i) {
  return reinterpret_cast<uint32_t*>(&x)[i];
}

// slot classes, kept in bits 30-31 of the last word of the slot's prefix product (a top limb:
// < 2^5 for values below 2p)
enum : uint32_t { AC_COPY = 0, AC_ADD = 1, AC_DBL = 2, AC_IDENT = 3 };

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

// A thread's slots cover one contiguous range of the level's input: cursors walk it with the
// current bucket's bounds in registers (memory is read only when a bucket ends), so no slot waits
// on a chain of dependent loads.
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

// x of record e (PK: a packed table record), and its point-at-infinity flag
template <class A, bool PK>
__device__ __forceinline__ void load_x(const uint32_t* src, uint32_t rec, uint32_t e, typename A::T& x, bool& ident) {
  constexpr int XQ = PK ? A::XQ_PK : A::XQ_RAW;
  const uint4* q = reinterpret_cast<const uint4*>(src + (size_t)(e & 0x7fffffffu) * rec);
  uint32_t w[4 * XQ];
#pragma unroll
  for (int k = 0; k < XQ; k++) {
    const uint4 v = q[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
  ident = !PK && (w[13] & AFF_IDENT) != 0;
  A::coord(w, PK && A::TABLE_PACKED, x);
}

// x and y of record e (y negated for a negative entry)
template <class A, bool PK>
__device__ __forceinline__ void decode_xy(const uint32_t* w, uint32_t e, typename A::T& x, typename A::T& y) {
  constexpr int YOFF = PK ? A::XQ_PK * 4 : A::NC;  // (table record: x's pieces)
  A::coord(w, PK && A::TABLE_PACKED, x);
  A::coord(w + YOFF, PK && A::TABLE_PACKED, y);
  if (e >> 31) y = A::neg(y);  // p - y, in (0, p]
}

template <class A, bool PK>
__device__ __forceinline__ void load_xy(const uint32_t* src, uint32_t rec, uint32_t e, typename A::T& x,
                                        typename A::T& y) {
  constexpr int Q = PK ? A::Q_PK : A::Q_RAW;
  const uint4* q = reinterpret_cast<const uint4*>(src + (size_t)(e & 0x7fffffffu) * rec);
  uint32_t w[4 * Q];
#pragma unroll
  for (int k = 0; k < Q; k++) {
    const uint4 v = q[k];
    w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
  }
  decode_xy<A, PK>(w, e, x, y);
}

template <class A>
__device__ __forceinline__ void store_rec(uint32_t* dst, const typename A::T& x, const typename A::T& y, bool ident) {
  uint32_t w[2 * A::NC];
  const uint32_t* xs = reinterpret_cast<const uint32_t*>(&x);
  const uint32_t* ys = reinterpret_cast<const uint32_t*>(&y);
#pragma unroll
  for (int i = 0; i < A::NC; i++) {
    w[i] = ident ? 0u : xs[i];
    w[A::NC + i] = ident ? 0u : ys[i];
  }
  if (ident) w[13] = AFF_IDENT;
  uint4* q = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < A::Q_RAW; k++) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// A level runs as two kernels over the same thread -> slot map.  Thread t owns output records
// [t*K, t*K + K) of the level (bucket b's records at out_off[b] .. out_off[b+1]); record j of
// bucket b is the sum of input records in_off[b] + 2j and + 2j + 1 (when present).
//  * k_aff_fwd (few registers): classifies each slot, stores the prefix products of the
//    denominators (scratch planes, word (k*NC + w)*T + t, the slot class in the top bits) and the
//    thread's total (prod planes, word w*T + t); entries two slots ahead and the x coordinates one
//    slot ahead are in flight during the current slot's product.
//  * k_aff_bwd: inverts the total, then walks the slots backwards with the previous slot's two
//    records prefetched global -> LDS (global_load_lds, no VGPR cost) and its entries one further
//    slot ahead, during the current slot's arithmetic (as k_accumulate_pf does).
template <class A, bool PK>
__device__ __forceinline__ void aff_fwd(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                        const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt, uint32_t K,
                                        uint32_t* pre, uint32_t* prod) {
  using T = typename A::T;
  constexpr int NC = A::NC;
  const uint32_t TT = gridDim.x * blockDim.x;
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
  T cx0, cx1;
  bool cid0, cid1;
  load_x<A, PK>(src, rec, se.e0, cx0, cid0);
  load_x<A, PK>(src, rec, se.e1, cx1, cid1);
  T acc = A::one();
  for (uint32_t o = o0; o < o1; o++) {
    // classify slot o and store its prefix first, then put slot o+1's loads in flight: a load
    // issued before a store cannot be waited for without waiting for the store too (the
    // compiler's vmcnt treats pending loads and stores as completing out of order)
    uint32_t cls = AC_COPY;
    T d;
    if (se.has1 && !cid0 && !cid1) {
      d = A::template sub<2>(cx1, cx0);  // < 4p
      cls = AC_ADD;
      if (A::is_zero(d)) {  // rare: P0 = +-P1
        T x0, y0, x1, y1;
        load_xy<A, PK>(src, rec, se.e0, x0, y0);
        load_xy<A, PK>(src, rec, se.e1, x1, y1);
        if (A::is_zero(A::template sub<2>(y1, y0))) {
          cls = AC_DBL;
          d = A::add(y0, y0);  // 2 y0 < 4p, never 0 (no point of order 2)
        } else {
          cls = AC_IDENT;
        }
      }
    }
    {
      uint32_t* pk = pre + (size_t)(o - o0) * NC * TT + t;
      const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
#pragma unroll
      for (int l = 0; l < NC; l++) pk[(size_t)l * TT] = l == NC - 1 ? (aw[l] | (cls << 30)) : aw[l];
    }
    T nx0, nx1;
    bool nid0 = false, nid1 = false;
    SlotE snn = sn;
    if (o + 1 < o1) {  // slot o+1's x, slot o+2's entries
      load_x<A, PK>(src, rec, sn.e0, nx0, nid0);
      load_x<A, PK>(src, rec, sn.e1, nx1, nid1);
      if (o + 2 < o1) {
        snn = slot_entries(entries, cur.i, cur.has1());
        if (o + 3 < o1) cur.next(in_off);
      }
    }
    if (cls == AC_ADD || cls == AC_DBL) acc = A::mul(acc, d);
    se = sn;
    sn = snn;
    cx0 = nx0;
    cx1 = nx1;
    cid0 = nid0;
    cid1 = nid1;
  }
  const uint32_t* aw = reinterpret_cast<const uint32_t*>(&acc);
#pragma unroll
  for (int l = 0; l < NC; l++) prod[(size_t)l * TT + t] = aw[l];
}

template <class A, bool PK>
__device__ __forceinline__ void aff_bwd(const uint32_t* entries, const uint32_t* src, uint32_t rec,
                                        const uint32_t* in_off, const uint32_t* out_off, uint32_t nbt, uint32_t K,
                                        const uint32_t* pre, const uint32_t* prod, uint32_t* dst, uint4* lds_all) {
  using T = typename A::T;
  constexpr int NC = A::NC;
  constexpr int Q = PK ? A::Q_PK : A::Q_RAW;  // pieces per input record
  const uint32_t TT = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t Eo = out_off[nbt];
  const uint32_t o0 = t * K;
  if (o0 >= Eo) return;
  const uint32_t o1 = min(o0 + K, Eo);
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint4* lds = lds_all + (size_t)wv * 2 * Q * 64;  // this wave's: record 0 in pieces [0, Q), record 1 in [Q, 2Q)
  auto issue = [&](const SlotE& s) {
    const uint32_t* p0 = src + (size_t)(s.e0 & 0x7fffffffu) * rec;
    const uint32_t* p1 = src + (size_t)(s.e1 & 0x7fffffffu) * rec;
#pragma unroll
    for (int q = 0; q < Q; q++)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p0 + 4 * q),
                                       (__attribute__((address_space(3))) void*)&lds[q * 64], 16, 0, 0);
    if (s.has1) {
#pragma unroll
      for (int q = 0; q < Q; q++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p1 + 4 * q),
                                         (__attribute__((address_space(3))) void*)&lds[(Q + q) * 64], 16, 0, 0);
    }
  };
  auto load_pre = [&](uint32_t o, T& pf) {
    const uint32_t* pk = pre + (size_t)(o - o0) * NC * TT + t;
    uint32_t* pw = reinterpret_cast<uint32_t*>(&pf);
#pragma unroll
    for (int l = 0; l < NC; l++) pw[l] = pk[(size_t)l * TT];
  };
  T inv;
  {
    uint32_t* iw = reinterpret_cast<uint32_t*>(&inv);
#pragma unroll
    for (int l = 0; l < NC; l++) iw[l] = prod[(size_t)l * TT + t];
  }
  inv = A::inv(inv);
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
  T pfn;
  load_pre(o, pfn);
  T pxo, pyo;  // the previous slot's result, stored one slot late
  bool pido = false;
  for (;;) {
    __builtin_amdgcn_s_waitcnt(0x3f70);  // vmcnt(0): slot o's records are in LDS, its prefix in pfn
    uint32_t w0[4 * Q], w1[4 * Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
      const uint4 v0 = lds[q * 64 + lane], v1 = lds[(Q + q) * 64 + lane];
      w0[4 * q] = v0.x; w0[4 * q + 1] = v0.y; w0[4 * q + 2] = v0.z; w0[4 * q + 3] = v0.w;
      w1[4 * q] = v1.x; w1[4 * q + 1] = v1.y; w1[4 * q + 2] = v1.z; w1[4 * q + 3] = v1.w;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): read before the slots are refilled
    const SlotE cs = se;
    T pf = pfn;
    if (o > o0) {  // slot o-1's records and prefix, slot o-2's entries: in flight during slot o
      issue(sp);
      load_pre(o - 1, pfn);
      se = sp;
      if (o - 1 > o0) {
        sp = slot_entries(entries, cur.i, cur.has1());
        if (o - 2 > o0) cur.prev(in_off);
      }
    }
    // slot o+1's result, stored only now: the vmcnt(0) at the next slot's top then finds these
    // stores done (issued before slot o's arithmetic) instead of waiting for them
    if (o + 1 < o1) store_rec<A>(dst + (size_t)(o + 1) * A::REC, pxo, pyo, pido);
    const uint32_t cls = word<A>(pf, NC - 1) >> 30;
    word<A>(pf, NC - 1) &= FC::MASK;
    T x0, y0, x1, y1;
    decode_xy<A, PK>(w0, cs.e0, x0, y0);
    decode_xy<A, PK>(w1, cs.has1 ? cs.e1 : 0u, x1, y1);
    const bool id0 = !PK && (w0[13] & AFF_IDENT) != 0;
    const bool id1 = !cs.has1 || (!PK && (w1[13] & AFF_IDENT) != 0);
    T xo, yo;
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
      const T d = dbl ? A::add(y0, y0) : A::template sub<2>(x1, x0);
      const T dinv = A::mul(inv, pf);
      inv = A::mul(inv, d);
      T num;
      if (dbl) {
        const T xx = A::sqr(x0);
        num = A::add(A::add(xx, xx), xx);  // 3 x0^2 < 6p
      } else {
        num = A::template sub<2>(y1, y0);  // < 4p
      }
      const T lam = A::mul(num, dinv);  // < 2p
      const T sx = dbl ? A::add(x0, x0) : A::add(x0, x1);  // < 4p
      xo = A::below2p(A::template sub<4>(A::sqr(lam), sx));
      yo = A::below2p(A::template sub<2>(A::mul(lam, A::template sub<2>(x0, xo)), y0));
    }
    pxo = xo;
    pyo = yo;
    pido = ido;
    if (o == o0) break;
    o--;
  }
  store_rec<A>(dst + (size_t)o0 * A::REC, pxo, pyo, pido);
}

// per-level record counts ceil(count / 2^l) (l = 1..L; word nbt of each = 0 for the scan) and the
// last level's counts
static __global__ void __launch_bounds__(256) k_aff_counts(const uint32_t* counts, uint32_t nbt, int L, uint32_t* lv,
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

inline int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

using FwdK = void (*)(const uint32_t*, const uint32_t*, uint32_t, const uint32_t*, const uint32_t*, uint32_t, uint32_t,
                     uint32_t*, uint32_t*);
using BwdK = void (*)(const uint32_t*, const uint32_t*, uint32_t, const uint32_t*, const uint32_t*, uint32_t, uint32_t,
                      const uint32_t*, const uint32_t*, uint32_t*);

// Enqueue the levels of `pl` on st (caller holds ws.aff->mu): per-level offsets from the sort's
// counts, then level 0 (F0/B0: table records through the sorted entries) and the others (F1/B1:
// the previous level's records in order); the last level's max-span words for the tail.
template <class A, class WS>
hipError_t levels_run(WS& ws, hipStream_t st, const uint32_t* d_bases, uint32_t rec, const AffinePlan& pl, size_t nbt,
                      FwdK F0, BwdK B0, FwdK F1, BwdK B1, const uint32_t** final_pts) {
  *final_pts = nullptr;
  if (pl.levels == 0) return hipSuccess;
  hipError_t e;
  if ((e = affine_reserve(ws, nbt)) != hipSuccess) return e;
  size_t pre_words = 0;
  for (int l = 0; l < pl.levels; l++)
    pre_words = std::max(pre_words, (size_t)(pl.K[l] + 1) * A::NC * (size_t)pl.blocks[l] * 256);  // + the totals
  const size_t rb = (size_t)A::REC * 4;
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
    uint32_t* prod = pre + (size_t)pl.K[l] * A::NC * pl.blocks[l] * 256;
    hipLaunchKernelGGL(l ? F1 : F0, dim3(pl.blocks[l]), dim3(256), 0, st, ent, src, r, in_off, out_off, (uint32_t)nbt,
                       pl.K[l], pre, prod);
    hipLaunchKernelGGL(l ? B1 : B0, dim3(pl.blocks[l]), dim3(256), 0, st, ent, src, r, in_off, out_off, (uint32_t)nbt,
                       pl.K[l], (const uint32_t*)pre, (const uint32_t*)prod, dst);
    src = dst;
    ent = nullptr;
    in_off = out_off;
    r = A::REC;
  }
  *final_pts = src;
  // the last level's longest bucket span (segments of pl.S), read by the reduction tail
  if ((e = max_span(ws.acnt, ws.aoff + (size_t)(pl.levels - 1) * (nbt + 1), nbt, (uint32_t)pl.S, ws.aspan, nullptr,
                    st)) != hipSuccess)
    return e;
  return hipGetLastError();
}

// occupancy x CUs of a level kernel
inline size_t resident_of(const void* k) {
  int dev = 0, cus = 256, blocks = 1;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k, 256, 0) != hipSuccess || blocks < 1) blocks = 1;
  return (size_t)cus * (size_t)blocks * 256;
}

}  // namespace aff

// Plan of the levels for a group whose level kernel keeps `resident` threads on the device.
// BH_AFFINE=0 turns the levels off (A/B; BH_AFFINE_G1 / BH_AFFINE_G2 for one group);
// BH_AFF_ROUNDS (2): resident rounds of threads per level; BH_AFF_KMIN (16): the smallest K a level
// is run with; BH_AFF_LEVELS: at most this many; BH_AFF_MIN_E (2^18): fewer entries take the XYZZ
// accumulation alone.  Read on every call (tests set them around one multiexp); an accumulation
// and its reduction are enqueued under one setting.
AffinePlan affine_plan(size_t Emax, size_t nbt, int halves, size_t resident, bool g2);

}  // namespace bh
