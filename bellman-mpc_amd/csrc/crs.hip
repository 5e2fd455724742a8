// Device fixed-base scalar multiplication for CRS generation -- the GPU
// counterpart of the wNAF `g1_wnaf.scalar(..)` / `g2_wnaf.scalar(..)` calls of
// the classic generator (reference groth16/generator.rs:310-572) followed by
// batch_normalize.  Not on the proving hot path: it builds the Parameters the
// benchmark circuits need, since the fork's own generator only succeeds for
// 4-constraint circuits.
//
//   k_fixed_base : P_i = sum_w T[w][digit_w(k_i)], 8-bit windows, T[w][d] = d*2^(8w)*G
//                  (table affine, 32 x 255 entries, built on the host)
//   k_normalize  : XYZZ -> affine with one inversion per CHUNK points (Montgomery's
//                  trick), result packed canonical in the bh_srs layout.
#include "crs.h"
#include "msm.h"  // G1_TABLE_REC

#include <algorithm>

namespace bh {

template <class C>
struct FieldOf;
template <>
struct FieldOf<G1Ops> { using F = G1F; };
template <>
struct FieldOf<G2Ops> { using F = Fp2Ops; };

template <class C>
__device__ __forceinline__ typename C::A load_affine_packed(const uint32_t* base, size_t i) {
  using F = typename FieldOf<C>::F;
  constexpr int PW = F::PACKED_WORDS;
  typename C::A a;
  a.x = F::unpack(base + i * 2 * PW);
  a.y = F::unpack(base + i * 2 * PW + PW);
  return a;
}

template <class C>
__global__ void __launch_bounds__(256) k_fixed_base(const uint32_t* table, const uint32_t* scalars, size_t n,
                                                    typename C::P* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4* sp = reinterpret_cast<const uint4*>(scalars + i * 8);
  uint4 s0 = sp[0], s1 = sp[1];
  const uint32_t s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
  typename C::P acc = C::identity();
  for (int w = 0; w < 32; w++) {
    const uint32_t d = (s[w >> 2] >> ((w & 3) * 8)) & 0xffu;
    if (d) acc = C::madd(acc, load_affine_packed<C>(table, (size_t)w * 255 + (d - 1)));
  }
  out[i] = acc;
}

// x^(p-2) in the device Montgomery domain
__device__ DFp fp_inv(const DFp& x) {
  // p - 2, little-endian 32-bit words
  constexpr uint32_t E[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  DFp r = fe_one<FpCfg>();
  for (int w = 11; w >= 0; w--) {
    for (int b = 31; b >= 0; b--) {
      r = fe_sqr<FpCfg>(r);
      if ((E[w] >> b) & 1u) r = fe_mul<FpCfg>(r, x);
    }
  }
  return r;
}

// the same exponentiation over any Fp representation of the FpOpsT / FpSOps interface
template <class F>
__device__ typename F::T fp_inv_ops(const typename F::T& x) {
  constexpr uint32_t E[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                              0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
  typename F::T r = F::one();
  for (int w = 11; w >= 0; w--) {
    for (int b = 31; b >= 0; b--) {
      r = F::sqr(r);
      if ((E[w] >> b) & 1u) r = F::mul(r, x);
    }
  }
  return r;
}

template <class F>
struct Inv {  // Fp in any representation (G1F)
  static __device__ typename F::T run(const typename F::T& x) { return fp_inv_ops<F>(x); }
};
template <>
struct Inv<Fp2Ops> {
  static __device__ DFp2 run(const DFp2& x) {
    // (a + bu)^-1 = (a - bu) / (a^2 + b^2)
    DFp t = fe_add<FpCfg>(fe_sqr<FpCfg>(x.c0), fe_sqr<FpCfg>(x.c1));
    DFp ti = fp_inv(t);
    DFp2 r;
    r.c0 = fe_mul<FpCfg>(x.c0, ti);
    r.c1 = fe_mul<FpCfg>(fe_sub<FpCfg, 64>(fe_zero<FpCfg>(), x.c1), ti);
    return r;
  }
};

// one thread per CHUNK consecutive points; prefix products kept in `scratch`
template <class C, int CHUNK>
__global__ void __launch_bounds__(64) k_normalize(const typename C::P* pts, size_t n, typename FieldOf<C>::F::T* scratch,
                                                  uint32_t* out_packed, uint32_t rec, int limbs) {
  using F = typename FieldOf<C>::F;
  using T = typename F::T;
  constexpr int PW = F::PACKED_WORDS;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i0 = t * CHUNK;
  if (i0 >= n) return;
  const size_t i1 = (i0 + CHUNK < n) ? i0 + CHUNK : n;
  // prefix products of z_i = ZZ_i * ZZZ_i
  T acc = F::one();
  for (size_t i = i0; i < i1; i++) {
    const T z = F::mul(pts[i].ZZ, pts[i].ZZZ);
    scratch[i] = acc;  // product of z_i0..z_{i-1}
    acc = F::mul(acc, z);
  }
  T inv = Inv<F>::run(acc);
  for (size_t i = i1; i-- > i0;) {
    const typename C::P p = pts[i];
    const T z = F::mul(p.ZZ, p.ZZZ);
    const T zinv = F::mul(inv, scratch[i]);  // 1 / z_i
    inv = F::mul(inv, z);
    // 1/ZZ = ZZZ / z ; 1/ZZZ = ZZ / z
    const T x = F::reduce(F::mul(p.X, F::mul(p.ZZZ, zinv)));
    const T y = F::reduce(F::mul(p.Y, F::mul(p.ZZ, zinv)));
    if (limbs) {  // window-table record (G1_TABLE_REC / G2_TABLE_REC): raw limbs, x then y
      constexpr int NW = sizeof(T) / 4;
      const uint32_t* xw = reinterpret_cast<const uint32_t*>(&x);
      const uint32_t* yw = reinterpret_cast<const uint32_t*>(&y);
#pragma unroll
      for (int k = 0; k < NW; k++) {
        out_packed[i * rec + k] = xw[k];
        out_packed[i * rec + NW + k] = yw[k];
      }
    } else {
      F::pack(x, out_packed + i * rec);
      F::pack(y, out_packed + i * rec + PW);
    }
  }
}

template <class C>
hipError_t fixed_base_batch(const uint32_t* d_table, const uint32_t* d_scalars, size_t n, void* d_xyzz,
                            void* d_scratch, uint32_t* d_out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  using P = typename C::P;
  hipLaunchKernelGGL(k_fixed_base<C>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_table, d_scalars, n,
                     reinterpret_cast<P*>(d_xyzz));
  constexpr int CHUNK = 32;
  const size_t threads = (n + CHUNK - 1) / CHUNK;
  hipLaunchKernelGGL((k_normalize<C, CHUNK>), dim3((unsigned)((threads + 63) / 64)), dim3(64), 0, st,
                     reinterpret_cast<const P*>(d_xyzz), n,
                     reinterpret_cast<typename FieldOf<C>::F::T*>(d_scratch), d_out,
                     (uint32_t)(2 * FieldOf<C>::F::PACKED_WORDS), 0);
  return hipGetLastError();
}

// t-th point of the chunk: its W window multiples, doubling c times between windows
template <class C>
__global__ void __launch_bounds__(256) k_window_multiples(const uint32_t* pts, size_t i0, size_t cnt, int c, int W,
                                                          typename C::P* out) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  typename C::P acc = C::from_affine(load_affine_packed<C>(pts, i0 + t));
  out[t * W] = acc;
  for (int w = 1; w < W; w++) {
    for (int j = 0; j < c; j++) acc = C::dbl(acc);
    out[t * W + w] = acc;
  }
}

template <class C>
size_t window_table_scratch_bytes(size_t chunk, int W) {
  return chunk * (size_t)W * (sizeof(typename C::P) + sizeof(typename FieldOf<C>::F::T));
}

template <class C>
hipError_t window_table(const uint32_t* d_pts, size_t n, int c, int W, uint32_t* d_out, uint32_t rec,
                        void* d_scratch, size_t chunk, hipStream_t st) {
  using P = typename C::P;
  using T = typename FieldOf<C>::F::T;
  constexpr int PW = FieldOf<C>::F::PACKED_WORDS;
  constexpr int CHUNK = 32;
  P* xyzz = reinterpret_cast<P*>(d_scratch);
  T* prefix = reinterpret_cast<T*>(reinterpret_cast<char*>(d_scratch) + chunk * (size_t)W * sizeof(P));
  for (size_t i0 = 0; i0 < n; i0 += chunk) {
    const size_t cnt = std::min(chunk, n - i0);
    hipLaunchKernelGGL(k_window_multiples<C>, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, d_pts, i0, cnt,
                       c, W, xyzz);
    const size_t m = cnt * (size_t)W;
    const size_t threads = (m + CHUNK - 1) / CHUNK;
    hipLaunchKernelGGL((k_normalize<C, CHUNK>), dim3((unsigned)((threads + 63) / 64)), dim3(64), 0, st, xyzz, m,
                       prefix, d_out + i0 * (size_t)W * rec, rec,
                       (int)(std::is_same<C, G1Ops>::value ? rec == G1_TABLE_REC : rec == G2_TABLE_REC));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template size_t window_table_scratch_bytes<G1Ops>(size_t, int);
template size_t window_table_scratch_bytes<G2Ops>(size_t, int);
template hipError_t window_table<G1Ops>(const uint32_t*, size_t, int, int, uint32_t*, uint32_t, void*, size_t,
                                        hipStream_t);
template hipError_t window_table<G2Ops>(const uint32_t*, size_t, int, int, uint32_t*, uint32_t, void*, size_t,
                                        hipStream_t);

template hipError_t fixed_base_batch<G1Ops>(const uint32_t*, const uint32_t*, size_t, void*, void*, uint32_t*,
                                            hipStream_t);
template hipError_t fixed_base_batch<G2Ops>(const uint32_t*, const uint32_t*, size_t, void*, void*, uint32_t*,
                                            hipStream_t);

}  // namespace bh
