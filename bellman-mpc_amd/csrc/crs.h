// Host interface of the device fixed-base scalar multiplication (crs.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include "curve.cuh"

namespace bh {
// d_table: 32*255 packed affine points T[w][d-1] = d*2^(8w)*G (device Montgomery, canonical)
// d_scalars: n canonical scalars (8 LE u32 words); non-zero scalars only (results are never infinity)
// d_xyzz: n*sizeof(XYZZ) scratch; d_scratch: n*sizeof(field) scratch; d_out: n packed affine points
template <class C>
hipError_t fixed_base_batch(const uint32_t* d_table, const uint32_t* d_scalars, size_t n, void* d_xyzz,
                            void* d_scratch, uint32_t* d_out, hipStream_t st);

// Window table of a fixed base vector (the prover's SRS): out[i*W + w] = 2^(c*w) * P_i,
// packed affine like the input but in records of `rec` u32 words (a whole number of
// 128-byte lines: one line per G1 gather, two per G2), for the n points of d_pts (none
// may be the identity).
// Processed in chunks of `chunk` points; d_scratch must hold window_table_scratch_bytes.
template <class C>
size_t window_table_scratch_bytes(size_t chunk, int W);
template <class C>
hipError_t window_table(const uint32_t* d_pts, size_t n, int c, int W, uint32_t* d_out, uint32_t rec,
                        void* d_scratch, size_t chunk, hipStream_t st);
}  // namespace bh
