// kfec_xcd.hpp -- XCD spans: the chunk order of the dense single-tile launches (device code; .hip files only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#ifndef KFEC_XCD_ORDER
#define KFEC_XCD_ORDER 16  // S > 0: single-tile MAC and dense syndrome launches give each XCD runs of S adjacent chunks
#endif

namespace kfec {

// Single-tile grids (R <= 8) of at least kXcdMinGrid chunks with KFEC_XCD_ORDER = S: the grid is a multiple of
// 8 S and, within each run of 8 S workgroups, XCD x (workgroups x, x + 8, ...) takes the S adjacent chunks
// x S .. x S + S - 1, so the 128-byte lines that a group split between two of them shares (its rows at the split
// column; at B = 1400 also the line between two groups) are fetched into, and written back from, one L2
// instead of two, for 15 of every 16 splits.  Chunks past the last are padding and exit.  Measured
// (profiles/r05_xcd_span_ab.txt, three boxes): S = 16 takes the 20:3 encode 4% and its decode 1-2% faster, the
// 10:3 random decode 1-2%, the 8:4 encode 6%; one contiguous eighth per XCD made 20:3 6% slower.  Smaller grids
// (small flushes) keep the plain order and no padding.  The fused wire path's framed encode / decode kernels
// (kfec_frame.hip), whose shards sit at scattered arena offsets, measured the same with this order
// (profiles/r05_xcd_frame_ab.txt) and keep the plain one.
constexpr uint32_t kXcdMinGrid = 512;

__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b)
{
    constexpr uint32_t S = KFEC_XCD_ORDER;
    if constexpr (S == 0) {
        return b;
    } else {
        if (gridDim.x < kXcdMinGrid) return b;
        const uint32_t r = b % (8u * S);
        return (b - r) + (r & 7u) * S + (r >> 3);
    }
}

__host__ __device__ constexpr uint32_t xcd_grid(uint32_t chunks)
{
    return KFEC_XCD_ORDER && chunks >= kXcdMinGrid ? (chunks + 8u * KFEC_XCD_ORDER - 1u) / (8u * KFEC_XCD_ORDER) * (8u * KFEC_XCD_ORDER)
                                                    : chunks;
}

}  // namespace kfec
