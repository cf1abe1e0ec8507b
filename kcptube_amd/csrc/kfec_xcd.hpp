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

// Row-tiled grids (R > 8: fec=200:55's 7 tiles of 8 parity rows).  The tiles of one chunk are workgroups b, b + 8,
// b + 16, ... -- one XCD, back to back, so all but the first read the chunk's shards from that XCD's L2
// (block_chunk_tile) -- and with KFEC_XCD_TILE_SPAN = S the chunks an XCD takes in successive rounds are S adjacent
// ones instead of every 8th, so the group split at each chunk boundary has its 200 rows' shared lines fetched into
// one L2 instead of two (as xcd_chunk for single tiles).  Chunks are padded to a multiple of 8 S; padding exits.
// Measured at 200:55, 256k groups (profiles/r06_tile_span_ab.txt): the decode MAC's HBM traffic 116.45 -> 114.16 GB
// per launch (with its prep 1.21x -> 1.19x of the algorithmic 96.26 GB), decode 152.4-152.6 -> 151.4 ms; S = 4
// the same time; the VALU-bound encode unchanged.
#ifndef KFEC_XCD_TILE_SPAN
#define KFEC_XCD_TILE_SPAN 16
#endif
__host__ __device__ constexpr uint32_t xcd_tile_chunks(uint32_t chunks)
{
    return KFEC_XCD_TILE_SPAN && chunks >= kXcdMinGrid
               ? (chunks + 8u * KFEC_XCD_TILE_SPAN - 1u) / (8u * KFEC_XCD_TILE_SPAN) * (8u * KFEC_XCD_TILE_SPAN)
               : (chunks + 7u) & ~7u;
}

// round r of XCD x -> chunk (r = the XCD's r-th set of `tiles` workgroups); grid_chunks: xcd_tile_chunks(chunks)
__device__ __forceinline__ uint32_t xcd_tile_chunk(uint32_t r, uint32_t x, uint32_t grid_chunks)
{
    constexpr uint32_t S = KFEC_XCD_TILE_SPAN;
    if constexpr (S == 0) {
        return r * 8u + x;
    } else {
        // (a grid of >= kXcdMinGrid chunks is a multiple of 8 S: the host pads to it, or to 8 when chunks < 512,
        // which only reaches 512 itself -- a multiple of 8 S)
        static_assert(kXcdMinGrid % (8u * (S ? S : 1u)) == 0, "span must divide the minimum grid");
        if (grid_chunks < kXcdMinGrid) return r * 8u + x;
        return ((r / S) * 8u + x) * S + (r % S);
    }
}

}  // namespace kfec
