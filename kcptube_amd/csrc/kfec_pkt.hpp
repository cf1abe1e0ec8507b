// kfec_pkt.hpp -- 16-byte packet-block helpers shared by the AES-based packet kernels (kfec_gcm.hip,
// kfec_ocb.hip): packets sit at arbitrary byte offsets of a dword-aligned buffer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfec {
namespace {

__device__ __forceinline__ uint4 u4_xor(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

// 16 bytes at byte address a of a dword-aligned buffer of lim32 dwords (zero past it)
__device__ __forceinline__ uint4 load16(const uint32_t *b32, uint64_t lim32, uint64_t a)
{
    const uint64_t w = a >> 2;
    uint32_t d[5];
    if (w + 5 <= lim32) {
        const uint4 q = *reinterpret_cast<const uint4 *>(b32 + w);
        d[0] = q.x; d[1] = q.y; d[2] = q.z; d[3] = q.w;
        d[4] = b32[w + 4];
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) d[i] = w + i < lim32 ? b32[w + i] : 0u;
    }
    const uint32_t sh = (uint32_t)(a & 3u);
    return make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], sh), __builtin_amdgcn_alignbyte(d[2], d[1], sh),
                      __builtin_amdgcn_alignbyte(d[3], d[2], sh), __builtin_amdgcn_alignbyte(d[4], d[3], sh));
}

// keep the first rem bytes (0 < rem < 16)
__device__ __forceinline__ uint4 mask16(uint4 v, uint32_t rem)
{
    uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = (int)rem - 4 * i;
        d[i] = k >= 4 ? d[i] : k <= 0 ? 0u : d[i] & ((1u << (8 * k)) - 1u);
    }
    return make_uint4(d[0], d[1], d[2], d[3]);
}

}  // namespace
}  // namespace kfec
