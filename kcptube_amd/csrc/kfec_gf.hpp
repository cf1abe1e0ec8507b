// kfec_gf.hpp -- GF(2^8) arithmetic shared by the kfec HIP kernels.
//
// Field: polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator alpha = 2, exactly the field of the reference
// coder (fecpp.cpp:26-146: GF_EXP / GF_LOG / GF_INVERSE).  The log/antilog tables are generated at
// compile time (constexpr) and staged into LDS by the kernels that need random-access multiplies
// (matrix construction, per-group decode coefficients).  The bulk multiply-accumulate over shard bytes
// does NOT use them: it uses per-coefficient byte-permute tables (see kfec_kernels.hip, "perm MAC").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfec {

struct GfTables {
    uint8_t exp[512];  // exp[i] = alpha^(i mod 255), doubled so log a + log b needs no reduction
    uint8_t log[256];  // log[0] = 0xFF = 255: callers that multiply test for zero first, but the fused
                       // Lagrange prep (kfec_kernels.hip decode_prep_lagrange) relies on 255 = 0 mod 255
                       // (static_assert there); do not change the sentinel
};

constexpr GfTables make_gf_tables()
{
    GfTables t{};
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = (uint8_t)v;
        t.log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100) v ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
    t.log[0] = 0xFF;
    return t;
}

// multiply by alpha (x) in GF(2^8)/0x11D; input and output < 256
__host__ __device__ __forceinline__ uint32_t gf_xtime(uint32_t v)
{
    return ((v << 1) ^ ((v & 0x80u) ? 0x11Du : 0u)) & 0xFFu;
}

// Per-coefficient byte-permute tables for v_perm_b32 (see "perm MAC" in kfec_kernels.hip):
//   t[0] = c*{0,1,2,3}        t[1] = c*{4,5,6,7}          (3 low bits)
//   t[2] = c*{0,8,16,24}      t[3] = c*{32,40,48,56}      (bits 3..5)
//   t[4] = c*{0,64,128,192}                               (bits 6..7)
// Built from the 8 doublings of c by linearity (c*(a^b) = c*a ^ c*b): no table lookups.
__host__ __device__ __forceinline__ void gf_perm_tables(uint32_t c, uint32_t t[5])
{
    const uint32_t c1 = c & 0xFFu, c2 = gf_xtime(c1), c4 = gf_xtime(c2), c8 = gf_xtime(c4);
    const uint32_t c16 = gf_xtime(c8), c32 = gf_xtime(c16), c64 = gf_xtime(c32), c128 = gf_xtime(c64);
    const uint32_t lo0 = (c1 << 8) | (c2 << 16) | ((c1 ^ c2) << 24);
    const uint32_t lo1 = (c8 << 8) | (c16 << 16) | ((c8 ^ c16) << 24);
    t[0] = lo0;
    t[1] = lo0 ^ (c4 * 0x01010101u);
    t[2] = lo1;
    t[3] = lo1 ^ (c32 * 0x01010101u);
    t[4] = (c64 << 8) | (c128 << 16) | ((c64 ^ c128) << 24);
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96); hipcc emits two v_xor_b32 otherwise.
// The builtin (not inline asm) leaves the scheduler free to interleave independent accumulator chains.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^ c * x for 4 bytes, c given by its 5 permute tables (kfec_gf.hpp gf_perm_tables):
// three v_perm_b32 lookups (bits 0-2, 3-5, 6-7 of every byte) and two XORs
__device__ __forceinline__ uint32_t perm_mac(uint32_t acc, const uint32_t *t, uint32_t s0, uint32_t s1, uint32_t s2)
{
    const uint32_t p0 = __builtin_amdgcn_perm(t[1], t[0], s0);
    const uint32_t p1 = __builtin_amdgcn_perm(t[3], t[2], s1);
    const uint32_t p2 = __builtin_amdgcn_perm(t[4], t[4], s2);
    return xor3(acc, p0, p1) ^ p2;
}

}  // namespace kfec
