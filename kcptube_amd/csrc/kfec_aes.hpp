// kfec_aes.hpp -- AES-256 (FIPS 197) pieces shared by the AEAD kernels (kfec_gcm.hip, kfec_ocb.hip):
// the S-box (generated, not tabulated), the key schedule and a byte-oriented block encryption used at key
// setup and for the rare blocks the per-packet kernels do not cover with tables.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfec {
namespace {

struct Sbox {
    uint8_t s[256];
};

constexpr Sbox make_sbox()
{
    // inverse in GF(2^8) mod x^8 + x^4 + x^3 + x + 1 via exp / log of the generator 3, then the affine map
    uint8_t ex[256] = {}, lg[256] = {};
    uint32_t x = 1;
    for (int i = 0; i < 255; ++i) {
        ex[i] = (uint8_t)x;
        lg[x] = (uint8_t)i;
        uint32_t x2 = x << 1;
        if (x2 & 0x100u) x2 ^= 0x11Bu;
        x = (x2 ^ x) & 0xFFu;  // x * 3
    }
    Sbox b{};
    for (int a = 0; a < 256; ++a) {
        const uint32_t inv = a ? ex[(255 - lg[a]) % 255] : 0u;
        uint32_t y = inv;
        for (int k = 1; k < 5; ++k) y ^= ((inv << k) | (inv >> (8 - k))) & 0xFFu;
        b.s[a] = (uint8_t)(y ^ 0x63u);
    }
    return b;
}

__device__ const Sbox c_sbox = make_sbox();

__device__ __forceinline__ uint32_t xtime(uint32_t a) { return ((a << 1) ^ ((a & 0x80u) ? 0x1Bu : 0u)) & 0xFFu; }

// rk: 240 bytes of round keys
__device__ void aes256_encrypt(const uint8_t *rk, const uint8_t (&in)[16], uint8_t (&out)[16])
{
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 14; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = c_sbox.s[s[(i + 4 * (i % 4)) % 16]];  // SubBytes + ShiftRows
        if (r < 14) {
            for (int c = 0; c < 4; ++c) {  // MixColumns
                const uint32_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                const uint32_t e = a0 ^ a1 ^ a2 ^ a3;
                s[4 * c] = (uint8_t)(a0 ^ e ^ xtime(a0 ^ a1));
                s[4 * c + 1] = (uint8_t)(a1 ^ e ^ xtime(a1 ^ a2));
                s[4 * c + 2] = (uint8_t)(a2 ^ e ^ xtime(a2 ^ a3));
                s[4 * c + 3] = (uint8_t)(a3 ^ e ^ xtime(a3 ^ a0));
            }
        } else {
            for (int i = 0; i < 16; ++i) s[i] = t[i];
        }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];
    }
    for (int i = 0; i < 16; ++i) out[i] = s[i];
}

// key schedule: 240 bytes of round keys from the 8 key words (little-endian bytes of the SHA-3 digest)
__device__ void aes256_expand(const uint32_t *key, uint8_t (&w)[240])
{
    for (int i = 0; i < 32; ++i) w[i] = (uint8_t)(key[i / 4] >> (8 * (i % 4)));
    uint32_t rcon = 1;
    for (int i = 8; i < 60; ++i) {
        uint8_t t[4] = {w[4 * i - 4], w[4 * i - 3], w[4 * i - 2], w[4 * i - 1]};
        if (i % 8 == 0) {
            const uint8_t t0 = t[0];
            t[0] = (uint8_t)(c_sbox.s[t[1]] ^ rcon);
            t[1] = c_sbox.s[t[2]];
            t[2] = c_sbox.s[t[3]];
            t[3] = c_sbox.s[t0];
            rcon = xtime(rcon);
        } else if (i % 8 == 4) {
            for (int k = 0; k < 4; ++k) t[k] = c_sbox.s[t[k]];
        }
        for (int k = 0; k < 4; ++k) w[4 * i + k] = w[4 * i - 32 + k] ^ t[k];
    }
}

}  // namespace
}  // namespace kfec
