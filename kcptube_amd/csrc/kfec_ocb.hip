// kfec_ocb.hip -- kcptube's aes_ocb packet mode as gfx950 kernels (include/kfec_aead.h).
//
// encrypt_data / decrypt_data (data_operations.cpp:171-234, 373-435) over encrypt_decrypt<aes_256_ocb>
// (aead.hpp:314-400): Botan "AES-256/OCB" (RFC 7253, 128-bit tag) with kcptube's 12-byte nonce (iv_raw
// repeated 6 times); packet = C || tag || iv_raw; AD "KCP PortHopping" (aead.hpp:16).
//
// OCB enciphers every data block (C_i = Offset_i xor E_K(P_i xor Offset_i)), so unlike CTR the block cipher
// cannot be tabulated; what the key and the 16-bit iv_raw alone determine is: L_*, L_$, L_0..L_31, the hash of
// the fixed AD (HASH(K, A) = E_K((A || 0x80 || 0^) xor L_*), one block since |A| = 15) -- per key -- and
// Offset_0 -- per iv, a 1 MiB table.  Block i's offset has a closed form, Offset_i = Offset_0 xor XOR of L_j
// over the set bits j of gray(i) = i xor (i >> 1), so the blocks of a packet are independent: a row of 8
// lanes per packet, lane j taking blocks j + 1, j + 9, ...; the checksum is the row's XOR of the plaintext
// blocks, and one lane enciphers the tag.  AES runs from T-tables in LDS, replicated per bank so that the
// byte-indexed reads of a row never conflict (OcbLds below), with the round keys in LDS too (broadcast reads).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/kfec_aead.h"
#include "kfec_aes.hpp"
#include "kfec_gf.hpp"
#include "kfec_count.hpp"
#include "kfec_internal.hpp"
#include "kfec_pkt.hpp"

namespace kfec {

namespace {

// per-key record (ocb_key_kernel), 16-byte aligned pieces
struct OcbKey {
    uint4 rk[15];    // encryption round keys
    uint4 dk[15];    // decryption round keys of the equivalent inverse cipher
    uint4 lstar;     // L_* = E_K(0)
    uint4 ldollar;   // L_$ = double(L_*)
    uint4 l[32];     // L_0 = double(L_$), L_j = double(L_(j-1))
    uint4 sad;       // HASH(K, "KCP PortHopping")
    uint32_t te[4][256];
    uint32_t td[4][256];
    uint32_t isb[256];
    uint4 rkr[15];   // rk / dk with every word rotated by 16 (the per-packet kernel's scalar round-key loads)
    uint4 dkr[15];
};

__device__ __forceinline__ uint32_t gmul8(uint32_t a, uint32_t b)
{
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1u) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

__device__ __forceinline__ uint32_t pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3)
{
    return b0 | b1 << 8 | b2 << 16 | b3 << 24;
}

__device__ __forceinline__ uint4 bytes_to_u4(const uint8_t (&b)[16])
{
    return make_uint4(pack4(b[0], b[1], b[2], b[3]), pack4(b[4], b[5], b[6], b[7]), pack4(b[8], b[9], b[10], b[11]),
                      pack4(b[12], b[13], b[14], b[15]));
}

__device__ __forceinline__ void u4_to_bytes(uint4 v, uint8_t (&b)[16])
{
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(w[i / 4] >> (8 * (i % 4)));
}

// double(S) of RFC 7253: S << 1, xor 0x87 into the last byte when the first bit was set
__device__ void ocb_double(uint8_t (&s)[16])
{
    const uint32_t msb = s[0] >> 7;
    for (int i = 0; i < 15; ++i) s[i] = (uint8_t)((s[i] << 1) | (s[i + 1] >> 7));
    s[15] = (uint8_t)((s[15] << 1) ^ (msb ? 0x87u : 0u));
}

// T-tables and inverse S-box: one workgroup of 256 threads, thread = byte value
__global__ void ocb_tables_kernel(OcbKey *k)
{
    const uint32_t x = threadIdx.x;
    if (blockIdx.x || x >= 256) return;
    const uint32_t s = c_sbox.s[x];
    k->te[0][x] = pack4(xtime(s), s, s, xtime(s) ^ s);
    k->te[1][x] = pack4(xtime(s) ^ s, xtime(s), s, s);
    k->te[2][x] = pack4(s, xtime(s) ^ s, xtime(s), s);
    k->te[3][x] = pack4(s, s, xtime(s) ^ s, xtime(s));
    k->isb[s] = x;
    __syncthreads();
    const uint32_t is = k->isb[x];
    const uint32_t e = gmul8(is, 14), n9 = gmul8(is, 9), d = gmul8(is, 13), b = gmul8(is, 11);
    k->td[0][x] = pack4(e, n9, d, b);
    k->td[1][x] = pack4(b, e, n9, d);
    k->td[2][x] = pack4(d, b, e, n9);
    k->td[3][x] = pack4(n9, d, b, e);
}

// key schedule, the decryption round keys, L values and the AD hash: one thread
__global__ void ocb_key_kernel(const uint32_t *key, OcbKey *k)
{
    if (blockIdx.x || threadIdx.x) return;
    uint8_t w[240];
    aes256_expand(key, w);
    for (int r = 0; r < 15; ++r) {
        uint8_t b[16];
        for (int i = 0; i < 16; ++i) b[i] = w[16 * r + i];
        k->rk[r] = bytes_to_u4(b);
        // dk[r] = InvMixColumns(rk[14 - r]) for 0 < r < 14, the end keys unchanged
        for (int i = 0; i < 16; ++i) b[i] = w[16 * (14 - r) + i];
        if (r > 0 && r < 14) {
            uint8_t m[16];
            for (int c = 0; c < 4; ++c) {
                const uint32_t a0 = b[4 * c], a1 = b[4 * c + 1], a2 = b[4 * c + 2], a3 = b[4 * c + 3];
                m[4 * c] = (uint8_t)(gmul8(a0, 14) ^ gmul8(a1, 11) ^ gmul8(a2, 13) ^ gmul8(a3, 9));
                m[4 * c + 1] = (uint8_t)(gmul8(a0, 9) ^ gmul8(a1, 14) ^ gmul8(a2, 11) ^ gmul8(a3, 13));
                m[4 * c + 2] = (uint8_t)(gmul8(a0, 13) ^ gmul8(a1, 9) ^ gmul8(a2, 14) ^ gmul8(a3, 11));
                m[4 * c + 3] = (uint8_t)(gmul8(a0, 11) ^ gmul8(a1, 13) ^ gmul8(a2, 9) ^ gmul8(a3, 14));
            }
            for (int i = 0; i < 16; ++i) b[i] = m[i];
        }
        k->dk[r] = bytes_to_u4(b);
        auto r16 = [](uint4 v) {
            return make_uint4(v.x << 16 | v.x >> 16, v.y << 16 | v.y >> 16, v.z << 16 | v.z >> 16, v.w << 16 | v.w >> 16);
        };
        k->rkr[r] = r16(k->rk[r]);
        k->dkr[r] = r16(k->dk[r]);
    }
    uint8_t z[16] = {}, ls[16], t[16];
    aes256_encrypt(w, z, ls);  // L_*
    k->lstar = bytes_to_u4(ls);
    for (int i = 0; i < 16; ++i) t[i] = ls[i];
    ocb_double(t);  // L_$
    k->ldollar = bytes_to_u4(t);
    for (int j = 0; j < 32; ++j) {
        ocb_double(t);
        k->l[j] = bytes_to_u4(t);
    }
    // HASH(K, A) for the 15-byte AD: no full block; E_K((A || 0x80) xor L_*)
    const char *ad = "KCP PortHopping";
    uint8_t in[16], o[16];
    for (int i = 0; i < 16; ++i) in[i] = (uint8_t)((i < 15 ? (uint8_t)ad[i] : 0x80u) ^ ls[i]);
    aes256_encrypt(w, in, o);
    k->sad = bytes_to_u4(o);
}

// Offset_0 of every iv (RFC 7253 4.2, TAGLEN 128, 12-byte nonce): one thread per iv
__global__ void ocb_iv_kernel(const uint32_t *key, uint4 *off0)
{
    const uint32_t iv = blockIdx.x * blockDim.x + threadIdx.x;
    if (iv >= 65536u) return;
    uint8_t w[240];
    aes256_expand(key, w);
    uint8_t nonce[16] = {0, 0, 0, 1};
    for (int i = 4; i < 16; ++i) nonce[i] = (uint8_t)(i % 2 ? iv >> 8 : iv);  // iv_raw (little-endian) x 6
    const uint32_t bottom = nonce[15] & 0x3Fu;
    nonce[15] &= 0xC0u;
    uint8_t ktop[16];
    aes256_encrypt(w, nonce, ktop);
    uint64_t hi = 0, lo = 0;
    for (int i = 0; i < 8; ++i) {
        hi = hi << 8 | ktop[i];
        lo = lo << 8 | ktop[8 + i];
    }
    // Stretch = Ktop || (Ktop[1..64] xor Ktop[9..72]); Offset_0 = Stretch[1 + bottom .. 128 + bottom]
    const uint64_t x = hi ^ (hi << 8 | lo >> 56);
    uint64_t oh = hi, ol = lo;
    if (bottom) {
        oh = hi << bottom | lo >> (64 - bottom);
        ol = lo << bottom | x >> (64 - bottom);
    }
    uint8_t o[16];
    for (int i = 0; i < 8; ++i) {
        o[i] = (uint8_t)(oh >> (56 - 8 * i));
        o[8 + i] = (uint8_t)(ol >> (56 - 8 * i));
    }
    off0[iv] = bytes_to_u4(o);
}

// ---- per-packet kernel -------------------------------------------------------------------------------
#ifndef KFEC_OCB_BITOP3
#define KFEC_OCB_BITOP3 1  // byte-1 table addresses by v_bitop3_b32 instead of v_perm_b32 (A/B knob)
#endif
#ifndef KFEC_OCB_PAIR
#define KFEC_OCB_PAIR 1  // two-block cipher: two rounds per loop trip, no register moves between trips (A/B knob)
#endif
#ifndef KFEC_OCB_ILP
#define KFEC_OCB_ILP 2  // full blocks per lane through the AES rounds together (1 or 2; A/B knob)
#endif
#ifndef KFEC_OCB_KSGPR
#define KFEC_OCB_KSGPR 1  // the two-block rounds' keys by scalar loads, not LDS broadcast reads (A/B knob)
#endif
#ifndef KFEC_OCB_T4
#define KFEC_OCB_T4 1  // four replicated tables (128 KiB, 1024-lane workgroups) and no rotate per column (A/B knob)
#endif
#if KFEC_OCB_T4
#define OCB_RKEY rk  // the round keys as they are (no rotated half to fold them into)
#define OCB_DKEY dk
#else
#define OCB_RKEY rkr
#define OCB_DKEY dkr
#endif
constexpr int kRow = 8;
constexpr int kOcbBlock = KFEC_OCB_T4 ? 1024 : 512;
constexpr int kRowsPerBlock = kOcbBlock / kRow;

struct OcbArgs {
    const uint32_t *src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint32_t *len;
    const uint16_t *iv;
    uint8_t *dst;
    uint64_t dst_pitch;
    uint32_t *out_len;
    uint8_t *ok;
    const OcbKey *key;
    const uint4 *off0;
    uint64_t P;
    uint32_t *done;  // counted launch (kfec_count.hpp)
};

// What one workgroup stages into LDS.  AES is LDS-bound here: 16 byte-indexed table reads per round on random
// bytes, and with one table shared by the 32 lanes of a read (32 banks) those reads took ~2.3 LDS cycles
// each.  Tables are kept in 32 copies laid out so that copy c sits in bank c -- row lane c reads rep[v][c],
// and the 32 lanes of a read hit 32 different banks whatever their bytes: no conflicts.  Te2 / Te3 are Te0 /
// Te1 rotated by 16 bits (Td likewise), so a column is T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d]) ^ k: two
// replicated tables and one rotate per column.
//   seal: te[v][j][c] = Te_j[v], j = 0, 1 (64 KiB).  open: td[v][j][c] = Td_j[v] (64 KiB), isb4 / isb = the
//   inverse S-box bytes 4w .. 4w + 3 (8 KiB), and Te0 once (the pad of a partial block and the tag: at most
//   two blocks per packet).
constexpr int kRep = 32;
#ifndef KFEC_OCB_ISB4
#define KFEC_OCB_ISB4 1  // open's last round from a byte-replicated InvS table, columns joined by permutes (A/B knob)
#endif
template <bool OPEN>
struct OcbLds;
//   KFEC_OCB_T4: Te2 / Te3 (Td2 / Td3) replicated as well, in a second 64 KiB half right after the first, so a
//   column is T0[a] ^ T1[b] ^ T2[c] ^ T3[d] ^ k with no rotate (a 4-cycle op on gfx950, one of ~7 per column);
//   128 KiB per workgroup, so one 1024-lane workgroup per CU keeps the 4 waves per SIMD of two 512-lane ones.
#if KFEC_OCB_T4
template <>
struct OcbLds<false> {
    uint32_t te[256][2][kRep];    // row v: the 32 copies of Te0[v], then of Te1[v] (256 B)
    uint32_t te23[256][2][kRep];  // the same for Te2 / Te3, at te + 64 KiB
    uint4 rk[15];
    uint4 dk[15];
    uint4 l[32];
    uint4 rkr[15];
    uint4 dkr[15];
};
template <>
struct OcbLds<true> {
    uint32_t td[256][2][kRep];
    uint32_t td23[256][2][kRep];
    uint4 rk[15];
    uint4 dk[15];
    uint4 l[32];
    uint4 rkr[15];
    uint4 dkr[15];
#else
template <>
struct OcbLds<false> {
    uint4 rk[15];
    uint4 dk[15];
    uint4 l[32];
    uint4 rkr[15];              // the round keys with every word rotated by 16 (tcol folds the key into the rotate)
    uint4 dkr[15];
    uint32_t te[256][2][kRep];  // row v: the 32 copies of Te0[v], then of Te1[v] (256 B)
};
template <>
struct OcbLds<true> {
    uint4 rk[15];
    uint4 dk[15];
    uint4 l[32];
    uint4 rkr[15];
    uint4 dkr[15];
    uint32_t td[256][2][kRep];
#endif
#if KFEC_OCB_ISB4
    uint32_t isb4[256][8];  // row v: 8 copies of InvS(v) in all four bytes (8 KiB; copy = lane % 8)
#else
    uint32_t isb[64][kRep];
#endif
    uint32_t te0[256];
};

__device__ __forceinline__ uint32_t b0(uint32_t x) { return x & 0xFFu; }
__device__ __forceinline__ uint32_t b1(uint32_t x) { return (x >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t b2(uint32_t x) { return (x >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t b3(uint32_t x) { return x >> 24; }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int k) { return __builtin_amdgcn_alignbit(x, x, 32 - k); }

// Table J's copy c of entry (byte K of x): a row is 256 bytes, so the byte offset is byte K of x in bits 8..15
// and 4 c (< 128) in bits 0..7 -- one v_perm_b32 (the shift-and-or form was two VALU ops per read) -- plus
// 128 J, the read's immediate offset
template <int J, int K>
__device__ __forceinline__ uint32_t rep_at(const uint32_t (*T)[2][kRep], uint32_t x, uint32_t c4)
{
    // byte 1 is already in bits 8..15: (x & 0xFF00) | c4 is one v_bitop3_b32, a full-rate op (v_perm_b32 is not)
    const uint32_t o = K == 1 && KFEC_OCB_BITOP3 ? __builtin_amdgcn_bitop3_b32(x, 0xFF00u, c4, 0xEA)
                                                 : __builtin_amdgcn_perm(x, c4, 0x0C0C0000u | ((4u + K) << 8));
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(T) + o + 128 * J);
}

#if KFEC_OCB_T4
// one column of a round from the four tables: T0[b0(a)] ^ T1[b1(b)] ^ T2[b2(cc)] ^ T3[b3(d)] ^ k.  T2 / T3 sit
// 64 KiB above T0 / T1: byte 2 of their lane term (c4 | 0x10000, loop-invariant) carries it through the same
// single permute that places the state byte, so the halves cost the same address work and no rotate is left
__device__ __forceinline__ uint32_t tcol(const uint32_t (*T)[2][kRep], uint32_t c4, uint32_t a, uint32_t b, uint32_t cc,
                                         uint32_t d, uint32_t k)
{
    const uint8_t *base = reinterpret_cast<const uint8_t *>(T);
    const uint32_t c4h = c4 | 0x10000u;
    const uint32_t o0 = __builtin_amdgcn_perm(a, c4, 0x0C0C0400u);
    const uint32_t o1 = KFEC_OCB_BITOP3 ? __builtin_amdgcn_bitop3_b32(b, 0xFF00u, c4, 0xEA)
                                        : __builtin_amdgcn_perm(b, c4, 0x0C0C0500u);
    const uint32_t o2 = __builtin_amdgcn_perm(cc, c4h, 0x0C020600u);
    const uint32_t o3 = __builtin_amdgcn_perm(d, c4h, 0x0C020700u);
    auto at = [&](uint32_t o, uint32_t imm) { return *reinterpret_cast<const uint32_t *>(base + o + imm); };
    return xor3(xor3(at(o0, 0), at(o1, 128), at(o2, 0)), at(o3, 128), k);
}
static_assert(offsetof(OcbLds<false>, te23) == offsetof(OcbLds<false>, te) + 65536, "T2 / T3 half at +64 KiB");
static_assert(offsetof(OcbLds<true>, td23) == offsetof(OcbLds<true>, td) + 65536, "Td2 / Td3 half at +64 KiB");
#else
// one column of a round: T0[b0(a)] ^ T1[b1(b)] ^ rotl16(T0[b2(cc)] ^ T1[b3(d)]) ^ k, with kr = rotl16(k) folded
// into the rotated half: rotl16(T0[..] ^ T1[..] ^ kr) = rotl16(T0[..] ^ T1[..]) ^ k -- three VALU ops, not four
__device__ __forceinline__ uint32_t tcol(const uint32_t (*T)[2][kRep], uint32_t c4, uint32_t a, uint32_t b, uint32_t cc,
                                         uint32_t d, uint32_t kr)
{
    const uint32_t hi = xor3(rep_at<0, 2>(T, cc, c4), rep_at<1, 3>(T, d, c4), kr);
    return xor3(rep_at<0, 0>(T, a, c4), rep_at<1, 1>(T, b, c4), rotl(hi, 16));
}
#endif

// Te0 holds S(x) in byte 1 (Te0[x] = {2S, S, S, 3S})
__device__ __forceinline__ uint32_t sbox_col(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3)
{
    // byte 1 of each word: two v_perm_b32 gather two bytes each, one OR joins the halves
    const uint32_t lo = __builtin_amdgcn_perm(w1, w0, 0x0C0C0501u);  // {w0.b1, w1.b1, 0, 0}
    const uint32_t hi = __builtin_amdgcn_perm(w3, w2, 0x05010C0Cu);  // {0, 0, w2.b1, w3.b1}
    return lo | hi;
}

// encryption from the replicated tables (seal), row lane c (c4 = 4 c)
__device__ __forceinline__ uint4 aes_enc(const OcbLds<false> &t, uint32_t c4, uint4 in)
{
    uint32_t s0 = in.x ^ t.rk[0].x, s1 = in.y ^ t.rk[0].y, s2 = in.z ^ t.rk[0].z, s3 = in.w ^ t.rk[0].w;
#pragma unroll 1
    for (int r = 1; r < 14; ++r) {
        const uint4 k = t.OCB_RKEY[r];
        const uint32_t t0 = tcol(t.te, c4, s0, s1, s2, s3, k.x);
        const uint32_t t1 = tcol(t.te, c4, s1, s2, s3, s0, k.y);
        const uint32_t t2 = tcol(t.te, c4, s2, s3, s0, s1, k.z);
        const uint32_t t3 = tcol(t.te, c4, s3, s0, s1, s2, k.w);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = t.rk[14];
    const uint32_t (*T)[2][kRep] = t.te;
    const uint32_t o0 = sbox_col(rep_at<0, 0>(T, s0, c4), rep_at<0, 1>(T, s1, c4), rep_at<0, 2>(T, s2, c4), rep_at<0, 3>(T, s3, c4));
    const uint32_t o1 = sbox_col(rep_at<0, 0>(T, s1, c4), rep_at<0, 1>(T, s2, c4), rep_at<0, 2>(T, s3, c4), rep_at<0, 3>(T, s0, c4));
    const uint32_t o2 = sbox_col(rep_at<0, 0>(T, s2, c4), rep_at<0, 1>(T, s3, c4), rep_at<0, 2>(T, s0, c4), rep_at<0, 3>(T, s1, c4));
    const uint32_t o3 = sbox_col(rep_at<0, 0>(T, s3, c4), rep_at<0, 1>(T, s0, c4), rep_at<0, 2>(T, s1, c4), rep_at<0, 3>(T, s2, c4));
    return make_uint4(o0 ^ k.x, o1 ^ k.y, o2 ^ k.z, o3 ^ k.w);
}

// encryption from the single Te0 (open: the partial block's pad and the tag only)
__device__ __forceinline__ uint4 aes_enc(const OcbLds<true> &t, uint32_t, uint4 in)
{
    const uint32_t *T = t.te0;
    uint32_t s0 = in.x ^ t.rk[0].x, s1 = in.y ^ t.rk[0].y, s2 = in.z ^ t.rk[0].z, s3 = in.w ^ t.rk[0].w;
#pragma unroll 1
    for (int r = 1; r < 14; ++r) {
        const uint4 k = t.rk[r];
        const uint32_t t0 = xor3(T[b0(s0)], rotl(T[b1(s1)], 8), rotl(T[b2(s2)], 16)) ^ xor3(rotl(T[b3(s3)], 24), k.x, 0u);
        const uint32_t t1 = xor3(T[b0(s1)], rotl(T[b1(s2)], 8), rotl(T[b2(s3)], 16)) ^ xor3(rotl(T[b3(s0)], 24), k.y, 0u);
        const uint32_t t2 = xor3(T[b0(s2)], rotl(T[b1(s3)], 8), rotl(T[b2(s0)], 16)) ^ xor3(rotl(T[b3(s1)], 24), k.z, 0u);
        const uint32_t t3 = xor3(T[b0(s3)], rotl(T[b1(s0)], 8), rotl(T[b2(s1)], 16)) ^ xor3(rotl(T[b3(s2)], 24), k.w, 0u);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = t.rk[14];
    const uint32_t o0 = sbox_col(T[b0(s0)], T[b1(s1)], T[b2(s2)], T[b3(s3)]);
    const uint32_t o1 = sbox_col(T[b0(s1)], T[b1(s2)], T[b2(s3)], T[b3(s0)]);
    const uint32_t o2 = sbox_col(T[b0(s2)], T[b1(s3)], T[b2(s0)], T[b3(s1)]);
    const uint32_t o3 = sbox_col(T[b0(s3)], T[b1(s0)], T[b2(s1)], T[b3(s2)]);
    return make_uint4(o0 ^ k.x, o1 ^ k.y, o2 ^ k.z, o3 ^ k.w);
}

#if KFEC_OCB_ISB4
// InvS of byte K of x, replicated in all four bytes: row v is 32 bytes, so the offset is byte K of x in bits
// 5..12 and 4 (lane % 8) in bits 2..4 (c4 & 31)
template <int K>
__device__ __forceinline__ uint32_t isb4_at(const OcbLds<true> &t, uint32_t c4, uint32_t x)
{
    const uint32_t o = (K == 0 ? x << 5 : x >> (8 * K - 5)) & 0x1FE0u;
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t.isb4) + (o | (c4 & 31u)));
}

// the last round's column: InvS of byte 0 of a0, byte 1 of a1, byte 2 of a2, byte 3 of a3, joined by permutes
__device__ __forceinline__ uint32_t isb_col(const OcbLds<true> &t, uint32_t c4, uint32_t a0, uint32_t a1, uint32_t a2,
                                            uint32_t a3)
{
    const uint32_t lo = __builtin_amdgcn_perm(isb4_at<1>(t, c4, a1), isb4_at<0>(t, c4, a0), 0x0C0C0400u);
    const uint32_t hi = __builtin_amdgcn_perm(isb4_at<3>(t, c4, a3), isb4_at<2>(t, c4, a2), 0x04000C0Cu);
    return lo | hi;
}
#else
// inverse S-box byte K of x from the replicated packed table
template <int K>
__device__ __forceinline__ uint32_t isb(const OcbLds<true> &t, uint32_t c4, uint32_t x)
{
    const uint32_t v = (x >> (8 * K)) & 0xFFu;
    return (t.isb[v >> 2][c4 >> 2] >> (8 * (v & 3u))) & 0xFFu;
}

__device__ __forceinline__ uint32_t isb_col(const OcbLds<true> &t, uint32_t c4, uint32_t a0, uint32_t a1, uint32_t a2,
                                            uint32_t a3)
{
    return isb<0>(t, c4, a0) | isb<1>(t, c4, a1) << 8 | isb<2>(t, c4, a2) << 16 | isb<3>(t, c4, a3) << 24;
}
#endif

// the equivalent inverse cipher (FIPS 197 5.3.5) from the replicated Td0 / Td1, row lane c (c4 = 4 c)
__device__ __forceinline__ uint4 aes_dec(const OcbLds<true> &t, uint32_t c4, uint4 in)
{
    uint32_t s0 = in.x ^ t.dk[0].x, s1 = in.y ^ t.dk[0].y, s2 = in.z ^ t.dk[0].z, s3 = in.w ^ t.dk[0].w;
#pragma unroll 1
    for (int r = 1; r < 14; ++r) {
        const uint4 k = t.OCB_DKEY[r];
        // InvShiftRows: output column c row r takes input column c - r
        const uint32_t t0 = tcol(t.td, c4, s0, s3, s2, s1, k.x);
        const uint32_t t1 = tcol(t.td, c4, s1, s0, s3, s2, k.y);
        const uint32_t t2 = tcol(t.td, c4, s2, s1, s0, s3, k.z);
        const uint32_t t3 = tcol(t.td, c4, s3, s2, s1, s0, k.w);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint4 k = t.dk[14];
    const uint32_t o0 = isb_col(t, c4, s0, s3, s2, s1);
    const uint32_t o1 = isb_col(t, c4, s1, s0, s3, s2);
    const uint32_t o2 = isb_col(t, c4, s2, s1, s0, s3);
    const uint32_t o3 = isb_col(t, c4, s3, s2, s1, s0);
    return make_uint4(o0 ^ k.x, o1 ^ k.y, o2 ^ k.z, o3 ^ k.w);
}

// two blocks through the rounds together (KFEC_OCB_ILP 2): twice the independent table reads in flight per
// wave, for the latency the 4 waves per SIMD that the tables' LDS allows do not hide
// round key r of a uniform table in global memory, by scalar loads (the address space of constant data)
__device__ __forceinline__ uint4 key_at(const uint4 *tab, int r)
{
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(4))) v4u cu4;
    const v4u v = ((const cu4 *)tab)[r];
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void aes_enc2(const OcbLds<false> &t, const OcbKey *key, uint32_t c4, uint4 &x, uint4 &y)
{
    uint32_t s0 = x.x ^ t.rk[0].x, s1 = x.y ^ t.rk[0].y, s2 = x.z ^ t.rk[0].z, s3 = x.w ^ t.rk[0].w;
    uint32_t u0 = y.x ^ t.rk[0].x, u1 = y.y ^ t.rk[0].y, u2 = y.z ^ t.rk[0].z, u3 = y.w ^ t.rk[0].w;
#if KFEC_OCB_PAIR
    // rounds 1 .. 13, two per loop trip with the state alternating between (s, u) and (p, q), so no trip
    // ends in register moves
    auto round = [&](int r, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t b0, uint32_t b1,
                     uint32_t b2, uint32_t b3, uint32_t &o0, uint32_t &o1, uint32_t &o2, uint32_t &o3, uint32_t &e0,
                     uint32_t &e1, uint32_t &e2, uint32_t &e3) {
        const uint4 k = KFEC_OCB_KSGPR ? key_at(key->OCB_RKEY, r) : t.OCB_RKEY[r];
        o0 = tcol(t.te, c4, a0, a1, a2, a3, k.x);
        e0 = tcol(t.te, c4, b0, b1, b2, b3, k.x);
        o1 = tcol(t.te, c4, a1, a2, a3, a0, k.y);
        e1 = tcol(t.te, c4, b1, b2, b3, b0, k.y);
        o2 = tcol(t.te, c4, a2, a3, a0, a1, k.z);
        e2 = tcol(t.te, c4, b2, b3, b0, b1, k.z);
        o3 = tcol(t.te, c4, a3, a0, a1, a2, k.w);
        e3 = tcol(t.te, c4, b3, b0, b1, b2, k.w);
    };
    uint32_t p0, p1, p2, p3, q0, q1, q2, q3;
    round(1, s0, s1, s2, s3, u0, u1, u2, u3, p0, p1, p2, p3, q0, q1, q2, q3);
#pragma unroll 1
    for (int r = 2; r < 14; r += 2) {
        round(r, p0, p1, p2, p3, q0, q1, q2, q3, s0, s1, s2, s3, u0, u1, u2, u3);
        round(r + 1, s0, s1, s2, s3, u0, u1, u2, u3, p0, p1, p2, p3, q0, q1, q2, q3);
    }
    s0 = p0; s1 = p1; s2 = p2; s3 = p3;
    u0 = q0; u1 = q1; u2 = q2; u3 = q3;
#else
#pragma unroll 1
    for (int r = 1; r < 14; ++r) {
        const uint4 k = KFEC_OCB_KSGPR ? key_at(key->OCB_RKEY, r) : t.OCB_RKEY[r];
        const uint32_t t0 = tcol(t.te, c4, s0, s1, s2, s3, k.x);
        const uint32_t v0 = tcol(t.te, c4, u0, u1, u2, u3, k.x);
        const uint32_t t1 = tcol(t.te, c4, s1, s2, s3, s0, k.y);
        const uint32_t v1 = tcol(t.te, c4, u1, u2, u3, u0, k.y);
        const uint32_t t2 = tcol(t.te, c4, s2, s3, s0, s1, k.z);
        const uint32_t v2 = tcol(t.te, c4, u2, u3, u0, u1, k.z);
        const uint32_t t3 = tcol(t.te, c4, s3, s0, s1, s2, k.w);
        const uint32_t v3 = tcol(t.te, c4, u3, u0, u1, u2, k.w);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        u0 = v0; u1 = v1; u2 = v2; u3 = v3;
    }
#endif
    const uint4 k = t.rk[14];
    const uint32_t (*T)[2][kRep] = t.te;
    auto last = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
        return sbox_col(rep_at<0, 0>(T, a0, c4), rep_at<0, 1>(T, a1, c4), rep_at<0, 2>(T, a2, c4), rep_at<0, 3>(T, a3, c4));
    };
    x = make_uint4(last(s0, s1, s2, s3) ^ k.x, last(s1, s2, s3, s0) ^ k.y, last(s2, s3, s0, s1) ^ k.z, last(s3, s0, s1, s2) ^ k.w);
    y = make_uint4(last(u0, u1, u2, u3) ^ k.x, last(u1, u2, u3, u0) ^ k.y, last(u2, u3, u0, u1) ^ k.z, last(u3, u0, u1, u2) ^ k.w);
}

__device__ __forceinline__ void aes_dec2(const OcbLds<true> &t, const OcbKey *key, uint32_t c4, uint4 &x, uint4 &y)
{
    uint32_t s0 = x.x ^ t.dk[0].x, s1 = x.y ^ t.dk[0].y, s2 = x.z ^ t.dk[0].z, s3 = x.w ^ t.dk[0].w;
    uint32_t u0 = y.x ^ t.dk[0].x, u1 = y.y ^ t.dk[0].y, u2 = y.z ^ t.dk[0].z, u3 = y.w ^ t.dk[0].w;
#if KFEC_OCB_PAIR
    auto round = [&](int r, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t b0, uint32_t b1,
                     uint32_t b2, uint32_t b3, uint32_t &o0, uint32_t &o1, uint32_t &o2, uint32_t &o3, uint32_t &e0,
                     uint32_t &e1, uint32_t &e2, uint32_t &e3) {
        const uint4 k = KFEC_OCB_KSGPR ? key_at(key->OCB_DKEY, r) : t.OCB_DKEY[r];
        o0 = tcol(t.td, c4, a0, a3, a2, a1, k.x);
        e0 = tcol(t.td, c4, b0, b3, b2, b1, k.x);
        o1 = tcol(t.td, c4, a1, a0, a3, a2, k.y);
        e1 = tcol(t.td, c4, b1, b0, b3, b2, k.y);
        o2 = tcol(t.td, c4, a2, a1, a0, a3, k.z);
        e2 = tcol(t.td, c4, b2, b1, b0, b3, k.z);
        o3 = tcol(t.td, c4, a3, a2, a1, a0, k.w);
        e3 = tcol(t.td, c4, b3, b2, b1, b0, k.w);
    };
    uint32_t p0, p1, p2, p3, q0, q1, q2, q3;
    round(1, s0, s1, s2, s3, u0, u1, u2, u3, p0, p1, p2, p3, q0, q1, q2, q3);
#pragma unroll 1
    for (int r = 2; r < 14; r += 2) {
        round(r, p0, p1, p2, p3, q0, q1, q2, q3, s0, s1, s2, s3, u0, u1, u2, u3);
        round(r + 1, s0, s1, s2, s3, u0, u1, u2, u3, p0, p1, p2, p3, q0, q1, q2, q3);
    }
    s0 = p0; s1 = p1; s2 = p2; s3 = p3;
    u0 = q0; u1 = q1; u2 = q2; u3 = q3;
#else
#pragma unroll 1
    for (int r = 1; r < 14; ++r) {
        const uint4 k = KFEC_OCB_KSGPR ? key_at(key->OCB_DKEY, r) : t.OCB_DKEY[r];
        const uint32_t t0 = tcol(t.td, c4, s0, s3, s2, s1, k.x);
        const uint32_t v0 = tcol(t.td, c4, u0, u3, u2, u1, k.x);
        const uint32_t t1 = tcol(t.td, c4, s1, s0, s3, s2, k.y);
        const uint32_t v1 = tcol(t.td, c4, u1, u0, u3, u2, k.y);
        const uint32_t t2 = tcol(t.td, c4, s2, s1, s0, s3, k.z);
        const uint32_t v2 = tcol(t.td, c4, u2, u1, u0, u3, k.z);
        const uint32_t t3 = tcol(t.td, c4, s3, s2, s1, s0, k.w);
        const uint32_t v3 = tcol(t.td, c4, u3, u2, u1, u0, k.w);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        u0 = v0; u1 = v1; u2 = v2; u3 = v3;
    }
#endif
    const uint4 k = t.dk[14];
    auto last = [&](uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
        return isb_col(t, c4, a0, a1, a2, a3);
    };
    x = make_uint4(last(s0, s3, s2, s1) ^ k.x, last(s1, s0, s3, s2) ^ k.y, last(s2, s1, s0, s3) ^ k.z, last(s3, s2, s1, s0) ^ k.w);
    y = make_uint4(last(u0, u3, u2, u1) ^ k.x, last(u1, u0, u3, u2) ^ k.y, last(u2, u1, u0, u3) ^ k.z, last(u3, u2, u1, u0) ^ k.w);
}

template <class Lds>
__device__ __forceinline__ uint4 ocb_offset(const Lds &t, uint4 o0, uint32_t i)
{
    uint32_t g = i ^ (i >> 1);
    while (g) {
        o0 = u4_xor(o0, t.l[__builtin_ctz(g)]);
        g &= g - 1;
    }
    return o0;
}

// A row's work per packet is its full blocks, spread over the 8 lanes, plus up to two enciphers that only one
// lane can do: the pad of a partial last block, E_K(Offset_*), and the tag.  A lane that takes a different code
// path makes the whole wave wait for it, so done per packet those two cost the row two extra AES times on top
// of the ~12 it spends on 91 blocks (fec-sized 1449-byte packets).  Instead a row takes its packets 8 at a time:
// the full blocks of each packet in turn, then lane b finishes packet b of the batch -- pad, checksum, tag --
// so the pads of 8 packets cost one AES time, and so do their tags.
template <bool OPEN>
__global__ void __launch_bounds__(kOcbBlock, 4) ocb_kernel(OcbArgs a)  // (4 waves per SIMD: two 512-lane or one 1024-lane workgroup per CU)
{
    __shared__ OcbLds<OPEN> s;
    {
        // stage the round keys, L values and tables (open: the decryption half and Te0 once)
        const uint32_t *k32 = reinterpret_cast<const uint32_t *>(a.key);
        uint32_t *s32 = reinterpret_cast<uint32_t *>(s.rk);
        constexpr int kKeys = (int)((offsetof(OcbLds<OPEN>, l) - offsetof(OcbLds<OPEN>, rk)) / 4) + 32 * 4;
        for (int i = threadIdx.x; i < kKeys; i += kOcbBlock) {
            // OcbLds: rk, dk, l -- OcbKey: rk, dk, lstar, ldollar, l
            const int src = i < 120 ? i : i + 8;
            s32[i] = k32[src];
        }
        uint32_t *r32 = reinterpret_cast<uint32_t *>(s.rkr);  // rkr then dkr, as rk then dk
        for (int i = threadIdx.x; i < 120; i += kOcbBlock) r32[i] = rotl(k32[i], 16);
        if constexpr (OPEN) {
            for (int i = threadIdx.x; i < 2 * 256 * kRep; i += kOcbBlock)
                s.td[i / (2 * kRep)][i / kRep % 2][i % kRep] = a.key->td[i / kRep % 2][i / (2 * kRep)];
#if KFEC_OCB_T4
            for (int i = threadIdx.x; i < 2 * 256 * kRep; i += kOcbBlock)
                s.td23[i / (2 * kRep)][i / kRep % 2][i % kRep] = a.key->td[2 + i / kRep % 2][i / (2 * kRep)];
#endif
#if KFEC_OCB_ISB4
            for (int i = threadIdx.x; i < 256 * 8; i += kOcbBlock) s.isb4[i / 8][i % 8] = a.key->isb[i / 8] * 0x01010101u;
#else
            for (int i = threadIdx.x; i < 64 * kRep; i += kOcbBlock) {
                const int w = i / kRep;
                s.isb[w][i % kRep] = a.key->isb[4 * w] | a.key->isb[4 * w + 1] << 8 | a.key->isb[4 * w + 2] << 16 |
                                     a.key->isb[4 * w + 3] << 24;
            }
#endif
            for (int i = threadIdx.x; i < 256; i += kOcbBlock) s.te0[i] = a.key->te[0][i];
        } else {
            for (int i = threadIdx.x; i < 2 * 256 * kRep; i += kOcbBlock)
                s.te[i / (2 * kRep)][i / kRep % 2][i % kRep] = a.key->te[i / kRep % 2][i / (2 * kRep)];
#if KFEC_OCB_T4
            for (int i = threadIdx.x; i < 2 * 256 * kRep; i += kOcbBlock)
                s.te23[i / (2 * kRep)][i / kRep % 2][i % kRep] = a.key->te[2 + i / kRep % 2][i / (2 * kRep)];
#endif
        }
        __syncthreads();
    }
    const uint4 lstar = a.key->lstar, ldollar = a.key->ldollar, sad = a.key->sad;
    const uint32_t lane = threadIdx.x % kRow, c = 4 * (threadIdx.x % kRep);  // c: this lane's table copy, in bytes
    const uint64_t stride = (uint64_t)gridDim.x * kRowsPerBlock;
    for (uint64_t p0 = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRow; p0 < a.P; p0 += kRow * stride) {
        // lane b's packet of the batch: what its tail needs
        bool t_on = false;       // a packet to finish (valid length)
        uint64_t t_p = 0, t_off = 0;
        uint32_t t_n = 0, t_iv = 0;
        uint4 t_sum = make_uint4(0u, 0u, 0u, 0u), t_fo = t_sum, t_part = t_sum, t_ptag = t_sum;
        for (uint32_t b = 0; b < kRow; ++b) {
            const uint64_t p = p0 + b * stride;
            if (p >= a.P) break;  // (uniform over the row)
            const uint32_t L = a.len[p];
            const uint64_t off = a.off[p];
            uint32_t n, iv;
            if (OPEN) {
                if (L < KFEC_AEAD_OVERHEAD || L - KFEC_AEAD_OVERHEAD > a.dst_pitch) {
                    if (lane == 0) {
                        a.out_len[p] = 0;
                        a.ok[p] = 0;
                    }
                    continue;
                }
                n = L - KFEC_AEAD_OVERHEAD;
                iv = lane == b ? load16(a.src, a.src_dw, off + n + 16).x & 0xFFFFu : 0u;
            } else {
                if (L == 0 || (uint64_t)L + KFEC_AEAD_OVERHEAD > a.dst_pitch) {  // "empty data" / no room
                    if (lane == 0) a.out_len[p] = 0;
                    continue;
                }
                n = L;
                iv = a.iv[p];
            }
            if (OPEN) iv = __shfl(iv, b, kRow);
            const uint4 o0 = a.off0[iv];
            const uint32_t m = n / 16, rem = n % 16;
            uint8_t *dst = a.dst + p * a.dst_pitch;
            uint4 sum = make_uint4(0u, 0u, 0u, 0u);
#if KFEC_OCB_ILP == 2
            for (uint32_t i = 1 + lane; i <= m; i += 2 * kRow) {  // blocks i and i + 8 (1-based) together
                const bool two = i + kRow <= m;
                const uint32_t j = two ? i + kRow : i;
                const uint4 ia = load16(a.src, a.src_dw, off + 16 * (i - 1));
                const uint4 ib = load16(a.src, a.src_dw, off + 16 * (j - 1));
                const uint4 oa = ocb_offset(s, o0, i), ob = ocb_offset(s, o0, j);
                uint4 xa = u4_xor(ia, oa), xb = u4_xor(ib, ob);
                if constexpr (OPEN) aes_dec2(s, a.key, c, xa, xb);
                else aes_enc2(s, a.key, c, xa, xb);
                xa = u4_xor(xa, oa);
                xb = u4_xor(xb, ob);
                if constexpr (OPEN) {
                    sum = u4_xor(sum, xa);
                    if (two) sum = u4_xor(sum, xb);
                } else {
                    sum = u4_xor(sum, ia);
                    if (two) sum = u4_xor(sum, ib);
                }
                *reinterpret_cast<uint4 *>(dst + 16 * (i - 1)) = xa;
                if (two) *reinterpret_cast<uint4 *>(dst + 16 * (j - 1)) = xb;
            }
#else
            for (uint32_t i = 1 + lane; i <= m; i += kRow) {  // the full blocks (1-based index)
                const uint32_t qb = 16 * (i - 1);
                const uint4 in = load16(a.src, a.src_dw, off + qb);
                const uint4 oi = ocb_offset(s, o0, i);
                uint4 out;
                if constexpr (OPEN) {
                    out = u4_xor(aes_dec(s, c, u4_xor(in, oi)), oi);
                    sum = u4_xor(sum, out);
                } else {
                    out = u4_xor(aes_enc(s, c, u4_xor(in, oi)), oi);
                    sum = u4_xor(sum, in);
                }
                *reinterpret_cast<uint4 *>(dst + qb) = out;
            }
#endif
#pragma unroll
            for (int d = 1; d < kRow; d <<= 1) {
                sum.x ^= __shfl_xor(sum.x, d, kRow);
                sum.y ^= __shfl_xor(sum.y, d, kRow);
                sum.z ^= __shfl_xor(sum.z, d, kRow);
                sum.w ^= __shfl_xor(sum.w, d, kRow);
            }
            if (lane == b) {
                t_on = true;
                t_p = p;
                t_off = off;
                t_n = n;
                t_iv = iv;
                t_sum = sum;
                // Offset_* = Offset_m, xor L_* after a partial block: the pad's input and the tag's offset
                t_fo = ocb_offset(s, o0, m);
                if (rem) {
                    t_fo = u4_xor(t_fo, lstar);
                    t_part = mask16(load16(a.src, a.src_dw, off + 16 * m), rem);
                }
                if (OPEN) t_ptag = load16(a.src, a.src_dw, off + n);
            }
        }
        // lane b finishes packet b: the pads of the row's packets in one AES time, then their tags in another
        const uint32_t rem = t_n % 16, m = t_n / 16;
        const uint4 pad = aes_enc(s, c, t_fo);
        uint8_t *dst = a.dst + t_p * a.dst_pitch;
        if (t_on && rem) {
            const uint4 out = mask16(u4_xor(t_part, pad), rem);
            const uint4 pt = OPEN ? out : t_part;
            uint32_t w[4] = {pt.x, pt.y, pt.z, pt.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) w[q] |= (uint32_t)q == rem / 4 ? 0x80u << (8 * (rem % 4)) : 0u;
            t_sum = u4_xor(t_sum, make_uint4(w[0], w[1], w[2], w[3]));
            const uint32_t o4[4] = {out.x, out.y, out.z, out.w};
            uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + 16 * m);
            // open: whole dwords (the zero pad is part of the output); seal: bytes below n only
            const uint32_t nd = OPEN ? (rem + 3) / 4 : rem / 4;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((uint32_t)q < nd) d32[q] = o4[q];
            if (!OPEN && (rem & 3)) {
                uint8_t *bp = dst + 16 * m + 4 * (rem / 4);
                for (uint32_t q = 0; q < (rem & 3); ++q) bp[q] = (uint8_t)(o4[rem / 4] >> (8 * q));
            }
        }
        // Tag = E_K(Checksum xor Offset_* xor L_$) xor HASH(K, A)
        const uint4 tg = u4_xor(aes_enc(s, c, u4_xor(u4_xor(t_sum, t_fo), ldollar)), sad);
        if (!t_on) continue;
        if (OPEN) {
            const bool good = tg.x == t_ptag.x && tg.y == t_ptag.y && tg.z == t_ptag.z && tg.w == t_ptag.w;
            if (!good) {  // no unauthenticated plaintext leaves the kernel (the row's stores came first)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
                const uint32_t nd = (t_n + 3) / 4;
                for (uint32_t i = 0; i < nd; ++i) d32[i] = 0u;
            }
            a.out_len[t_p] = good ? t_n : 0u;
            a.ok[t_p] = good ? 1 : 0;
        } else {
            // tag || iv_raw || zeros to the next multiple of 4: bytes n .. round4(n + 18)
            const uint32_t tag[4] = {tg.x, tg.y, tg.z, tg.w};
            const uint32_t end = (t_n + KFEC_AEAD_OVERHEAD + 3) & ~3u;
            for (uint32_t i = 0; t_n + i < end; ++i) {
                const uint32_t w = i < 4 ? tag[0] : i < 8 ? tag[1] : i < 12 ? tag[2] : i < 16 ? tag[3] : t_iv;
                dst[t_n + i] = (uint8_t)(i < 18 ? (w >> (8 * (i & 3))) & 0xFFu : 0u);
            }
            a.out_len[t_p] = t_n + KFEC_AEAD_OVERHEAD;
        }
        (void)t_off;
    }
    count_workgroup_done(a.done);
}

}  // namespace

int ocb_setup(kfec_aead *k, const uint32_t *d_key, hipStream_t s)
{
    if (hipMalloc(&k->d_ocb, sizeof(OcbKey)) != hipSuccess || hipMalloc(&k->d_ivt, 65536 * 16) != hipSuccess)
        return KFEC_ENOMEM;
    OcbKey *ok = reinterpret_cast<OcbKey *>(k->d_ocb);
    hipLaunchKernelGGL(ocb_key_kernel, dim3(1), dim3(64), 0, s, d_key, ok);
    hipLaunchKernelGGL(ocb_tables_kernel, dim3(1), dim3(256), 0, s, ok);
    hipLaunchKernelGGL(ocb_iv_kernel, dim3(65536 / 256), dim3(256), 0, s, d_key,
                       reinterpret_cast<uint4 *>(k->d_ivt));
    return hipGetLastError() == hipSuccess ? KFEC_OK : KFEC_EHIP;
}

int launch_ocb(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
               const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
               hipStream_t s, uint32_t *done, uint32_t *blocks)
{
    if (blocks) *blocks = 0;
    if (P == 0) return 0;
    OcbArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.iv = iv;
    a.dst = static_cast<uint8_t *>(dst);
    a.dst_pitch = dst_pitch;
    a.out_len = out_len;
    a.ok = ok;
    a.key = reinterpret_cast<const OcbKey *>(k->d_ocb);
    a.off0 = reinterpret_cast<const uint4 *>(k->d_ivt);
    a.P = P;
    a.done = done;
    const int cus = current_device_cus();
    // one workgroup per resident slot (LDS tables and VGPRs decide how many fit on a CU)
    auto occupancy = [](const void *f) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, kOcbBlock, 0) != hipSuccess || b < 1) b = 1;
        return b;
    };
    static const int fit_open = occupancy(reinterpret_cast<const void *>(&ocb_kernel<true>));  // thread-safe init
    static const int fit_seal = occupancy(reinterpret_cast<const void *>(&ocb_kernel<false>));
    const int fit = open ? fit_open : fit_seal;
    const uint64_t want = (P + kRowsPerBlock - 1) / kRowsPerBlock;
    const dim3 grid((uint32_t)std::min<uint64_t>(want, (uint64_t)cus * fit));
    if (blocks && done) *blocks = grid.x;
    if (open) hipLaunchKernelGGL(ocb_kernel<true>, grid, dim3(kOcbBlock), 0, s, a);
    else hipLaunchKernelGGL(ocb_kernel<false>, grid, dim3(kOcbBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace kfec
