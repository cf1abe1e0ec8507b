// kfec_seal.hip -- the per-packet integrity step either side of FEC on the wire,
// for kcptube's non-AEAD encryption modes:
//   encrypt_data (data_operations.cpp:171-234), modes "none" (default branch) and plain_xor:
//     append checksum16(data) (simple_hashing.hpp:10-25: CRC-32 of the data, its two 16-bit halves XORed),
//     then, for plain_xor, xor_forward over data + checksum (data_operations.cpp:120-128).
//   decrypt_data (data_operations.cpp:373-435): plain_xor first undoes xor_backward (:140-148), then the
//     trailing two bytes are compared with checksum16 of the rest.
// (The AEAD modes are kfec_aead.hip / kfec_gcm.hip / kfec_ocb.hip.)
//
// Half a wave per packet (see "parallel CRC-32" below): each lane owns 16-byte chunks, chunk CRCs are
// combined with GF(2)-linear shift tables, so a packet's bytes are read with 16-byte loads by consecutive
// lanes instead of serially by one thread.  CRC-32 is reflected, polynomial 0xEDB88320, init and final XOR
// 0xFFFFFFFF (Botan's "CRC32").  xor_forward is out[i] = in[i] ^ in[i+1]; xor_backward is the suffix XOR
// out[i] = XOR_{k >= i} in[k] = T ^ (exclusive prefix XOR), T the XOR of all bytes: a lane-level scan.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>

#include "../../include/kfec_frame.h"
#include "kfec_count.hpp"
#include "kfec_internal.hpp"

namespace kfec {

namespace {

constexpr int kSealBlock = 512;  // 16 packets share one LDS copy of the tables

struct Crc32Tables {
    uint32_t t[4][256];
};

constexpr Crc32Tables make_crc32_tables()
{
    Crc32Tables c{};
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t v = i;
        for (int b = 0; b < 8; ++b) v = (v >> 1) ^ ((v & 1u) ? 0xEDB88320u : 0u);
        c.t[0][i] = v;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i) c.t[k][i] = (c.t[k - 1][i] >> 8) ^ c.t[0][c.t[k - 1][i] & 0xFFu];
    return c;
}

__constant__ Crc32Tables c_crc = make_crc32_tables();

// ---- parallel CRC-32 -------------------------------------------------------------------------------
// Half a wave (32 lanes) per packet; lane l takes the 16-byte chunk l of each 512-byte round, computes its raw
// CRC (zero init, slicing-by-16) and folds it into its own running sum across rounds (Horner with shift_512);
// the 32 lanes' sums are combined once per packet:
//   CRC(A || B) = shift_|B|(CRC(A)) ^ CRC(B),   shift_d(r) = r advanced through d zero bytes,
// a GF(2)-linear map (linearity makes the per-lane sums combine exactly like one round's chunk CRCs).  The
// streaming rows right-align the message into the rounds (leading zero bytes leave a CRC computed from a zero
// register unchanged); the register rows left-align it and take the trailing zeros back out at the end
// (unshift).  The standard 0xFFFFFFFF init is folded in by complementing the first 4 message bytes (messages
// >= 4 bytes; shorter ones run serially on one lane), and the result is complemented at the end.
constexpr int kRowLanes = 32;
constexpr int kCrcLane = 16;                       // bytes of a round per lane
constexpr int kCrcRound = kCrcLane * kRowLanes;    // 512 B
#ifndef KFEC_SEAL_BATCH
#define KFEC_SEAL_BATCH 1  // >1 issues several rounds' loads together but the compiler then needs 134-150 VGPRs
#endif
#ifndef KFEC_SEAL_U4
#define KFEC_SEAL_U4 1
#endif
#ifndef KFEC_SEAL_SHFL
#define KFEC_SEAL_SHFL 1
#endif
constexpr int kCrcBatch = KFEC_SEAL_BATCH;         // rounds whose loads are issued together
constexpr int kRowsPerBlock = kSealBlock / kRowLanes;

#ifndef KFEC_SEAL_REG
#define KFEC_SEAL_REG 1  // 0: every packet takes the streaming rows (A/B knob)
#endif

#ifndef KFEC_SEAL_PREFETCH
#define KFEC_SEAL_PREFETCH 1  // 0: no kernel prefetches the next packet (A/B knob)
#endif
#ifndef KFEC_SEAL_OPEN_PF
#define KFEC_SEAL_OPEN_PF 1  // 0: open loads each packet when it reaches it (A/B knob)
#endif
#ifndef KFEC_SEAL_AB
#define KFEC_SEAL_AB 0  // ablation (timing only, wrong results): 1 = the register rows skip the CRC
#endif

// The CRC tables each workgroup stages into LDS (60 KiB; all maps GF(2)-linear, so table lookups of the
// input's bytes XORed together):
//   s16[k][v]:   raw CRC (zero init) of a 16-byte chunk with byte v at position k and zeros elsewhere
//                (slicing-by-16: a chunk's CRC is 16 independent lookups; s16[12..15] are slicing-by-4's tables)
//   sh[m][j][v]: byte j = v of a CRC register advanced through 16 << m zero bytes (m = 5: Horner over rounds;
//                m < 5: the in-place kernel's butterfly)
//   col[i][l]:   register bit i of row lane l advanced past the 31 - l chunks of its round after it, so the
//                row's 32 lane sums combine as XOR_l XOR_i bit_i(R_l) col[i][l]: one conflict-free lookup
//                per bit (lane l reads bank l) and no dependent chain, instead of a 5-level tree of shifts
// Measured and dropped: per-lane copies of the bytewise table and a diagonal layout of s16 (both
// conflict-free, both slower: dependent chains / a per-lane byte rotation), nibble tables (conflict-free, twice
// the lookups and a third more VALU: slower).
struct CrcLds {
    uint32_t s16[16][256];
    uint32_t sh[6][4][256];
    uint32_t col[32][kRowLanes];
};
constexpr int kCrcWords = (int)(sizeof(CrcLds) / 4);
// what the in-place kernel stages (28 KiB, for its occupancy): slicing-by-4's tables (s16[12..15]) and sh
struct CrcLdsIP {
    uint32_t s4[4][256];
    uint32_t sh[6][4][256];
};
__device__ __forceinline__ const uint32_t (*s4_of(const CrcLds &t))[256] { return t.s16 + 12; }
__device__ __forceinline__ const uint32_t (*s4_of(const CrcLdsIP &t))[256] { return t.s4; }
// after the LDS tables, in global memory only (one row of 32 dwords read per packet): unshift[d][i] = the CRC
// register 1 << i taken back through d zero bytes (d < 512) -- the inverse of advancing it, which exists
// because the reflected CRC-32 table's top bytes T[v] >> 24 are a permutation of v
constexpr int kUnshiftWords = kCrcRound * 32;
constexpr int kTabWords = kCrcWords + kUnshiftWords;

struct InvTop {
    uint8_t v[256];
};
constexpr InvTop make_inv_top()
{
    InvTop r{};
    const Crc32Tables c = make_crc32_tables();
    for (uint32_t i = 0; i < 256; ++i) r.v[c.t[0][i] >> 24] = (uint8_t)i;
    return r;
}
__constant__ InvTop c_inv_top = make_inv_top();

__device__ uint32_t advance(uint32_t r, int d)  // r through d zero bytes
{
    for (int i = 0; i < d; ++i) r = (r >> 8) ^ c_crc.t[0][r & 0xFFu];
    return r;
}

__global__ void crc_tables_kernel(uint32_t *tab)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    constexpr int kS16 = 16 * 256, kSh = kS16 + 6 * 4 * 256;
    uint32_t r;
    if (e < kS16) {  // s16[k][v]
        r = advance(c_crc.t[0][e & 255], 15 - e / 256);
    } else if (e < kSh) {  // sh[m][j][v]
        const int f = e - kS16, m = f / 1024, j = (f / 256) & 3, v = f & 255;
        r = advance((uint32_t)v << (8 * j), kCrcLane << m);
    } else if (e < kCrcWords) {
        const int f = e - kSh, i = f / kRowLanes, l = f % kRowLanes;
        r = advance(1u << i, kCrcLane * (kRowLanes - 1 - l));
    } else if (e < kTabWords) {  // unshift[d][i]: undo d single-byte steps r' = (r >> 8) ^ T[r & 0xFF]
        const int d = (e - kCrcWords) / 32, i = (e - kCrcWords) % 32;
        r = 1u << i;
        for (int k = 0; k < d; ++k) {
            const uint32_t b = c_inv_top.v[r >> 24];
            r = ((r ^ c_crc.t[0][b]) << 8) | b;
        }
    } else {
        return;
    }
    tab[e] = r;
}

// raw CRC (zero init) of the 16-byte chunk o: 16 independent lookups (slicing-by-16)
__device__ __forceinline__ uint32_t crc_chunk(const CrcLds &t, const uint32_t (&o)[4], uint32_t)
{
    uint32_t c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        c[i] = t.s16[4 * i][o[i] & 0xFFu] ^ t.s16[4 * i + 1][(o[i] >> 8) & 0xFFu] ^
               t.s16[4 * i + 2][(o[i] >> 16) & 0xFFu] ^ t.s16[4 * i + 3][o[i] >> 24];
    return c[0] ^ c[1] ^ c[2] ^ c[3];
}

// the same by slicing-by-4 (a chain of 4 steps, s16[12..15] as its tables): fewer VALU, for the in-place kernel
template <class T>
__device__ __forceinline__ uint32_t crc_chunk4(const T &t, const uint32_t (&o)[4])
{
    const uint32_t (*s)[256] = s4_of(t);
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = c ^ o[i];
        c = s[0][x & 0xFFu] ^ s[1][(x >> 8) & 0xFFu] ^ s[2][(x >> 16) & 0xFFu] ^ s[3][x >> 24];
    }
    return c;
}

// the register r advanced through 16 << m zero bytes
template <class T>
__device__ __forceinline__ uint32_t crc_shift(const T &t, int m, uint32_t r)
{
    const uint32_t (*s)[256] = t.sh[m];
    return s[0][r & 0xFFu] ^ s[1][(r >> 8) & 0xFFu] ^ s[2][(r >> 16) & 0xFFu] ^ s[3][r >> 24];
}

__device__ __forceinline__ uint32_t crc_shift512(const CrcLds &t, uint32_t r) { return crc_shift(t, 5, r); }

// the 32 lane sums of a row, each advanced past the chunks after it in the round (col), XORed over the row
__device__ __forceinline__ uint32_t row_combine(const CrcLds &t, uint32_t R, uint32_t lane)
{
    uint32_t Z = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) Z ^= (uint32_t)((int32_t)(R << (31 - i)) >> 31) & t.col[i][lane];
#pragma unroll
    for (int k = 0; k < 5; ++k) Z ^= __shfl_xor(Z, 1 << k, kRowLanes);
    return Z;
}

template <class T>
__device__ __forceinline__ uint32_t crc_byte(const T &t, uint32_t c, uint32_t byte)
{
    return (c >> 8) ^ s4_of(t)[3][(c ^ byte) & 0xFFu];
}

// 16 bytes [q0, q0 + 16) of base[start, start + len), zero outside (dword-aligned base, dwords < lim32):
// one 16-byte load at the covering dword (dword alignment suffices on gfx950) and one more dword
__device__ __forceinline__ void chunk16(const uint32_t *base32, uint64_t lim32, uint64_t start, uint32_t len,
                                        int32_t q0, uint32_t (&o)[4])
{
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = 0u;
    if (q0 + 16 <= 0 || q0 >= (int32_t)len) return;
    const uint64_t a4 = start + (uint64_t)(int64_t)(q0 + 16);
    const uint64_t w4 = a4 >> 2;
    const uint32_t sh = (uint32_t)(a4 & 3u);
    uint32_t d[5];
    if (KFEC_SEAL_U4 && w4 >= 4 && w4 + 1 <= lim32) {
        const uint4 x = *reinterpret_cast<const uint4 *>(base32 + (w4 - 4));
        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
        d[4] = (sh && w4 < lim32) ? base32[w4] : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint64_t w = w4 - 4 + i;
            d[i] = (w4 + i >= 4 && w < lim32) ? base32[w] : 0u;
        }
    }
    const int lo = max(0, -q0), hi = min(16, (int32_t)len - q0);  // valid bytes [lo, hi) of the chunk
    const uint32_t M = ((1u << hi) - 1u) & ~((1u << lo) - 1u);    // one bit per valid byte (branch-free masks)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;  // bit b of nib -> byte b
        o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & bm;
    }
}

// standard CRC-32 of base[start, start + len), computed by the 32 lanes of a row (all lanes get it)
__device__ __forceinline__ uint32_t row_crc32(const CrcLds &tab, const uint32_t *base32, uint64_t lim32, uint64_t start,
                              uint32_t len, uint32_t lane)
{
    if (len < 4) {  // the init cannot be folded into message bytes: one lane, byte by byte
        uint32_t c = 0xFFFFFFFFu;
        if (lane == 0) {
            uint32_t o[4];
            chunk16(base32, lim32, start, len, 0, o);
            for (uint32_t i = 0; i < len; ++i) c = crc_byte(tab, c, o[0] >> (8 * i));
        }
        return ~__shfl(c, 0, kRowLanes);
    }
    const uint32_t rounds = (len + kCrcRound - 1) / kCrcRound, pad = rounds * kCrcRound - len;
    uint32_t R = 0;
    for (uint32_t r0 = 0; r0 < rounds; r0 += kCrcBatch) {
        // issue the loads of up to kCrcBatch rounds before the dependent CRC chains: latency, not LDS, bounds
        // this kernel (measured: one round in flight per row ran at 2.0-2.2 TB/s)
        uint32_t o[kCrcBatch][4];
#pragma unroll
        for (int u = 0; u < kCrcBatch; ++u) {
            const int32_t q0 = (int32_t)((r0 + u) * kCrcRound + kCrcLane * lane) - (int32_t)pad;
            chunk16(base32, lim32, start, len, r0 + u < rounds ? q0 : (int32_t)len, o[u]);
            if (q0 <= 3 && q0 > -16) {  // complement message bytes 0..3 (the 0xFFFFFFFF init)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int32_t q = q0 + 4 * i + b;
                        if (q >= 0 && q < 4) o[u][i] ^= 0xFFu << (8 * b);
                    }
            }
        }
#pragma unroll
        for (int u = 0; u < kCrcBatch; ++u) {  // fixed trip count (a break here sent o[][] to scratch)
            const uint32_t c = crc_chunk(tab, o[u], lane);
            // Horner over this lane's chunks: R = XOR_r shift_{(rounds-1-r)*512}(chunk CRC of round r)
            if (r0 + u < rounds) R = crc_shift512(tab, R) ^ c;
        }
    }
    // by linearity the 32 lanes' Horner sums combine exactly as one round's chunk CRCs do
    R = row_combine(tab, R, lane);
    return ~R;
}

// row_crc32 in the round-1 form the in-place kernel measures fastest with (`tools/gpu_seal_ab.sh`, same call:
// 1.97-2.00 ms against 2.06-2.16 for the register rows, where nothing else hides the CRC): slicing-by-4
// chains and a butterfly of shift maps, fewer VALU than slicing-by-16 and the column combine
template <class T>
__device__ __forceinline__ uint32_t row_crc32_bf(const T &tab, const uint32_t *base32, uint64_t lim32, uint64_t start,
                                                 uint32_t len, uint32_t lane)
{
    if (len < 4) {  // the init cannot be folded into message bytes: one lane, byte by byte
        uint32_t c = 0xFFFFFFFFu;
        if (lane == 0) {
            uint32_t o[4];
            chunk16(base32, lim32, start, len, 0, o);
            for (uint32_t i = 0; i < len; ++i) c = crc_byte(tab, c, o[0] >> (8 * i));
        }
        return ~__shfl(c, 0, kRowLanes);
    }
    const uint32_t rounds = (len + kCrcRound - 1) / kCrcRound, pad = rounds * kCrcRound - len;
    uint32_t R = 0;
    for (uint32_t r = 0; r < rounds; ++r) {
        uint32_t o[4];
        const int32_t q0 = (int32_t)(r * kCrcRound + kCrcLane * lane) - (int32_t)pad;
        chunk16(base32, lim32, start, len, q0, o);
        if (q0 <= 3 && q0 > -16) {  // complement message bytes 0..3 (the 0xFFFFFFFF init)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int32_t q = q0 + 4 * i + b;
                    if (q >= 0 && q < 4) o[i] ^= 0xFFu << (8 * b);
                }
        }
        R = crc_shift(tab, 5, R) ^ crc_chunk4(tab, o);  // Horner over this lane's chunks
    }
    // butterfly: level k, the lane holding the earlier block A shifts it past the later block B (16 << k bytes)
    for (int k = 0; k < 5; ++k) {
        const uint32_t other = __shfl_xor(R, 1 << k, kRowLanes);
        const bool later = lane & (1u << k);
        R = crc_shift(tab, k, later ? other : R) ^ (later ? R : other);
    }
    return ~R;
}

// checksum16 bytes as a little-endian u16 (simple_hashing.hpp:17-23): Botan's CRC32::final_result stores
// the CRC big-endian, and the two 16-bit halves are XORed in host (little-endian) order
__device__ __forceinline__ uint32_t checksum16(uint32_t c)
{
    return (((c >> 24) ^ (c >> 8)) & 0xFFu) | ((((c >> 16) ^ c) & 0xFFu) << 8);
}

// ---- register-resident rows -------------------------------------------------------------------------
// A packet of up to kRegRounds rounds (2 KiB, every kcptube datagram at its MTUs) is loaded whole into
// left-aligned chunks -- lane l holds chunk j = 32 r + l = bytes [16 j, 16 j + 16) of round r -- with every
// load of the row issued before any arithmetic, and the CRC, the xor modes and the output all come from
// those registers: the packet is read once and written once.  (The rows above stream round by round, one
// round in flight per row, and read each packet twice: latency-bound.)  Longer packets take those rows.
constexpr int kRegRounds = 4;
constexpr uint32_t kRegBytes = kRegRounds * kCrcRound;

__device__ uint4 g_zero16;  // never written: the target of the loads a register row does not need

// The register rows load without a branch: both loads of a chunk are always issued, a chunk past the packet
// (or a dword it does not need) reading g_zero16 instead.  A load under a branch makes the compiler wait for
// it at the join (the loaded value is a phi there), which serialised every chunk of a row behind the one
// before.  The bytes past len in the packet's last partial chunk are left for mask_tail(); every window read
// must lie inside the buffer, so row_fits() is checked for the row first.
__device__ __forceinline__ bool row_fits(uint64_t start, uint32_t len, uint64_t lim32)
{
    return ((start + 16 * (uint64_t)((len + 15) / 16)) >> 2) + 1 <= lim32;
}

__device__ __forceinline__ void load_row(const uint32_t *base32, uint64_t start, uint32_t len, uint32_t lane,
                                         uint32_t (&o)[kRegRounds][4])
{
    const uint32_t sh = (uint32_t)(start & 3u);
    const uint32_t *rp = base32 + (start >> 2) + 4 * lane;  // chunk r of this lane: the 5 dwords at rp + 128 r
#pragma unroll
    for (int r = 0; r < kRegRounds; ++r) {
        const bool any = (uint32_t)(r * kCrcRound) + kCrcLane * lane < len;
        const uint4 x = *(any ? reinterpret_cast<const uint4 *>(rp + 128 * r) : &g_zero16);
        const uint32_t x4 = *(any && sh ? rp + 128 * r + 4 : &g_zero16.x);
        o[r][0] = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
        o[r][1] = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
        o[r][2] = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
        o[r][3] = __builtin_amdgcn_alignbyte(x4, x.w, sh);
    }
}

// keep the bytes of chunk o (at packet position q0 >= 0) below len
__device__ __forceinline__ void mask_chunk(uint32_t (&o)[4], int32_t q0, uint32_t len)
{
    const int32_t hi = min(16, max(0, (int32_t)len - q0));
    const uint32_t M = (1u << hi) - 1u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        o[i] &= ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;
    }
}

// zero the bytes at and past len (only the chunk holding position len has any that are not zero already)
__device__ __forceinline__ void mask_tail(uint32_t (&o)[kRegRounds][4], uint32_t len, uint32_t lane)
{
#pragma unroll
    for (int r = 0; r < kRegRounds; ++r) {
        const int32_t q0 = (int32_t)(r * kCrcRound + kCrcLane * lane);
        if (q0 < (int32_t)len && (int32_t)len < q0 + 16) mask_chunk(o[r], q0, len);
    }
}

// byte pos (0 <= pos < 16) of chunk o, through a 128-bit shift: any form that selects o[i] by pos (o[pos >> 2],
// or the selects / conditional updates LLVM turns back into it) sends the whole row to scratch
__device__ __forceinline__ unsigned __int128 as128(const uint32_t (&o)[4])
{
    return (unsigned __int128)o[0] | ((unsigned __int128)o[1] << 32) | ((unsigned __int128)o[2] << 64) |
           ((unsigned __int128)o[3] << 96);
}

__device__ __forceinline__ uint32_t get_byte(const uint32_t (&o)[4], int32_t pos)
{
    return (uint32_t)(as128(o) >> (8 * pos)) & 0xFFu;
}

__device__ __forceinline__ void or_byte(uint32_t (&o)[4], int32_t pos, uint32_t byte)
{
    const unsigned __int128 v = (unsigned __int128)byte << (8 * pos);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] |= (uint32_t)(v >> (32 * i));
}

// standard CRC-32 of the first n bytes held left-aligned in o (bytes at and past n zero).  Horner over the
// rounds and the row combine of row_crc32 give the raw CRC of M || 0^pad, pad = rounds * 512 - n the zero bytes
// that close the last round; one linear map, the unshift by pad (u = row pad of the unshift table on lane i
// (the caller reads it early), bit i of the register on lane i), takes it back to the raw CRC of M.
__device__ __forceinline__ uint32_t crc_regs(const CrcLds &tab, uint32_t u, const uint32_t (&o)[kRegRounds][4],
                                             uint32_t n, uint32_t lane)
{
    if (KFEC_SEAL_AB == 1) return u;
    if (n < 4) {  // the init cannot be folded into message bytes: byte by byte from lane 0's first dword
        uint32_t c = 0xFFFFFFFFu;
        for (uint32_t i = 0; i < n; ++i) c = crc_byte(tab, c, o[0][0] >> (8 * i));
        return ~__shfl(c, 0, kRowLanes);
    }
    const uint32_t rounds = (n + kCrcRound - 1) / kCrcRound;
    uint32_t R = 0;
#pragma unroll
    for (int r = 0; r < kRegRounds; ++r) {
        if ((uint32_t)r < rounds) {
            const uint32_t x[4] = {o[r][0] ^ (r == 0 && lane == 0 ? 0xFFFFFFFFu : 0u), o[r][1], o[r][2], o[r][3]};
            const uint32_t c = crc_chunk(tab, x, lane);
            R = r == 0 ? c : crc_shift512(tab, R) ^ c;  // Horner: R = shift_512(R) ^ chunk CRC
        }
    }
    R = row_combine(tab, R, lane);
    uint32_t v = (R >> lane) & 1u ? u : 0u;
#pragma unroll
    for (int k = 0; k < 5; ++k) v ^= __shfl_xor(v, 1 << k, kRowLanes);
    return ~v;
}

struct SealArgs {
    const uint32_t *src;
    uint64_t src_dw;
    uint64_t src_bytes;
    const uint64_t *off;
    const uint32_t *len;
    uint8_t *dst;
    uint64_t dst_pitch;
    uint32_t *out_len;
    uint8_t *ok;
    const uint32_t *tab;
    const uint32_t *unshift;  // tab + kCrcWords
    uint64_t P;
    int mode;
    uint32_t *done;  // optional completion count in coherent pinned host memory (launch_seal)
};

// The queues' small sealed flushes (kfec_pipeline.cpp, up to kSealCountRows rows) wait for this count instead of
// the stream: every wave waits for its own stores, the workgroup meets at a barrier, and one lane releases at
// system scope and adds the workgroup in (the producer form of MI355X_MICROARCH.md's hand-off recipe, with the
// host as the consumer).  The host sees the rows once the last workgroup has counted itself, without the
// runtime's completion signal and stream wait: one 20:3 group's flush waits 15-16 -> 10-11 us.  With many
// workgroups it loses (16 groups: 24 -> 40 us, whether the release is a system-scope fence in every thread or
// this one per workgroup, and 56 us with every output store written through at system scope instead).
__device__ __forceinline__ void count_done(const SealArgs &a) { count_workgroup_done(a.done); }

__device__ __forceinline__ uint32_t *dst_row(const SealArgs &a, uint64_t p)
{
    return reinterpret_cast<uint32_t *>(a.dst + p * a.dst_pitch);
}

__device__ __forceinline__ void stage_tables(const uint32_t *tab, CrcLds &s_tab)
{
    uint32_t *flat = reinterpret_cast<uint32_t *>(&s_tab);
    for (int i = threadIdx.x; i < kCrcWords; i += kSealBlock) flat[i] = tab[i];
    __syncthreads();
}

// store the dwords of 16-byte chunk j of a row that lie below nd (whole chunk: one 16-byte store)
__device__ __forceinline__ void store_chunk(uint32_t *dst, uint32_t j, uint32_t nd, const uint32_t (&o)[4])
{
    if (4 * j + 4 <= nd) {
        *reinterpret_cast<uint4 *>(dst + 4 * j) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (4 * j + i < nd) dst[4 * j + i] = o[i];
    }
}

// ---- the streaming rows: packets longer than the register rows hold ------------------------------------
__device__ __forceinline__ void seal_stream_row(const SealArgs &a, const CrcLds &s_tab, uint64_t p, uint32_t L,
                                                uint64_t off, uint32_t lane)
{
    const uint32_t n = L + KFEC_SEAL_TRAILER, nd = (n + 3) / 4;
    uint32_t *dst = dst_row(a, p);
    const uint32_t cs = checksum16(row_crc32(s_tab, a.src, a.src_dw, off, L, lane));
    for (uint32_t j0 = 0; 16 * j0 < n; j0 += kRowLanes) {  // whole rounds: the shuffle needs every lane
        const uint32_t j = j0 + lane;
        uint32_t o[5];
        uint32_t q[4];
        chunk16(a.src, a.src_dw, off, L, 16 * (int32_t)j, q);
        o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3];
        // the checksum bytes at S positions L and L + 1 (positions relative to the chunk: c, c + 1)
        const int32_t c = (int32_t)L - 16 * (int32_t)j;
        o[4] = 0u;
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int32_t t = 4 * i + b - c;  // checksum byte index at chunk position 4i + b
                if (t == 0 || t == 1) o[i] |= ((cs >> (8 * t)) & 0xFFu) << (8 * b);
            }
        if (a.mode == KFEC_SEAL_PLAIN_XOR) {
            // S[16j + 16]: the next chunk's first byte -- the next lane's, or a load for the round's last lane
            uint32_t nx = KFEC_SEAL_SHFL ? __shfl_down(o[0], 1, kRowLanes) & 0xFFu : 0u;
            if (!KFEC_SEAL_SHFL || lane == kRowLanes - 1) {
                uint32_t t4[4];
                chunk16(a.src, a.src_dw, off, L, 16 * (int32_t)j + 16, t4);
                nx = t4[0] & 0xFFu;
                const int32_t t0 = c - 16;  // position of S byte L (checksum byte 0) inside the next chunk
                if (t0 == 0) nx = cs & 0xFFu;
                else if (t0 == -1) nx = (cs >> 8) & 0xFFu;
            }
            o[4] |= nx;
        }
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            w[i] = a.mode == KFEC_SEAL_PLAIN_XOR ? o[i] ^ ((o[i] >> 8) | (o[i + 1] << 24)) : o[i];
        if (16 * j < n) store_chunk(dst, j, nd, w);
    }    if (lane == 0) a.out_len[p] = n;
}

__device__ __forceinline__ void open_stream_row(const SealArgs &a, const CrcLds &s_tab, uint64_t p, uint32_t L,
                                                uint64_t off, uint32_t lane)
{
    const bool px = a.mode == KFEC_SEAL_PLAIN_XOR;
    const uint32_t n = L - KFEC_SEAL_TRAILER, nd = (n + 3) / 4;
    // xor_backward: plain[i] = T ^ (XOR of cipher[0..i)), T = XOR of every cipher byte
    uint32_t T = 0;
    if (px) {
        uint32_t x = 0;
        for (uint32_t j = lane; 16 * j < L; j += kRowLanes) {
            uint32_t o[4];
            chunk16(a.src, a.src_dw, off, L, 16 * (int32_t)j, o);
            x ^= o[0] ^ o[1] ^ o[2] ^ o[3];
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) x ^= __shfl_xor(x, 1 << k, kRowLanes);
        x ^= x >> 16;
        x ^= x >> 8;
        T = (x & 0xFFu) * 0x01010101u;
    }
    uint32_t *dst = reinterpret_cast<uint32_t *>(a.dst + p * a.dst_pitch);
    uint32_t carry = 0;    // XOR of the cipher bytes before this round (broadcast byte)
    uint32_t trailer = 0;  // plaintext bytes n, n + 1 (little-endian u16), gathered from the owning lanes
    for (uint32_t j0 = 0; 16 * j0 < L; j0 += kRowLanes) {
        const uint32_t j = j0 + lane;
        uint32_t o[4];
        chunk16(a.src, a.src_dw, off, L, 16 * (int32_t)j, o);
        if (px) {
            // exclusive prefix XOR of the round's chunks across lanes, then bytewise inside the chunk
            uint32_t cx = o[0] ^ o[1] ^ o[2] ^ o[3];
            cx ^= cx >> 16;
            cx ^= cx >> 8;
            cx = (cx & 0xFFu) * 0x01010101u;  // this chunk's XOR, broadcast
            uint32_t incl = cx;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint32_t v = __shfl_up(incl, 1 << k, kRowLanes);
                if (lane >= (1u << k)) incl ^= v;
            }
            uint32_t run = carry ^ incl ^ cx;  // bytes before this chunk
            carry ^= __shfl(incl, kRowLanes - 1, kRowLanes);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t in = o[i] ^ (o[i] << 8);
                in ^= in << 16;  // byte b: XOR of bytes 0..b of this dword
                const uint32_t x = T ^ run ^ (in << 8);
                run ^= (in >> 24) * 0x01010101u;
                o[i] = x;
            }
            // mask to the packet
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t b0 = 16 * (int64_t)j + 4 * i;
                const int64_t k = (int64_t)L - b0;
                if (k <= 0) o[i] = 0u;
                else if (k < 4) o[i] &= (1u << (8 * k)) - 1u;
            }
        }
        // trailer bytes n and n + 1
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int64_t t = 16 * (int64_t)j + 4 * i + b - n;  // trailer byte index at this position
                if (t == 0 || t == 1) trailer |= ((o[i] >> (8 * b)) & 0xFFu) << (8 * t);
            }
        // plaintext bytes below n
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t k = (int64_t)n - (16 * (int64_t)j + 4 * i);
            if (k <= 0) o[i] = 0u;
            else if (k < 4) o[i] &= (1u << (8 * k)) - 1u;
        }
        if (16 * j < n) store_chunk(dst, j, nd, o);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) trailer |= __shfl_xor(trailer, 1 << k, kRowLanes);
    // CRC of the plaintext: for "none" it is the packet's own first n bytes; for plain_xor the plaintext
    // just written (same wave: drain the stores first)
    uint32_t crc;
    if (px) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        crc = row_crc32(s_tab, dst, nd, 0, n, lane);
    } else {
        crc = row_crc32(s_tab, a.src, a.src_dw, off, n, lane);
    }    if (lane == 0) {
        a.out_len[p] = n;
        a.ok[p] = checksum16(crc) == trailer;
    }
}

// ---- the row walker ------------------------------------------------------------------------------------
// Each row takes packets p, p + S, p + 2S, ... (S = the grid's rows) and keeps the next packet's bytes in
// flight while it computes the current one: (len, off) are read two packets ahead, the bytes one ahead
// (load_len(L) of them: 0 for a packet the streaming rows take, or none), and the unshift row of the
// current packet is read before that prefetch is issued, so that waiting for it (vmcnt counts in issue
// order) does not wait for the prefetch.  body(p, L, off, o, u) gets the packet's registers.  PF = false
// loads the packet when the row reaches it (fewer VGPRs: measured faster for open and the in-place kernel,
// prefetch faster for seal).
template <bool PF, class LoadLen, class CrcLen, class Body>
__device__ __forceinline__ void for_each_row(const SealArgs &a, uint32_t lane, LoadLen load_len, CrcLen crc_len, Body body)
{
    const uint64_t S = (uint64_t)gridDim.x * kRowsPerBlock;
    uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRowLanes;
    uint32_t L1 = 0, L2 = 0;
    uint64_t off1 = 0, off2 = 0;
    if (p < a.P) {
        L1 = a.len[p];
        off1 = a.off[p];
    }
    if (p + S < a.P) {
        L2 = a.len[p + S];
        off2 = a.off[p + S];
    }
    uint32_t nx[kRegRounds][4];
    if (PF) load_row(a.src, off1, p < a.P ? load_len(L1, off1) : 0u, lane, nx);
    for (; p < a.P; p += S) {
        const uint32_t L = L1;
        const uint64_t off = off1;
        uint32_t o[kRegRounds][4];
#pragma unroll
        for (int r = 0; r < kRegRounds; ++r)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[r][i] = nx[r][i];
        const uint32_t nc = crc_len(L);
        const uint32_t pad = (kCrcRound - nc % kCrcRound) % kCrcRound;
        const uint32_t u = load_len(L, off) && nc >= 4 ? a.unshift[pad * 32 + lane] : 0u;
        L1 = L2;
        off1 = off2;
        if (p + 2 * S < a.P) {
            L2 = a.len[p + 2 * S];
            off2 = a.off[p + 2 * S];
        }
        if (PF) load_row(a.src, off1, p + S < a.P ? load_len(L1, off1) : 0u, lane, nx);
        else load_row(a.src, off, load_len(L, off), lane, o);
        body(p, L, off, o, u);
    }
}

// the plaintext bytes n, n + 1 (a little-endian u16) from the lanes holding them, on every lane of the row
__device__ __forceinline__ uint32_t row_trailer(const uint32_t (&o)[kRegRounds][4], uint32_t n, uint32_t lane)
{
    uint32_t t = 0;
#pragma unroll
    for (int r = 0; r < kRegRounds; ++r) {
        const int32_t c = (int32_t)n - (int32_t)(r * kCrcRound + kCrcLane * lane);
        if (c >= -1 && c < 16) {
            if (c >= 0) t |= get_byte(o[r], c);
            if (c + 1 < 16) t |= get_byte(o[r], c + 1) << 8;
        }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) t |= __shfl_xor(t, 1 << k, kRowLanes);
    return t;
}

__global__ void __launch_bounds__(kSealBlock) __attribute__((amdgpu_waves_per_eu(4))) seal_kernel(SealArgs a)
{
    __shared__ CrcLds s_tab;
    stage_tables(a.tab, s_tab);
    const uint32_t lane = threadIdx.x % kRowLanes;
    // encrypt_data: "empty data" (:173-174), or no room in dst
    auto valid = [&](uint32_t L) { return L != 0 && L + KFEC_SEAL_TRAILER <= a.dst_pitch; };
    auto load_len = [&](uint32_t L, uint64_t off) {
        return KFEC_SEAL_REG && valid(L) && L + KFEC_SEAL_TRAILER <= kRegBytes && row_fits(off, L, a.src_dw) ? L : 0u;
    };
    auto crc_len = [](uint32_t L) { return L; };
    for_each_row<KFEC_SEAL_PREFETCH != 0>(a, lane, load_len, crc_len, [&](uint64_t p, uint32_t L, uint64_t off, uint32_t (&o)[kRegRounds][4], uint32_t u) {
        if (!valid(L)) {
            if (lane == 0) a.out_len[p] = 0;
            return;
        }
        if (!load_len(L, off)) {
            seal_stream_row(a, s_tab, p, L, off, lane);
            return;
        }
        // sealed packet S = data || cs, xor_forward'ed for plain_xor (out[i] = S[i] ^ S[i + 1])
        const uint32_t n = L + KFEC_SEAL_TRAILER, nd = (n + 3) / 4;
        mask_tail(o, L, lane);
        const uint32_t cs = checksum16(crc_regs(s_tab, u, o, L, lane));
#pragma unroll
        for (int r = 0; r < kRegRounds; ++r) {
            const int32_t c = (int32_t)L - (int32_t)(r * kCrcRound + kCrcLane * lane);  // cs byte 0 at chunk position c
            if (c >= -1 && c < 16) {
                if (c >= 0) or_byte(o[r], c, cs & 0xFFu);
                if (c + 1 < 16) or_byte(o[r], c + 1, cs >> 8);
            }
        }
        uint32_t *dst = dst_row(a, p);
#pragma unroll
        for (int r = 0; r < kRegRounds; ++r) {
            uint32_t w[4] = {o[r][0], o[r][1], o[r][2], o[r][3]};
            if (a.mode == KFEC_SEAL_PLAIN_XOR) {
                // S[16 j + 16]: the next lane's first byte; for the row's last lane, lane 0's of the next round
                const uint32_t down = __shfl_down(o[r][0], 1, kRowLanes);
                const uint32_t wrap = r + 1 < kRegRounds ? __shfl(o[r + 1 < kRegRounds ? r + 1 : r][0], 0, kRowLanes) : 0u;
                const uint32_t next[4] = {o[r][1], o[r][2], o[r][3], (lane == kRowLanes - 1 ? wrap : down) & 0xFFu};
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] ^= (o[r][i] >> 8) | (next[i] << 24);
            }
            const uint32_t j = r * kRowLanes + lane;
            if (16 * j < n) store_chunk(dst, j, nd, w);
        }
        if (lane == 0) a.out_len[p] = n;
    });
    count_done(a);
}

__global__ void __launch_bounds__(kSealBlock) __attribute__((amdgpu_waves_per_eu(4))) open_kernel(SealArgs a)
{
    __shared__ CrcLds s_tab;
    stage_tables(a.tab, s_tab);
    const uint32_t lane = threadIdx.x % kRowLanes;
    const bool px = a.mode == KFEC_SEAL_PLAIN_XOR;
    // decrypt_data: bad length (nothing besides the trailer), or no room in dst
    auto valid = [&](uint32_t L) { return L > KFEC_SEAL_TRAILER && L - KFEC_SEAL_TRAILER <= a.dst_pitch; };
    auto load_len = [&](uint32_t L, uint64_t off) {
        return KFEC_SEAL_REG && valid(L) && L <= kRegBytes && row_fits(off, L, a.src_dw) ? L : 0u;
    };
    auto crc_len = [](uint32_t L) { return L - KFEC_SEAL_TRAILER; };
    for_each_row<KFEC_SEAL_OPEN_PF != 0>(a, lane, load_len, crc_len, [&](uint64_t p, uint32_t L, uint64_t off, uint32_t (&o)[kRegRounds][4], uint32_t u) {
        if (!valid(L)) {
            if (lane == 0) {
                a.out_len[p] = 0;
                a.ok[p] = 0;
            }
            return;
        }
        if (!load_len(L, off)) {
            open_stream_row(a, s_tab, p, L, off, lane);
            return;
        }
        const uint32_t n = L - KFEC_SEAL_TRAILER, nd = (n + 3) / 4;
        if (px) {  // xor_backward: plain[i] = T ^ (XOR of cipher[0..i)), T = XOR of every cipher byte
            mask_tail(o, L, lane);
            // one scan for all rounds: byte r of cx is the XOR of this lane's chunk of round r, so the exclusive
            // prefix over the row's lanes of every round comes out of one 5-level scan (XOR is bytewise)
            uint32_t cx = 0;
#pragma unroll
            for (int r = 0; r < kRegRounds; ++r) {
                uint32_t c = o[r][0] ^ o[r][1] ^ o[r][2] ^ o[r][3];
                c ^= c >> 16;
                c ^= c >> 8;
                cx |= (c & 0xFFu) << (8 * r);
            }
            uint32_t incl = cx;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const uint32_t v = __shfl_up(incl, 1 << k, kRowLanes);
                if (lane >= (1u << k)) incl ^= v;
            }
            const uint32_t tot = __shfl(incl, kRowLanes - 1, kRowLanes);  // byte r: XOR of round r's bytes
            uint32_t before = tot << 8;                                    // byte r: XOR of the rounds before r
            before ^= before << 8;
            before ^= before << 16;
            uint32_t T = tot ^ (tot >> 16);  // XOR of every cipher byte, broadcast
            T ^= T >> 8;
            T = (T & 0xFFu) * 0x01010101u;
            const uint32_t ex = before ^ incl ^ cx;  // byte r: cipher bytes before this lane's chunk of round r
#pragma unroll
            for (int r = 0; r < kRegRounds; ++r) {
                uint32_t run = ((ex >> (8 * r)) & 0xFFu) * 0x01010101u;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t in = o[r][i] ^ (o[r][i] << 8);
                    in ^= in << 16;  // byte b: XOR of bytes 0..b of this dword
                    const uint32_t y = T ^ run ^ (in << 8);
                    run ^= (in >> 24) * 0x01010101u;
                    o[r][i] = y;
                }
            }
        }
        const uint32_t trailer = row_trailer(o, n, lane);
        uint32_t *dst = dst_row(a, p);
#pragma unroll
        for (int r = 0; r < kRegRounds; ++r) {
            // past the plaintext: the trailer, and for plain_xor the scan's bytes past L (chunks after the one
            // holding n are zeroed whole)
            const int32_t q0 = (int32_t)(r * kCrcRound + kCrcLane * lane);
            if ((int32_t)n < q0 + 16) mask_chunk(o[r], q0, n);
            const uint32_t j = r * kRowLanes + lane;
            if (16 * j < n) store_chunk(dst, j, nd, o[r]);
        }
        const uint32_t crc = crc_regs(s_tab, u, o, n, lane);
        if (lane == 0) {
            a.out_len[p] = n;
            a.ok[p] = checksum16(crc) == trailer;
        }
    });
    count_done(a);
}

// Checksum mode in place (kfec_seal_batch / kfec_open_batch with d_dst == NULL): the packets stay where they
// are; seal appends the two checksum bytes after each packet, open verifies the trailer.  The CRC reads the
// packet once and nothing else moves (separate kernels: a per-packet in-place test inside seal_kernel cost
// its out-of-place path 24%).  Seal writes a trailer only where it fits the packet's slot (a.dst_pitch =
// the slot size from d_off, e.g. pkt_pitch) and the buffer: a packet filling its slot would otherwise get
// its trailer written over the next packet while another row is still reading that packet for its CRC.
__global__ void __launch_bounds__(kSealBlock) seal_in_place_kernel(SealArgs a, bool open)
{
    __shared__ CrcLdsIP s_tab;
    {
        uint32_t *flat = reinterpret_cast<uint32_t *>(&s_tab);
        const uint32_t *src = a.tab + offsetof(CrcLds, s16) / 4 + 12 * 256;  // s16[12..15], then sh: contiguous
        for (int i = threadIdx.x; i < (int)(sizeof(CrcLdsIP) / 4); i += kSealBlock) flat[i] = src[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x % kRowLanes;
    uint8_t *base = const_cast<uint8_t *>(reinterpret_cast<const uint8_t *>(a.src));
    for (uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRowLanes; p < a.P;
         p += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint32_t L = a.len[p];
        const uint64_t off = a.off[p];
        if (open ? L <= KFEC_SEAL_TRAILER : L == 0) {  // decrypt_data: bad length / encrypt_data: empty data
            if (lane == 0) {
                a.out_len[p] = 0;
                if (open) a.ok[p] = 0;
            }
            continue;
        }
        if (!open && ((uint64_t)L + KFEC_SEAL_TRAILER > a.dst_pitch || off + L + KFEC_SEAL_TRAILER > a.src_bytes)) {
            if (lane == 0) a.out_len[p] = 0;  // no room for the trailer: "does not fit", nothing written
            continue;
        }
        if (open && off + L > a.src_bytes) {  // the packet runs past the buffer: a bad length, nothing read
            if (lane == 0) {
                a.out_len[p] = 0;
                a.ok[p] = 0;
            }
            continue;
        }
        const uint32_t n = open ? L - KFEC_SEAL_TRAILER : L;  // bytes under the checksum
        const uint32_t cs = checksum16(row_crc32_bf(s_tab, a.src, a.src_dw, off, n, lane));
        if (lane == 0) {
            uint8_t *t = base + off + n;
            if (open) {
                a.ok[p] = cs == ((uint32_t)t[0] | ((uint32_t)t[1] << 8));
                a.out_len[p] = n;
            } else {
                t[0] = (uint8_t)cs;
                t[1] = (uint8_t)(cs >> 8);
                a.out_len[p] = L + KFEC_SEAL_TRAILER;
            }
        }
    }
}

uint32_t *crc_tables(hipStream_t s)
{
    static std::mutex mu;
    static uint32_t *tabs[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!tabs[dev]) {
        uint32_t *t = nullptr;
        if (hipMalloc(&t, kTabWords * sizeof(uint32_t)) != hipSuccess) return nullptr;
        hipLaunchKernelGGL(crc_tables_kernel, dim3((kTabWords + 255) / 256), dim3(256), 0, s, t);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return nullptr;
        tabs[dev] = t;
    }
    return tabs[dev];
}

}  // namespace

int launch_seal(bool open, int mode, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
                const uint32_t *len, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok, hipStream_t s,
                uint32_t *done, uint32_t *blocks)
{
    if (blocks) *blocks = 0;
    if (P == 0) return 0;
    SealArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.src_bytes = src_bytes;
    a.off = off;
    a.len = len;
    a.dst = static_cast<uint8_t *>(dst);
    a.dst_pitch = dst_pitch;
    a.out_len = out_len;
    a.ok = ok;
    a.P = P;
    a.mode = mode;
    a.done = dst ? done : nullptr;  // (the in-place kernel does not count)
    a.tab = crc_tables(s);
    if (!a.tab) return -3;
    a.unshift = a.tab + kCrcWords;
    const int cus = current_device_cus();
    // one workgroup per resident slot (the LDS tables and the VGPRs decide how many fit on a CU); each loops
    // over rows of 16 packets
    // resident workgroups per CU, once per kernel (thread-safe static initialisation)
    auto occupancy = [](const void *f) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, f, kSealBlock, 0) != hipSuccess || b < 1) b = 1;
        return b;
    };
    static const int fit_in_place = occupancy(reinterpret_cast<const void *>(&seal_in_place_kernel));
    static const int fit_open = occupancy(reinterpret_cast<const void *>(&open_kernel));
    static const int fit_seal = occupancy(reinterpret_cast<const void *>(&seal_kernel));
    const int fit = !dst ? fit_in_place : open ? fit_open : fit_seal;
    const uint64_t want = (P + kRowsPerBlock - 1) / kRowsPerBlock;
    const dim3 grid((uint32_t)std::min<uint64_t>(want, (uint64_t)cus * fit));
    if (blocks && a.done) *blocks = grid.x;
    if (!dst) hipLaunchKernelGGL(seal_in_place_kernel, grid, dim3(kSealBlock), 0, s, a, open);  // checksum mode
    else if (open) hipLaunchKernelGGL(open_kernel, grid, dim3(kSealBlock), 0, s, a);
    else hipLaunchKernelGGL(seal_kernel, grid, dim3(kSealBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace kfec
