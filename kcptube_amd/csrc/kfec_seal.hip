// kfec_seal.hip -- the per-packet integrity step either side of FEC on the wire,
// for kcptube's non-AEAD encryption modes:
//   encrypt_data (data_operations.cpp:171-234), modes "none" (default branch) and plain_xor:
//     append checksum16(data) (simple_hashing.hpp:10-25: CRC-32 of the data, its two 16-bit halves XORed),
//     then, for plain_xor, xor_forward over data + checksum (data_operations.cpp:120-128).
//   decrypt_data (data_operations.cpp:373-435): plain_xor first undoes xor_backward (:140-148), then the
//     trailing two bytes are compared with checksum16 of the rest.
// The AEAD modes (AES-GCM/OCB, (X)ChaCha20-Poly1305) need Botan, which is absent here: out of scope.
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
#include "kfec_internal.hpp"

namespace kfec {

namespace {

constexpr int kSealBlock = 512;  // 16 packets share one LDS copy of the tables (28 KiB): 4 workgroups = 32 waves per CU

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
// Half a wave (32 lanes) per packet.  The message is right-aligned into 512-byte rounds (leading zero bytes
// leave a CRC computed from a zero register unchanged); lane l takes the 16-byte chunk l of a round and
// computes its raw CRC (zero init, slicing-by-4) and folds it into its own running sum across rounds
// (Horner with shift_512); the 32 lanes' sums are combined once per packet in 5 butterfly levels:
//   CRC(A || B) = shift_|B|(CRC(A)) ^ CRC(B),   shift_d(r) = r advanced through d zero bytes,
// a GF(2)-linear map applied as 4 byte-indexed table lookups (linearity makes the per-lane sums combine
// exactly like one round's chunk CRCs).  The
// standard 0xFFFFFFFF init is folded in by complementing the first 4 message bytes (messages >= 4 bytes;
// shorter ones run serially on one lane), and the result is complemented at the end.
//   tables: [0] slicing-by-4 (4 x 256), [1 + k] shift by 16 << k bytes (k = 0..5), each 4 x 256 u32
constexpr int kCrcMaps = 7;
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

#ifndef KFEC_SEAL_NIB
#define KFEC_SEAL_NIB 0  // 1: nibble-indexed tables -- no LDS bank conflicts, but +33% VALU and slower
#endif

// The CRC tables each workgroup stages into LDS.
//  nibble form (KFEC_SEAL_NIB): every map is GF(2)-linear, so it is the XOR of one 16-entry table per input
//    nibble.  A 16-entry table is 16 consecutive dwords -- 16 distinct banks -- and all lanes of one
//    ds_read_b32 read the same table, so distinct entries never share a bank: no conflicts (the byte tables'
//    256 entries over 32 banks gave ~4-5-way conflicts on random data).  The 32 chunk lookups of a 16-byte
//    chunk are also independent of each other, where slicing-by-4 chains the four dwords of a chunk.
//      chunk[k][v]:    raw CRC (zero init) of a 16-byte chunk holding nibble v at nibble k, zeros elsewhere
//      shift[m][j][v]: nibble j = v of a CRC register advanced through 16 << m zero bytes (m = 5: 512)
//      byte0[v]:       the bytewise table, for packets of fewer than 4 bytes
//  byte form: [0] slicing-by-4 (4 x 256), [1 + m] the shift maps, each 4 x 256
struct CrcLds {
#if KFEC_SEAL_NIB
    uint32_t chunk[32][16];
    uint32_t shift[6][8][16];
    uint32_t byte0[256];
#else
    uint32_t t[kCrcMaps][4][256];
#endif
};
constexpr int kCrcWords = (int)(sizeof(CrcLds) / 4);

__global__ void crc_tables_kernel(uint32_t *tab)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCrcWords) return;
#if KFEC_SEAL_NIB
    uint32_t r = 0;
    if (e < 32 * 16) {  // chunk[k][v]
        const int k = e / 16, v = e % 16;
        for (int i = 0; i < 16; ++i) {
            const uint32_t byte = i == k / 2 ? (uint32_t)v << (4 * (k & 1)) : 0u;
            r = (r >> 8) ^ c_crc.t[0][(r ^ byte) & 0xFFu];
        }
    } else if (e < 32 * 16 + 6 * 8 * 16) {  // shift[m][j][v]
        const int f = e - 32 * 16, m = f / 128, j = (f / 16) & 7, v = f % 16;
        r = (uint32_t)v << (4 * j);
        const int d = kCrcLane << m;
        for (int i = 0; i < d; ++i) r = (r >> 8) ^ c_crc.t[0][r & 0xFFu];
    } else {
        r = c_crc.t[0][e - 32 * 16 - 6 * 8 * 16];
    }
    tab[e] = r;
#else
    const int map = e / 1024, j = (e / 256) & 3, v = e & 255;  // e = ((map * 4) + j) * 256 + v
    if (map == 0) {
        tab[e] = c_crc.t[j][v];
        return;
    }
    uint32_t r = (uint32_t)v << (8 * j);
    const int d = kCrcLane << (map - 1);
    for (int i = 0; i < d; ++i) r = (r >> 8) ^ c_crc.t[0][r & 0xFFu];
    tab[e] = r;
#endif
}

#if KFEC_SEAL_NIB
// entry at byte offset bo (= 4 * nibble) of a 16-entry table
__device__ __forceinline__ uint32_t nib_at(const uint32_t *t16, uint32_t bo)
{
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(t16) + bo);
}

// raw CRC (zero init) of the 16-byte chunk o: 32 independent lookups
__device__ __forceinline__ uint32_t crc_chunk(const CrcLds &t, const uint32_t (&o)[4])
{
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t lo = (o[i] << 2) & 0x3C3C3C3Cu, hi = (o[i] >> 2) & 0x3C3C3C3Cu;  // 4 x nibble per byte
#pragma unroll
        for (int b = 0; b < 4; ++b)
            c ^= nib_at(t.chunk[8 * i + 2 * b], (lo >> (8 * b)) & 0xFFu) ^
                 nib_at(t.chunk[8 * i + 2 * b + 1], (hi >> (8 * b)) & 0xFFu);
    }
    return c;
}

// map m applied to the register r
__device__ __forceinline__ uint32_t crc_shift(const CrcLds &t, int m, uint32_t r)
{
    const uint32_t lo = (r << 2) & 0x3C3C3C3Cu, hi = (r >> 2) & 0x3C3C3C3Cu;
    uint32_t c = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
        c ^= nib_at(t.shift[m][2 * b], (lo >> (8 * b)) & 0xFFu) ^ nib_at(t.shift[m][2 * b + 1], (hi >> (8 * b)) & 0xFFu);
    return c;
}

__device__ __forceinline__ uint32_t crc_byte(const CrcLds &t, uint32_t c, uint32_t byte)
{
    return (c >> 8) ^ t.byte0[(c ^ byte) & 0xFFu];
}
#else
__device__ __forceinline__ uint32_t crc_dword(const uint32_t (*t)[256], uint32_t c, uint32_t d)
{
    const uint32_t x = c ^ d;
    return t[3][x & 0xFFu] ^ t[2][(x >> 8) & 0xFFu] ^ t[1][(x >> 16) & 0xFFu] ^ t[0][x >> 24];
}

__device__ __forceinline__ uint32_t crc_chunk(const CrcLds &t, const uint32_t (&o)[4])
{
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) c = crc_dword(t.t[0], c, o[i]);
    return c;
}

__device__ __forceinline__ uint32_t crc_shift(const CrcLds &t, int m, uint32_t r)
{
    const uint32_t (*s)[256] = t.t[1 + m];
    return s[0][r & 0xFFu] ^ s[1][(r >> 8) & 0xFFu] ^ s[2][(r >> 16) & 0xFFu] ^ s[3][r >> 24];
}

__device__ __forceinline__ uint32_t crc_byte(const CrcLds &t, uint32_t c, uint32_t byte)
{
    return (c >> 8) ^ t.t[0][0][(c ^ byte) & 0xFFu];
}
#endif

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
            const uint32_t c = crc_chunk(tab, o[u]);
            // Horner over this lane's chunks: R = XOR_r shift_{(rounds-1-r)*512}(chunk CRC of round r)
            if (r0 + u < rounds) R = crc_shift(tab, 5, R) ^ c;
        }
    }
    // one butterfly per packet (not per round): by linearity the 32 lanes' Horner sums combine exactly as
    // one round's chunk CRCs do.  Level k: the lane holding the earlier block A shifts it past the later
    // block B (16 << k bytes): A' = shift(A) ^ B -- one table shift per lane, the operands picked by lane bit
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
    uint64_t P;
    int mode;
};

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

__global__ void __launch_bounds__(kSealBlock) seal_kernel(SealArgs a)
{
    __shared__ CrcLds s_tab;
    stage_tables(a.tab, s_tab);
    const uint32_t lane = threadIdx.x % kRowLanes;
    for (uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRowLanes; p < a.P;
         p += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint32_t L = a.len[p];
        const uint64_t off = a.off[p];
        if (L == 0 || L + KFEC_SEAL_TRAILER > a.dst_pitch) {  // encrypt_data: "empty data" (:173-174); no room
            if (lane == 0) a.out_len[p] = 0;
            continue;
        }
        const uint32_t cs = checksum16(row_crc32(s_tab, a.src, a.src_dw, off, L, lane));
        // sealed packet S = data || cs, xor_forward'ed for plain_xor (out[i] = S[i] ^ S[i + 1])
        const uint32_t n = L + KFEC_SEAL_TRAILER, nd = (n + 3) / 4;
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.dst + p * a.dst_pitch);
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
        }
        if (lane == 0) a.out_len[p] = n;
    }
}

__global__ void __launch_bounds__(kSealBlock) open_kernel(SealArgs a)
{
    __shared__ CrcLds s_tab;
    stage_tables(a.tab, s_tab);
    const uint32_t lane = threadIdx.x % kRowLanes;
    const bool px = a.mode == KFEC_SEAL_PLAIN_XOR;
    for (uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRowLanes; p < a.P;
         p += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint32_t L = a.len[p];
        const uint64_t off = a.off[p];
        if (L <= KFEC_SEAL_TRAILER || L - KFEC_SEAL_TRAILER > a.dst_pitch) {  // decrypt_data: bad length
            if (lane == 0) {
                a.out_len[p] = 0;
                a.ok[p] = 0;
            }
            continue;
        }
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
        }
        if (lane == 0) {
            a.out_len[p] = n;
            a.ok[p] = checksum16(crc) == trailer;
        }
    }
}

// Checksum mode in place (kfec_seal_batch / kfec_open_batch with d_dst == NULL): the packets stay where they
// are; seal appends the two checksum bytes after each packet, open verifies the trailer.  The CRC reads the
// packet once and nothing else moves (separate kernels: a per-packet in-place test inside seal_kernel cost
// its out-of-place path 24%).  Seal writes a trailer only where it fits the packet's slot (a.dst_pitch =
// the slot size from d_off, e.g. pkt_pitch) and the buffer: a packet filling its slot would otherwise get
// its trailer written over the next packet while another row is still reading that packet for its CRC.
__global__ void __launch_bounds__(kSealBlock) seal_in_place_kernel(SealArgs a, bool open)
{
    __shared__ CrcLds s_tab;
    stage_tables(a.tab, s_tab);
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
        const uint32_t n = open ? L - KFEC_SEAL_TRAILER : L;  // bytes under the checksum
        const uint32_t cs = checksum16(row_crc32(s_tab, a.src, a.src_dw, off, n, lane));
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
        if (hipMalloc(&t, kCrcWords * sizeof(uint32_t)) != hipSuccess) return nullptr;
        hipLaunchKernelGGL(crc_tables_kernel, dim3((kCrcWords + 255) / 256), dim3(256), 0, s, t);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return nullptr;
        tabs[dev] = t;
    }
    return tabs[dev];
}

}  // namespace

int launch_seal(bool open, int mode, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
                const uint32_t *len, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok, hipStream_t s)
{
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
    a.tab = crc_tables(s);
    if (!a.tab) return -3;
    static int cus = [] {
        int d = 0, n = 0;
        if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) !=
                                                  hipSuccess)
            n = 256;
        return std::max(n, 1);
    }();
    // 28 KiB of tables per 512-thread workgroup: 4 resident per CU; each loops over rows of 16 packets
    const uint64_t want = (P + kRowsPerBlock - 1) / kRowsPerBlock;
    const dim3 grid((uint32_t)std::min<uint64_t>(want, (uint64_t)cus * 4));
    if (!dst) hipLaunchKernelGGL(seal_in_place_kernel, grid, dim3(kSealBlock), 0, s, a, open);  // checksum mode
    else if (open) hipLaunchKernelGGL(open_kernel, grid, dim3(kSealBlock), 0, s, a);
    else hipLaunchKernelGGL(seal_kernel, grid, dim3(kSealBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace kfec
