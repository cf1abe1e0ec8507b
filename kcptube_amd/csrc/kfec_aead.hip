// kfec_aead.hip -- kcptube's chacha20 / xchacha20 packet modes as gfx950 kernels (include/kfec_aead.h).
//
// encrypt_data / decrypt_data (data_operations.cpp:171-234, 373-435) over encrypt_decrypt<chacha20> and
// encrypt_decrypt<xchacha20> (aead.hpp:402-562): Botan's ChaCha20Poly1305 with an 8-byte nonce (original
// construction: 64-bit counter, MAC over AD || le64(|AD|) || C || le64(|C|)) or a 24-byte one (XChaCha20:
// HChaCha20 subkey, then RFC 8439: MAC over AD || pad16 || C || pad16 || le64(|AD|) || le64(|C|)).
//
// Layout: a row of 8 lanes per packet, 32 rows per 256-lane workgroup.  In round t, lane j of a row owns
// the 64-byte ciphertext chunk c = 8t + j: it runs ChaCha20 block c + 1 (block 0 keys Poly1305), XORs the
// chunk, and stores it.  The Poly1305 message is header || ciphertext || trailer, with the header 23 (or
// 16) bytes long, so the 64-byte message chunk c is the previous chunk's last header-length bytes followed
// by this chunk's first ones: the previous lane's tail arrives by one row shuffle (the row's last lane
// carries it into the next round, and the header itself is the carry into round 0).  Each lane splits its
// message chunk into 4 Poly1305 blocks and keeps one Horner accumulator per block slot, stepping by
// r^32 (a row round covers 32 blocks); at the end slot i is multiplied by r^(NB - b) for its last block b
// (1 <= NB - b <= 32), and the 32 accumulators are summed across the row.  Arithmetic is radix 2^26 with
// 32x32->64 multiply-adds (donna-32 style); r^1..r^8 come from a 3-step scan across the row, r^16, r^24,
// r^32 from them.
//
// The nonce depends only on the 16-bit iv_raw, so the Poly1305 key (ChaCha20 block 0) and, for xchacha20,
// the HChaCha20 subkey are tabulated for all 65536 iv values when the key is set (kfec_aead_create), and
// looked up per packet: no per-packet HChaCha20 and no block-0 ChaCha20.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <new>

#include "../../include/kfec_aead.h"
#include "kfec_count.hpp"
#include "kfec_internal.hpp"
#include "kfec_pkt.hpp"

namespace kfec {

namespace {

// ---- SHA-3(256) (FIPS 202): the password hash of set_key (aead.hpp:416-418, 497-499); one thread ---------
__device__ const uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

__device__ void keccak_f1600(uint64_t (&s)[25])
{
    // rotation offsets of lane x + 5y
    constexpr int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (int round = 0; round < 24; ++round) {
        uint64_t c[5], b[25];
        for (int x = 0; x < 5; ++x) c[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
        for (int x = 0; x < 5; ++x) {
            const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
            for (int y = 0; y < 25; y += 5) s[x + y] ^= d;
        }
        for (int x = 0; x < 5; ++x)  // rho and pi: B[y, 2x + 3y] = rot(A[x, y])
            for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(s[x + 5 * y], rho[x + 5 * y]);
        for (int y = 0; y < 25; y += 5)
            for (int x = 0; x < 5; ++x) s[x + y] = b[x + y] ^ (~b[(x + 1) % 5 + y] & b[(x + 2) % 5 + y]);
        s[0] ^= kKeccakRC[round];
    }
}

__global__ void sha3_256_kernel(const uint8_t *msg, uint64_t len, uint32_t *out)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    constexpr int kRate = 136;
    uint64_t s[25] = {};
    uint64_t pos = 0;
    for (;;) {
        const uint64_t take = len - pos < (uint64_t)kRate ? len - pos : (uint64_t)kRate;
        for (uint64_t i = 0; i < take; ++i) s[i / 8] ^= (uint64_t)msg[pos + i] << (8 * (i % 8));
        pos += take;
        if (take < (uint64_t)kRate) {  // pad10*1 with the SHA-3 domain bits 01: 0x06 ... 0x80
            s[take / 8] ^= 0x06ull << (8 * (take % 8));
            s[(kRate - 1) / 8] ^= 0x80ull << (8 * ((kRate - 1) % 8));
            keccak_f1600(s);
            break;
        }
        keccak_f1600(s);
    }
    for (int i = 0; i < 8; ++i) out[i] = (uint32_t)(s[i / 2] >> (32 * (i % 2)));
}

// ---- ChaCha20 ----------------------------------------------------------------------------------------
constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646Eu, kSigma2 = 0x79622D32u, kSigma3 = 0x6B206574u;

#define KFEC_QR(a, b, c, d)                                 \
    x[a] += x[b]; x[d] = __builtin_rotateleft32(x[d] ^ x[a], 16); \
    x[c] += x[d]; x[b] = __builtin_rotateleft32(x[b] ^ x[c], 12); \
    x[a] += x[b]; x[d] = __builtin_rotateleft32(x[d] ^ x[a], 8);  \
    x[c] += x[d]; x[b] = __builtin_rotateleft32(x[b] ^ x[c], 7);

__device__ __forceinline__ void chacha_rounds(uint32_t (&x)[16])
{
#pragma unroll 2
    for (int i = 0; i < 10; ++i) {
        KFEC_QR(0, 4, 8, 12) KFEC_QR(1, 5, 9, 13) KFEC_QR(2, 6, 10, 14) KFEC_QR(3, 7, 11, 15)
        KFEC_QR(0, 5, 10, 15) KFEC_QR(1, 6, 11, 12) KFEC_QR(2, 7, 8, 13) KFEC_QR(3, 4, 9, 14)
    }
}
#undef KFEC_QR

// keystream block: key k, words 12..15 = (ctr, 0, nw, nw).  For both nonce sizes kcptube uses, this is the
// state: 8-byte nonce = iv_raw x 4 in words 14-15 under a 64-bit counter (words 12-13); XChaCha's inner
// 12-byte nonce = 0^4 || iv_raw x 4 under a 32-bit counter.  Counters stay below 2^32 for any packet.
__device__ __forceinline__ void chacha_block(const uint32_t (&k)[8], uint32_t ctr, uint32_t nw, uint32_t (&o)[16])
{
    uint32_t x[16] = {kSigma0, kSigma1, kSigma2, kSigma3, k[0], k[1], k[2], k[3],
                      k[4],    k[5],    k[6],    k[7],    ctr,  0u,   nw,   nw};
    chacha_rounds(x);
    o[0] = x[0] + kSigma0; o[1] = x[1] + kSigma1; o[2] = x[2] + kSigma2; o[3] = x[3] + kSigma3;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[4 + i] = x[4 + i] + k[i];
    o[12] = x[12] + ctr; o[13] = x[13]; o[14] = x[14] + nw; o[15] = x[15] + nw;
}

// per-iv table (kfec_aead_create): polykey = block 0; xchacha20: subkey = HChaCha20(key, iv_raw x 8) first
__global__ void iv_table_kernel(int mode, const uint32_t *key, uint32_t *tab)
{
    const uint32_t iv = blockIdx.x * blockDim.x + threadIdx.x;
    if (iv >= 65536u) return;
    const uint32_t nw = iv | (iv << 16);
    uint32_t k[8];
    for (int i = 0; i < 8; ++i) k[i] = key[i];
    uint32_t *e = tab + (size_t)iv * (mode == KFEC_AEAD_XCHACHA20 ? 16 : 8);
    if (mode == KFEC_AEAD_XCHACHA20) {
        uint32_t x[16] = {kSigma0, kSigma1, kSigma2, kSigma3, k[0], k[1], k[2], k[3],
                          k[4],    k[5],    k[6],    k[7],    nw,   nw,   nw,   nw};
        chacha_rounds(x);
        for (int i = 0; i < 4; ++i) {
            k[i] = x[i];
            k[4 + i] = x[12 + i];
        }
        for (int i = 0; i < 8; ++i) e[i] = k[i];
        e += 8;
    }
    uint32_t o[16];
    chacha_block(k, 0u, nw, o);
    for (int i = 0; i < 8; ++i) e[i] = o[i];
}

// keystream table (16-lane kernels): the first kChaKsBytes of every iv's keystream (blocks 1 ..), thread per
// (iv, 64-byte block); the key is the connection's (chacha20) or the iv's HChaCha20 subkey (xchacha20)
#ifndef KFEC_AEAD_KS
#define KFEC_AEAD_KS 1  // 16-lane kernels read the keystream from a per-iv table (0: ChaCha20 in the kernel)
#endif
constexpr uint32_t kChaKsBytes = 2048;

__global__ void chacha_ks_kernel(int mode, const uint32_t *key, const uint32_t *tab, uint32_t *ks)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr uint32_t kBlocks = kChaKsBytes / 64;
    if (e >= 65536ull * kBlocks) return;
    const uint32_t iv = (uint32_t)(e / kBlocks), blk = (uint32_t)(e % kBlocks);
    const bool x = mode == KFEC_AEAD_XCHACHA20;
    uint32_t k[8];
    for (int i = 0; i < 8; ++i) k[i] = x ? tab[(size_t)iv * 16 + i] : key[i];
    uint32_t o[16];
    chacha_block(k, blk + 1, iv | (iv << 16), o);
    uint4 *d = reinterpret_cast<uint4 *>(ks + ((size_t)iv * kChaKsBytes + 64 * (size_t)blk) / 4);
    for (int i = 0; i < 4; ++i) d[i] = make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

// ---- Poly1305, radix 2^26 ----------------------------------------------------------------------------
constexpr uint32_t kM26 = 0x3FFFFFFu;

struct F5 {
    uint32_t v[5];
};

__device__ __forceinline__ F5 f5_zero() { return F5{{0u, 0u, 0u, 0u, 0u}}; }

__device__ __forceinline__ void f5_add(F5 &a, const F5 &b)
{
#pragma unroll
    for (int i = 0; i < 5; ++i) a.v[i] += b.v[i];
}

// a * b mod 2^130 - 5, partially reduced (limbs < 2^26 except v[1] < 2^26 + 2^11).  Inputs: a limbs < 2^27,
// b limbs < 2^26 + 2^11 -- products < 2^56.4, sums of five < 2^59.
__device__ __forceinline__ F5 f5_mul(const F5 &a, const F5 &b)
{
    const uint32_t s1 = b.v[1] * 5u, s2 = b.v[2] * 5u, s3 = b.v[3] * 5u, s4 = b.v[4] * 5u;
    const uint64_t a0 = a.v[0], a1 = a.v[1], a2 = a.v[2], a3 = a.v[3], a4 = a.v[4];
    uint64_t d0 = a0 * b.v[0] + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
    uint64_t d1 = a0 * b.v[1] + a1 * b.v[0] + a2 * s4 + a3 * s3 + a4 * s2;
    uint64_t d2 = a0 * b.v[2] + a1 * b.v[1] + a2 * b.v[0] + a3 * s4 + a4 * s3;
    uint64_t d3 = a0 * b.v[3] + a1 * b.v[2] + a2 * b.v[1] + a3 * b.v[0] + a4 * s4;
    uint64_t d4 = a0 * b.v[4] + a1 * b.v[3] + a2 * b.v[2] + a3 * b.v[1] + a4 * b.v[0];
    F5 h;
    d1 += d0 >> 26; h.v[0] = (uint32_t)d0 & kM26;
    d2 += d1 >> 26; h.v[1] = (uint32_t)d1 & kM26;
    d3 += d2 >> 26; h.v[2] = (uint32_t)d2 & kM26;
    d4 += d3 >> 26; h.v[3] = (uint32_t)d3 & kM26;
    h.v[4] = (uint32_t)d4 & kM26;
    const uint64_t t = (uint64_t)h.v[0] + (d4 >> 26) * 5u;
    h.v[0] = (uint32_t)t & kM26;
    h.v[1] += (uint32_t)(t >> 26);
    return h;
}

__device__ __forceinline__ F5 f5_shfl(const F5 &a, int src)
{
    F5 r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.v[i] = __shfl(a.v[i], src, 8);
    return r;
}

__device__ __forceinline__ F5 f5_shfl_up(const F5 &a, int d)
{
    F5 r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.v[i] = __shfl_up(a.v[i], d, 8);
    return r;
}

// a 16-byte message block (four little-endian dwords) with its 2^(8*len) bit, len = 16 for a full block
__device__ __forceinline__ F5 f5_block(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int len)
{
    uint32_t hib = 1u << 24;
    if (len < 16) {  // only the last block of an 8-byte-nonce message: its bytes past len are already zero
        hib = 0u;
        const uint32_t bit = 1u << (8 * (len & 3));
        const int q = len >> 2;
        w0 |= q == 0 ? bit : 0u;
        w1 |= q == 1 ? bit : 0u;
        w2 |= q == 2 ? bit : 0u;
        w3 |= q == 3 ? bit : 0u;
    }
    return F5{{w0 & kM26, ((w0 >> 26) | (w1 << 6)) & kM26, ((w1 >> 20) | (w2 << 12)) & kM26,
               ((w2 >> 14) | (w3 << 18)) & kM26, (w3 >> 8) | hib}};
}

// (h mod 2^130 - 5) + s mod 2^128, h's limbs < 2^31
__device__ __forceinline__ void f5_tag(F5 h, const uint32_t (&s)[4], uint32_t (&tag)[4])
{
    for (int pass = 0; pass < 3; ++pass) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            h.v[i] += c;
            c = h.v[i] >> 26;
            h.v[i] &= kM26;
        }
        h.v[0] += c * 5u;
    }
    // every limb < 2^26 but v[0] (< 2^26 + 5): carry it through without a fold -- v[4] may reach 2^26,
    // i.e. h >= 2^130, which the h - p step below takes care of
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        h.v[i + 1] += h.v[i] >> 26;
        h.v[i] &= kM26;
    }
    // h - p = h + 5 - 2^130: take it when it does not borrow
    uint32_t g[5], c = 5;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        g[i] = h.v[i] + c;
        c = g[i] >> 26;
        g[i] &= kM26;
    }
    if (c) {  // h + 5 >= 2^130
#pragma unroll
        for (int i = 0; i < 5; ++i) h.v[i] = g[i];
    }
    const uint32_t w0 = h.v[0] | (h.v[1] << 26), w1 = (h.v[1] >> 6) | (h.v[2] << 20),
                   w2 = (h.v[2] >> 12) | (h.v[3] << 14), w3 = (h.v[3] >> 18) | (h.v[4] << 8);
    uint64_t t = (uint64_t)w0 + s[0];
    tag[0] = (uint32_t)t;
    t = (uint64_t)w1 + s[1] + (t >> 32);
    tag[1] = (uint32_t)t;
    t = (uint64_t)w2 + s[2] + (t >> 32);
    tag[2] = (uint32_t)t;
    t = (uint64_t)w3 + s[3] + (t >> 32);
    tag[3] = (uint32_t)t;
}

// ---- kcptube's MAC header: "KCP PortHopping" (aead.hpp:16) with its length or its pad ---------------------
__host__ __device__ constexpr uint32_t ad_byte(int i)
{
    return i < 0 || i >= 15 ? 0u : (uint32_t)(uint8_t)("KCP PortHopping"[i]);
}

// byte q (0..63) of the virtual 64-byte chunk that precedes ciphertext chunk 0: the header right-aligned
template <bool IETF>
__host__ __device__ constexpr uint32_t hdr_byte(int q)
{
    constexpr int H = IETF ? 16 : 23;
    const int i = q - (64 - H);  // header byte index
    if (i < 0) return 0u;
    if (i < 15) return ad_byte(i);
    return (!IETF && i == 15) ? 15u : 0u;  // le64(15) (8-byte nonce) or the zero pad byte (IETF)
}

template <bool IETF>
__host__ __device__ constexpr uint32_t hdr_dword(int d)
{
    return hdr_byte<IETF>(4 * d) | (hdr_byte<IETF>(4 * d + 1) << 8) | (hdr_byte<IETF>(4 * d + 2) << 16) |
           (hdr_byte<IETF>(4 * d + 3) << 24);
}

// ---- packet loads / stores -------------------------------------------------------------------------------
// 64 bytes at byte address a of a dword-aligned buffer of lim32 dwords (zero past the buffer)
__device__ __forceinline__ void load64(const uint32_t *b32, uint64_t lim32, uint64_t a, uint32_t (&o)[16])
{
    const uint64_t w = a >> 2;
    uint32_t d[17];
    if (w + 17 <= lim32) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 q = *reinterpret_cast<const uint4 *>(b32 + w + 4 * i);
            d[4 * i] = q.x; d[4 * i + 1] = q.y; d[4 * i + 2] = q.z; d[4 * i + 3] = q.w;
        }
        d[16] = b32[w + 16];
    } else {
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = w + i < lim32 ? b32[w + i] : 0u;
    }
    const uint32_t sh = (uint32_t)(a & 3u);
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
}

// 4 bytes at byte address a (zero past the buffer)
__device__ __forceinline__ uint32_t load4(const uint32_t *b32, uint64_t lim32, uint64_t a)
{
    const uint64_t w = a >> 2;
    const uint32_t lo = w < lim32 ? b32[w] : 0u, hi = w + 1 < lim32 ? b32[w + 1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(a & 3u));
}

// keep the first rem bytes (0 < rem < 64) of a 64-byte chunk
__device__ __forceinline__ void mask64(uint32_t (&o)[16], int rem)
{
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int k = rem - 4 * i;
        o[i] = k >= 4 ? o[i] : k <= 0 ? 0u : o[i] & ((1u << (8 * k)) - 1u);
    }
}

#ifndef KFEC_AEAD_ROW16
#define KFEC_AEAD_ROW16 1  // 16-lane rows (aead16_kernel); 0: the 8-lane rows of aead_kernel
#endif
#ifndef KFEC_AEAD_AB
#define KFEC_AEAD_AB 0  // timing ablations only (wrong output): bit 0 = no Poly1305 arithmetic, bit 1 = no ChaCha20 rounds
#endif

constexpr int kRow = 8;                  // lanes per packet
constexpr int kAeadBlock = 256;          // 32 packets per workgroup
constexpr int kRowsPerBlock = kAeadBlock / kRow;

struct AeadArgs {
    const uint32_t *src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint32_t *len;
    const uint16_t *iv;
    uint8_t *dst;
    uint64_t dst_pitch;
    uint32_t *out_len;
    uint8_t *ok;
    const uint32_t *tab;
    const uint4 *ks;  // keystream table (16-lane kernels, KFEC_AEAD_KS)
    uint64_t P;
    uint32_t key[8];
    uint32_t *done;   // counted launch (kfec_count.hpp)
};

// seal (OPEN = false) or open one packet per row.  IETF: xchacha20 (subkey from the table, RFC 8439 MAC)
template <bool IETF, bool OPEN>
__global__ void __launch_bounds__(kAeadBlock) aead_kernel(AeadArgs a)
{
    constexpr int H = IETF ? 16 : 23;   // MAC header bytes before the ciphertext
    constexpr int TL = IETF ? 16 : 8;   // MAC trailer bytes
    constexpr int S = 64 - H;           // message chunk c = bytes [S, S + 64) of (chunk c-1 || chunk c)
    constexpr int S4 = S / 4, SB = S % 4;
    constexpr int T0 = S4;              // first dword of a chunk's tail the next message chunk needs
    constexpr int NT = 16 - T0;
    const int lane = threadIdx.x % kRow;
    for (uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRow; p < a.P;
         p += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint32_t L = a.len[p];
        const uint64_t off = a.off[p];
        uint32_t n, iv;
        uint32_t ptag[4] = {0u, 0u, 0u, 0u};
        if (OPEN) {
            if (L < KFEC_AEAD_OVERHEAD || L - KFEC_AEAD_OVERHEAD > a.dst_pitch) {
                if (lane == 0) {
                    a.out_len[p] = 0;
                    a.ok[p] = 0;
                }
                continue;
            }
            n = L - KFEC_AEAD_OVERHEAD;
            // the packet's tag (lanes 0-3 one dword each, gathered later) and iv_raw
            const uint32_t tw = load4(a.src, a.src_dw, off + n + 4 * (lane & 3));
#pragma unroll
            for (int i = 0; i < 4; ++i) ptag[i] = __shfl(tw, i, kRow);
            iv = load4(a.src, a.src_dw, off + n + 16) & 0xFFFFu;
        } else {
            if (L == 0 || (uint64_t)L + KFEC_AEAD_OVERHEAD > a.dst_pitch) {  // "empty data" / no room
                if (lane == 0) a.out_len[p] = 0;
                continue;
            }
            n = L;
            iv = a.iv[p];
        }
        const uint32_t nw = iv | (iv << 16);
        const uint32_t *e = a.tab + (size_t)iv * (IETF ? 16 : 8);
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) k[i] = IETF ? e[i] : a.key[i];
        const uint32_t *pk = e + (IETF ? 8 : 0);
        // r (clamped) and s of the Poly1305 key
        const uint32_t t0 = pk[0], t1 = pk[1], t2 = pk[2], t3 = pk[3];
        const uint32_t sk[4] = {pk[4], pk[5], pk[6], pk[7]};
        const F5 r{{t0 & 0x3FFFFFFu, ((t0 >> 26) | (t1 << 6)) & 0x3FFFF03u, ((t1 >> 20) | (t2 << 12)) & 0x3FFC0FFu,
                    ((t2 >> 14) | (t3 << 18)) & 0x3F03FFFu, (t3 >> 8) & 0x00FFFFFu}};
        // lane j: r^(j+1); then r^8, r^16, r^24, r^32
        F5 pw = r;
#pragma unroll
        for (int d = 1; d < ((KFEC_AEAD_AB & 1) ? 1 : kRow); d <<= 1) {
            const F5 y = f5_shfl_up(pw, d);
            if (lane >= d) pw = f5_mul(pw, y);
        }
        const F5 r8 = f5_shfl(pw, kRow - 1);
        const F5 r16 = f5_mul(r8, r8);
        const F5 r24 = f5_mul(r16, r8);
        const F5 r32 = f5_mul(r16, r16);

        const uint32_t tpos = IETF ? (n + 15u) & ~15u : n;  // trailer position in the ciphertext stream
        const uint32_t M = H + tpos + TL;                   // MAC message bytes
        const uint32_t NB = (M + 15) / 16, NC = (M + 63) / 64;
        const uint32_t rounds = (NC + kRow - 1) / kRow;
        uint32_t carry[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) carry[i] = hdr_dword<IETF>(T0 + i);
        F5 acc[4] = {f5_zero(), f5_zero(), f5_zero(), f5_zero()};
        int blast[4] = {-1, -1, -1, -1};
        uint8_t *dst = a.dst + p * a.dst_pitch;
        for (uint32_t t = 0; t < rounds; ++t) {
            const uint32_t c = t * kRow + lane;
            const uint32_t cs = 64u * c;  // ciphertext offset of this lane's chunk
            uint32_t ct[16];
            if (cs < n) {
                uint32_t ks[16], in[16];
                if (KFEC_AEAD_AB & 2) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) ks[i] = k[i & 7] + c;
                } else {
                    chacha_block(k, c + 1, nw, ks);
                }
                load64(a.src, a.src_dw, off + cs, in);
                const bool part = cs + 64 > n;
                if (part) mask64(in, (int)(n - cs));
                uint32_t out[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) out[i] = in[i] ^ ks[i];
                if (part) mask64(out, (int)(n - cs));  // the keystream past n is not ciphertext
#pragma unroll
                for (int i = 0; i < 16; ++i) ct[i] = OPEN ? in[i] : out[i];
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + cs);
                if (!part) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        *reinterpret_cast<uint4 *>(d32 + 4 * i) =
                            make_uint4(out[4 * i], out[4 * i + 1], out[4 * i + 2], out[4 * i + 3]);
                } else {
                    const uint32_t rem = n - cs;  // 1..63
                    // open: whole dwords (the zero pad to a multiple of 4 is part of the output); seal: the
                    // last partial dword byte by byte, the tag follows it
                    const uint32_t nd = OPEN ? (rem + 3) / 4 : rem / 4;
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if ((uint32_t)i < nd) d32[i] = out[i];
                    if (!OPEN && (rem & 3)) {
                        const uint32_t q = rem / 4;
                        uint32_t v = 0;
#pragma unroll
                        for (int i = 0; i < 16; ++i) v = (uint32_t)i == q ? out[i] : v;
                        uint8_t *b = dst + cs + 4 * q;
                        for (uint32_t i = 0; i < (rem & 3); ++i) b[i] = (uint8_t)(v >> (8 * i));
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) ct[i] = 0u;
            }
            // the MAC trailer continues the ciphertext stream at tpos: le64(n) (8-byte nonce) or le64(15) ||
            // le64(n) (IETF); n < 2^32, so its high dword is zero
            if (cs + 64 > tpos && cs < tpos + TL) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int kk = (int)(cs + 4 * i) - (int)tpos;  // trailer byte at this dword's start
                    if (IETF) {
                        ct[i] |= kk == 0 ? 15u : kk == 8 ? n : 0u;
                    } else if (kk > -4 && kk < 4) {
                        ct[i] |= kk >= 0 ? n >> (8 * kk) : n << (-8 * kk);
                    }
                }
            }
            // the message chunk: [S, S + 64) of (previous chunk's tail || this chunk)
            uint32_t prev[NT];
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const uint32_t up = __shfl_up(ct[T0 + i], 1, kRow);
                prev[i] = lane == 0 ? carry[i] : up;
                carry[i] = __shfl(ct[T0 + i], kRow - 1, kRow);
            }
            uint32_t msg[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int x0 = S4 + i, x1 = S4 + i + 1;  // indices into prev (10.. 15 / 12..15) ++ ct
                const uint32_t lo = x0 < 16 ? prev[x0 - T0] : ct[x0 - 16];
                const uint32_t hi = x1 < 16 ? prev[x1 - T0] : ct[x1 - 16];
                msg[i] = SB ? __builtin_amdgcn_alignbyte(hi, lo, SB) : lo;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t b = 4 * c + i;
                if (b < NB) {
                    const int blen = (int)min(16u, M - 16 * b);
                    const F5 m = f5_block(msg[4 * i], msg[4 * i + 1], msg[4 * i + 2], msg[4 * i + 3], blen);
                    if (t && !(KFEC_AEAD_AB & 1)) acc[i] = f5_mul(acc[i], r32);
                    f5_add(acc[i], m);
                    blast[i] = (int)b;
                }
            }
        }
        // slot i's accumulator times r^(NB - b_last), 1 <= NB - b_last <= 32 = r^(8q) * r^(e'), then row sum
        F5 h = f5_zero();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e1 = blast[i] >= 0 ? (int)NB - blast[i] - 1 : 0;  // 0..31
            F5 rp = f5_shfl(pw, e1 & 7);
            const int q = e1 >> 3;
            const F5 rq = q == 1 ? r8 : q == 2 ? r16 : r24;
            if (KFEC_AEAD_AB & 1) {
                f5_add(h, acc[i]);
                f5_add(h, rq);
                continue;
            }
            if (q) rp = f5_mul(rp, rq);
            if (blast[i] >= 0) f5_add(h, f5_mul(acc[i], rp));
        }
#pragma unroll
        for (int d = 1; d < kRow; d <<= 1)
#pragma unroll
            for (int i = 0; i < 5; ++i) h.v[i] += __shfl_xor(h.v[i], d, kRow);
        uint32_t tag[4];
        f5_tag(h, sk, tag);
        if (OPEN) {
            const bool good = tag[0] == ptag[0] && tag[1] == ptag[1] && tag[2] == ptag[2] && tag[3] == ptag[3];
            if (!good) {  // no unauthenticated plaintext leaves the kernel: zero what was written
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
                const uint32_t nd = (n + 3) / 4;
                for (uint32_t i = lane; i < nd; i += kRow) d32[i] = 0u;
            }
            if (lane == 0) {
                a.out_len[p] = good ? n : 0u;
                a.ok[p] = good ? 1 : 0;
            }
        } else {
            // tag || iv_raw || zeros up to the next multiple of 4, bytes n .. n + 21, 3 per lane
            const uint32_t end = (n + KFEC_AEAD_OVERHEAD + 3) & ~3u;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const uint32_t i = 3 * lane + q;
                if (n + i < end) {
                    const uint32_t w = i < 4 ? tag[0] : i < 8 ? tag[1] : i < 12 ? tag[2] : i < 16 ? tag[3] : iv;
                    const uint32_t v = i < 18 ? (w >> (8 * (i & 3))) & 0xFFu : 0u;
                    dst[n + i] = (uint8_t)v;
                }
            }
            if (lane == 0) a.out_len[p] = n + KFEC_AEAD_OVERHEAD;
        }
    }
    count_workgroup_done(a.done);
}

// ---- 16-lane rows (KFEC_AEAD_ROW16) --------------------------------------------------------------------
// A row of 16 lanes per packet, each lane moving 16 contiguous bytes per round (256 per row: the copy rate of
// this layout is 4.1 TB/s against 2.5 for 8 lanes x 64 bytes, profiles/r02_rowcopy.json).  In round t, lane l
// owns ciphertext piece q = 16 t + l and message block b = 16 t + l.
//  * ChaCha20: the four lanes of a quad compute the quad's 64-byte block together, one state column each
//    (column rounds in place; for the diagonal rounds rows 1-3 are rotated across the quad by DPP quad_perm
//    and back), and a final quad transpose hands lane c the block's row c = its 16 keystream bytes.
//  * Poly1305: message block b is bytes [32 - H, 48 - H) of (piece b - 2 || piece b - 1) -- the pieces of the
//    two lanes before (the previous round's lanes 14, 15 through a carry; the MAC header before round 0).
//    Lane l's accumulator steps by r^16 and ends times r^(NB - b_last) from the row's powers r^1..r^16
//    (4-step scan), and the 16 accumulators are summed across the row.
constexpr int kRow16 = 16;

__device__ __forceinline__ uint32_t quad_rot(uint32_t v, int s)
{
    // lane c of each quad receives v from lane (c + s) % 4
    if (s == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x39, 0xF, 0xF, false);
    if (s == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x93, 0xF, 0xF, false);
}

#define KFEC_QR4(a, b, c, d)                                      \
    a += b; d = __builtin_rotateleft32(d ^ a, 16);                \
    c += d; b = __builtin_rotateleft32(b ^ c, 12);                \
    a += b; d = __builtin_rotateleft32(d ^ a, 8);                 \
    c += d; b = __builtin_rotateleft32(b ^ c, 7);

// 16 keystream bytes: row c (= lane % 4) of ChaCha20 block (key k, counter ctr, nonce words nw, nw)
__device__ __forceinline__ uint4 chacha_quad(const uint32_t (&k)[8], uint32_t ctr, uint32_t nw, uint32_t c)
{
    // two-level selects (a select chain over k[] becomes a dynamically indexed private array)
    const bool c1 = c & 1u, c2 = c & 2u;
    const uint32_t a0 = c2 ? (c1 ? kSigma3 : kSigma2) : (c1 ? kSigma1 : kSigma0);
    const uint32_t b0 = c2 ? (c1 ? k[3] : k[2]) : (c1 ? k[1] : k[0]);
    const uint32_t c0 = c2 ? (c1 ? k[7] : k[6]) : (c1 ? k[5] : k[4]);
    const uint32_t d0 = c == 0 ? ctr : c == 1 ? 0u : nw;
    uint32_t a = a0, b = b0, cc = c0, d = d0;
#pragma unroll 2
    for (int i = 0; i < 10; ++i) {
        KFEC_QR4(a, b, cc, d)
        b = quad_rot(b, 1); cc = quad_rot(cc, 2); d = quad_rot(d, 3);
        KFEC_QR4(a, b, cc, d)
        b = quad_rot(b, 3); cc = quad_rot(cc, 2); d = quad_rot(d, 1);
    }
    a += a0; b += b0; cc += c0; d += d0;
    // lane j holds column j (rows a, b, cc, d); lane c wants row c: word j of it from lane j's register c
    uint32_t row[4];
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
        // lane j sends its register (j - sft) & 3 -- the row the receiving lane (j - sft) & 3 wants
        const uint32_t r = (c - (uint32_t)sft) & 3u;
        const uint32_t v = r == 0 ? a : r == 1 ? b : r == 2 ? cc : d;
        const uint32_t got = sft ? quad_rot(v, sft) : v;
        // received from lane (c + sft) & 3: word (c + sft) & 3 of row c
        const uint32_t w = (c + (uint32_t)sft) & 3u;
        row[0] = w == 0 ? got : (sft ? row[0] : 0u);
        row[1] = w == 1 ? got : (sft ? row[1] : 0u);
        row[2] = w == 2 ? got : (sft ? row[2] : 0u);
        row[3] = w == 3 ? got : (sft ? row[3] : 0u);
    }
    return make_uint4(row[0], row[1], row[2], row[3]);
}
#undef KFEC_QR4

template <bool IETF>
__host__ __device__ constexpr uint32_t vpiece_dword(int piece, int d)
{
    // dword d of virtual ciphertext piece -1 or -2: the MAC header at stream positions [-H, 0)
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
        const int pos = 16 * piece + 4 * d + i;  // stream position (< 0)
        const int hb = pos + (IETF ? 16 : 23);   // header byte
        uint32_t byte = 0;
        if (hb >= 0) byte = hb < 15 ? ad_byte(hb) : (!IETF && hb == 15) ? 15u : 0u;
        v |= byte << (8 * i);
    }
    return v;
}

template <bool IETF, bool OPEN>
__global__ void __launch_bounds__(kAeadBlock) aead16_kernel(AeadArgs a)
{
    constexpr int H = IETF ? 16 : 23;
    constexpr int TL = IETF ? 16 : 8;
    constexpr int S = 32 - H;  // message block = bytes [S, S + 16) of (piece b - 2 || piece b - 1)
    constexpr int S4 = S / 4, SB = S % 4;
    constexpr int rows = kAeadBlock / kRow16;
    const uint32_t lane = threadIdx.x % kRow16, quad = lane & 3u;
    for (uint64_t p = (uint64_t)blockIdx.x * rows + threadIdx.x / kRow16; p < a.P;
         p += (uint64_t)gridDim.x * rows) {
        const uint32_t L = a.len[p];
        const uint64_t off = a.off[p];
        uint32_t n, iv, ptag = 0;
        if (OPEN) {
            if (L < KFEC_AEAD_OVERHEAD || L - KFEC_AEAD_OVERHEAD > a.dst_pitch) {
                if (lane == 0) {
                    a.out_len[p] = 0;
                    a.ok[p] = 0;
                }
                continue;
            }
            n = L - KFEC_AEAD_OVERHEAD;
            ptag = load4(a.src, a.src_dw, off + n + 4 * (lane & 3));
            iv = load4(a.src, a.src_dw, off + n + 16) & 0xFFFFu;
        } else {
            if (L == 0 || (uint64_t)L + KFEC_AEAD_OVERHEAD > a.dst_pitch) {
                if (lane == 0) a.out_len[p] = 0;
                continue;
            }
            n = L;
            iv = a.iv[p];
        }
        const uint32_t nw = iv | (iv << 16);
        const uint32_t *e = a.tab + (size_t)iv * (IETF ? 16 : 8);
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) k[i] = IETF ? e[i] : a.key[i];
        const uint32_t *pk = e + (IETF ? 8 : 0);
        const uint32_t t0 = pk[0], t1 = pk[1], t2 = pk[2], t3 = pk[3];
        const uint32_t sk[4] = {pk[4], pk[5], pk[6], pk[7]};
        const F5 r{{t0 & 0x3FFFFFFu, ((t0 >> 26) | (t1 << 6)) & 0x3FFFF03u, ((t1 >> 20) | (t2 << 12)) & 0x3FFC0FFu,
                    ((t2 >> 14) | (t3 << 18)) & 0x3F03FFFu, (t3 >> 8) & 0x00FFFFFu}};
        // lane l: r^(l+1); r^16 from lane 15
        F5 pw = r;
#pragma unroll
        for (int d = 1; d < kRow16; d <<= 1) {
            F5 y;
#pragma unroll
            for (int i = 0; i < 5; ++i) y.v[i] = __shfl_up(pw.v[i], d, kRow16);
            if (lane >= (uint32_t)d) pw = f5_mul(pw, y);
        }
        F5 r16;
#pragma unroll
        for (int i = 0; i < 5; ++i) r16.v[i] = __shfl(pw.v[i], kRow16 - 1, kRow16);

        const uint32_t tpos = IETF ? (n + 15u) & ~15u : n;
        const uint32_t M = H + tpos + TL, NB = (M + 15) / 16;
        const uint32_t rounds = (NB + kRow16 - 1) / kRow16;
        // carries: the previous round's pieces of lanes 14 and 15 (the header before round 0)
        uint32_t c14[4], c15[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            c14[i] = vpiece_dword<IETF>(-2, i);
            c15[i] = vpiece_dword<IETF>(-1, i);
        }
        F5 acc = f5_zero();
        int blast = -1;
        uint8_t *dst = a.dst + p * a.dst_pitch;
        uint32_t ctail = 0;
        for (uint32_t t = 0; t < rounds; ++t) {
            const uint32_t q = t * kRow16 + lane, qb = 16 * q;
            uint32_t ct[4] = {0u, 0u, 0u, 0u};
            // the quad's ChaCha20 block (counter 4 t + lane / 4 + 1), when it holds ciphertext
            const uint32_t blk = 4 * t + lane / 4;
            if (64 * blk < n) {
                uint4 ks;
                if (KFEC_AEAD_AB & 2) ks = make_uint4(k[0] + blk, k[1], k[2], k[3]);
                else if (KFEC_AEAD_KS && 64 * blk + 64 <= kChaKsBytes) ks = a.ks[(size_t)iv * (kChaKsBytes / 16) + q];
                else ks = chacha_quad(k, blk + 1, nw, quad);  // the quad's block: uniform per quad
                if (qb < n) {
                    uint4 in = load16(a.src, a.src_dw, off + qb);
                    const uint32_t rem = n - qb;
                    if (rem < 16) in = mask16(in, rem);
                    uint4 out = u4_xor(in, ks);
                    if (rem < 16) out = mask16(out, rem);
                    const uint4 c4 = OPEN ? in : out;
                    ct[0] = c4.x; ct[1] = c4.y; ct[2] = c4.z; ct[3] = c4.w;
                    uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + qb);
                    if (rem >= 16) {
                        *reinterpret_cast<uint4 *>(d32) = out;
                    } else {
                        const uint32_t o4[4] = {out.x, out.y, out.z, out.w};
                        const uint32_t nd = OPEN ? (rem + 3) / 4 : rem / 4;
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if ((uint32_t)i < nd) d32[i] = o4[i];
                        if (!OPEN && (rem & 3)) ctail = o4[rem / 4];
                    }
                }
            }
            // the MAC trailer continues the ciphertext stream at tpos (n < 2^32: its high dword is zero)
            if (qb + 16 > tpos && qb < tpos + TL) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int kk = (int)(qb + 4 * i) - (int)tpos;
                    if (IETF) ct[i] |= kk == 0 ? 15u : kk == 8 ? n : 0u;
                    else if (kk > -4 && kk < 4) ct[i] |= kk >= 0 ? n >> (8 * kk) : n << (-8 * kk);
                }
            }
            // pieces b - 1 and b - 2 from the lanes before (carries across the round boundary)
            uint32_t x[8];  // piece b - 2 || piece b - 1
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t u1 = __shfl_up(ct[i], 1, kRow16), u2 = __shfl_up(ct[i], 2, kRow16);
                x[4 + i] = lane >= 1 ? u1 : c15[i];
                x[i] = lane >= 2 ? u2 : lane == 1 ? c15[i] : c14[i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                c14[i] = __shfl(ct[i], kRow16 - 2, kRow16);
                c15[i] = __shfl(ct[i], kRow16 - 1, kRow16);
            }
            uint32_t msg[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) msg[i] = SB ? __builtin_amdgcn_alignbyte(x[S4 + i + 1], x[S4 + i], SB) : x[S4 + i];
            const uint32_t b = q;  // message block
            if (b < NB) {
                const int blen = (int)min(16u, M - 16 * b);
                const F5 m = f5_block(msg[0], msg[1], msg[2], msg[3], blen);
                if (t && !(KFEC_AEAD_AB & 1)) acc = f5_mul(acc, r16);
                f5_add(acc, m);
                blast = (int)b;
            }
        }
        // times r^(NB - b_last), 1..16, then the row sum
        {
            const int e1 = blast >= 0 ? (int)NB - blast - 1 : 0;
            F5 rp;
#pragma unroll
            for (int i = 0; i < 5; ++i) rp.v[i] = __shfl(pw.v[i], e1, kRow16);
            acc = blast >= 0 && !(KFEC_AEAD_AB & 1) ? f5_mul(acc, rp) : blast >= 0 ? acc : f5_zero();
        }
#pragma unroll
        for (int d = 1; d < kRow16; d <<= 1)
#pragma unroll
            for (int i = 0; i < 5; ++i) acc.v[i] += __shfl_xor(acc.v[i], d, kRow16);
        uint32_t tag[4];
        f5_tag(acc, sk, tag);
        if (OPEN) {
            const uint32_t l4 = lane & 3;
            const uint32_t mine = l4 == 0 ? tag[0] : l4 == 1 ? tag[1] : l4 == 2 ? tag[2] : tag[3];
            uint32_t bad = mine != ptag ? 1u : 0u;
#pragma unroll
            for (int d = 1; d < kRow16; d <<= 1) bad |= __shfl_xor(bad, d, kRow16);
            if (bad) {  // no unauthenticated plaintext leaves the kernel
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
                const uint32_t nd = (n + 3) / 4;
                for (uint32_t i = lane; i < nd; i += kRow16) d32[i] = 0u;
            }
            if (lane == 0) {
                a.out_len[p] = bad ? 0u : n;
                a.ok[p] = bad ? 0 : 1;
            }
        } else {
            // dwords from floor4(n): the ciphertext's last n % 4 bytes || tag || iv_raw || zero pad (5 or 6),
            // one per lane; the partial dword comes from the lane of the last ciphertext piece
            const uint32_t o = n & 3u, n4 = n & ~3u;
            const uint32_t cp = __shfl(ctail, (int)(((n - 1) / 16) % kRow16), kRow16);
            const uint32_t cnt = (((n + KFEC_AEAD_OVERHEAD + 3u) & ~3u) - n4) / 4u;
            const uint32_t w[7] = {o ? cp << (8 * (4 - o)) : 0u, tag[0], tag[1], tag[2], tag[3], iv, 0u};
            uint32_t w1 = 0, w0 = 0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                w1 = lane == (uint32_t)i ? w[i + 1] : w1;
                w0 = lane == (uint32_t)i ? w[i] : w0;
            }
            const uint32_t v = o ? __builtin_amdgcn_alignbyte(w1, w0, 4 - o) : w1;
            if (lane < cnt) reinterpret_cast<uint32_t *>(dst + n4)[lane] = v;
            if (lane == 0) a.out_len[p] = n + KFEC_AEAD_OVERHEAD;
        }
    }
    count_workgroup_done(a.done);
}

int aead_cus() { return current_device_cus(); }

}  // namespace

int launch_aead(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
                const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
                hipStream_t s, uint32_t *done, uint32_t *blocks)
{
    if (blocks) *blocks = 0;
    if (P == 0) return 0;
    if (k->mode == KFEC_AEAD_AES_GCM)
        return launch_gcm(k, open, P, src, src_bytes, off, len, iv, dst, dst_pitch, out_len, ok, s, done, blocks);
    if (k->mode == KFEC_AEAD_AES_OCB)
        return launch_ocb(k, open, P, src, src_bytes, off, len, iv, dst, dst_pitch, out_len, ok, s, done, blocks);
    AeadArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.iv = iv;
    a.dst = static_cast<uint8_t *>(dst);
    a.dst_pitch = dst_pitch;
    a.out_len = out_len;
    a.ok = ok;
    a.tab = k->d_tab;
    a.ks = reinterpret_cast<const uint4 *>(k->d_ks);
    a.P = P;
    a.done = done;
    for (int i = 0; i < 8; ++i) a.key[i] = k->key[i];
    const bool x = k->mode == KFEC_AEAD_XCHACHA20;
    if (KFEC_AEAD_ROW16) {
        const uint64_t rows = kAeadBlock / kRow16;
        const dim3 grid16((uint32_t)std::min<uint64_t>((P + rows - 1) / rows, (uint64_t)aead_cus() * 16));
        if (blocks && done) *blocks = grid16.x;
        if (x && open) hipLaunchKernelGGL((aead16_kernel<true, true>), grid16, dim3(kAeadBlock), 0, s, a);
        else if (x) hipLaunchKernelGGL((aead16_kernel<true, false>), grid16, dim3(kAeadBlock), 0, s, a);
        else if (open) hipLaunchKernelGGL((aead16_kernel<false, true>), grid16, dim3(kAeadBlock), 0, s, a);
        else hipLaunchKernelGGL((aead16_kernel<false, false>), grid16, dim3(kAeadBlock), 0, s, a);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    const uint64_t want = (P + kRowsPerBlock - 1) / kRowsPerBlock;
    const dim3 grid((uint32_t)std::min<uint64_t>(want, (uint64_t)aead_cus() * 16));
    if (blocks && done) *blocks = grid.x;
    if (x && open) hipLaunchKernelGGL((aead_kernel<true, true>), grid, dim3(kAeadBlock), 0, s, a);
    else if (x) hipLaunchKernelGGL((aead_kernel<true, false>), grid, dim3(kAeadBlock), 0, s, a);
    else if (open) hipLaunchKernelGGL((aead_kernel<false, true>), grid, dim3(kAeadBlock), 0, s, a);
    else hipLaunchKernelGGL((aead_kernel<false, false>), grid, dim3(kAeadBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int aead_setup_on(kfec_aead *k, const void *password, size_t len, hipStream_t s);

// key derivation and per-iv tables on the current device (synchronous: once per connection).  It runs on a
// private non-blocking stream and waits for that stream only, so in-flight work of other streams is not stalled.
int aead_setup(kfec_aead *k, const void *password, size_t len)
{
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return KFEC_EHIP;
    const int rc = aead_setup_on(k, password, len, s);
    (void)hipStreamDestroy(s);
    return rc;
}

int aead_setup_on(kfec_aead *k, const void *password, size_t len, hipStream_t s)
{
    uint8_t *d_pw = nullptr;
    uint32_t *d_key = nullptr;
    const bool gcm = k->mode == KFEC_AEAD_AES_GCM, ocb = k->mode == KFEC_AEAD_AES_OCB;
    const size_t entries = k->mode == KFEC_AEAD_XCHACHA20 ? 16 : 8;
    if (hipMalloc(&d_pw, len) != hipSuccess) return KFEC_ENOMEM;
    if (hipMalloc(&d_key, 32) != hipSuccess) {
        (void)hipFree(d_pw);
        return KFEC_ENOMEM;
    }
    int rc = KFEC_OK;
    if (!gcm && !ocb && hipMalloc(&k->d_tab, 65536 * entries * sizeof(uint32_t)) != hipSuccess) {
        k->d_tab = nullptr;
        rc = KFEC_ENOMEM;
    }
    if (rc == KFEC_OK && hipMemcpyAsync(d_pw, password, len, hipMemcpyHostToDevice, s) != hipSuccess) rc = KFEC_EHIP;
    if (rc == KFEC_OK) {
        hipLaunchKernelGGL(sha3_256_kernel, dim3(1), dim3(64), 0, s, d_pw, (uint64_t)len, d_key);
        if (gcm) {
            rc = gcm_setup(k, d_key, s);
        } else if (ocb) {
            rc = ocb_setup(k, d_key, s);
        } else {
            hipLaunchKernelGGL(iv_table_kernel, dim3(65536 / 256), dim3(256), 0, s, k->mode, d_key, k->d_tab);
            if (KFEC_AEAD_ROW16 && KFEC_AEAD_KS) {
                if (hipMalloc(&k->d_ks, (size_t)65536 * kChaKsBytes) != hipSuccess) {
                    k->d_ks = nullptr;
                    rc = KFEC_ENOMEM;
                } else {
                    k->ks_bytes = kChaKsBytes;
                    const uint64_t th = 65536ull * (kChaKsBytes / 64);
                    hipLaunchKernelGGL(chacha_ks_kernel, dim3((uint32_t)((th + 255) / 256)), dim3(256), 0, s,
                                       k->mode, d_key, k->d_tab, reinterpret_cast<uint32_t *>(k->d_ks));
                }
            }
        }
        if (rc == KFEC_OK && (hipGetLastError() != hipSuccess ||
                              hipMemcpyAsync(k->key, d_key, 32, hipMemcpyDeviceToHost, s) != hipSuccess ||
                              hipStreamSynchronize(s) != hipSuccess))
            rc = KFEC_EHIP;
    }
    (void)hipStreamSynchronize(s);  // (a failed launch sequence: nothing may still read d_pw / d_key)
    (void)hipFree(d_pw);
    (void)hipFree(d_key);
    if (rc != KFEC_OK) {
        if (k->d_tab) (void)hipFree(k->d_tab);
        k->d_tab = nullptr;
        gcm_free(k);
    }
    return rc;
}

}  // namespace kfec

extern "C" {

int kfec_aead_create(int mode, const void *password, size_t password_len, kfec_aead **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if ((mode != KFEC_AEAD_AES_GCM && mode != KFEC_AEAD_AES_OCB && mode != KFEC_AEAD_CHACHA20 &&
         mode != KFEC_AEAD_XCHACHA20) ||
        !password || password_len == 0)
        return KFEC_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return KFEC_ENODEV;
    kfec_aead *k = new (std::nothrow) kfec_aead;
    if (!k) return KFEC_ENOMEM;
    k->mode = mode;
    if (hipGetDevice(&k->device) != hipSuccess) {
        delete k;
        return KFEC_EHIP;
    }
    const int rc = kfec::aead_setup(k, password, password_len);
    if (rc != KFEC_OK) {
        delete k;
        return rc;
    }
    *out = k;
    return KFEC_OK;
}

void kfec_aead_destroy(kfec_aead *a)
{
    if (!a) return;
    (void)hipSetDevice(a->device);  // the tables live on the cipher's device
    if (a->d_tab) (void)hipFree(a->d_tab);
    kfec::gcm_free(a);
    delete a;
}

int kfec_aead_mode(const kfec_aead *a) { return a ? a->mode : KFEC_EINVAL; }

int kfec_aead_key(const kfec_aead *a, uint8_t key[32])
{
    if (!a || !key) return KFEC_EINVAL;
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(a->key[i / 4] >> (8 * (i % 4)));
    return KFEC_OK;
}

static bool aead_al4(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

int kfec_aead_seal_batch(const kfec_aead *a, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                         const uint32_t *d_len, const uint16_t *d_iv, void *d_dst, size_t dst_pitch,
                         uint32_t *d_out_len, void *stream)
{
    if (!a || dst_pitch % 4) return KFEC_EINVAL;
    if (P && (!d_src || !aead_al4(d_src) || !d_off || !d_len || !d_iv || !d_dst || !aead_al4(d_dst) || !d_out_len))
        return KFEC_EINVAL;
    if (hipSetDevice(a->device) != hipSuccess) return KFEC_EHIP;  // launch where the cipher's tables live
    return kfec::launch_aead(a, false, P, d_src, src_bytes, d_off, d_len, d_iv, d_dst, dst_pitch, d_out_len, nullptr,
                             static_cast<hipStream_t>(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

int kfec_aead_open_batch(const kfec_aead *a, size_t P, const void *d_src, size_t src_bytes, const uint64_t *d_off,
                         const uint32_t *d_len, void *d_dst, size_t dst_pitch, uint32_t *d_out_len, uint8_t *d_ok,
                         void *stream)
{
    if (!a || dst_pitch % 4) return KFEC_EINVAL;
    if (P && (!d_src || !aead_al4(d_src) || !d_off || !d_len || !d_dst || !aead_al4(d_dst) || !d_out_len || !d_ok))
        return KFEC_EINVAL;
    if (hipSetDevice(a->device) != hipSuccess) return KFEC_EHIP;  // launch where the cipher's tables live
    return kfec::launch_aead(a, true, P, d_src, src_bytes, d_off, d_len, nullptr, d_dst, dst_pitch, d_out_len, d_ok,
                             static_cast<hipStream_t>(stream))
               ? KFEC_EHIP
               : KFEC_OK;
}

}  // extern "C"
