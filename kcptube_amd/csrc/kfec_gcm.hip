// kfec_gcm.hip -- kcptube's aes_gcm packet mode as gfx950 kernels (include/kfec_aead.h).
//
// encrypt_data / decrypt_data (data_operations.cpp:171-234, 373-435) over encrypt_decrypt<aes_256_gcm>
// (aead.hpp:237-312): Botan "AES-256/GCM" with kcptube's 16-byte nonce (iv_raw repeated 8 times), so
// J0 = GHASH_H(IV || 0^64 || be64(128)) (NIST SP 800-38D 7.1); CTR from inc32(J0); tag = E_K(J0) xor
// GHASH_H(AD || pad || C || pad || be64(8|AD|) || be64(8|C|)); packet = C || tag || iv_raw.
//
// The MI355X-first part: everything the key and the 16-bit iv_raw determine is computed once per key, on the
// device, for all 65536 iv values -- J0, E_K(J0) and the first kKsBytes of the CTR keystream (128 MiB at
// 2 KiB per iv, which covers kcptube's packets) -- so per packet AES is a table read; only blocks past
// kKsBytes run AES in the kernel.  GHASH runs lane-parallel: a row of 4 lanes per packet, lane j owning
// message blocks j, j + 4, ...; each lane keeps a Horner accumulator stepped by H^4 and ends by one multiply
// by H^e, 1 <= e <= 4, and the row XORs the four.  A multiply by a fixed power of H is 32 lookups of
// 16-byte entries (one 16-entry table per input nibble, Shoup) from LDS: 16 entries of 16 bytes span the
// 64 banks once, so the lookups of one instruction never conflict.  The message block of lane j is the
// ciphertext block the same lane just produced (the AD is exactly one block), so no data crosses lanes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/kfec_aead.h"
#include "kfec_aes.hpp"
#include "kfec_pkt.hpp"
#include "kfec_gf.hpp"
#include "kfec_count.hpp"
#include "kfec_internal.hpp"

namespace kfec {

namespace {

#ifndef KFEC_GCM_KS_BYTES
#define KFEC_GCM_KS_BYTES 2048  // keystream bytes tabulated per iv (multiple of 16)
#endif
constexpr uint32_t kKsBytes = KFEC_GCM_KS_BYTES;
#ifndef KFEC_GCM_AB
#define KFEC_GCM_AB 0  // timing ablations only (wrong output): bit 0 = no GHASH multiplies, bit 1 = no keystream loads
#endif

// ---- GHASH multiply, bit-serial (setup only): z = x * y in GF(2^128), SP 800-38D 6.3 bit order ---------
__device__ void gf128_mul(const uint8_t (&x)[16], const uint8_t (&y)[16], uint8_t (&z)[16])
{
    uint8_t v[16], r[16] = {};
    for (int i = 0; i < 16; ++i) v[i] = y[i];
    for (int i = 0; i < 128; ++i) {
        if ((x[i / 8] >> (7 - i % 8)) & 1)
            for (int k = 0; k < 16; ++k) r[k] ^= v[k];
        const uint32_t lsb = v[15] & 1u;
        for (int k = 15; k > 0; --k) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xE1u;
    }
    for (int i = 0; i < 16; ++i) z[i] = r[i];
}

// key schedule and H = E_K(0^128): one thread
__global__ void gcm_key_kernel(const uint32_t *key, uint8_t *rk, uint8_t *h)
{
    if (blockIdx.x || threadIdx.x) return;
    uint8_t w[240];
    aes256_expand(key, w);
    for (int i = 0; i < 240; ++i) rk[i] = w[i];
    uint8_t z[16] = {}, o[16];
    aes256_encrypt(w, z, o);
    for (int i = 0; i < 16; ++i) h[i] = o[i];
}

// Shoup tables of H^(2^p), p = 0..4 (H, H^2, H^4, H^8, H^16): gh[p][k][v] = (the block whose byte k / 2 is
// v << 4 (k & 1), zeros elsewhere) * H^(2^p), 16 bytes each; thread per entry
constexpr int kGhTables = 5;
__global__ void gcm_tables_kernel(const uint8_t *h, uint8_t *gh)
{
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kGhTables * 32 * 16) return;
    const int p = e / 512, k = (e / 16) % 32, v = e % 16;
    uint8_t hp[16];
    for (int i = 0; i < 16; ++i) hp[i] = h[i];
    for (int q = 0; q < p; ++q) {  // square p times
        uint8_t t[16];
        gf128_mul(hp, hp, t);
        for (int i = 0; i < 16; ++i) hp[i] = t[i];
    }
    uint8_t x[16] = {}, z[16];
    x[k / 2] = (uint8_t)(v << (4 * (k & 1)));
    gf128_mul(x, hp, z);
    for (int i = 0; i < 16; ++i) gh[16 * e + i] = z[i];
}

// per iv: J0 and E_K(J0) (iv table, 32 bytes per iv)
__global__ void gcm_iv_kernel(const uint8_t *rk, const uint8_t *h, uint8_t *ivt)
{
    const uint32_t iv = blockIdx.x * blockDim.x + threadIdx.x;
    if (iv >= 65536u) return;
    uint8_t hh[16], y[16], t[16], mask[16];
    for (int i = 0; i < 16; ++i) {
        hh[i] = h[i];
        y[i] = (uint8_t)(i % 2 ? iv >> 8 : iv);  // the nonce: iv_raw (little-endian) x 8
    }
    gf128_mul(y, hh, t);  // GHASH(IV || len block): (IV * H ^ L) * H, L = 0^64 || be64(128)
    t[15] ^= 0x80u;
    gf128_mul(t, hh, y);
    aes256_encrypt(rk, y, mask);
    for (int i = 0; i < 16; ++i) {
        ivt[32 * (size_t)iv + i] = y[i];
        ivt[32 * (size_t)iv + 16 + i] = mask[i];
    }
}

// counter block i (i >= 1) of a packet: inc32^i(J0)
__device__ __forceinline__ void ctr_block(const uint8_t *j0, uint32_t i, uint8_t (&c)[16])
{
    for (int k = 0; k < 12; ++k) c[k] = j0[k];
    const uint32_t v = ((uint32_t)j0[12] << 24 | (uint32_t)j0[13] << 16 | (uint32_t)j0[14] << 8 | j0[15]) + i;
    c[12] = (uint8_t)(v >> 24);
    c[13] = (uint8_t)(v >> 16);
    c[14] = (uint8_t)(v >> 8);
    c[15] = (uint8_t)v;
}

// the first kKsBytes of keystream of every iv: thread per (iv, 16-byte block)
__global__ void gcm_ks_kernel(const uint8_t *rk, const uint8_t *ivt, uint8_t *ks)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    constexpr uint32_t kBlocks = kKsBytes / 16;
    if (e >= 65536ull * kBlocks) return;
    const uint32_t iv = (uint32_t)(e / kBlocks), q = (uint32_t)(e % kBlocks);
    uint8_t c[16], o[16];
    ctr_block(ivt + 32 * (size_t)iv, q + 1, c);
    aes256_encrypt(rk, c, o);
    uint4 *d = reinterpret_cast<uint4 *>(ks + (size_t)iv * kKsBytes + 16 * (size_t)q);
    uint32_t wv[4];
    for (int i = 0; i < 4; ++i)
        wv[i] = (uint32_t)o[4 * i] | (uint32_t)o[4 * i + 1] << 8 | (uint32_t)o[4 * i + 2] << 16 |
                (uint32_t)o[4 * i + 3] << 24;
    *d = make_uint4(wv[0], wv[1], wv[2], wv[3]);
}

// ---- the packet kernel ---------------------------------------------------------------------------------
constexpr int kRow = 16;  // lanes per packet (16 bytes each: 256 contiguous bytes per row per round)
#ifndef KFEC_GCM_BLOCK
#define KFEC_GCM_BLOCK 512  // 32 packets per workgroup share one LDS copy of the 40 KiB of tables
#endif
constexpr int kGcmBlock = KFEC_GCM_BLOCK;
constexpr int kRowsPerBlock = kGcmBlock / kRow;

struct GcmArgs {
    const uint32_t *src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint32_t *len;
    const uint16_t *iv;
    uint8_t *dst;
    uint64_t dst_pitch;
    uint32_t *out_len;
    uint8_t *ok;
    const uint4 *gh;      // [4][32][16] Shoup tables of H^1..H^4
    const uint8_t *ivt;   // [65536][32] J0, E_K(J0)
    const uint8_t *ks;    // [65536][kKsBytes] keystream
    const uint8_t *rk;    // AES round keys (blocks past the table)
    uint64_t P;
    uint32_t *done;       // counted launch (kfec_count.hpp)
};

// a * H^(p+1) from the LDS tables T = s_gh[p] ([32][16] entries): per input dword 8 lookups in flight, folded
// in with 3-input XORs (v_bitop3_b32)
__device__ __forceinline__ uint4 gh_mul(const uint4 (*T)[16], uint4 a)
{
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    // a rolled loop over the input dwords: one dword's 8 lookups (32 VGPRs) in flight, where the unrolled form
    // let the scheduler hoist all 32 (128 VGPRs) and cost a wave per SIMD
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        const uint32_t d = i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w;
        const uint32_t lo = (d << 4) & 0xF0F0F0F0u, hi = d & 0xF0F0F0F0u;  // 16 * nibble per byte
        const uint4(*Ti)[16] = T + 8 * i;
        uint4 e[8];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            e[2 * b] = *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint8_t *>(Ti[2 * b]) + ((lo >> (8 * b)) & 0xFFu));
            e[2 * b + 1] =
                *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint8_t *>(Ti[2 * b + 1]) + ((hi >> (8 * b)) & 0xFFu));
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            r0 = xor3(r0, e[2 * m].x, e[2 * m + 1].x);
            r1 = xor3(r1, e[2 * m].y, e[2 * m + 1].y);
            r2 = xor3(r2, e[2 * m].z, e[2 * m + 1].z);
            r3 = xor3(r3, e[2 * m].w, e[2 * m + 1].w);
        }
    }
    return make_uint4(r0, r1, r2, r3);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// keystream block i (i >= 1) computed here, for blocks past the table: out of line, so that its byte arrays do
// not weigh on the packet loop's registers
__device__ __noinline__ uint4 ctr_keystream(const uint8_t *rk, const uint8_t *j0, uint32_t i)
{
    uint8_t c[16], o[16];
    ctr_block(j0, i, c);
    aes256_encrypt(rk, c, o);
    return make_uint4((uint32_t)o[0] | o[1] << 8 | o[2] << 16 | (uint32_t)o[3] << 24,
                      (uint32_t)o[4] | o[5] << 8 | o[6] << 16 | (uint32_t)o[7] << 24,
                      (uint32_t)o[8] | o[9] << 8 | o[10] << 16 | (uint32_t)o[11] << 24,
                      (uint32_t)o[12] | o[13] << 8 | o[14] << 16 | (uint32_t)o[15] << 24);
}

#ifndef KFEC_GCM_WPE
#define KFEC_GCM_WPE 6  // waves per SIMD the register allocation must allow
#endif

template <bool OPEN>
__global__ void __launch_bounds__(kGcmBlock) __attribute__((amdgpu_waves_per_eu(KFEC_GCM_WPE))) gcm_kernel(GcmArgs a)
{
    __shared__ uint4 s_gh[kGhTables][32][16];  // 40 KiB: H, H^2, H^4, H^8, H^16
    {
        uint4 *flat = &s_gh[0][0][0];
        for (int i = threadIdx.x; i < kGhTables * 32 * 16; i += kGcmBlock) flat[i] = a.gh[i];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x % kRow;
    // the AD block: "KCP PortHopping" || 0x00 (aead.hpp:16) as little-endian dwords
    const uint4 ad = make_uint4(0x2050434Bu, 0x74726F50u, 0x70706F48u, 0x00676E69u);
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    for (uint64_t p = (uint64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kRow; p < a.P;
         p += (uint64_t)gridDim.x * kRowsPerBlock) {
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
            ptag = load16(a.src, a.src_dw, off + n + 4 * (lane & 3)).x;  // tag dword lane % 4
            iv = load16(a.src, a.src_dw, off + n + 16).x & 0xFFFFu;
        } else {
            if (L == 0 || (uint64_t)L + KFEC_AEAD_OVERHEAD > a.dst_pitch) {  // "empty data" / no room
                if (lane == 0) a.out_len[p] = 0;
                continue;
            }
            n = L;
            iv = a.iv[p];
        }
        const uint8_t *ivrow = a.ivt + 32 * (size_t)iv;
        const uint4 *ksrow = reinterpret_cast<const uint4 *>(a.ks + (size_t)iv * kKsBytes);
        const uint32_t nc = (n + 15) / 16;             // ciphertext blocks
        const uint32_t NB = nc + 2;                    // AD block, ciphertext blocks, length block
        const uint32_t pad = (kRow - NB % kRow) % kRow;  // leading zero blocks: the last block lands on lane 15
        const uint32_t rounds = (NB + pad) / kRow;
        uint8_t *dst = a.dst + p * a.dst_pitch;
        uint4 acc = zero;
        uint32_t ctail = 0;  // seal: the ciphertext's partial last dword
        for (uint32_t t = 0; t < rounds; ++t) {
            const int b = (int)(t * kRow + lane) - (int)pad;  // message block of this lane
            uint4 x = zero;
            if (b == 0) {
                x = ad;
            } else if (b == (int)NB - 1) {  // be64(8 * 15) || be64(8 * n)
                x = make_uint4(0u, bswap32(120u), bswap32(n >> 29), bswap32(n << 3));
            } else if (b > 0 && b < (int)NB - 1) {
                const uint32_t q = (uint32_t)b - 1, qb = 16 * q;
                uint4 ks = zero;
                if (qb + 16 <= kKsBytes) {
                    if (!(KFEC_GCM_AB & 2)) ks = ksrow[q];
                } else {  // past the table: AES of the counter block here
                    ks = ctr_keystream(a.rk, ivrow, q + 1);
                }
                uint4 in = load16(a.src, a.src_dw, off + qb);
                const uint32_t rem = n - qb;  // > 0
                if (rem < 16) in = mask16(in, rem);
                uint4 out = u4_xor(in, ks);
                if (rem < 16) out = mask16(out, rem);
                x = OPEN ? in : out;
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + qb);
                if (rem >= 16) {
                    *reinterpret_cast<uint4 *>(d32) = out;
                } else {
                    const uint32_t o4[4] = {out.x, out.y, out.z, out.w};
                    // open: whole dwords (the zero pad is part of the output); seal: whole dwords below n,
                    // the last partial dword goes out with the tag
                    const uint32_t nd = OPEN ? (rem + 3) / 4 : rem / 4;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if ((uint32_t)i < nd) d32[i] = o4[i];
                    if (!OPEN && (rem & 3)) ctail = o4[rem / 4];
                }
            }
            if (t && !(KFEC_GCM_AB & 1)) acc = gh_mul(s_gh[4], acc);  // * H^16
            acc = u4_xor(acc, x);
        }
        // lane l's accumulator ends on padded block 16 (rounds - 1) + l, so it carries H^(16 - l): fold the 16
        // lanes pairwise (the earlier lane of a pair of distance d times H^d), then times H
#pragma unroll 1
        for (int lv = 0; lv < 4; ++lv) {  // not unrolled: one multiply's 32 lookups in flight at a time
            const int d = 1 << lv;
            const uint4 other = make_uint4(__shfl_xor(acc.x, d, kRow), __shfl_xor(acc.y, d, kRow),
                                           __shfl_xor(acc.z, d, kRow), __shfl_xor(acc.w, d, kRow));
            const bool earlier = (lane & d) == 0;
            acc = u4_xor(gh_mul(s_gh[lv], earlier ? acc : other), earlier ? other : acc);
        }
        acc = gh_mul(s_gh[0], acc);
        const uint4 mask = *reinterpret_cast<const uint4 *>(ivrow + 16);
        const uint32_t tag[4] = {acc.x ^ mask.x, acc.y ^ mask.y, acc.z ^ mask.z, acc.w ^ mask.w};
        if (OPEN) {
            const uint32_t l4 = lane & 3;
            const uint32_t mine = l4 == 0 ? tag[0] : l4 == 1 ? tag[1] : l4 == 2 ? tag[2] : tag[3];
            uint32_t bad = mine != ptag ? 1u : 0u;
#pragma unroll
            for (int d = 1; d < kRow; d <<= 1) bad |= __shfl_xor(bad, d, kRow);
            if (bad) {  // no unauthenticated plaintext leaves the kernel
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                uint32_t *d32 = reinterpret_cast<uint32_t *>(dst);
                const uint32_t nd = (n + 3) / 4;
                for (uint32_t i = lane; i < nd; i += kRow) d32[i] = 0u;
            }
            if (lane == 0) {
                a.out_len[p] = bad ? 0u : n;
                a.ok[p] = bad ? 0 : 1;
            }
        } else {
            // dwords from floor4(n): the ciphertext's last n % 4 bytes || tag || iv_raw || zero pad (5 or 6
            // dwords, one per lane); the partial dword comes from the lane of ciphertext block nc - 1
            const uint32_t o = n & 3u, n4 = n & ~3u;
            const uint32_t cp = __shfl(ctail, (int)((nc + pad) % kRow), kRow);
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

}  // namespace

int gcm_setup(kfec_aead *k, const uint32_t *d_key, hipStream_t s)
{
    if (hipMalloc(&k->d_rk, 240) != hipSuccess || hipMalloc(&k->d_h, 16) != hipSuccess ||
        hipMalloc(&k->d_gh, kGhTables * 32 * 16 * 16) != hipSuccess || hipMalloc(&k->d_ivt, 65536 * 32) != hipSuccess ||
        hipMalloc(&k->d_ks, (size_t)65536 * kKsBytes) != hipSuccess)
        return KFEC_ENOMEM;
    k->ks_bytes = kKsBytes;
    hipLaunchKernelGGL(gcm_key_kernel, dim3(1), dim3(64), 0, s, d_key, k->d_rk, k->d_h);
    hipLaunchKernelGGL(gcm_tables_kernel, dim3(kGhTables * 32 * 16 / 256), dim3(256), 0, s, k->d_h, k->d_gh);
    hipLaunchKernelGGL(gcm_iv_kernel, dim3(65536 / 256), dim3(256), 0, s, k->d_rk, k->d_h, k->d_ivt);
    const uint64_t ks_threads = 65536ull * (kKsBytes / 16);
    hipLaunchKernelGGL(gcm_ks_kernel, dim3((uint32_t)((ks_threads + 255) / 256)), dim3(256), 0, s, k->d_rk,
                       k->d_ivt, k->d_ks);
    return hipGetLastError() == hipSuccess ? KFEC_OK : KFEC_EHIP;
}

void gcm_free(kfec_aead *k)
{
    for (void *p : {(void *)k->d_rk, (void *)k->d_h, (void *)k->d_gh, (void *)k->d_ivt, (void *)k->d_ks,
                    (void *)k->d_ocb})
        if (p) (void)hipFree(p);
    k->d_rk = k->d_h = k->d_gh = k->d_ivt = k->d_ks = k->d_ocb = nullptr;
}

int launch_gcm(const kfec_aead *k, bool open, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
               const uint32_t *len, const uint16_t *iv, void *dst, size_t dst_pitch, uint32_t *out_len, uint8_t *ok,
               hipStream_t s, uint32_t *done, uint32_t *blocks)
{
    if (blocks) *blocks = 0;
    if (P == 0) return 0;
    GcmArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.iv = iv;
    a.dst = static_cast<uint8_t *>(dst);
    a.dst_pitch = dst_pitch;
    a.out_len = out_len;
    a.ok = ok;
    a.gh = reinterpret_cast<const uint4 *>(k->d_gh);
    a.ivt = k->d_ivt;
    a.ks = k->d_ks;
    a.rk = k->d_rk;
    a.P = P;
    a.done = done;
    const int cus = current_device_cus();
    // 40 KiB of GHASH tables per workgroup: 3 resident per CU at 512 lanes (6 waves per SIMD), 4 at 256;
    // grid-stride over packets
    const uint64_t want = (P + kRowsPerBlock - 1) / kRowsPerBlock;
    const dim3 grid((uint32_t)std::min<uint64_t>(want, (uint64_t)cus * (kGcmBlock >= 512 ? 3 : 4)));
    if (blocks && done) *blocks = grid.x;
    if (open) hipLaunchKernelGGL(gcm_kernel<true>, grid, dim3(kGcmBlock), 0, s, a);
    else hipLaunchKernelGGL(gcm_kernel<false>, grid, dim3(kGcmBlock), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace kfec
