// kfec_frame.hip -- gfx950 kernels of the framing and wire layer around the coder (include/kfec_frame.h):
// shard framing on both sides (compact_into_container, data_operations.cpp:610-667), datagram extraction
// (extract_from_container, :697-704), FEC wire packets (connections.cpp:395-430, 488-511) and the device
// form of the receive cache's shard insert (client.cpp:851-892).
//
// All of it is byte movement: HBM-bound, one dword per lane per item, consecutive lanes on consecutive
// dwords of one slot / packet so that every wave-instruction stores 256 contiguous bytes.  Payloads sit at
// arbitrary byte offsets and are re-based by a 2-, 9- or 13-byte header, so each output dword is
// assembled from the two aligned source dwords that cover it (v_alignbyte_b32) and masked to the payload;
// the neighbouring lanes' overlapping source dwords come from the same cache lines, so HBM sees each
// payload byte about once.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/kfec_frame.h"
#include "kfec_gf.hpp"
#include "kfec_internal.hpp"

namespace kfec {

namespace {

constexpr int kFrameBlock = 256;
constexpr uint64_t kMaxGrid = 1u << 24;

// 16 bytes [q0, q0 + 16) of the payload base[start, start + len) as 4 dwords, zero outside it: one 16-byte
// load at the covering dword (dword aligned is enough on gfx950, as the MAC kernel's granules rely on) and
// one more dword, re-based with v_alignbyte_b32.  Dwords at or beyond lim32 read as zero.
__device__ __forceinline__ void payload_quad(const uint32_t *base32, uint64_t lim32, uint64_t start, uint32_t len,
                                             int64_t q0l, uint32_t (&o)[4])
{
    const int32_t q0 = (int32_t)q0l;                     // |q0| < 2^17: slot and packet offsets
    const int lo = max(0, -q0), hi = min(16, (int32_t)len - q0);  // payload bytes [lo, hi) of the chunk
    if (hi <= lo) {  // nothing of the payload here (zero padding, headers): no loads
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = 0u;
        return;
    }
    const uint64_t a4 = start + (uint64_t)(int64_t)(q0 + 16);  // first byte's address + 16 (q0 >= -15)
    const uint64_t w4 = a4 >> 2;                                // its dword index + 4
    const uint32_t sh = (uint32_t)(a4 & 3u);
    uint32_t d[5];
    if (w4 >= 4 && w4 + 1 <= lim32) {
        const uint4 x = *reinterpret_cast<const uint4 *>(base32 + (w4 - 4));
        d[0] = x.x; d[1] = x.y; d[2] = x.z; d[3] = x.w;
        d[4] = (sh && w4 < lim32) ? base32[w4] : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint64_t w = w4 - 4 + i;  // may wrap below zero: then >= lim32 and read as 0
            d[i] = (w4 + i >= 4 && w < lim32) ? base32[w] : 0u;
        }
    }
    const uint32_t M = ((1u << hi) - 1u) & ~((1u << lo) - 1u);  // valid bytes of the 16 (hi <= 16)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;  // bit b of nib -> byte b
        o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & bm;
    }
}

// header bytes [4k, 4k + 4) of an H-byte header packed little-endian into h[0..3]
__device__ __forceinline__ uint32_t header_dword(const uint32_t (&h)[4], uint32_t H, uint64_t k)
{
    if (4 * k >= H) return 0u;
    const uint32_t w = k == 0 ? h[0] : (k == 1 ? h[1] : (k == 2 ? h[2] : h[3]));
    const uint32_t n = H - 4 * (uint32_t)k;
    return n >= 4 ? w : (w & ((1u << (8 * n)) - 1u));
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// ---- alignment (block size) per group ------------------------------------------------------------------

// send: align = max len + 2 (data_operations.cpp:613-616); receive: max(len + 2 for data, len for parity)
// over the present shards (:638-646).  0 when a shard does not fit in B.
__global__ void __launch_bounds__(kFrameBlock) align_kernel(uint64_t G, uint32_t S, uint32_t K, const uint16_t *len,
                                                            const uint64_t *present, uint32_t B, uint16_t *align)
{
    const uint64_t g = blockIdx.x * (uint64_t)kFrameBlock + threadIdx.x;
    if (g >= G) return;
    uint32_t a = 0;
    bool over = false;
    for (uint32_t s = 0; s < S; ++s) {
        if (present && !((present[g * 4 + (s >> 6)] >> (s & 63)) & 1ull)) continue;
        const uint32_t need = len[g * S + s] + (s < K ? KFEC_FEC_CONTAINER_HEADER : 0u);
        a = max(a, need);
        over |= need > B;
    }
    align[g] = over ? 0 : (uint16_t)a;
}

// ---- framing: one dword of one shard slot per item ----------------------------------------------------
struct FrameArgs {
    const uint32_t *__restrict__ src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint16_t *len;
    const uint64_t *present;  // null on the send side (every slot written)
    const uint16_t *align;
    uint8_t *data;
    uint8_t *parity;
    uint64_t pitch;
    uint64_t rows;  // G * S
    uint32_t S, K, R, cols;
};

// Half a wave (32 lanes) per row: a 1,444-byte shard slot is 91 chunks of 16 B = 32 + 32 + 27, so lanes stay
// busy (one row per 64 lanes would leave the second pass 42% occupied).
constexpr uint32_t kRowLanes = 32;
constexpr uint32_t kRowsPerBlock = kFrameBlock / kRowLanes;

__device__ __forceinline__ uint32_t row_in_block() { return threadIdx.x / kRowLanes; }

// Write dwords [0, nd) of one row: an H-byte header followed by payload bytes [0, len) of base[start..],
// zero after the payload.  Lane l of the row's 32 writes 16-byte chunks l, l + 32, ...; a row's last chunk, when it is
// partial, is written dword by dword so that nothing past dword nd is touched.
#ifndef KFEC_FRAME_REG
#define KFEC_FRAME_REG 1  // 0: every row streams round by round (A/B knob)
#endif
constexpr uint32_t kQuadRounds = 4;  // rows of up to 2 KiB are loaded whole (every kcptube slot and packet)

__device__ uint4 g_zero16;  // never written: the target of the loads a lane does not need

// payload_quad without a branch: both loads are always issued (a chunk without payload reads g_zero16), so
// the loads of all the rounds of a row are in flight together.  A load under a branch is waited for at the
// join (its value is a phi there), which kept one round per row in flight.  The caller checks that every
// window lies inside the buffer.
__device__ __forceinline__ void payload_quad_nb(const uint32_t *base32, uint64_t start, uint32_t len, int32_t q0,
                                                uint32_t (&o)[4])
{
    const int lo = max(0, -q0), hi = min(16, (int32_t)len - q0);  // payload bytes [lo, hi) of the chunk
    const bool any = hi > lo;
    const uint64_t a4 = start + (uint64_t)(int64_t)(q0 + 16);
    const uint64_t w4 = a4 >> 2;
    const uint32_t sh = (uint32_t)(a4 & 3u);
    const uint4 x = *(any ? reinterpret_cast<const uint4 *>(base32 + (w4 - 4)) : &g_zero16);
    const uint32_t x4 = *(any && sh ? base32 + w4 : &g_zero16.x);
    const uint32_t d[5] = {x.x, x.y, x.z, x.w, x4};
    const uint32_t M = any ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & (((nib * 0x00204081u) & 0x01010101u) * 0xFFu);
    }
}

__device__ __forceinline__ void store_quads(uint32_t *__restrict__ dst, uint32_t nd, const uint32_t (&h)[4], uint32_t H,
                                            const uint32_t *__restrict__ base, uint64_t lim32, uint64_t start,
                                            uint32_t len, uint32_t lane)
{
    if (KFEC_FRAME_REG && nd <= 4 * kRowLanes * kQuadRounds && start >= H && ((start + len + 15) >> 2) + 1 <= lim32) {
        uint32_t o[kQuadRounds][4];
#pragma unroll
        for (uint32_t r = 0; r < kQuadRounds; ++r)
            payload_quad_nb(base, start, len, (int32_t)(16 * (r * kRowLanes + lane)) - (int32_t)H, o[r]);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) o[0][i] |= header_dword(h, H, i);
        }
#pragma unroll
        for (uint32_t r = 0; r < kQuadRounds; ++r) {
            const uint32_t j = r * kRowLanes + lane;
            if (4 * j + 4 <= nd) {
                *reinterpret_cast<uint4 *>(dst + 4 * j) = make_uint4(o[r][0], o[r][1], o[r][2], o[r][3]);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (4 * j + i < nd) dst[4 * j + i] = o[r][i];
            }
        }
        return;
    }
    for (uint32_t j = lane; 4 * j < nd; j += kRowLanes) {
        uint32_t o[4];
        payload_quad(base, lim32, start, len, (int64_t)(16 * j) - H, o);
        if (j == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] |= header_dword(h, H, i);
        }
        if (4 * j + 4 <= nd) {
            *reinterpret_cast<uint4 *>(dst + 4 * j) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (4 * j + i < nd) dst[4 * j + i] = o[i];
        }
    }
}

__global__ void __launch_bounds__(kFrameBlock) frame_kernel(FrameArgs a)
{
    const uint32_t lane = threadIdx.x % kRowLanes;
    for (uint64_t slot = (uint64_t)blockIdx.x * kRowsPerBlock + row_in_block(); slot < a.rows;
         slot += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint64_t g = slot / a.S;
        const uint32_t s = (uint32_t)(slot - g * a.S);
        if (a.present && !((a.present[g * 4 + (s >> 6)] >> (s & 63)) & 1ull)) continue;
        uint32_t *dst = reinterpret_cast<uint32_t *>(s < a.K ? a.data + (g * a.K + s) * a.pitch
                                                             : a.parity + (g * a.R + (s - a.K)) * a.pitch);
        const bool ok = a.align[g] != 0;
        const uint32_t n = ok ? a.len[slot] : 0u;
        const uint64_t off = ok ? a.off[slot] : 0u;
        const uint32_t H = (ok && s < a.K) ? KFEC_FEC_CONTAINER_HEADER : 0u;
        const uint32_t h[4] = {(n >> 8) | ((n & 0xFFu) << 8), 0u, 0u, 0u};  // htons(length)
        store_quads(dst, a.cols, h, H, a.src, a.src_dw, off, n, lane);
    }
}

// ---- extraction of recovered datagrams ----------------------------------------------------------------
struct UnframeArgs {
    const uint8_t *out;
    const uint8_t *out_idx;
    uint16_t *rec_len;
    uint8_t *dst;
    uint64_t pitch, dst_pitch, rows;
    uint32_t R, B;
};

__global__ void __launch_bounds__(kFrameBlock) unframe_kernel(UnframeArgs a)
{
    const uint32_t lane = threadIdx.x % kRowLanes;
    for (uint64_t slot = (uint64_t)blockIdx.x * kRowsPerBlock + row_in_block(); slot < a.rows;
         slot += (uint64_t)gridDim.x * kRowsPerBlock) {
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(a.out + slot * a.pitch);
        uint32_t n = 0xFFFFu;
        if (a.out_idx[slot] != 0xFF) {
            const uint32_t d0 = s32[0];
            n = ((d0 & 0xFFu) << 8) | ((d0 >> 8) & 0xFFu);  // ntohs(data_length)
            if (n + KFEC_FEC_CONTAINER_HEADER > a.B) n = 0xFFFFu;
        }
        if (lane == 0) a.rec_len[slot] = (uint16_t)n;
        if (!a.dst || n == 0xFFFFu) continue;
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.dst + slot * a.dst_pitch);
        const uint32_t h0[4] = {0u, 0u, 0u, 0u};
        store_quads(dst, (n + 3) / 4, h0, 0u, s32, a.pitch / 4, KFEC_FEC_CONTAINER_HEADER, n, lane);
    }
}

// ---- wire packets ---------------------------------------------------------------------------------------
struct PackArgs {
    const uint32_t *__restrict__ src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint16_t *len;
    const uint8_t *parity;
    const uint16_t *align;
    const uint32_t *sn, *conv;
    uint8_t *pkt;
    uint16_t *pkt_len;
    uint64_t pitch, pkt_pitch, rows;
    uint32_t K, N, which, timestamp, nsel, s0;
};

__global__ void __launch_bounds__(kFrameBlock) pack_kernel(PackArgs a)
{
    const uint32_t lane = threadIdx.x % kRowLanes;
    for (uint64_t pk = (uint64_t)blockIdx.x * kRowsPerBlock + row_in_block(); pk < a.rows;
         pk += (uint64_t)gridDim.x * kRowsPerBlock) {
        // rows run over the selected kinds only: row pk is packet s0 + k of group g (k < nsel)
        const uint64_t g = pk / a.nsel;
        const uint32_t s = a.s0 + (uint32_t)(pk - g * a.nsel);
        const bool red = s >= a.K;
        // output slot: (g, s) of [G][N], or of [G][emitted kinds] with KFEC_PACK_COMPACT
        const uint64_t slot = (a.which & KFEC_PACK_COMPACT) ? pk : g * a.N + s;
        const uint32_t H = red ? KFEC_PKT_REDUNDANT_HEADER : KFEC_PKT_DATA_HEADER;
        const uint32_t n = red ? a.align[g] : a.len[g * a.K + s];
        const bool fits = H + n <= a.pkt_pitch && !(red && n == 0);
        if (lane == 0) a.pkt_len[slot] = fits ? (uint16_t)(H + n) : (uint16_t)0;
        if (!fits) continue;
        uint32_t h[4];
        h[0] = a.timestamp;      // host_to_little_endian
        h[1] = bswap32(a.sn[g]);  // htonl
        const uint32_t cv = red ? bswap32(a.conv[g]) : 0u;
        h[2] = s | (cv << 8);
        h[3] = cv >> 24;
        const uint32_t *base;
        uint64_t lim, off;
        if (red) {
            base = reinterpret_cast<const uint32_t *>(a.parity + (g * (a.N - a.K) + (s - a.K)) * a.pitch);
            lim = a.pitch / 4;
            off = 0;
        } else {
            base = a.src;
            lim = a.src_dw;
            off = a.off[g * a.K + s];
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.pkt + slot * a.pkt_pitch);
        store_quads(dst, (H + n + 3) / 4, h, H, base, lim, off, n, lane);
    }
}

__global__ void __launch_bounds__(kFrameBlock) unpack_kernel(uint64_t P, uint32_t K, const uint8_t *src,
                                                             const uint64_t *off, const uint32_t *len,
                                                             kfec_pkt_hdr *hdr)
{
    const uint64_t p = blockIdx.x * (uint64_t)kFrameBlock + threadIdx.x;
    if (p >= P) return;
    const uint8_t *b = src + off[p];
    const uint32_t n = len[p];
    kfec_pkt_hdr h{};
    h.kind = KFEC_PKT_KIND_MALFORMED;
    if (n >= KFEC_PKT_DATA_HEADER) {
        h.timestamp = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
        h.sn = ((uint32_t)b[4] << 24) | ((uint32_t)b[5] << 16) | ((uint32_t)b[6] << 8) | (uint32_t)b[7];
        h.sub_sn = b[8];
        const bool red = h.sub_sn >= K;
        const uint32_t H = red ? KFEC_PKT_REDUNDANT_HEADER : KFEC_PKT_DATA_HEADER;
        if (n >= H && n - H <= 0xFFFFu) {
            h.kind = red ? KFEC_PKT_KIND_REDUNDANT : KFEC_PKT_KIND_DATA;
            h.payload_off = off[p] + H;
            h.payload_len = (uint16_t)(n - H);
            const uint8_t *q = b + H;
            if (red)
                h.conv = ((uint32_t)b[9] << 24) | ((uint32_t)b[10] << 16) | ((uint32_t)b[11] << 8) | (uint32_t)b[12];
            else if (n - H >= 4)
                h.conv = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        }
    }
    hdr[p] = h;
}

// Receive-cache insert in three passes, so that a duplicated (sn, sub_sn) resolves to ONE packet -- the one
// with the highest index, i.e. the last to arrive, as fec_rcv_cache[sn][sub_sn] = ... overwrites
// (client.cpp:869,887) -- and its offset and length are never mixed with another copy's:
//   clear:  off[e] = 0 for every targeted entry
//   claim:  atomicMax(off[e], TAG | p)           (TAG = bit 63: no payload offset carries it)
//   commit: the packet whose tag survived writes off / len and sets its present bit
__device__ __forceinline__ int64_t scatter_entry(const kfec_pkt_hdr &h, uint64_t p, uint32_t N, const int32_t *slot_of,
                                                 uint32_t sn_base, uint64_t G)
{
    if (h.kind == KFEC_PKT_KIND_MALFORMED || h.sub_sn >= N) return -1;
    const int64_t slot = slot_of ? (int64_t)slot_of[p] : (int64_t)(uint32_t)(h.sn - sn_base);
    if (slot < 0 || (uint64_t)slot >= G) return -1;
    return slot * (int64_t)N + h.sub_sn;
}

constexpr uint64_t kScatterTag = 1ull << 63;

__global__ void __launch_bounds__(kFrameBlock) scatter_kernel(int pass, uint64_t P, uint32_t N, const kfec_pkt_hdr *hdr,
                                                              const int32_t *slot_of, uint32_t sn_base, uint64_t G,
                                                              unsigned long long *present, uint64_t *off,
                                                              uint16_t *len)
{
    const uint64_t p = blockIdx.x * (uint64_t)kFrameBlock + threadIdx.x;
    if (p >= P) return;
    const kfec_pkt_hdr h = hdr[p];
    const int64_t e = scatter_entry(h, p, N, slot_of, sn_base, G);
    if (e < 0) return;
    if (pass == 0) {
        off[e] = 0;
    } else if (pass == 1) {
        atomicMax(reinterpret_cast<unsigned long long *>(off + e), (unsigned long long)(kScatterTag | p));
    } else if (off[e] == (kScatterTag | p)) {
        off[e] = h.payload_off;
        len[e] = h.payload_len;
        atomicOr(&present[(uint64_t)e / N * 4 + (h.sub_sn >> 6)], 1ull << (h.sub_sn & 63));
    }
}

// ---- fused compact_into_container + encode ---------------------------------------------------------------
// Parity of framed groups without materialising the framed slots: lane (group, 32-byte column) assembles the
// column of framed slot j -- [BE16 len][datagram][zeros] -- straight from the datagram arena (two 16-byte
// re-based loads) and runs the same perm MAC as mac_kernel, with the coefficient tables of the encoding
// matrix read by scalar loads.  Saves the slot write and re-read of frame_data + encode (2 x G*K*B bytes).
// The workgroup stages the (offset, length) of its groups' datagrams in LDS.
struct FramedArgs {
    const uint32_t *src;
    uint64_t src_dw;
    const uint64_t *off;
    const uint16_t *len;
    uint16_t *align;        // written: max length + 2, 0 for a group holding a datagram too long for B (its
                            // slots, hence parity, are zero)
    uint8_t *parity;
    const uint32_t *etab;   // [K][etab_rows][5] perm tables (kfec_internal.hpp enc_tab_*)
    uint64_t pitch;
    uint32_t total, cols, K, R, B, etab_rows, gmax;
    // data packets (framed_encode_kernel<MT, true>): pkt[g][N][pkt_pitch], pkt_len[g][N], as kfec_pack_batch
    uint8_t *pkt;
    uint16_t *pkt_len;
    const uint32_t *sn;
    uint64_t pkt_pitch;
    uint32_t N, timestamp;
};

// 32 bytes [q0, q0 + 32) of the payload base[start, start + len) as 8 dwords, zero outside it (q0 > -32;
// a window reaching below the arena's start reads those dwords as zero).
// Nine dword-aligned dwords (two 16-byte loads and one dword; per-dword guarded loads only where the window
// touches the ends of the arena) re-based by v_alignbyte_b32, then masked without branches: the window's
// valid bytes form one 32-bit mask M (bit k = byte k), and dword i's byte mask is its nibble of M spread to
// bytes by a multiply.  About 6 VALU per dword, against ~15 for two masked payload_quad calls.
__device__ __forceinline__ void payload_window(const uint32_t *base32, uint64_t lim32, uint64_t start, uint32_t len,
                                               int32_t q0, uint32_t (&o)[8])
{
    const int lo = max(0, -q0), hi = min(32, (int32_t)len - q0);  // payload bytes [lo, hi) of the window
    if (hi <= lo) {  // nothing of the payload here (zero padding, headers): no loads
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = 0u;
        return;
    }
    const int64_t ab = (int64_t)start + q0;  // the window's first byte (below the arena for a header window)
    const int64_t w0 = ab >> 2;               // its dword (floor)
    const uint32_t sh = (uint32_t)(ab & 3);
    uint32_t d[9];
    if (w0 >= 0 && w0 + 9 <= (int64_t)lim32) {
        const uint4 p = *reinterpret_cast<const uint4 *>(base32 + w0);
        const uint4 q = *reinterpret_cast<const uint4 *>(base32 + w0 + 4);
        d[0] = p.x; d[1] = p.y; d[2] = p.z; d[3] = p.w;
        d[4] = q.x; d[5] = q.y; d[6] = q.z; d[7] = q.w;
        d[8] = base32[w0 + 8];
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const int64_t w = w0 + i;
            d[i] = (w >= 0 && w < (int64_t)lim32) ? base32[w] : 0u;
        }
    }
    const uint32_t mhi = hi >= 32 ? 0xFFFFFFFFu : (1u << hi) - 1u;
    const uint32_t M = mhi & ~((1u << lo) - 1u);  // lo < hi <= 32, so lo < 32
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;  // bit b of nib -> byte b
        o[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh) & bm;
    }
}

// framed bytes [32 col, 32 col + 32) of a slot holding an n-byte datagram at byte `off` of the arena
__device__ __forceinline__ void framed_gran(const uint32_t *src, uint64_t lim, uint64_t off, uint32_t n, uint32_t col,
                                            uint32_t (&x)[8])
{
    payload_window(src, lim, off, n, (int32_t)(32 * col) - KFEC_FEC_CONTAINER_HEADER, x);
    if (col == 0) x[0] |= (n >> 8) | ((n & 0xFFu) << 8);  // htons(length)
}

// create_fec_data_packet (connections.cpp:395-411) for datagram j of group g, by the lanes of its columns:
// lane `col` writes the 16-byte-aligned packet bytes [32 cc, 32 cc + 32) for cc = col, col + cols, ... below
// the packet's length (windows past the framed columns exist only for a datagram too long for B), re-read
// from the arena -- the lines the MAC just loaded -- and lane 0 adds the 9-byte header.  Same bytes and
// lengths as pack_kernel's data packets.
__device__ __forceinline__ void data_packet(const FramedArgs &a, uint64_t g, uint32_t j, uint32_t col, uint64_t off,
                                            uint32_t n)
{
    const uint32_t plen = KFEC_PKT_DATA_HEADER + n, nd = (plen + 3) / 4;
    uint32_t *dst = reinterpret_cast<uint32_t *>(a.pkt + (g * a.N + j) * a.pkt_pitch);
    const bool fits = plen <= a.pkt_pitch;
    if (col == 0) a.pkt_len[g * a.N + j] = fits ? (uint16_t)plen : (uint16_t)0;
    if (!fits) return;
    for (uint32_t cc = col; 32 * cc < plen; cc += a.cols) {
        uint32_t w[8];
        // packet byte q holds datagram byte q - 9: the window starts 9 bytes before the datagram for cc = 0
        payload_window(a.src, a.src_dw, off, n, (int32_t)(32 * cc) - (int32_t)KFEC_PKT_DATA_HEADER, w);
        if (cc == 0) {
            w[0] = a.timestamp;                 // host_to_little_endian
            w[1] = __builtin_bswap32(a.sn[g]);  // htonl
            w[2] |= j;                          // sub_sn
        }
        const uint32_t d0 = 8 * cc;
        if (d0 + 8 <= nd) {
            typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u32x4_t{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4_t *>(dst + d0));
            __builtin_nontemporal_store(u32x4_t{w[4], w[5], w[6], w[7]}, reinterpret_cast<u32x4_t *>(dst + d0 + 4));
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (d0 + i < nd) dst[d0 + i] = w[i];
        }
    }
}

template <int MT, bool DPK = false>
__global__ void __launch_bounds__(256) framed_encode_kernel(FramedArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s_raw[];
    uint64_t *s_off = reinterpret_cast<uint64_t *>(s_raw);
    // s_len: the datagram's length, bit 31 set when its group's slots read as zeros (a datagram too long for B)
    uint32_t *s_len = reinterpret_cast<uint32_t *>(s_raw + (size_t)a.gmax * a.K * 8);
    uint32_t *s_al = s_len + (size_t)a.gmax * a.K;  // per group: max length + 2 (the align), then the flag pass
    const uint32_t K = a.K, cols = a.cols;
    const uint32_t base = blockIdx.x * 256u, item = base + threadIdx.x;
    const uint32_t gfirst = base / cols, glast = min(base + 255u, a.total - 1) / cols, ng = glast - gfirst + 1;
    // align of the send side (data_operations.cpp:613-616) computed here, per workgroup, for its groups
    for (uint32_t gs = threadIdx.x; gs < ng; gs += 256) s_al[gs] = 0;
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < ng * K; e += 256) {
        const uint32_t gs = e / K, j = e - gs * K;
        const uint64_t gj = (uint64_t)(gfirst + gs) * K + j;
        const uint32_t n = a.len[gj];
        s_off[e] = a.off[gj];
        s_len[e] = n;
        atomicMax(&s_al[gs], n + KFEC_FEC_CONTAINER_HEADER);
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < ng * K; e += 256)
        if (s_al[e / K] > a.B) s_len[e] |= 0x80000000u;  // a datagram too long for B: the slots read as zeros
    if (blockIdx.y == 0)  // every workgroup touching a group writes the same value
        for (uint32_t gs = threadIdx.x; gs < ng; gs += 256)
            a.align[gfirst + gs] = s_al[gs] > a.B ? (uint16_t)0 : (uint16_t)s_al[gs];
    __syncthreads();
    const uint32_t row0 = blockIdx.y * MT;
    const uint32_t rows = a.R > row0 ? min((uint32_t)MT, a.R - row0) : 0u;
    if (item >= a.total || rows == 0) return;
    const uint32_t g = item / cols, col = item - g * cols, gs = g - gfirst;
    uint32_t acc[MT][8];
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) acc[r][w] = 0;
    auto load = [&](uint32_t j, uint32_t (&x)[8]) {
        const uint32_t n = s_len[gs * K + j];
        if (n & 0x80000000u) {
#pragma unroll
            for (int w = 0; w < 8; ++w) x[w] = 0;
        } else {
            framed_gran(a.src, a.src_dw, s_off[gs * K + j], n, col, x);
        }
    };
    uint32_t x0[8], x1[8];
    load(0, x0);
    if (K > 1) load(1, x1);
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    // one shard: MAC the granule in x, then refill x with shard jj + 2 (two shards' loads in flight)
    auto step = [&](uint32_t jj, uint32_t (&x)[8]) {
        uint32_t cur[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) cur[w] = x[w];
        if (jj + 2 < K) load(jj + 2, x);
        const cu32 *tg = (const cu32 *)(a.etab + ((size_t)jj * a.etab_rows + row0) * 5);
        uint32_t t[5 * MT];
#pragma unroll
        for (int i = 0; i < 5 * MT; ++i) t[i] = tg[i];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t xv = cur[w];
            const uint32_t s0 = xv & 0x07070707u, s1 = (xv >> 3) & 0x07070707u, s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < MT; ++r) acc[r][w] = perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
        }
        if constexpr (DPK) {
            if (blockIdx.y == 0) data_packet(a, g, jj, col, s_off[gs * K + jj], s_len[gs * K + jj] & 0xFFFFu);
        }
    };
    for (uint32_t j = 0; j < K; j += 2) {
        step(j, x0);
        if (j + 1 < K) step(j + 1, x1);
    }
    const uint32_t nd = (col + 1) * 32 > a.B ? (a.B - col * 32 + 3) / 4 : 8u;  // dwords of this column below B
#pragma unroll
    for (int r = 0; r < MT; ++r) {
        if ((uint32_t)r >= rows) continue;
        uint32_t *o = reinterpret_cast<uint32_t *>(a.parity + ((uint64_t)g * a.R + row0 + r) * a.pitch) + col * 8;
        if (nd == 8) {
            typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u32x4_t{acc[r][0], acc[r][1], acc[r][2], acc[r][3]}, reinterpret_cast<u32x4_t *>(o));
            __builtin_nontemporal_store(u32x4_t{acc[r][4], acc[r][5], acc[r][6], acc[r][7]},
                                        reinterpret_cast<u32x4_t *>(o + 4));
        } else {
#pragma unroll
            for (int w = 0; w < 8; ++w)
                if ((uint32_t)w < nd) o[w] = acc[r][w];
        }
    }
}

// ---- fused receive compact_into_container + decode ---------------------------------------------------------
// The recovered data shards of G cached groups straight from the packet arena: decode_prep_* has chosen each
// group's K shares and written the coefficient rows of its missing data shards (decode records, as for
// kfec_decode_batch); lane (group, 32-byte column) assembles column `col` of each chosen share on the fly --
// a data shard framed as [BE16 len][payload][zeros], a parity shard raw and zero-padded -- and runs the perm
// MAC.  Saves frame_shards' write of every present shard and the decoder's re-read of it.  The workgroup stages
// its groups' (offset, length, kind) of the chosen shares and their perm tables in LDS.
struct FramedDecArgs {
    const uint32_t *src;
    uint64_t src_dw;
    const uint64_t *off;    // [G][N]
    const uint16_t *len;    // [G][N]
    const uint16_t *align;  // 0: a present shard does not fit in B (the group's shards read as zeros)
    const uint8_t *rec;     // decode records (kfec_internal.hpp record_stride)
    uint8_t *out;           // [G][R][pitch]
    uint64_t pitch;
    uint32_t total, cols, K, N, R, B, gmax, rec_stride;
};

constexpr uint32_t kDecData = 0x80000000u;  // s_len flag: a data shard (framed on the fly)
constexpr uint32_t kDecZero = 0xFFFFFFFFu;  // s_len: reads as zeros

template <int MT>
__global__ void __launch_bounds__(256) framed_decode_kernel(FramedDecArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s_raw[];
    const uint32_t K = a.K, cols = a.cols, K4 = (K + 3) & ~3u;
    const uint32_t base = blockIdx.x * 256u, item = base + threadIdx.x;
    const uint32_t gfirst = base / cols, glast = min(base + 255u, a.total - 1) / cols, ng = glast - gfirst + 1;
    uint32_t *s_tab = reinterpret_cast<uint32_t *>(s_raw);                              // [ng][K][MT][5]
    uint64_t *s_off = reinterpret_cast<uint64_t *>(s_raw + (size_t)a.gmax * K * MT * 20);  // [ng][K]
    uint32_t *s_len = reinterpret_cast<uint32_t *>(s_off + (size_t)a.gmax * K);           // [ng][K]
    const uint32_t row0 = blockIdx.y * MT;
    for (uint32_t e = threadIdx.x; e < ng * K; e += 256) {
        const uint32_t gs = e / K, j = e - gs * K, g = gfirst + gs;
        const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
        const uint32_t st = rec[0], m = rec[1];
        const bool work = st == 0 && m > row0;
        uint32_t n = kDecZero;
        uint64_t o = 0;
        if (work && a.align[g] != 0) {
            const uint32_t src = rec[4 + j];
            const uint64_t idx = (uint64_t)g * a.N + src;
            o = a.off[idx];
            n = (uint32_t)a.len[idx] | (src < K ? kDecData : 0u);
        }
        s_off[e] = o;
        s_len[e] = n;
#pragma unroll
        for (int r = 0; r < MT; ++r) {
            const uint32_t u = row0 + r;
            const uint32_t c = (work && u < m) ? rec[4 + K4 + u * K4 + j] : 0u;
            uint32_t t[5];
            gf_perm_tables(c, t);
#pragma unroll
            for (int i = 0; i < 5; ++i) s_tab[((size_t)e * MT + r) * 5 + i] = t[i];
        }
    }
    __syncthreads();
    if (item >= a.total) return;
    const uint32_t g = item / cols, col = item - g * cols, gs = g - gfirst;
    uint32_t rows = 0;
    {
        const uint8_t *rec = a.rec + (uint64_t)g * a.rec_stride;
        const uint32_t st = rec[0], m = rec[1];
        rows = (st == 0 && m > row0) ? min((uint32_t)MT, m - row0) : 0u;
    }
    if (rows == 0) return;
    uint32_t acc[MT][8];
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) acc[r][w] = 0;
    auto load = [&](uint32_t j, uint32_t (&x)[8]) {
        const uint32_t n = s_len[gs * K + j];
        const uint64_t o = s_off[gs * K + j];
        if (n == kDecZero) {
#pragma unroll
            for (int w = 0; w < 8; ++w) x[w] = 0;
        } else if (n & kDecData) {
            framed_gran(a.src, a.src_dw, o, n & 0xFFFFu, col, x);
        } else {
            payload_window(a.src, a.src_dw, o, n, (int32_t)(32 * col), x);
        }
    };
    uint32_t x0[8], x1[8];
    load(0, x0);
    if (K > 1) load(1, x1);
    auto step = [&](uint32_t jj, uint32_t (&x)[8]) {
        uint32_t cur[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) cur[w] = x[w];
        if (jj + 2 < K) load(jj + 2, x);
        const uint32_t *tp = s_tab + ((size_t)(gs * K + jj) * MT) * 5;
        uint32_t t[5 * MT];
#pragma unroll
        for (int i = 0; i < 5 * MT; ++i) t[i] = tp[i];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            const uint32_t xv = cur[w];
            const uint32_t s0 = xv & 0x07070707u, s1 = (xv >> 3) & 0x07070707u, s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
            for (int r = 0; r < MT; ++r) acc[r][w] = perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
        }
    };
    for (uint32_t j = 0; j < K; j += 2) {
        step(j, x0);
        if (j + 1 < K) step(j + 1, x1);
    }
    const uint32_t nd = (col + 1) * 32 > a.B ? (a.B - col * 32 + 3) / 4 : 8u;  // dwords of this column below B
#pragma unroll
    for (int r = 0; r < MT; ++r) {
        if ((uint32_t)r >= rows) continue;
        uint32_t *o = reinterpret_cast<uint32_t *>(a.out + ((uint64_t)g * a.R + row0 + r) * a.pitch) + col * 8;
        if (nd == 8) {
            typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(u32x4_t{acc[r][0], acc[r][1], acc[r][2], acc[r][3]}, reinterpret_cast<u32x4_t *>(o));
            __builtin_nontemporal_store(u32x4_t{acc[r][4], acc[r][5], acc[r][6], acc[r][7]},
                                        reinterpret_cast<u32x4_t *>(o + 4));
        } else {
#pragma unroll
            for (int w = 0; w < 8; ++w)
                if ((uint32_t)w < nd) o[w] = acc[r][w];
        }
    }
}

uint32_t grid_for(uint64_t total)
{
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((total + kFrameBlock - 1) / kFrameBlock, kMaxGrid));
}

uint32_t grid_rows(uint64_t rows)
{
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((rows + kRowsPerBlock - 1) / kRowsPerBlock, kMaxGrid));
}

int launched() { return hipGetLastError() == hipSuccess ? 0 : -3; }

// packet descriptors of a row-major packet array (the pack kernel's output) for the seal / open kernels
__global__ void __launch_bounds__(kFrameBlock) pkt_desc_kernel(uint64_t P, uint64_t pitch, const uint16_t *len16,
                                                               uint64_t *off, uint32_t *len32)
{
    const uint64_t i = blockIdx.x * (uint64_t)kFrameBlock + threadIdx.x;
    if (i >= P) return;
    off[i] = i * pitch;
    len32[i] = len16[i];
}

}  // namespace

int launch_pkt_desc(size_t P, size_t pitch, const uint16_t *len16, uint64_t *off, uint32_t *len32, hipStream_t s)
{
    if (P == 0) return 0;
    hipLaunchKernelGGL(pkt_desc_kernel, dim3((uint32_t)((P + kFrameBlock - 1) / kFrameBlock)), dim3(kFrameBlock), 0, s,
                       (uint64_t)P, (uint64_t)pitch, len16, off, len32);
    return launched();
}

// 0 on success, 1 when the fused kernel does not apply (the caller frames, then encodes), -3 on a HIP error
int launch_framed_encode(const uint8_t *d_enc, int K, int N, size_t G, const void *src, size_t src_bytes,
                         const uint64_t *off, const uint16_t *len, size_t B, size_t pitch, void *parity,
                         uint16_t *align, hipStream_t s, const DataPackets *dp)
{
    const int R = N - K;
    if (G == 0) return 0;
    const uint32_t cols = (uint32_t)((B + 31) / 32);
    const uint32_t gmax = (uint32_t)std::min<size_t>(G, 255 / cols + 2);
    const size_t lds = (size_t)gmax * K * 12 + (size_t)gmax * 4;
    const int mt = R <= 4 ? std::max(R, 1) : 8;
    if (R == 0 || lds > 32 * 1024 || (uint64_t)G * cols > 0x7FFFFFFFull || pitch % 4 || B > 0xFFFF) return 1;
    FramedArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.align = align;
    a.parity = static_cast<uint8_t *>(parity);
    a.etab = reinterpret_cast<const uint32_t *>(d_enc + enc_tab_offset(K, N));
    a.pitch = pitch;
    a.total = (uint32_t)(G * cols);
    a.cols = cols;
    a.K = K;
    a.R = R;
    a.B = (uint32_t)B;
    a.etab_rows = (uint32_t)enc_tab_rows(R);
    a.gmax = gmax;
    const dim3 grid((a.total + 255) / 256, (R + mt - 1) / mt);
    if (dp) {
        a.pkt = static_cast<uint8_t *>(dp->pkt);
        a.pkt_len = dp->pkt_len;
        a.sn = dp->sn;
        a.pkt_pitch = dp->pkt_pitch;
        a.N = N;
        a.timestamp = dp->timestamp;
        switch (mt) {
        case 1: hipLaunchKernelGGL((framed_encode_kernel<1, true>), grid, dim3(256), lds, s, a); break;
        case 2: hipLaunchKernelGGL((framed_encode_kernel<2, true>), grid, dim3(256), lds, s, a); break;
        case 3: hipLaunchKernelGGL((framed_encode_kernel<3, true>), grid, dim3(256), lds, s, a); break;
        case 4: hipLaunchKernelGGL((framed_encode_kernel<4, true>), grid, dim3(256), lds, s, a); break;
        default: hipLaunchKernelGGL((framed_encode_kernel<8, true>), grid, dim3(256), lds, s, a); break;
        }
        return launched();
    }
    switch (mt) {
    case 1: hipLaunchKernelGGL(framed_encode_kernel<1>, grid, dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL(framed_encode_kernel<2>, grid, dim3(256), lds, s, a); break;
    case 3: hipLaunchKernelGGL(framed_encode_kernel<3>, grid, dim3(256), lds, s, a); break;
    case 4: hipLaunchKernelGGL(framed_encode_kernel<4>, grid, dim3(256), lds, s, a); break;
    default: hipLaunchKernelGGL(framed_encode_kernel<8>, grid, dim3(256), lds, s, a); break;
    }
    return launched();
}

int launch_framed_decode(const DeviceInfo &di, const uint8_t *d_enc, int K, int N, size_t G, const void *src,
                         size_t src_bytes, const uint64_t *off, const uint16_t *len, const uint64_t *present, size_t B,
                         size_t pitch, void *out, uint8_t *out_idx, uint8_t *status, uint16_t *align,
                         void *workspace, hipStream_t s)
{
    const int R = N - K;
    if (G == 0) return 0;
    const uint32_t cols = (uint32_t)((B + 31) / 32);
    const uint32_t gmax = (uint32_t)std::min<size_t>(G, 255 / std::max<uint32_t>(cols, 1) + 2);
    const int mt = R <= 4 ? std::max(R, 1) : 8;
    const size_t lds = (size_t)gmax * K * ((size_t)mt * 20 + 12);
    if (R == 0 || B == 0 || lds > 64 * 1024 || (uint64_t)G * cols > 0x7FFFFFFFull || pitch % 4 || B > 0xFFFF) return 1;
    hipLaunchKernelGGL(align_kernel, dim3(grid_for(G)), dim3(kFrameBlock), 0, s, (uint64_t)G, (uint32_t)N, (uint32_t)K,
                       len, present, (uint32_t)B, align);
    if (launched()) return -3;
    if (launch_decode_prep(di, d_enc, K, N, G, present, out_idx, status, workspace, s)) return -3;
    FramedDecArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.align = align;
    a.rec = static_cast<const uint8_t *>(workspace);
    a.out = static_cast<uint8_t *>(out);
    a.pitch = pitch;
    a.total = (uint32_t)(G * cols);
    a.cols = cols;
    a.K = K;
    a.N = N;
    a.R = R;
    a.B = (uint32_t)B;
    a.gmax = gmax;
    a.rec_stride = (uint32_t)record_stride(K, R);
    const dim3 grid((a.total + 255) / 256, (R + mt - 1) / mt);
    switch (mt) {
    case 1: hipLaunchKernelGGL(framed_decode_kernel<1>, grid, dim3(256), lds, s, a); break;
    case 2: hipLaunchKernelGGL(framed_decode_kernel<2>, grid, dim3(256), lds, s, a); break;
    case 3: hipLaunchKernelGGL(framed_decode_kernel<3>, grid, dim3(256), lds, s, a); break;
    case 4: hipLaunchKernelGGL(framed_decode_kernel<4>, grid, dim3(256), lds, s, a); break;
    default: hipLaunchKernelGGL(framed_decode_kernel<8>, grid, dim3(256), lds, s, a); break;
    }
    return launched();
}

int launch_frame(int K, int N, bool recv, size_t G, const void *src, size_t src_bytes, const uint64_t *off,
                 const uint16_t *len, const uint64_t *present, size_t B, size_t pitch, void *data, void *parity,
                 uint16_t *align, hipStream_t s)
{
    if (G == 0) return 0;
    const uint32_t S = recv ? N : K;
    hipLaunchKernelGGL(align_kernel, dim3(grid_for(G)), dim3(kFrameBlock), 0, s, (uint64_t)G, S, (uint32_t)K, len,
                       recv ? present : nullptr, (uint32_t)B, align);
    if (launched()) return -3;
    if (!data && !parity) return 0;  // align only (the R = 0 encode: there are no slots to write)
    FrameArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.present = recv ? present : nullptr;
    a.align = align;
    a.data = static_cast<uint8_t *>(data);
    a.parity = static_cast<uint8_t *>(parity);
    a.pitch = pitch;
    a.S = S;
    a.K = K;
    a.R = N - K;
    a.cols = (uint32_t)((B + 3) / 4);
    a.rows = (uint64_t)G * S;
    hipLaunchKernelGGL(frame_kernel, dim3(grid_rows(a.rows)), dim3(kFrameBlock), 0, s, a);
    return launched();
}

int launch_unframe(int K, int N, size_t G, size_t B, size_t pitch, const void *out, const uint8_t *out_idx,
                   uint16_t *rec_len, void *dst, size_t dst_pitch, hipStream_t s)
{
    const uint32_t R = N - K;
    if (G == 0 || R == 0) return 0;
    UnframeArgs a{};
    a.out = static_cast<const uint8_t *>(out);
    a.out_idx = out_idx;
    a.rec_len = rec_len;
    a.dst = static_cast<uint8_t *>(dst);
    a.pitch = pitch;
    a.dst_pitch = dst_pitch;
    a.R = R;
    a.B = (uint32_t)B;
    a.rows = (uint64_t)G * R;
    hipLaunchKernelGGL(unframe_kernel, dim3(grid_rows(a.rows)), dim3(kFrameBlock), 0, s, a);
    return launched();
}

int launch_pack(int K, int N, size_t G, unsigned which, const void *src, size_t src_bytes, const uint64_t *off,
                const uint16_t *len, size_t pitch, const void *parity, const uint16_t *align, const uint32_t *sn,
                const uint32_t *conv, uint32_t timestamp, void *pkt, size_t pkt_pitch, uint16_t *pkt_len,
                hipStream_t s)
{
    if (G == 0) return 0;
    PackArgs a{};
    a.src = static_cast<const uint32_t *>(src);
    a.src_dw = (src_bytes + 3) / 4;
    a.off = off;
    a.len = len;
    a.parity = static_cast<const uint8_t *>(parity);
    a.align = align;
    a.sn = sn;
    a.conv = conv;
    a.pkt = static_cast<uint8_t *>(pkt);
    a.pkt_len = pkt_len;
    a.pitch = pitch;
    a.pkt_pitch = pkt_pitch;
    a.K = K;
    a.N = N;
    a.which = which;
    a.timestamp = timestamp;
    a.nsel = ((which & KFEC_PACK_DATA) ? K : 0) + ((which & KFEC_PACK_REDUNDANT) ? N - K : 0);
    a.s0 = (which & KFEC_PACK_DATA) ? 0 : K;
    a.rows = (uint64_t)G * a.nsel;
    if (a.rows == 0) return 0;
    hipLaunchKernelGGL(pack_kernel, dim3(grid_rows(a.rows)), dim3(kFrameBlock), 0, s, a);
    return launched();
}

int launch_unpack(int K, size_t P, const void *src, const uint64_t *off, const uint32_t *len, kfec_pkt_hdr *hdr,
                  hipStream_t s)
{
    if (P == 0) return 0;
    hipLaunchKernelGGL(unpack_kernel, dim3((uint32_t)((P + kFrameBlock - 1) / kFrameBlock)), dim3(kFrameBlock), 0, s,
                       (uint64_t)P, (uint32_t)K, static_cast<const uint8_t *>(src), off, len, hdr);
    return launched();
}

int launch_scatter(int N, size_t P, const kfec_pkt_hdr *hdr, const int32_t *slot, uint32_t sn_base, size_t G,
                   uint64_t *present, uint64_t *off, uint16_t *len, hipStream_t s)
{
    if (P == 0) return 0;
    for (int pass = 0; pass < 3; ++pass) {
        hipLaunchKernelGGL(scatter_kernel, dim3((uint32_t)((P + kFrameBlock - 1) / kFrameBlock)), dim3(kFrameBlock), 0,
                           s, pass, (uint64_t)P, (uint32_t)N, hdr, slot, sn_base, (uint64_t)G,
                           reinterpret_cast<unsigned long long *>(present), off, len);
        if (launched()) return -3;
    }
    return 0;
}

}  // namespace kfec
