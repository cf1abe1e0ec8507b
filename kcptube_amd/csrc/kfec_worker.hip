// kfec_worker.hip -- the per-call latency path of the fecpp::fec_code drop-in (kfec_encode / kfec_decode on
// ONE group from host memory, fecpp.cpp:495-513 and 518-587): a resident device worker instead of a kernel
// launch + stream synchronisation per call.
//
// Why: the reference codes a 20:3 group in ~8 us on the KCP updater thread while it holds the KCP mutex
// (kcp.cpp:144, client.cpp:775 -> fec_maker :797).  A launch + hipStreamSynchronize alone costs more than
// that, so the per-call path cannot pay one per group.
//
// How: a worker is W resident workgroups (default 8, one per CU) that poll a doorbell word in fine-grained
// (coherent) pinned host memory (each with 8 / W loads in flight; see KFEC_WORKER_POLL).  The caller copies the group's shares into the slot's pinned stage, writes
// the doorbell (sequence number + op + K, N, B in ONE 64-bit store) and spins on the slot's completion words.
// Workgroup w owns the 16-byte column granules [w*G/W, (w+1)*G/W) of every shard (G = pitch / 16): it pulls its
// slice of the request body's shares into LDS in one burst of 16-byte loads over PCIe, computes its slice of
// the output rows, writes them straight back into the pinned stage, publishes them with a system-scope
// release and stores its completion word.  Splitting the columns over CUs splits the PCIe reads, the GF work
// and the write-back acknowledgements of one small group W ways.
//
//   encode  parity_r = XOR_j enc[K+r][j] * D_j                       (fecpp.cpp:504-510)
//   decode  rows in the reference's selection order (fecpp.cpp:528-548, done by the caller: bookkeeping only),
//           y_t = share(row M_t) ^ XOR_{j present} enc[P_t][j] * D_j  (syndrome of the used parity share P_t)
//           out_u = XOR_t Sinv[u][t] * y_t,  S[t][u] = enc[P_t][M_u]  (the missing rows of the K x K inverse,
//           fecpp.cpp:564-583; the inverse is unique, so the bytes equal the reference's Gauss-Jordan result)
//
// All GF products use the perm MAC of kfec_gf.hpp with tables in LDS; the parity-row tables of the coder's
// matrix are copied from its device allocation (enc_tab_offset) once per matrix and kept in LDS while the
// same matrix is used.  Lifetime: workgroup 0 leaves after KFEC_WORKER_IDLE_US without a request (default
// 20 ms) or, between requests, once the launch is KFEC_WORKER_LEASE_US old (default 2 ms: the bound on how long
// another thread's hipFree / hipDeviceSynchronize waits for this stream), and relays a quit value through the
// device-memory word the other workgroups poll; all leave on op STOP.  Each
// writes its generation to its exit word; the host relaunches the worker on the next request.  Every wave
// reaches the exit: the loop's only waits are the bounded doorbell / quit poll and workgroup barriers.
#include "kfec_gf.hpp"
#include "kfec_internal.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>

namespace kfec {
namespace {

constexpr int kWThreads = 256;             // threads per worker workgroup
constexpr int kMaxW = 8;                   // workgroups per worker
constexpr int kMaxR = 16;                  // parity rows (encode) / missing rows (decode) a worker takes
constexpr size_t kStageMax = 36 * 1024;    // (K + R) * pitch of a request
constexpr size_t kTabMax = 16 * 1024;      // R * K * 32 bytes: parity-row perm tables (8-dword entries) in LDS
constexpr size_t kSliceMax = 16 * 1024;    // K * ceil(G / W) * 16 bytes: one workgroup's slice of the shares
// LDS carve of one workgroup (bytes, all 16-aligned)
constexpr size_t kLdsData = 0;
constexpr size_t kLdsTab = kLdsData + kSliceMax;
constexpr size_t kLdsCinv = kLdsTab + kTabMax;                    // m x m perm tables of Sinv (8-dword entries)
constexpr size_t kLdsGj = kLdsCinv + kMaxR * kMaxR * 32;          // m x 2m Gauss-Jordan matrix (u32 entries)
constexpr size_t kLdsPart = kLdsGj + kMaxR * 2 * kMaxR * 4;       // partial sums of the share groups [JS][4][ncw]
constexpr size_t kLdsGf = kLdsPart + 4 * 1024;                    // exp[512] + log[256]
constexpr size_t kLdsBody = kLdsGf + 768;                         // the request body (128 bytes)
constexpr size_t kLdsDtab = kLdsBody + 128;                       // decode: perm tables of the host's D (m x K)
constexpr size_t kLdsBytes = kLdsDtab + kTabMax;
static_assert(kLdsBytes <= 64 * 1024, "a worker workgroup fits the default 64 KiB of LDS");

// Slot layout in pinned host memory (offsets in bytes).  The host writes the doorbell, the body and the shares;
// the device writes the completion / exit words (lines of their own), the output rows and the debug times.
constexpr size_t kOffDoorbell = 0;
constexpr size_t kOffBody = 256;    // WorkerBody
constexpr size_t kOffTrace = 512;   // u64: device-side phase times (KFEC_WORKER_DEBUG=2)
constexpr size_t kOffDone = 1024;   // u64 per workgroup, 128 bytes apart: seq | status << 32
constexpr size_t kOffExited = 2048; // u64 per workgroup, 128 bytes apart: generation of a workgroup that has left
constexpr size_t kLineW = 128;      // (one line per workgroup: no two CUs write into one host cache line)
constexpr size_t kOffCinv = 3072;   // decode, host-solved: D = S^-1 [E | I] over the K staged rows, m x K bytes
constexpr size_t kOffShares = 4096; // K rows x pitch: the shares, in row order; then the output rows
constexpr size_t kSlotBytes = kOffShares + 2 * kStageMax;

enum : uint32_t { kOpPing = 0, kOpEncode = 1, kOpDecode = 2, kOpStop = 3 };  // ping: answered at once
constexpr uint32_t kSeqMask = (1u << 30) - 1;
constexpr int kWorkerDead = -1000;  // post_and_wait: the worker did not answer (the device's workers are disabled)

// doorbell: seq (30 bits) | op (2) | K - 1 (8) | N - 1 (8) | B (16)
__host__ __device__ inline uint64_t db_pack(uint32_t seq, uint32_t op, uint32_t K, uint32_t N, uint32_t B)
{
    return (uint64_t)(seq & kSeqMask) | ((uint64_t)op << 30) | ((uint64_t)(K - 1) << 32) | ((uint64_t)(N - 1) << 40) |
           ((uint64_t)B << 48);
}
__host__ __device__ inline uint32_t db_seq(uint64_t v) { return (uint32_t)v & kSeqMask; }
__host__ __device__ inline uint32_t db_op(uint64_t v) { return (uint32_t)(v >> 30) & 3u; }

// Decodes with m <= kHostSolveMax lost shares and m * m * K <= kHostSolveWork have their whole decode matrix
// solved on the host: out_u = XOR_j D[u][j] * row_j over the K staged rows, D = S^-1 * (the rows' columns of
// [E | I]) -- a few hundred table multiplies (~0.2 us), where the device's solve + syndromes + mix took 3.2 us
// on the request's critical path.  The device then runs the encode MAC with D's tables (one pass, no solve).
constexpr int kHostSolveMax = 8;
constexpr int kHostSolveWork = 1024;
constexpr int kCinvLoads = 512 / 16;  // 16-byte loads of D (m * K <= 512: shape_ok's R * K bound)
static_assert(kOffExited + 8 * kLineW <= kOffCinv && kOffCinv + kCinvLoads * 16 <= kOffShares, "slot layout");

// ---- batch requests (the queues' small flushes, kfec_pipeline.cpp) -------------------------------------
// A doorbell with B = 0 is a batch request: its K / N fields carry the request's length in 16-byte units, and
// the request -- a BatchBody, then the shard descriptors, then (decode) one record per group -- sits at
// kOffShares of the request side.  Every workgroup copies the whole request into LDS in one burst (one
// dependent round trip, however many groups), then takes a contiguous range of the batch's (group, 16-byte
// column) items.  The shards themselves are read from the queue's staging arena: device memory the host
// wrote through the BAR as each datagram / shard arrived, so a flush moves no bulk bytes across PCIe before
// the doorbell.  Outputs go straight to the queue's coherent pinned output rows.
//   encode (kOpEncode): framed shards ([BE16 len][payload][zeros], compact_into_container, data_operations.cpp
//     :610-631) -> the R parity rows of each group (the coder's matrix tables, as the single-group encode);
//   decode (kOpDecode): the K selected shares of each group (data shards framed, parity shares raw, zero
//     padded; data_operations.cpp:633-667) -> out_u = XOR_j D[u][j] * row_j with D = S^-1 [E | I] solved by
//     the host per group (host_solve, the single-group decode's coefficients), rows u < m of the group.
constexpr size_t kBatchReqMax = 16 * 1024;  // request bytes (body + descriptors + records): copied into LDS
constexpr int kBatchMaxR = 8;               // parity rows (encode) / decode rows (m <= R) per group
constexpr int kBatchMaxKS = 32;             // shards per lane (K / share split): bounds the loads in flight
struct BatchBody {             // 128 bytes
    uint64_t enc;              // encode: the coder's matrix allocation (N x K bytes, then its tables)
    uint64_t mat_id;           // encode: LDS table-cache key
    uint64_t arena;            // device address of the staging arena (64 bytes of headroom before and after)
    uint64_t out;              // host address of the output rows: row (g, r) at out + (g * R + r) * opitch + ooff
    uint32_t n, K, N, B;       // groups, shape, shard bytes (framed: datagram + 2)
    uint32_t opitch, ooff;     // output row stride and the data's offset inside a row
    uint32_t rec_off;          // decode: byte offset (from the body) of the group records
    uint32_t rec_stride;       // decode: bytes per group record: [0] m, [16, 16 + R * K) D row-major (rows >= m zero)
    uint8_t pad[128 - 64];
};
static_assert(sizeof(BatchBody) == 128, "batch body is one 128-byte block");
// shard descriptor (u64, kfec_internal.hpp batch_desc): bits 0-39 byte offset in the arena, 40-55 payload
// length, 56 raw (1: a parity share as received, no container header) or framed (0: a data shard, BE16 length
// prepended)

struct WorkerBody {          // 128 bytes
    uint64_t enc;            // device address of the coder's matrix allocation (N x K bytes, then its tables)
    uint64_t mat_id;         // unique per built matrix: the LDS table cache key
    uint64_t miss[4];        // decode: bit j set <=> row j holds a parity share (data share j is missing)
    uint32_t m;              // decode: number of missing data shares (<= kMaxR)
    uint32_t solved;         // decode: 1 = the host sent D (m x K bytes, row-major) at kOffCinv
    uint8_t M[kMaxR];        // missing data ids, ascending (row t of the output)
    uint8_t P[kMaxR];        // the parity share id used for M[t] (fecpp.cpp:538-544)
    uint8_t pad[128 - 88];
};
static_assert(sizeof(WorkerBody) == 128, "body is one 128-byte block");

__constant__ GfTables w_gf = make_gf_tables();

__device__ __forceinline__ uint32_t wk_gmul(const uint8_t *e, const uint8_t *l, uint32_t a, uint32_t b)
{
    return (a && b) ? e[l[a] + l[b]] : 0u;
}

// acc ^ c * x with c's perm tables at an 8-dword (32-byte aligned) LDS entry: two 16-byte LDS reads
__device__ __forceinline__ uint32_t tab_mac(uint32_t acc, const uint32_t *ent, uint32_t s0, uint32_t s1, uint32_t s2)
{
    const uint4 a = *reinterpret_cast<const uint4 *>(ent);
    const uint32_t t[5] = {a.x, a.y, a.z, a.w, ent[4]};
    return perm_mac(acc, t, s0, s1, s2);
}

// acc[q] ^= XOR_{j0 <= j < K} tab(j, rows[q]) * X[j][c] for q < RT (RT a compile-time row count: no per-row branches),
// shares j with skip bit set contribute nothing (their dword is replaced by 0: c * 0 = 0, no branch).  Shares
// are taken 4 at a time so their LDS reads (and the broadcast table reads) are issued together.
template <int RT>
__device__ __forceinline__ void rows_mac(uint32_t (&acc)[4], const uint32_t *X, int nc, int c, int j0, int K,
                                         const uint32_t *tab, int R, const int (&rows)[4], const uint64_t (&skip)[4])
{
    auto skipped = [&](int j) -> bool { return (skip[j >> 6] >> (j & 63)) & 1ull; };
    int j = j0;
    for (; j + 4 <= K; j += 4) {
        // every LDS read of the 4 shares (their dwords and all 4 * RT tables) is issued before the first MAC: the
        // per-table load-use order left one LDS round trip per table on the critical path (1.3 us per request)
        uint32_t x[4];
        uint4 ta[4][RT];
        uint32_t tb[4][RT];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = skipped(j + u) ? 0u : X[(j + u) * nc + c];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                const uint32_t *ent = tab + ((j + u) * R + rows[q]) * 8;
                ta[u][q] = *reinterpret_cast<const uint4 *>(ent);
                tb[u][q] = ent[4];
            }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t s0 = x[u] & 0x07070707u, s1 = (x[u] >> 3) & 0x07070707u, s2 = (x[u] >> 6) & 0x03030303u;
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                const uint32_t t[5] = {ta[u][q].x, ta[u][q].y, ta[u][q].z, ta[u][q].w, tb[u][q]};
                acc[q] = perm_mac(acc[q], t, s0, s1, s2);
            }
        }
    }
    for (; j < K; ++j) {
        const uint32_t x = skipped(j) ? 0u : X[j * nc + c];
        const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
#pragma unroll
        for (int q = 0; q < RT; ++q) acc[q] = tab_mac(acc[q], tab + (j * R + rows[q]) * 8, s0, s1, s2);
    }
}

template <typename F>
__device__ __forceinline__ void by_rows(int n, F &&f)  // f(std::integral_constant-like RT) for the uniform row count n
{
    if (n >= 4) f(std::integral_constant<int, 4>());
    else if (n == 3) f(std::integral_constant<int, 3>());
    else if (n == 2) f(std::integral_constant<int, 2>());
    else f(std::integral_constant<int, 1>());
}

__device__ __forceinline__ uint64_t uniform64(uint64_t x)
{
    // (readfirstlane returns int: widen through uint32_t, or bit 31 -- op 2 -- sign-extends)
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

}  // namespace

// s_waitcnt immediate for vmcnt(0) with expcnt / lgkmcnt left at their maxima (gfx9 encoding: vmcnt[3:0] and
// [15:14], expcnt [6:4], lgkmcnt [11:8])
constexpr int kVmcntZero = (0x7 << 4) | (0xF << 8);

// an output dword: light -> a system-scope store, written through L2 to host memory (sc0 sc1)
__device__ __forceinline__ void put_out(uint32_t *p, uint32_t v, int light)
{
    if (light) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else *p = v;
}

__device__ uint4 w_zero16;  // never written: the target of the loads a lane does not need

// 16 bytes [16c, 16c + 16) of a shard row whose payload (len bytes at arena byte offset off, 4-aligned) follows
// an H-byte header (H = 2: the container's BE16 length, compact_into_container; H = 0: a raw parity share),
// zero past the payload.  Both loads are always issued (a granule without payload reads w_zero16), so every
// shard's loads can be in flight together.
__device__ __forceinline__ uint4 shard_granule(const uint32_t *arena32, uint64_t d, int c)
{
    const uint64_t off = d & 0xFFFFFFFFFFull;
    const int len = (int)((d >> 40) & 0xFFFFu), H = (d >> 56) & 1 ? 0 : 2;
    const int q0 = 16 * c - H;                               // payload index of the granule's first byte
    const int lo = max(0, -q0), hi = min(16, len - q0);      // payload bytes [lo, hi) of the granule
    const bool any = hi > lo;
    const uint64_t a4 = off + (uint64_t)(int64_t)(q0 + 16);  // (>= off + 14: the arena has headroom before it)
    const uint64_t w4 = a4 >> 2;
    const uint32_t sh = (uint32_t)(a4 & 3u);
    const uint4 x = *(any ? reinterpret_cast<const uint4 *>(arena32 + (w4 - 4)) : &w_zero16);
    const uint32_t x4 = *(any && sh ? arena32 + w4 : &w_zero16.x);
    const uint32_t dw[5] = {x.x, x.y, x.z, x.w, x4};
    const uint32_t M = any ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
    uint32_t o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t nib = (M >> (4 * i)) & 0xFu;
        o[i] = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], sh) & (((nib * 0x00204081u) & 0x01010101u) * 0xFFu);
    }
    if (H && c == 0) o[0] |= ((uint32_t)len >> 8) | (((uint32_t)len & 0xFFu) << 8);  // htons(data_length)
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// 16 bytes to host memory at system scope (written through L2: the light release is a wait for the acks)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_sys(uint8_t *p, uint4 v)
{
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(x) : "memory");
}

// One batch request (see BatchBody).  s_req: the request, copied into LDS by the caller.
template <int RT>
__device__ __forceinline__ void batch_items(const BatchBody &b, const uint64_t *s_desc, const uint8_t *s_rec,
                                            const uint32_t *tab, int g_lo, int i0, int i1, int r0, bool decode)
{
    const int K = (int)b.K, R = (int)(b.N - b.K), G16 = ((int)b.B + 15) >> 4;
    const int nitems = i1 - i0;
    // S lanes per item, each over the shards j = s, s + S, ...: a batch of few items still spreads its GF work
    // over every wave; the S partial sums meet by lane shuffles
    int S = 1;
    while (S < 16 && S < K && nitems * S * 2 <= kWThreads) S *= 2;
    while ((K + S - 1) / S > kBatchMaxKS) S *= 2;  // (the host refuses shapes that would need S > 64)
    const uint32_t *arena32 = reinterpret_cast<const uint32_t *>(b.arena);
    const int tid = threadIdx.x;
    for (int base = 0; base < nitems * S; base += kWThreads) {  // (uniform trip count: the shuffles need every lane)
        const int t = base + tid;
        const bool valid = t < nitems * S;
        const int item = i0 + (valid ? t / S : 0), s = t & (S - 1);
        const int g = item / G16, c = item - g * G16;
        const uint64_t *dsc = s_desc + (size_t)g * K;
        const uint32_t *gtab = decode ? tab + (size_t)(g - g_lo) * K * R * 8 : tab;
        uint32_t acc[RT][4];
#pragma unroll
        for (int q = 0; q < RT; ++q) acc[q][0] = acc[q][1] = acc[q][2] = acc[q][3] = 0u;
        // this lane's shards, 8 at a time with every load of a chunk issued before its MACs
        for (int j0 = s; j0 < K; j0 += 8 * S) {
            uint4 x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + u * S;
                // (no branch around the loads: a lane without this shard takes descriptor 0, an empty payload,
                //  whose granule loads read w_zero16)
                const uint64_t dj = dsc[min(j, K - 1)];
                x[u] = shard_granule(arena32, (valid && j < K) ? dj : 0ull, c);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = min(j0 + u * S, K - 1);  // (a clamped row multiplies a zero granule)
                const uint32_t xv[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
                uint4 ta[RT];
                uint32_t tb[RT];
#pragma unroll
                for (int q = 0; q < RT; ++q) {
                    const uint32_t *ent = gtab + ((size_t)j * R + r0 + q) * 8;
                    ta[q] = *reinterpret_cast<const uint4 *>(ent);
                    tb[q] = ent[4];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t s0 = xv[i] & 0x07070707u, s1 = (xv[i] >> 3) & 0x07070707u, s2 = (xv[i] >> 6) & 0x03030303u;
#pragma unroll
                    for (int q = 0; q < RT; ++q) {
                        const uint32_t tt[5] = {ta[q].x, ta[q].y, ta[q].z, ta[q].w, tb[q]};
                        acc[q][i] = perm_mac(acc[q][i], tt, s0, s1, s2);
                    }
                }
            }
        }
        for (int d = 1; d < S; d <<= 1)
#pragma unroll
            for (int q = 0; q < RT; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[q][i] ^= (uint32_t)__shfl_xor((int)acc[q][i], d);
        if (valid && s == 0) {
            const int m = decode ? (int)s_rec[(size_t)g * b.rec_stride] : R;
            uint8_t *out = reinterpret_cast<uint8_t *>(b.out) + (size_t)b.ooff + 16 * (size_t)c;
#pragma unroll
            for (int q = 0; q < RT; ++q)
                if (r0 + q < m)
                    store16_sys(out + ((size_t)g * R + r0 + q) * b.opitch, make_uint4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]));
        }
    }
}

__device__ __forceinline__ void serve_batch(const uint8_t *in, uint8_t *smem, uint64_t &s_mat, uint32_t op, uint32_t len16)
{
    const int tid = threadIdx.x, w = blockIdx.x, W = gridDim.x;
    // 1. the whole request into LDS: one burst of 16-byte loads
    uint4 *s16 = reinterpret_cast<uint4 *>(smem + kLdsData);
    const uint4 *src = reinterpret_cast<const uint4 *>(in + kOffShares);
    const int n16 = min((int)len16, (int)(kBatchReqMax / 16));
    for (int i0 = 0; i0 < n16; i0 += kWThreads * 4) {
        uint4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = src[min(i0 + u * kWThreads + tid, n16 - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i0 + u * kWThreads + tid < n16) s16[i0 + u * kWThreads + tid] = r[u];
    }
    __syncthreads();
    const BatchBody &b = *reinterpret_cast<const BatchBody *>(smem + kLdsData);
    const bool decode = op == kOpDecode;
    const int K = (int)b.K, N = (int)b.N, R = N - K, G16 = ((int)b.B + 15) >> 4;
    const int I = (int)b.n * G16;
    const int i0 = (int)((int64_t)w * I / W), i1 = (int)((int64_t)(w + 1) * I / W);
    const uint64_t *s_desc = reinterpret_cast<const uint64_t *>(smem + kLdsData + sizeof(BatchBody));
    const uint8_t *s_rec = smem + kLdsData + b.rec_off;
    const int g_lo = i0 / max(G16, 1), g_hi = i1 > i0 ? (i1 - 1) / G16 : g_lo - 1;
    // 2. tables: encode -- the matrix's parity-row tables (the single-group encode's LDS cache); decode -- the
    //    perm tables of D for this workgroup's groups, [group][j][u]
    const uint32_t *tab;
    if (!decode) {
        uint32_t *s_tab = reinterpret_cast<uint32_t *>(smem + kLdsTab);
        if (b.mat_id != s_mat) {
            const uint32_t *g_tab =
                reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(b.enc) + enc_tab_offset(K, N));
            const int rows = (int)enc_tab_rows(R), ne = K * R * 5;
            for (int i = tid; i < ne; i += kWThreads) {
                const int e = i / 5, q = i - e * 5, j = e / R, r = e - j * R;
                s_tab[e * 8 + q] = g_tab[(j * rows + r) * 5 + q];
            }
            __syncthreads();
            if (tid == 0) s_mat = b.mat_id;
        }
        tab = s_tab;
    } else {
        uint32_t *s_dtab = reinterpret_cast<uint32_t *>(smem + kLdsDtab);
        const int ne = (g_hi - g_lo + 1) * K * R;
        for (int e = tid; e < ne; e += kWThreads) {
            const int gl = e / (K * R), rem = e - gl * K * R, j = rem / R, u = rem - j * R;
            uint32_t tb[5];
            gf_perm_tables(s_rec[(size_t)(g_lo + gl) * b.rec_stride + 16 + u * K + j], tb);
            *reinterpret_cast<uint4 *>(s_dtab + e * 8) = uint4{tb[0], tb[1], tb[2], tb[3]};
            s_dtab[e * 8 + 4] = tb[4];
        }
        tab = s_dtab;
    }
    __syncthreads();
    // 3. the items, row tiles of up to 4
    for (int r0 = 0; r0 < R; r0 += 4)
        by_rows(R - r0, [&](auto rt) {
            constexpr int RT = decltype(rt)::value;
            batch_items<RT>(b, s_desc, s_rec, tab, g_lo, i0, i1, r0, decode);
        });
}

__global__ void __launch_bounds__(kWThreads) kfec_worker_kernel(uint8_t *slot, const uint8_t *in, uint64_t *relay,
                                                                uint32_t gen, uint32_t last_seq, uint64_t idle_ticks,
                                                                uint64_t lease_ticks, int debug, int direct, int light,
                                                                int deaf)
{
    const uint64_t t_start = wall_clock64();  // (the lease: see the poll below)
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t s_db;
    __shared__ uint64_t s_mat;
    __shared__ int s_singular;
    const int tid = threadIdx.x, w = blockIdx.x, W = gridDim.x;
    uint8_t *s_exp = smem + kLdsGf, *s_log = smem + kLdsGf + 512;
    for (int i = tid; i < 512; i += kWThreads) s_exp[i] = w_gf.exp[i];
    for (int i = tid; i < 256; i += kWThreads) s_log[i] = w_gf.log[i];
    if (tid == 0) s_mat = 0;  // matrix ids start at 1
    // (the request side -- doorbell, body, shares -- is `in`: the slot itself, or device memory the host writes
    //  through the BAR; the answer side -- completion words, output rows -- is always the slot in host memory)
    uint64_t *doorbell = reinterpret_cast<uint64_t *>(const_cast<uint8_t *>(in) + kOffDoorbell);
    uint64_t *done = reinterpret_cast<uint64_t *>(slot + kOffDone + kLineW * w);
    uint64_t *exited = reinterpret_cast<uint64_t *>(slot + kOffExited + kLineW * w);
    uint64_t *trace = reinterpret_cast<uint64_t *>(slot + kOffTrace);
    const uint4 *h_body = reinterpret_cast<const uint4 *>(in + kOffBody);
    const uint4 *h_rows = reinterpret_cast<const uint4 *>(in + kOffShares);
    const uint4 *h_cinv = reinterpret_cast<const uint4 *>(in + kOffCinv);
    uint32_t last = last_seq;

    for (;;) {
        // Wave 0 polls -- the whole wave, the value made wave-uniform: a loop under `tid == 0` leaves lanes 1-63
        // free to run on to the next barrier while lane 0 spins, and the compiler's structurized loop then
        // replays the previous request forever.  Rolling: NP loads in flight ~0.1 us apart, each checked as it
        // returns and reissued.  Two ways to spread a doorbell over the workgroups (KFEC_WORKER_POLL):
        //   relay  (0): workgroup 0 alone polls the host line (8 loads in flight) and relays each new doorbell
        //               through a device-memory word the others poll;
        //   direct (1): every workgroup polls the host line with 8 / W loads in flight (one line read by many CUs
        //               with 64 loads in flight serialised in the root complex: ping 12 us), no relay hop; the
        //               device word then carries only workgroup 0's quit.
        if (tid < 64) {
            const bool host = w == 0 || direct;
            const uint64_t t0 = wall_clock64();
            uint64_t v = 0;
            auto poll_loop = [&](auto np) {
                constexpr int NP = decltype(np)::value;
                uint64_t xs[NP];
                auto poll = [&]() -> uint64_t {
                    return host ? __hip_atomic_load(doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                : __hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
#pragma unroll
                for (int k = 0; k < NP; ++k) {
                    xs[k] = poll();
                    __builtin_amdgcn_s_sleep(3);
                }
                bool hit = false;
                for (;;) {
#pragma unroll
                    for (int k = 0; k < NP; ++k) {
                        const uint64_t u = uniform64(xs[k]);
                        // (0: nothing relayed since the launch's memset; deaf: the fallback test's knob, which
                        //  ignores requests but never the relay's quit value ~0, or relay-mode followers spin on)
                        if (!hit && u != 0 && db_seq(u) != last && (!deaf || u == ~0ull)) {
                            v = u;  // (the relay's quit value ~0 has seq kSeqMask, never posted, and makes v ~0)
                            hit = true;
                        }
                        if (!hit) {
                            xs[k] = poll();
                            __builtin_amdgcn_s_sleep(3);
                        }
                    }
                    if (hit) break;
                    if (w == 0) {
                        const uint64_t now = wall_clock64();
                        if (now - t0 > idle_ticks || now - t_start > lease_ticks) {  // idle or lease over: workgroup 0
                                                                                     // decides, the others follow
                            v = ~0ull;
                            break;
                        }
                    } else if (direct && uniform64(__hip_atomic_load(relay, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == ~0ull) {
                        v = ~0ull;
                        break;
                    }
                }
            };
            // The lease: workgroup 0 also leaves once the kernel has been resident for lease_ticks, checked only
            // inside the poll loop after a round of polls found no new doorbell (never ahead of a pending request,
            // which the other workgroups may already be serving).  Any device-wide synchronisation of the process
            // -- hipFree, hipHostFree, hipDeviceSynchronize, which wait for every stream -- then waits at most
            // about one lease, even while other threads keep calling; the next request relaunches the worker (a
            // launch, ~10 us, once per lease).
            if (w == 0 || !direct || W <= 1) poll_loop(std::integral_constant<int, 8>());
            else if (W <= 4) poll_loop(std::integral_constant<int, 2>());
            else poll_loop(std::integral_constant<int, 1>());
            if (w == 0 && W > 1 && (!direct || v == ~0ull)) __hip_atomic_store(relay, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tid == 0) s_db = v == ~0ull ? 0 : v;
        }
        __syncthreads();
        const uint64_t v = s_db;
        if (v == 0) break;
        const uint64_t ts_seen = debug == 2 ? wall_clock64() : 0;
        // the stage and body written before the doorbell.  light: they are in uncached device memory or coherent
        // host memory, which no L2 line holds, so only this CU's L1 is dropped (agent scope), not the whole L2
        if (light) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        last = db_seq(v);
        const uint32_t op = db_op(v);
        uint32_t status = 0;
        if (op == kOpStop || op == kOpPing) {
            if (tid == 0) {
                if (light) __hip_atomic_store(done, (uint64_t)last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else __hip_atomic_store(done, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if (op == kOpStop) break;
            continue;
        }
        if ((v >> 48) == 0) {  // B = 0: a batch request (the queues' small flushes)
            serve_batch(in, smem, s_mat, op, (uint32_t)((v >> 32) & 0xFFFF));
            __builtin_amdgcn_s_waitcnt(kVmcntZero);  // every output store acknowledged (system scope)
            __syncthreads();
            if (tid == 0) __hip_atomic_store(done, (uint64_t)last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        const int K = (int)((v >> 32) & 0xFF) + 1, N = (int)((v >> 40) & 0xFF) + 1, R = N - K;
        const int B = (int)(v >> 48);
        const int pitch = (B + 15) & ~15, G = pitch >> 4, P4 = pitch >> 2;
        // a request outside the worker's shapes (the host never posts one) is answered, not executed
        if (R < 1 || R > kMaxR || B < 1 || (size_t)(K + R) * pitch > kStageMax || (size_t)R * K * 32 > kTabMax) {
            __syncthreads();
            if (tid == 0)
                __hip_atomic_store(done, (uint64_t)last | (3ull << 32), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        // this workgroup's granules [ga, ga + ng) of every row; nc dword columns
        const int ga = (int)((int64_t)w * G / W), ng = (int)((int64_t)(w + 1) * G / W) - ga, nc = 4 * ng;
        if ((size_t)K * ((G + W - 1) / W) * 16 > kSliceMax) {  // (the host checks the same bound)
            __syncthreads();
            if (tid == 0)
                __hip_atomic_store(done, (uint64_t)last | (3ull << 32), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        // thread roles: JS groups of shares, each over ncw column lanes (so a workgroup slice of <= 64 columns
        // keeps all 4 waves busy, each on a quarter of the shares; the groups' partial sums meet in LDS)
        const int ncw = nc <= 64 ? 64 : (nc <= 128 ? 128 : kWThreads), JS = kWThreads / ncw;
        // (ncw is a multiple of 64: the share group is wave-uniform -- say so, or the share loop, its skip tests
        //  and the table addresses all run as per-lane VALU code with exec masks)
        const int jg = __builtin_amdgcn_readfirstlane(tid / ncw), cl = tid - jg * ncw;
        uint32_t *s_part = reinterpret_cast<uint32_t *>(smem + kLdsPart);  // [JS][4][ncw]
        // 1. one burst of 16-byte loads: the body and the K rows' slices (clamped indices keep r[] in VGPRs; the
        //    clamped duplicates store the same bytes)
        {
            const int n16 = K * ng;
            uint4 *s16 = reinterpret_cast<uint4 *>(smem + kLdsData);
            uint4 *b16 = reinterpret_cast<uint4 *>(smem + kLdsBody);
            const uint4 bq = h_body[tid & 7];
            const bool cl16 = op == kOpDecode && tid < kCinvLoads;  // (used only if the body says solved)
            const uint4 cq = cl16 ? h_cinv[tid] : uint4{0, 0, 0, 0};
            for (int i0 = 0; i0 < n16; i0 += kWThreads * 4) {
                uint4 r[4];
                int dst[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = max(min(i0 + u * kWThreads + tid, n16 - 1), 0);
                    const int j = i / max(ng, 1), g = i - j * max(ng, 1);
                    dst[u] = i;
                    r[u] = h_rows[j * G + ga + g];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) s16[dst[u]] = r[u];
            }
            if (tid < 8) b16[tid] = bq;
            if (cl16) reinterpret_cast<uint4 *>(smem + kLdsCinv)[tid] = cq;
        }
        __syncthreads();
        const uint64_t ts_loaded = debug == 2 ? wall_clock64() : 0;
        const uint64_t ck_loaded = debug == 2 ? __builtin_amdgcn_s_memtime() : 0;
        const WorkerBody *body = reinterpret_cast<const WorkerBody *>(smem + kLdsBody);
        uint32_t *s_tab = reinterpret_cast<uint32_t *>(smem + kLdsTab);
        uint32_t *s_rows = reinterpret_cast<uint32_t *>(smem + kLdsData);  // [K][nc] dwords
        // 2. parity-row perm tables of this matrix: s_tab[(j * R + r) * 8 + i], kept while the matrix is reused
        const bool fused = op == kOpDecode && body->solved;  // (LDS broadcast: uniform)
        if (!fused && body->mat_id != s_mat) {
            const uint32_t *g_tab =
                reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(body->enc) + enc_tab_offset(K, N));
            const int rows = (int)enc_tab_rows(R), n = K * R * 5;
            for (int i = tid; i < n; i += kWThreads) {
                const int e = i / 5, q = i - e * 5, j = e / R, r = e - j * R;
                s_tab[e * 8 + q] = g_tab[(j * rows + r) * 5 + q];
            }
            __syncthreads();
            if (tid == 0) s_mat = body->mat_id;
        }
        uint32_t *out = reinterpret_cast<uint32_t *>(slot + kOffShares + (size_t)K * pitch) + ga * 4;
        const uint64_t ts_tab = debug == 2 ? __builtin_amdgcn_s_memtime() : 0;
        uint64_t ts_mac = 0, ts_solve = 0, ts_syn = 0;
        if (op == kOpEncode || fused) {
            // encode: the R parity rows from the matrix's tables; fused decode: the m output rows from the
            // tables of the host's D, built here from its bytes (one entry per thread)
            const uint32_t *tab = s_tab;
            int RR = R;
            if (fused) {
                RR = __builtin_amdgcn_readfirstlane(min((int)body->m, R));
                if (debug == 2) ts_solve = __builtin_amdgcn_s_memtime();  // (fused: "solve" = building D's tables)
                uint32_t *s_dtab = reinterpret_cast<uint32_t *>(smem + kLdsDtab);
                const uint8_t *coef = smem + kLdsCinv;  // D[u][j], as loaded in step 1
                for (int e = tid; e < RR * K; e += kWThreads) {
                    const int j = e / RR, u = e - j * RR;
                    uint32_t tb[5];
                    gf_perm_tables(coef[u * K + j], tb);
                    *reinterpret_cast<uint4 *>(s_dtab + e * 8) = uint4{tb[0], tb[1], tb[2], tb[3]};
                    s_dtab[e * 8 + 4] = tb[4];
                }
                __syncthreads();
                tab = s_dtab;
            }
            // row tiles of 4 (uniform across the workgroup); thread = (share group, column)
            const uint64_t none[4] = {0, 0, 0, 0};
            const int jlo = jg * K / JS, jhi = (jg + 1) * K / JS;
            for (int r0 = 0; r0 < RR; r0 += 4) {
                const int rows[4] = {r0, r0 + 1, r0 + 2, r0 + 3}, rt_n = min(4, RR - r0);
                by_rows(rt_n, [&](auto rt) {
                    constexpr int RT = decltype(rt)::value;
                    for (int c = cl; c < nc; c += ncw) {
                        uint32_t acc[4] = {0, 0, 0, 0};
                        rows_mac<RT>(acc, s_rows, nc, c, jlo, jhi, tab, RR, rows, none);
#pragma unroll
                        for (int q = 0; q < RT; ++q) {
                            if (JS == 1) put_out(out + (r0 + q) * P4 + c, acc[q], light);
                            else s_part[(jg * 4 + q) * ncw + c] = acc[q];
                        }
                    }
                });
                if (debug == 2 && r0 == 0) ts_mac = ts_syn = __builtin_amdgcn_s_memtime();  // (fused: "syndromes")
                if (JS > 1) {
                    __syncthreads();
                    for (int e = tid; e < rt_n * nc; e += kWThreads) {
                        const int q = e / nc, c = e - q * nc;
                        uint32_t a = 0;
                        for (int g = 0; g < JS; ++g) a ^= s_part[(g * 4 + q) * ncw + c];
                        put_out(out + (r0 + q) * P4 + c, a, light);
                    }
                    __syncthreads();
                }
            }
        } else {
            const int m = __builtin_amdgcn_readfirstlane(min((int)body->m, R));  // (the host sends 1 <= m <= R)
            uint32_t *s_gj = reinterpret_cast<uint32_t *>(smem + kLdsGj);
            uint32_t *s_cinv = reinterpret_cast<uint32_t *>(smem + kLdsCinv);
            // 3. [S | I], S[t][u] = enc[P_t][M_u] (byte 1 of table word 0 is c * 1 = c)
            const int Wd = 2 * m, ne = m * Wd;  // ne <= 512: at most 2 entries per thread
            auto gj_init = [&](int e) {
                const int t = e / Wd, u = e - t * Wd;
                s_gj[e] = u < m ? (s_tab[((int)body->M[u] * R + ((int)body->P[t] - K)) * 8] >> 8) & 0xFFu
                                : (uint32_t)(u - m == t);
            };
            auto cinv_build = [&]() {  // perm tables of Sinv[uu][t] (the right half of the reduced [S | I])
                if (tid < m * m) {
                    const int uu = tid / m, t = tid - uu * m;
                    uint32_t tb[5];
                    gf_perm_tables(s_gj[uu * Wd + m + t], tb);
#pragma unroll
                    for (int i = 0; i < 5; ++i) s_cinv[tid * 8 + i] = tb[i];
                }
            };
            // Gauss-Jordan without pivot search: every leading minor of a square submatrix of the parity part
            // of this systematic MDS generator is non-singular; a zero pivot is still detected and reported.
            if (ne <= 64) {
                // m <= 5 (every kcptube-sized loss): wave 0 alone, wave-synchronously (a wave's LDS operations
                // complete in order; the fences keep the compiler from moving reads above writes), while the
                // other waves go on to their share of step 4 -- the solve is off the critical path, and it costs
                // no workgroup barrier.  Step 5 reads the tables after step 4's barrier.
                if (tid < 64) {
                    if (tid < ne) gj_init(tid);
                    if (tid == 0) s_singular = 0;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    const int t = tid / Wd, u = tid - t * Wd;
                    for (int c = 0; c < m; ++c) {
                        const uint32_t piv = s_gj[c * Wd + c];
                        if (piv == 0 && tid == 0) s_singular = 1;
                        const uint32_t inv = piv ? s_exp[255 - s_log[piv]] : 0u;
                        uint32_t f = 0, pv = 0;
                        if (tid < ne) {
                            f = s_gj[t * Wd + c];
                            pv = wk_gmul(s_exp, s_log, s_gj[c * Wd + u], inv);
                        }
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                        if (tid < ne) s_gj[tid] = (t == c) ? pv : (s_gj[tid] ^ wk_gmul(s_exp, s_log, f, pv));
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    }
                    cinv_build();
                    if (debug == 2) ts_solve = __builtin_amdgcn_s_memtime();
                }
            } else {
                for (int e = tid; e < ne; e += kWThreads) gj_init(e);
                if (tid == 0) s_singular = 0;
                __syncthreads();
                for (int c = 0; c < m; ++c) {
                    uint32_t f[2] = {0, 0}, pv[2] = {0, 0};
                    const uint32_t piv = s_gj[c * Wd + c];
                    if (piv == 0 && tid == 0) s_singular = 1;
                    const uint32_t inv = piv ? s_exp[255 - s_log[piv]] : 0u;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int e = tid + k * kWThreads;
                        if (e < ne) {
                            const int t = e / Wd, u = e - t * Wd;
                            f[k] = s_gj[t * Wd + c];
                            pv[k] = wk_gmul(s_exp, s_log, s_gj[c * Wd + u], inv);
                        }
                    }
                    __syncthreads();
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int e = tid + k * kWThreads;
                        if (e < ne) s_gj[e] = (e / Wd == c) ? pv[k] : (s_gj[e] ^ wk_gmul(s_exp, s_log, f[k], pv[k]));
                    }
                    __syncthreads();
                }
                cinv_build();
            }
            // 4. syndromes of the used parity shares over the present data rows, 4 at a time (uniform tiles), each
            //    share group's partial sums meeting in LDS; y_t overwrites row M_t in place
            if (debug == 2 && ne > 64) ts_solve = __builtin_amdgcn_s_memtime();
            const uint64_t miss[4] = {uniform64(body->miss[0]), uniform64(body->miss[1]), uniform64(body->miss[2]),
                                      uniform64(body->miss[3])};
            const int jlo = jg * K / JS, jhi = (jg + 1) * K / JS;
            for (int t0 = 0; t0 < m; t0 += 4) {
                int pr[4], mr[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int t = min(t0 + q, m - 1);
                    pr[q] = __builtin_amdgcn_readfirstlane((int)body->P[t] - K);
                    mr[q] = __builtin_amdgcn_readfirstlane((int)body->M[t]);
                }
                const int rt_n = min(4, m - t0);
                by_rows(rt_n, [&](auto rt) {
                    constexpr int RT = decltype(rt)::value;
                    for (int c = cl; c < nc; c += ncw) {
                        uint32_t y[4] = {0, 0, 0, 0};
                        if (JS == 1) {
#pragma unroll
                            for (int q = 0; q < RT; ++q) y[q] = s_rows[mr[q] * nc + c];
                        }
                        rows_mac<RT>(y, s_rows, nc, c, jlo, jhi, s_tab, R, pr, miss);
#pragma unroll
                        for (int q = 0; q < RT; ++q) {
                            if (JS == 1) s_rows[mr[q] * nc + c] = y[q];
                            else s_part[(jg * 4 + q) * ncw + c] = y[q];
                        }
                    }
                });
                if (JS > 1) {
                    __syncthreads();
                    for (int e = tid; e < rt_n * nc; e += kWThreads) {
                        const int q = e / nc, c = e - q * nc;
                        uint32_t a = s_rows[mr[q] * nc + c];
                        for (int g = 0; g < JS; ++g) a ^= s_part[(g * 4 + q) * ncw + c];
                        s_rows[mr[q] * nc + c] = a;
                    }
                    __syncthreads();
                }
            }
            __syncthreads();
            if (debug == 2) ts_syn = __builtin_amdgcn_s_memtime();
            // 5. out_u = XOR_t Sinv[u][t] * y_t, 4 output rows at a time: the same MAC over the m y rows (gathered
            //    through a row map) with the m x m tables of Sinv
            for (int u0 = 0; u0 < m; u0 += 4) {
                by_rows(m - u0, [&](auto rt) {
                    constexpr int RT = decltype(rt)::value;
                    for (int c = tid; c < nc; c += kWThreads) {
                        uint32_t o[4] = {0, 0, 0, 0};
                        for (int t = 0; t < m; ++t) {
                            const uint32_t x = s_rows[(int)body->M[t] * nc + c];
                            const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
#pragma unroll
                            for (int q = 0; q < RT; ++q) o[q] = tab_mac(o[q], s_cinv + ((u0 + q) * m + t) * 8, s0, s1, s2);
                        }
#pragma unroll
                        for (int q = 0; q < RT; ++q) put_out(out + (u0 + q) * P4 + c, o[q], light);
                    }
                });
            }
            status = (uint32_t)s_singular;
        }
        const uint64_t ts_comp = debug == 2 ? wall_clock64() : 0;
        const uint64_t ck_comp = debug == 2 ? __builtin_amdgcn_s_memtime() : 0;
        // 6. publish: every thread's output stores complete at system scope before the completion word.  light:
        //    the output stores were written through to the system (put_out), so waiting for their
        //    acknowledgements is the whole release -- no L2 write-back pass
        if (light) __builtin_amdgcn_s_waitcnt(kVmcntZero);
        else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (debug == 2 && tid == 0 && w == 0) {  // device-side phase times of this request (100 MHz ticks)
            const uint64_t ts_pub = wall_clock64();
            __hip_atomic_store(trace + 0, ts_loaded - ts_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 1, ts_comp - ts_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 2, ts_pub - ts_comp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 3, ck_comp - ck_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // (shader clocks) encode: tables-check, mac, reduce+store, compute; decode: tables-check, solve
            // (wave 0), syndromes (all waves, from the tables), mix + store
            const bool e = op == kOpEncode;
            __hip_atomic_store(trace + 4, ts_tab - ck_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 5, e ? ts_mac - ts_tab : ts_solve - ts_tab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 6, e ? ck_comp - ts_mac : ts_syn - ts_tab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(trace + 7, e ? ck_comp - ck_loaded : ck_comp - ts_syn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (tid == 0) {
            if (light)
                __hip_atomic_store(done, (uint64_t)last | ((uint64_t)status << 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            else
                __hip_atomic_store(done, (uint64_t)last | ((uint64_t)status << 32), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (tid == 0) __hip_atomic_store(exited, (uint64_t)gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace {

// ---------------------------------------------------------------------------------------------------
// host side: per-device slots, each with its own stream and (at most) one resident worker
// ---------------------------------------------------------------------------------------------------
struct Slot {
    std::mutex mu;
    uint8_t *h = nullptr;        // kSlotBytes of fine-grained pinned host memory
    uint64_t *d_relay = nullptr; // device-memory doorbell relay from workgroup 0 (zeroed before every launch)
    uint8_t *in = nullptr;       // request side (doorbell, body, shares): d_in (BAR) or h
    uint8_t *d_in = nullptr;     // uncached device memory the host writes through the BAR (large-BAR devices;
                                 // uncached so that no L2 line of an earlier request outlives the host's writes)
    hipStream_t stream = nullptr;
    uint32_t seq = 0;            // last posted sequence number (0 = none yet)
    uint32_t gen = 0;            // generation of the last launched worker
    bool running = false;        // a worker of generation `gen` was launched and has not been seen to exit
};

constexpr int kMaxSlots = 8;
struct DevWorkers {
    std::mutex init_mu;
    bool init = false;
    std::atomic<bool> failed{false};
    int nslots = 0;
    Slot slots[kMaxSlots];
};
DevWorkers g_dev[64];

// KFEC_WORKER: unset = on, falling back to the launch path (with one warning) if the worker does not answer;
// "1" = required (a worker that does not answer is an error); "0" = off (the launch path; A/B)
int env_mode()
{
    static const int mode = [] {
        const char *e = getenv("KFEC_WORKER");
        if (e && std::string(e) == "0") return 0;
        if (e && std::string(e) == "1") return 2;
        return 1;
    }();
    return mode;
}
bool env_enabled() { return env_mode() != 0; }
std::atomic<uint64_t> g_served{0};
std::atomic<uint64_t> g_batches{0};

int env_int(const char *name, int def, int lo, int hi)
{
    const char *e = getenv(name);
    int v = e ? atoi(e) : def;
    return v < lo ? lo : (v > hi ? hi : v);
}

int n_wgs()
{
    static const int n = env_int("KFEC_WORKER_WGS", kMaxW, 1, kMaxW);
    return n;
}

// the worker of this device did not answer: required -> error; otherwise warn once and use the launch path
int worker_dead(DevWorkers &d)
{
    d.failed = true;
    if (env_mode() == 2) return KFEC_EHIP;
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true)) fprintf(stderr, "kfec: resident worker did not answer; using the launch path\n");
    return 1;
}

uint64_t idle_ticks()
{
    static const uint64_t t = (uint64_t)env_int("KFEC_WORKER_IDLE_US", 20000, 100, 10000000) * 100;  // 100 MHz clock
    return t;
}

// KFEC_WORKER_LEASE_US: longest residency of one worker launch (default 2 ms): the bound on how long a
// device-wide synchronisation elsewhere in the process waits for the worker's stream while calls continue
uint64_t lease_ticks()
{
    static const uint64_t t = (uint64_t)env_int("KFEC_WORKER_LEASE_US", 2000, 100, 10000000) * 100;
    return t;
}

// KFEC_WORKER_TEST_DEAF=1 (tests only): the worker never answers a request, so the caller's 2 s "did not
// answer" fallback to the launch path runs
int test_deaf()
{
    static const int d = env_int("KFEC_WORKER_TEST_DEAF", 0, 0, 1);
    return d;
}

// KFEC_WORKER_POLL: 0 relay, 1 direct (see the kernel's poll; direct measured faster at every W: 20:3 encode
// 9.3 vs 11.4 us per call at W = 8, profiles/r03_worker_sweep.txt)
int poll_mode()
{
    static const int m = env_int("KFEC_WORKER_POLL", 1, 0, 1);
    return m;
}

// KFEC_WORKER_DEBUG=2: device-side phase times of workgroup 0, summed and printed when the workers stop
// KFEC_WORKER_FENCES: 1 (default) = light fences (see the kernel's steps 0 and 6), 0 = full system-scope
// acquire / release (an L2 invalidate per request, an L2 write-back per completion)
int light_fences()
{
    static const int f = env_int("KFEC_WORKER_FENCES", 1, 0, 1);
    return f;
}

int debug_level()
{
    static const int d = env_int("KFEC_WORKER_DEBUG", 0, 0, 2);
    return d;
}
std::atomic<uint64_t> g_dbg_n{0}, g_dbg_load{0}, g_dbg_comp{0}, g_dbg_pub{0}, g_dbg_clk{0};
std::atomic<uint64_t> g_dbg_ne{0}, g_dbg_etab{0}, g_dbg_emac{0}, g_dbg_ered{0}, g_dbg_ecomp{0};
std::atomic<uint64_t> g_dbg_nd{0}, g_dbg_dtab{0}, g_dbg_dsolve{0}, g_dbg_dsyn{0}, g_dbg_dmix{0};

// KFEC_WORKER_BAR: 1 = the request side lives in device memory the host writes through the PCIe BAR (posted
// writes: the worker then reads its shares from local HBM, not across PCIe), 0 = in the pinned slot; default:
// on where the device reports a large BAR.  (tools/bar_probe.hip: 28.8 KB by memcpy in 0.87 us.)
bool bar_staging(int dev)
{
    const char *e = getenv("KFEC_WORKER_BAR");
    if (e) return std::string(e) != "0";
    int large = 0;
    return hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, dev) == hipSuccess && large;
}

// Request writes.  Device memory through the BAR is write-combined: stores may reach the device in any order,
// so the body and shares are fenced before the doorbell, and the doorbell is fenced out (never read back: a
// read across the BAR costs a round trip).
// Into BAR memory by 32-byte stores: 28.8 KB in 0.68 us against memcpy's 0.82 (tools/bar_probe.hip on the box;
// `rep movsb` is as fast for one large copy but made the decode's per-row copies several us slower).
typedef uint8_t u8x32 __attribute__((vector_size(32), aligned(1)));  // (one ymm register under avx2)
__attribute__((target("avx2"))) void copy_wc_avx2(uint8_t *d, const uint8_t *s, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32) *reinterpret_cast<u8x32 *>(d + i) = *reinterpret_cast<const u8x32 *>(s + i);
    if (i < n) std::memcpy(d + i, s + i, n - i);
}

inline void put(Slot &s, size_t off, const void *src, size_t n)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (s.d_in && avx2) copy_wc_avx2(s.in + off, static_cast<const uint8_t *>(src), n);
    else std::memcpy(s.in + off, src, n);
}
inline void ring(Slot &s, uint64_t v)
{
    if (s.d_in) {
        __builtin_ia32_sfence();
        *reinterpret_cast<volatile uint64_t *>(s.in + kOffDoorbell) = v;
        __builtin_ia32_sfence();
    } else {
        __atomic_store_n(reinterpret_cast<uint64_t *>(s.in + kOffDoorbell), v, __ATOMIC_SEQ_CST);
    }
}

inline uint64_t load_acq(const uint8_t *p) { return __atomic_load_n(reinterpret_cast<const uint64_t *>(p), __ATOMIC_ACQUIRE); }

DevWorkers *get_dev(int dev)
{
    if (dev < 0 || dev >= 64) return nullptr;
    DevWorkers &d = g_dev[dev];
    std::lock_guard<std::mutex> lk(d.init_mu);
    if (d.init) return d.failed ? nullptr : &d;
    d.init = true;
    const int n = env_int("KFEC_WORKER_SLOTS", 2, 1, kMaxSlots);
    for (int i = 0; i < n; ++i) {
        Slot &s = d.slots[i];
        void *p = nullptr, *q = nullptr;
        if (hipHostMalloc(&p, kSlotBytes, hipHostMallocCoherent) != hipSuccess) break;
        if (hipMalloc(&q, 256) != hipSuccess) {
            (void)hipHostFree(p);
            break;
        }
        std::memset(p, 0, kOffShares);
        // The worker's stream gets the greatest priority: HIP maps streams onto a few hardware queues per priority
        // (GPU_MAX_HW_QUEUES, 4 by default) and a stream sharing the resident worker's in-order queue would wait
        // behind the worker kernel for up to its lease (measured: a queue's seal launch, 2.1 ms per small flush).
        // The library's and the caller's other streams are normal priority, so none lands on a worker's queue.
        int prio_lo = 0, prio_hi = 0;
        if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_hi = prio_lo = 0;
        if (hipStreamCreateWithPriority(&s.stream, hipStreamNonBlocking, prio_hi) != hipSuccess &&
            hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) {
            (void)hipHostFree(p);
            (void)hipFree(q);
            break;
        }
        s.h = static_cast<uint8_t *>(p);
        s.d_relay = static_cast<uint64_t *>(q);
        s.in = s.h;
        if (bar_staging(dev)) {
            void *b = nullptr;
            if (hipExtMallocWithFlags(&b, kOffShares + kStageMax, hipDeviceMallocUncached) == hipSuccess &&
                hipMemset(b, 0, kOffShares) == hipSuccess) {
                s.d_in = static_cast<uint8_t *>(b);
                s.in = s.d_in;
            } else if (b) {
                (void)hipFree(b);
            }
        }
        d.nslots = i + 1;
    }
    if (d.nslots == 0) d.failed = true;
    return d.failed ? nullptr : &d;
}

Slot &acquire(DevWorkers &d, std::unique_lock<std::mutex> &lk)
{
    for (int i = 0; i < d.nslots; ++i) {
        std::unique_lock<std::mutex> l(d.slots[i].mu, std::try_to_lock);
        if (l.owns_lock()) {
            lk = std::move(l);
            return d.slots[i];
        }
    }
    const size_t h = std::hash<std::thread::id>()(std::this_thread::get_id());
    Slot &s = d.slots[h % (size_t)d.nslots];
    lk = std::unique_lock<std::mutex>(s.mu);
    return s;
}

// workgroup 0 has left (idle) -- the others leave with it
bool leader_exited(const Slot &s) { return (uint32_t)load_acq(s.h + kOffExited) == s.gen; }

int launch_worker(Slot &s)
{
    s.gen += 1;
    // the relay word is cleared in stream order: after the previous worker's last workgroup, before this one
    if (hipMemsetAsync(s.d_relay, 0, 256, s.stream) != hipSuccess) return KFEC_EHIP;
    hipLaunchKernelGGL(kfec_worker_kernel, dim3(n_wgs()), dim3(kWThreads), kLdsBytes, s.stream, s.h, s.in, s.d_relay, s.gen,
                       s.seq - 1, idle_ticks(), lease_ticks(), debug_level(), poll_mode(), light_fences(), test_deaf());
    if (hipGetLastError() != hipSuccess) {
        s.running = false;
        return KFEC_EHIP;
    }
    s.running = true;
    return 0;
}

// the combined completion of `seq`: -1 while some workgroup has not finished it, else the largest status
int completion(const Slot &s, uint32_t seq, int W)
{
    uint32_t st = 0;
    for (int w = 0; w < W; ++w) {
        const uint64_t d = load_acq(s.h + kOffDone + kLineW * w);
        if (db_seq(d) != seq) return -1;
        st = st > (uint32_t)(d >> 32) ? st : (uint32_t)(d >> 32);
    }
    return (int)st;
}

// post the doorbell and wait for every workgroup's completion word; returns the status (0, 1 singular,
// 3 refused) or a KFEC_E* code.  hi: the doorbell's bits 32-63 (K, N, B; or a batch request's length)
int post_and_wait_db(Slot &s, uint32_t op, uint64_t hi)
{
    const int W = n_wgs();
    uint32_t seq = (s.seq + 1) & kSeqMask;
    if (seq == 0 || seq == kSeqMask) seq = 1;  // (kSeqMask: the seq of the relay's quit value)
    s.seq = seq;
    ring(s, (uint64_t)(seq & kSeqMask) | ((uint64_t)op << 30) | (hi << 32));
    if (!s.running || leader_exited(s)) {
        const int rc = launch_worker(s);
        if (rc) return rc;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t it = 1;; ++it) {
        const int st = completion(s, seq, W);
        if (st >= 0) {
            if (debug_level() == 2) {
                g_dbg_n += 1;
                g_dbg_load += load_acq(s.h + kOffTrace);
                g_dbg_comp += load_acq(s.h + kOffTrace + 8);
                g_dbg_pub += load_acq(s.h + kOffTrace + 16);
                g_dbg_clk += load_acq(s.h + kOffTrace + 24);
                if (op == kOpEncode) {
                    g_dbg_ne += 1;
                    g_dbg_etab += load_acq(s.h + kOffTrace + 32);
                    g_dbg_emac += load_acq(s.h + kOffTrace + 40);
                    g_dbg_ered += load_acq(s.h + kOffTrace + 48);
                    g_dbg_ecomp += load_acq(s.h + kOffTrace + 56);
                } else if (op == kOpDecode) {
                    g_dbg_nd += 1;
                    g_dbg_dtab += load_acq(s.h + kOffTrace + 32);
                    g_dbg_dsolve += load_acq(s.h + kOffTrace + 40);
                    g_dbg_dsyn += load_acq(s.h + kOffTrace + 48);
                    g_dbg_dmix += load_acq(s.h + kOffTrace + 56);
                }
            }
            return st;
        }
        if ((it & 255) == 0) {
            if (leader_exited(s)) {
                // the worker left its loop (idle timeout) before all of it saw this doorbell: launch a new one,
                // which starts behind the old one on the slot's stream and finds the doorbell pending (a slice
                // the old one already wrote is rewritten with the same bytes)
                if (completion(s, seq, W) >= 0) continue;
                const int rc = launch_worker(s);
                if (rc) return rc;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                if (debug_level())
                    fprintf(stderr, "kfec worker: no answer; seq %llx done[0] %llx exited[0] %llx gen %u stream %d\n",
                            (unsigned long long)s.seq, (unsigned long long)load_acq(s.h + kOffDone),
                            (unsigned long long)load_acq(s.h + kOffExited), s.gen, (int)hipStreamQuery(s.stream));
                // Post STOP so that a worker that is merely slow leaves at once; one that ignores its doorbell
                // still leaves by itself at its idle timeout or its lease (whichever comes first), and a kernel
                // that never reaches its poll again would hold its CUs until the process ends.
                uint32_t stop = (s.seq + 1) & kSeqMask;
                if (stop == 0 || stop == kSeqMask) stop = 1;
                s.seq = stop;
                ring(s, db_pack(stop, kOpStop, 1, 1, 0));
                s.running = false;
                return kWorkerDead;
            }
        }
        __builtin_ia32_pause();
    }
}

int post_and_wait(Slot &s, uint32_t op, int K, int N, int B)
{
    return post_and_wait_db(s, op, db_pack(0, op, (uint32_t)K, (uint32_t)N, (uint32_t)B) >> 32);
}

bool shape_ok(int K, int N, size_t B, int mrows)
{
    const int R = N - K, W = n_wgs();
    const size_t pitch = (B + 15) & ~size_t(15), G = pitch / 16;
    return B > 0 && B <= 0xFFFF && R >= 1 && R <= kMaxR && mrows <= kMaxR && (size_t)(K + R) * pitch <= kStageMax &&
           (size_t)R * K * 32 <= kTabMax && (size_t)K * ((G + W - 1) / W) * 16 <= kSliceMax;
}

}  // namespace

bool host_solve(const uint8_t *h_enc, int K, int m, const uint8_t *M, const uint8_t *P, uint8_t *D);

bool worker_enabled() { return env_enabled(); }

bool bar_writable(int device) { return bar_staging(device); }

void copy_to_bar(void *dst, const void *src, size_t n)
{
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) copy_wc_avx2(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n);
    else std::memcpy(dst, src, n);
}

void bar_fence() { __builtin_ia32_sfence(); }

// The largest number of groups one workgroup's item range touches (the decode's LDS tables hold that many).
static int batch_groups_per_wg(int n, int G16, int W)
{
    const int64_t I = (int64_t)n * G16;
    int most = 0;
    for (int w = 0; w < W; ++w) {
        const int64_t i0 = w * I / W, i1 = (w + 1) * I / W;
        if (i1 > i0) most = std::max(most, (int)((i1 - 1) / G16 - i0 / G16 + 1));
    }
    return most;
}

bool worker_batch_ok(const BatchSpec &b)
{
    if (!env_enabled() || b.n < 1 || b.K < 1 || b.N <= b.K || b.N > 256 || b.B < 1 || b.B > 0xFFFF) return false;
    const int R = b.N - b.K, G16 = (b.B + 15) / 16;
    if (R > kBatchMaxR || b.opitch < b.ooff + (size_t)G16 * 16 || (b.opitch & 15) || (b.ooff & 15)) return false;
    if ((size_t)b.K * R * 32 > kTabMax) return false;  // the matrix tables / one group's D tables
    size_t bytes = sizeof(BatchBody) + (size_t)b.n * b.K * 8;
    if (b.op == kBatchDecode) {
        if (b.rec_stride < 16 + (size_t)R * b.K || (b.rec_stride & 15)) return false;
        bytes = ((bytes + 15) & ~size_t(15)) + (size_t)b.n * b.rec_stride;
        if ((size_t)batch_groups_per_wg(b.n, G16, n_wgs()) * b.K * R * 32 > kTabMax) return false;
    }
    return bytes <= kBatchReqMax;
}

int worker_batch(int device, const BatchSpec &b)
{
    if (!worker_batch_ok(b)) return 1;
    DevWorkers *d = get_dev(device);
    if (!d) return env_mode() == 2 ? KFEC_EHIP : 1;
    std::unique_lock<std::mutex> lk;
    Slot &s = acquire(*d, lk);
    BatchBody body{};
    body.enc = reinterpret_cast<uint64_t>(b.enc);
    body.mat_id = b.mat_id;
    body.arena = reinterpret_cast<uint64_t>(b.arena);
    body.out = reinterpret_cast<uint64_t>(b.out);
    body.n = (uint32_t)b.n;
    body.K = (uint32_t)b.K;
    body.N = (uint32_t)b.N;
    body.B = (uint32_t)b.B;
    body.opitch = (uint32_t)b.opitch;
    body.ooff = (uint32_t)b.ooff;
    const size_t dbytes = (size_t)b.n * b.K * 8;
    size_t bytes = sizeof(BatchBody) + dbytes;
    if (b.op == kBatchDecode) {
        body.rec_off = (uint32_t)((bytes + 15) & ~size_t(15));
        body.rec_stride = (uint32_t)b.rec_stride;
        bytes = body.rec_off + (size_t)b.n * b.rec_stride;
    }
    put(s, kOffShares, &body, sizeof(body));
    put(s, kOffShares + sizeof(BatchBody), b.desc, dbytes);
    if (b.op == kBatchDecode) put(s, kOffShares + body.rec_off, b.rec, (size_t)b.n * b.rec_stride);
    const uint32_t len16 = (uint32_t)((bytes + 15) / 16);
    const int st = post_and_wait_db(s, b.op == kBatchDecode ? kOpDecode : kOpEncode, (uint64_t)len16);  // B = 0
    if (st == kWorkerDead) return worker_dead(*d);
    if (st < 0) return st;
    if (st) return KFEC_EHIP;
    g_batches.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

uint64_t worker_batches() { return g_batches.load(std::memory_order_relaxed); }

bool worker_solve(const uint8_t *h_enc, int K, int m, const uint8_t *M, const uint8_t *P, uint8_t *D)
{
    return m >= 1 && m <= kHostSolveMax && host_solve(h_enc, K, m, M, P, D);
}
uint64_t worker_served() { return g_served.load(std::memory_order_relaxed); }

int worker_encode(int device, const uint8_t *d_enc, uint64_t mat_id, int K, int N, size_t B, const uint8_t *input,
                  uint8_t *parity_out)
{
    if (!env_enabled() || !shape_ok(K, N, B, 0)) return 1;
    DevWorkers *d = get_dev(device);
    if (!d) return env_mode() == 2 ? KFEC_EHIP : 1;
    std::unique_lock<std::mutex> lk;
    Slot &s = acquire(*d, lk);
    const size_t pitch = (B + 15) & ~size_t(15), R = (size_t)(N - K);
    WorkerBody body{};
    body.enc = reinterpret_cast<uint64_t>(d_enc);
    body.mat_id = mat_id;
    put(s, kOffBody, &body, sizeof(body));
    if (pitch == B) {
        put(s, kOffShares, input, (size_t)K * B);
    } else {
        for (int j = 0; j < K; ++j) put(s, kOffShares + j * pitch, input + j * B, B);
    }
    const uint8_t *rows = s.h + kOffShares;  // (the output rows follow the K share rows, in the host slot)
    const int st = post_and_wait(s, kOpEncode, K, N, (int)B);
    if (st == kWorkerDead) return worker_dead(*d);
    if (st < 0) return st;
    if (st) return KFEC_EHIP;  // the worker refused the request's shape
    g_served.fetch_add(1, std::memory_order_relaxed);
    const uint8_t *out = rows + (size_t)K * pitch;
    if (pitch == B) {
        std::memcpy(parity_out, out, R * B);
    } else {
        for (size_t r = 0; r < R; ++r) std::memcpy(parity_out + r * B, out + r * pitch, B);
    }
    return 0;
}

// S = rows P_t, columns M_u of the coder's matrix; Gauss-Jordan on [S | I] (no pivot search, as on the
// device: every square submatrix of the parity part is non-singular), then D[u][j] for the K staged rows:
// Sinv[u][t] for row M_t (which holds parity share P_t), XOR_t Sinv[u][t] * E[P_t][j] for a present data row j
// (out_u = XOR_t Sinv[u][t] * (P_t - XOR_j E[P_t][j] * D_j), regrouped by row).  false: a zero pivot (the
// device solve then runs and reports it).
bool host_solve(const uint8_t *h_enc, int K, int m, const uint8_t *M, const uint8_t *P, uint8_t *D)
{
    static const GfTables gt = make_gf_tables();
    auto mul = [&](uint32_t a, uint32_t b) -> uint8_t { return (a && b) ? gt.exp[gt.log[a] + gt.log[b]] : 0; };
    uint8_t a[kHostSolveMax][2 * kHostSolveMax];
    for (int t = 0; t < m; ++t)
        for (int u = 0; u < m; ++u) {
            a[t][u] = h_enc[(size_t)P[t] * K + M[u]];
            a[t][m + u] = (uint8_t)(t == u);
        }
    for (int c = 0; c < m; ++c) {
        if (!a[c][c]) return false;
        const uint32_t inv = gt.exp[255 - gt.log[a[c][c]]];
        for (int u = 0; u < 2 * m; ++u) a[c][u] = mul(a[c][u], inv);
        for (int t = 0; t < m; ++t) {
            const uint32_t f = a[t][c];
            if (t == c || !f) continue;
            for (int u = 0; u < 2 * m; ++u) a[t][u] ^= mul(f, a[c][u]);
        }
    }
    int held[256];  // staged row -> t if it holds parity share P_t, else -1
    for (int j = 0; j < K; ++j) held[j] = -1;
    for (int t = 0; t < m; ++t) held[M[t]] = t;
    for (int u = 0; u < m; ++u) {
        uint8_t *d = D + (size_t)u * K;
        int ls[kHostSolveMax];  // log Sinv[u][t] (-1: zero)
        for (int t = 0; t < m; ++t) ls[t] = a[u][m + t] ? gt.log[a[u][m + t]] : -1;
        for (int j = 0; j < K; ++j) {
            if (held[j] >= 0) {
                d[j] = a[u][m + held[j]];
                continue;
            }
            uint32_t x = 0;
            for (int t = 0; t < m; ++t) {
                const uint32_t e = h_enc[(size_t)P[t] * K + j];
                if (e && ls[t] >= 0) x ^= gt.exp[ls[t] + gt.log[e]];
            }
            d[j] = (uint8_t)x;
        }
    }
    return true;
}

int worker_decode(int device, const uint8_t *d_enc, const uint8_t *h_enc, uint64_t mat_id, int K, int N, size_t B,
                  const uint8_t *const *row_ptr, int m, const uint8_t *M, const uint8_t *P, uint8_t *out)
{
    if (!env_enabled() || !shape_ok(K, N, B, m)) return 1;
    DevWorkers *d = get_dev(device);
    if (!d) return env_mode() == 2 ? KFEC_EHIP : 1;
    std::unique_lock<std::mutex> lk;
    Slot &s = acquire(*d, lk);
    const size_t pitch = (B + 15) & ~size_t(15);
    WorkerBody body{};  // built here, written once (never read back across the BAR)
    body.enc = reinterpret_cast<uint64_t>(d_enc);
    body.mat_id = mat_id;
    body.m = (uint32_t)m;
    for (int t = 0; t < m; ++t) {
        body.M[t] = M[t];
        body.P[t] = P[t];
        body.miss[M[t] >> 6] |= 1ull << (M[t] & 63);
    }
    uint8_t D[512];
    static const int host_solves = env_int("KFEC_WORKER_HOST_SOLVE", 1, 0, 1);  // 0: every solve on the device
    if (host_solves && h_enc && m <= kHostSolveMax && m * m * K <= kHostSolveWork && m * K <= 512 &&
        host_solve(h_enc, K, m, M, P, D)) {
        body.solved = 1;
        put(s, kOffCinv, D, (size_t)m * K);
    }
    put(s, kOffBody, &body, sizeof(body));
    for (int j = 0; j < K; ++j) put(s, kOffShares + j * pitch, row_ptr[j], B);
    const uint8_t *rows = s.h + kOffShares;
    const int st = post_and_wait(s, kOpDecode, K, N, (int)B);
    if (st == kWorkerDead) return worker_dead(*d);
    if (st < 0) return st;
    if (st == 3) return KFEC_EHIP;  // the worker refused the request's shape
    g_served.fetch_add(1, std::memory_order_relaxed);
    if (st) return KFEC_ESINGULAR;
    const uint8_t *o = rows + (size_t)K * pitch;
    if (pitch == B) {
        std::memcpy(out, o, (size_t)m * B);
    } else {
        for (int t = 0; t < m; ++t) std::memcpy(out + t * B, o + t * pitch, B);
    }
    return 0;
}

// One empty request (answered by every workgroup at once): the communication floor of the per-call path
int worker_ping(int device)
{
    if (!env_enabled()) return 1;
    DevWorkers *d = get_dev(device);
    if (!d) return env_mode() == 2 ? KFEC_EHIP : 1;
    std::unique_lock<std::mutex> lk;
    Slot &s = acquire(*d, lk);
    const int st = post_and_wait(s, kOpPing, 1, 2, 1);
    if (st == kWorkerDead) return worker_dead(*d);
    return st < 0 ? st : 0;
}

// Stop the resident workers of a device (no coder left on it): post STOP to every running slot and wait for
// the kernel to finish.  Bounded: a worker that does not answer within 2 s is left to its idle timeout.
void worker_stop(int device)
{
    if (device < 0 || device >= 64) return;
    if (debug_level() == 2 && g_dbg_n.load())
        fprintf(stderr, "kfec worker: %llu requests, device us per request (workgroup 0): loads %.2f compute %.2f publish %.2f; "
                        "shader clock during compute %.0f MHz\n",
                (unsigned long long)g_dbg_n.load(), g_dbg_load.load() / 100.0 / g_dbg_n.load(),
                g_dbg_comp.load() / 100.0 / g_dbg_n.load(), g_dbg_pub.load() / 100.0 / g_dbg_n.load(),
                g_dbg_comp.load() ? 100.0 * g_dbg_clk.load() / g_dbg_comp.load() : 0.0);
    // (the sub-phases are shader clocks: converted at the clock measured over the compute phases)
    const double mhz = g_dbg_comp.load() ? 100.0 * g_dbg_clk.load() / g_dbg_comp.load() : 2400.0;
    if (debug_level() == 2 && g_dbg_ne.load())
        fprintf(stderr, "kfec worker: encodes %llu: tables-check %.2f mac %.2f reduce+store %.2f compute %.2f us\n",
                (unsigned long long)g_dbg_ne.load(), g_dbg_etab.load() / mhz / g_dbg_ne.load(),
                g_dbg_emac.load() / mhz / g_dbg_ne.load(), g_dbg_ered.load() / mhz / g_dbg_ne.load(),
                g_dbg_ecomp.load() / mhz / g_dbg_ne.load());
    if (debug_level() == 2 && g_dbg_nd.load())
        fprintf(stderr, "kfec worker: decodes %llu: tables-check %.2f solve(wave 0) %.2f syndromes %.2f mix+store %.2f us\n",
                (unsigned long long)g_dbg_nd.load(), g_dbg_dtab.load() / mhz / g_dbg_nd.load(),
                g_dbg_dsolve.load() / mhz / g_dbg_nd.load(), g_dbg_dsyn.load() / mhz / g_dbg_nd.load(),
                g_dbg_dmix.load() / mhz / g_dbg_nd.load());
    DevWorkers &d = g_dev[device];
    {
        std::lock_guard<std::mutex> lk(d.init_mu);
        if (!d.init || d.failed) return;
    }
    const int W = n_wgs();
    for (int i = 0; i < d.nslots; ++i) {
        Slot &s = d.slots[i];
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.running) continue;
        auto all_exited = [&] {
            for (int w = 0; w < W; ++w)
                if ((uint32_t)load_acq(s.h + kOffExited + kLineW * w) != s.gen) return false;
            return true;
        };
        if (!all_exited()) {
            uint32_t seq = (s.seq + 1) & kSeqMask;
            if (seq == 0 || seq == kSeqMask) seq = 1;  // (kSeqMask: the seq of the relay's quit value)
            s.seq = seq;
            ring(s, db_pack(seq, kOpStop, 1, 1, 0));
            const auto t0 = std::chrono::steady_clock::now();
            while (!all_exited() && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) __builtin_ia32_pause();
        }
        if (all_exited()) (void)hipStreamSynchronize(s.stream);
        s.running = false;
    }
}

}  // namespace kfec
