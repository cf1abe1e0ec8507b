// kfec_worker.hip -- the per-call latency path of the fecpp::fec_code drop-in (kfec_encode / kfec_decode on
// ONE group from host memory, fecpp.cpp:495-513 and 518-587): a resident device worker instead of a kernel
// launch + stream synchronisation per call.
//
// Why: the reference codes a 20:3 group in ~8 us on the KCP updater thread while it holds the KCP mutex
// (kcp.cpp:144, client.cpp:775 -> fec_maker :797).  A launch + hipStreamSynchronize alone costs more than
// that, so the per-call path cannot pay one per group.
//
// How: each worker is a single 512-thread workgroup that stays resident on one CU and polls a doorbell word
// in fine-grained (coherent) pinned host memory.  The caller copies the group's shares into the slot's
// pinned stage, writes the doorbell (sequence number + op + K, N, B in ONE 64-bit store), and spins on the
// slot's completion word.  The worker sees the doorbell over PCIe, pulls the request body and the shares
// into LDS in one burst of 16-byte loads, computes, writes the parity / recovered shards straight back into
// the pinned stage, publishes them with a system-scope release, and stores the completion word.
//
//   encode  parity_r = XOR_j enc[K+r][j] * D_j                       (fecpp.cpp:504-510)
//   decode  rows in the reference's selection order (fecpp.cpp:528-548, done by the caller: bookkeeping only),
//           y_t = share(row M_t) ^ XOR_{j present} enc[P_t][j] * D_j  (syndrome of the used parity share P_t)
//           out_u = XOR_t Sinv[u][t] * y_t,  S[t][u] = enc[P_t][M_u]  (the missing rows of the K x K inverse,
//           fecpp.cpp:564-583; the inverse is unique, so the bytes equal the reference's Gauss-Jordan result)
//
// All GF products use the perm MAC of kfec_gf.hpp with tables in LDS; the parity-row tables of the coder's
// matrix are copied from its device allocation (enc_tab_offset) once per matrix and kept in LDS while the
// same matrix is used.  Lifetime: a worker exits when asked (op STOP), or after KFEC_WORKER_IDLE_US without a
// request (default 20 ms), and always writes its generation to the slot's exit word; the host relaunches it on
// the next request.  Every wave reaches the exit: the loop's only waits are the bounded doorbell poll and
// workgroup barriers.
#include "kfec_gf.hpp"
#include "kfec_internal.hpp"

#include <atomic>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

namespace kfec {
namespace {

constexpr int kWThreads = 512;
constexpr int kMaxR = 16;                  // parity rows (encode) / missing rows (decode) a worker takes
constexpr size_t kStageMax = 38 * 1024;    // (K + R) * pitch: LDS rows of the shares (20:3 at 1440 B: 33 KB)
constexpr size_t kTabMax = 16 * 1024;      // R * K * 20 bytes: parity-row perm tables in LDS
// LDS carve (bytes, all 16-aligned)
constexpr size_t kLdsData = 0;
constexpr size_t kLdsTab = kLdsData + kStageMax;
constexpr size_t kLdsCinv = kLdsTab + kTabMax;                    // m x m perm tables of Sinv
constexpr size_t kLdsGj = kLdsCinv + kMaxR * kMaxR * 20;          // m x 2m Gauss-Jordan matrix (u32 entries)
constexpr size_t kLdsGf = kLdsGj + kMaxR * 2 * kMaxR * 4;         // exp[512] + log[256]
constexpr size_t kLdsBody = kLdsGf + 768;                         // the request body (128 bytes)
constexpr size_t kLdsBytes = kLdsBody + 128;
static_assert(kLdsBytes <= 64 * 1024, "the worker fits the default 64 KiB workgroup LDS");

// Slot layout in pinned host memory (offsets in bytes).  The host writes [0, 8) and the body; the device
// writes the completion / exit words (their own 128-byte line) and the output rows.
constexpr size_t kOffDoorbell = 0;
constexpr size_t kOffDone = 128;    // u64: seq | status << 32
constexpr size_t kOffExited = 136;  // u64: generation of a worker that has left its loop
constexpr size_t kOffTrace = 144;   // u64: progress marker (KFEC_WORKER_DEBUG only): phase | seq << 8
constexpr size_t kOffBody = 256;    // WorkerBody
constexpr size_t kOffShares = 1024; // K rows x pitch: the shares, in row order
constexpr size_t kSlotBytes = kOffShares + 2 * kStageMax;  // shares + output rows

enum : uint32_t { kOpEncode = 1, kOpDecode = 2, kOpStop = 3 };
constexpr int kWorkerDead = -1000;  // post_and_wait: the worker did not answer (the device's workers are disabled)
constexpr uint32_t kSeqMask = (1u << 30) - 1;

// doorbell: seq (30 bits) | op (2) | K - 1 (8) | N - 1 (8) | B (16)
__host__ __device__ inline uint64_t db_pack(uint32_t seq, uint32_t op, uint32_t K, uint32_t N, uint32_t B)
{
    return (uint64_t)(seq & kSeqMask) | ((uint64_t)op << 30) | ((uint64_t)(K - 1) << 32) | ((uint64_t)(N - 1) << 40) |
           ((uint64_t)B << 48);
}
__host__ __device__ inline uint32_t db_seq(uint64_t v) { return (uint32_t)v & kSeqMask; }
__host__ __device__ inline uint32_t db_op(uint64_t v) { return (uint32_t)(v >> 30) & 3u; }

struct WorkerBody {          // 128 bytes
    uint64_t enc;            // device address of the coder's matrix allocation (N x K bytes, then its tables)
    uint64_t mat_id;         // unique per built matrix: the LDS table cache key
    uint64_t miss[4];        // decode: bit j set <=> row j holds a parity share (data share j is missing)
    uint32_t m;              // decode: number of missing data shares (<= kMaxR)
    uint32_t out_pitch;      // unused by the device; keeps the layout explicit
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

__device__ __forceinline__ uint32_t wk_apply(uint32_t acc, const uint32_t *t, uint32_t x)
{
    return perm_mac(acc, t, x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u);
}

}  // namespace

__global__ void __launch_bounds__(kWThreads) kfec_worker_kernel(uint8_t *slot, uint32_t gen, uint32_t last_seq,
                                                                uint64_t idle_ticks, int debug)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t s_db;
    __shared__ uint64_t s_mat;
    __shared__ int s_singular;
    const int tid = threadIdx.x;
    uint8_t *s_exp = smem + kLdsGf, *s_log = smem + kLdsGf + 512;
    for (int i = tid; i < 512; i += kWThreads) s_exp[i] = w_gf.exp[i];
    for (int i = tid; i < 256; i += kWThreads) s_log[i] = w_gf.log[i];
    if (tid == 0) s_mat = 0;  // matrix ids start at 1
    uint64_t *doorbell = reinterpret_cast<uint64_t *>(slot + kOffDoorbell);
    uint64_t *done = reinterpret_cast<uint64_t *>(slot + kOffDone);
    uint64_t *exited = reinterpret_cast<uint64_t *>(slot + kOffExited);
    const uint4 *h_body = reinterpret_cast<const uint4 *>(slot + kOffBody);
    const uint4 *h_rows = reinterpret_cast<const uint4 *>(slot + kOffShares);
    uint32_t last = last_seq;
    uint64_t *trace = reinterpret_cast<uint64_t *>(slot + kOffTrace);
    auto mark = [&](uint64_t phase) {  // (waits for the marker's own store: a later fault cannot drop it)
        if (debug && (tid & 63) == 0) {  // one marker per wave: trace[2 + wave]
            __hip_atomic_store(trace + (tid == 0 ? 0 : 2 + (tid >> 6)), phase | ((uint64_t)last << 8), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            if (tid == 0)
                __hip_atomic_store(trace + 2, phase | ((uint64_t)last << 8), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
    };
    mark(1);

    for (;;) {
        // The whole of wave 0 polls (all lanes load the same word; the value is made wave-uniform), never one
        // lane: a loop under `tid == 0` leaves lanes 1-63 of wave 0 free to run on to the next barrier while
        // lane 0 spins, and the compiler's structurized loop then replays the previous request forever.
        if (tid < 64) {
            const uint64_t t0 = wall_clock64();
            uint64_t v;
            for (;;) {
                const uint64_t x = __hip_atomic_load(doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                v = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
                    (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
                if (db_seq(v) != last) break;
                if (wall_clock64() - t0 > idle_ticks) {
                    v = 0;  // idle: leave (seq 0 is never posted)
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            if (tid == 0) s_db = v;
        }
        __syncthreads();
        const uint64_t v = s_db;
        if (v == 0) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the stage and body written before the doorbell
        last = db_seq(v);
        mark(2);
        const uint32_t op = db_op(v);
        uint32_t status = 0;
        if (op == kOpStop) {
            if (tid == 0) __hip_atomic_store(done, (uint64_t)last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        const int K = (int)((v >> 32) & 0xFF) + 1, N = (int)((v >> 40) & 0xFF) + 1, R = N - K;
        const int B = (int)(v >> 48);
        const int pitch = (B + 15) & ~15, P4 = pitch >> 2;
        // 1. one burst of 16-byte loads: the body and the K share rows (clamped indices keep r[] in VGPRs)
        {
            const int n16 = K * (pitch >> 4);
            uint4 *s16 = reinterpret_cast<uint4 *>(smem + kLdsData);
            uint4 *b16 = reinterpret_cast<uint4 *>(smem + kLdsBody);
            mark(10);
            const uint4 bq = h_body[tid & 7];
            for (int i0 = 0; i0 < n16; i0 += kWThreads * 8) {
                uint4 r[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) r[u] = h_rows[min(i0 + u * kWThreads + tid, n16 - 1)];
#pragma unroll
                for (int u = 0; u < 8; ++u) s16[min(i0 + u * kWThreads + tid, n16 - 1)] = r[u];  // (same bytes)
            }
            if (tid < 8) b16[tid] = bq;
            mark(11);
        }
        __syncthreads();
        mark(3);
        const WorkerBody *body = reinterpret_cast<const WorkerBody *>(smem + kLdsBody);
        uint32_t *s_tab = reinterpret_cast<uint32_t *>(smem + kLdsTab);
        const uint32_t *s_rows = reinterpret_cast<const uint32_t *>(smem + kLdsData);
        // 2. parity-row perm tables of this matrix: s_tab[(j * R + r) * 5 + i], kept while the matrix is reused
        if (debug && tid == 0)
            __hip_atomic_store(trace + 1, (uint64_t)body->m | ((uint64_t)body->M[0] << 8) | ((uint64_t)body->P[0] << 16) |
                                              ((uint64_t)K << 24) | ((uint64_t)R << 40) | ((uint64_t)(body->mat_id & 0xFF) << 56),
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (body->mat_id != s_mat) {
            const uint32_t *g_tab =
                reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(body->enc) + enc_tab_offset(K, N));
            const int rows = (int)enc_tab_rows(R), n = K * R * 5;
            for (int i = tid; i < n; i += kWThreads) {
                const int e = i / 5, w = i - e * 5, j = e / R, r = e - j * R;
                s_tab[i] = g_tab[(j * rows + r) * 5 + w];
            }
            __syncthreads();
            if (tid == 0) s_mat = body->mat_id;
        }
        uint32_t *out = reinterpret_cast<uint32_t *>(slot + kOffShares + (size_t)K * pitch);
        if (op == kOpEncode) {
            // items (r, c): parity row r, dword column c
            for (int it = tid; it < R * P4; it += kWThreads) {
                const int r = it / P4, c = it - r * P4;
                uint32_t acc = 0;
                for (int j = 0; j < K; ++j) acc = wk_apply(acc, s_tab + (j * R + r) * 5, s_rows[j * P4 + c]);
                out[it] = acc;
            }
        } else {
            mark(5);
            const int m = (int)body->m;
            uint32_t *s_gj = reinterpret_cast<uint32_t *>(smem + kLdsGj);
            uint32_t *s_cinv = reinterpret_cast<uint32_t *>(smem + kLdsCinv);
            uint32_t *s_y = reinterpret_cast<uint32_t *>(smem + kLdsData);  // y_t overwrites row M_t in place
            // 3. [S | I], S[t][u] = enc[P_t][M_u] (byte 1 of table word 0 is c * 1 = c)
            const int W = 2 * m;
            if (tid < m * W) {
                const int t = tid / W, u = tid - t * W;
                s_gj[tid] = u < m ? (s_tab[((int)body->M[u] * R + ((int)body->P[t] - K)) * 5] >> 8) & 0xFFu
                                  : (uint32_t)(u - m == t);
            }
            if (tid == 0) s_singular = 0;
            __syncthreads();
            // Gauss-Jordan without pivot search: every leading minor of a square submatrix of the parity part
            // of this systematic MDS generator is non-singular; a zero pivot is still detected and reported.
            for (int c = 0; c < m; ++c) {
                uint32_t f = 0, pv = 0;
                const bool mine = tid < m * W;
                const int t = mine ? tid / W : 0, u = mine ? tid - t * W : 0;
                if (mine) {
                    const uint32_t piv = s_gj[c * W + c];
                    if (piv == 0 && tid == 0) s_singular = 1;
                    const uint32_t inv = piv ? s_exp[255 - s_log[piv]] : 0u;
                    f = s_gj[t * W + c];
                    pv = wk_gmul(s_exp, s_log, s_gj[c * W + u], inv);
                }
                __syncthreads();
                if (mine) s_gj[tid] = (t == c) ? pv : (s_gj[tid] ^ wk_gmul(s_exp, s_log, f, pv));
                __syncthreads();
            }
            mark(6);
            if (tid < m * m) {
                const int uu = tid / m, t = tid - uu * m;
                uint32_t tb[5];
                gf_perm_tables(s_gj[uu * W + m + t], tb);
#pragma unroll
                for (int i = 0; i < 5; ++i) s_cinv[tid * 5 + i] = tb[i];
            }
            // 4. syndromes of the used parity shares over the present data rows
            const uint64_t miss0 = body->miss[0], miss1 = body->miss[1], miss2 = body->miss[2], miss3 = body->miss[3];
            for (int it = tid; it < m * P4; it += kWThreads) {
                const int t = it / P4, c = it - t * P4, pr = (int)body->P[t] - K;
                uint32_t y = s_rows[(int)body->M[t] * P4 + c];
                for (int j = 0; j < K; ++j) {
                    const uint64_t mw = j < 64 ? miss0 : j < 128 ? miss1 : j < 192 ? miss2 : miss3;
                    if ((mw >> (j & 63)) & 1ull) continue;
                    y = wk_apply(y, s_tab + (j * R + pr) * 5, s_rows[j * P4 + c]);
                }
                s_y[(int)body->M[t] * P4 + c] = y;  // row M_t is read by item (t, c) only
            }
            __syncthreads();
            mark(7);
            // 5. out_u = XOR_t Sinv[u][t] * y_t
            for (int it = tid; it < m * P4; it += kWThreads) {
                const int uu = it / P4, c = it - uu * P4;
                uint32_t o = 0;
                for (int t = 0; t < m; ++t) o = wk_apply(o, s_cinv + (uu * m + t) * 5, s_y[(int)body->M[t] * P4 + c]);
                out[it] = o;
            }
            status = (uint32_t)s_singular;
        }
        mark(4);
        // 6. publish: every thread's output stores complete at system scope before the completion word
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store(done, (uint64_t)last | ((uint64_t)status << 32), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
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
    static const uint64_t t = [] {
        const char *e = getenv("KFEC_WORKER_IDLE_US");
        long us = e ? atol(e) : 20000;
        if (us < 100) us = 100;
        if (us > 10000000) us = 10000000;
        return (uint64_t)us * 100;  // wall_clock64 runs at 100 MHz on gfx950
    }();
    return t;
}

inline uint64_t load_acq(const uint8_t *p) { return __atomic_load_n(reinterpret_cast<const uint64_t *>(p), __ATOMIC_ACQUIRE); }

DevWorkers *get_dev(int dev)
{
    if (dev < 0 || dev >= 64) return nullptr;
    DevWorkers &d = g_dev[dev];
    std::lock_guard<std::mutex> lk(d.init_mu);
    if (d.init) return d.failed ? nullptr : &d;
    d.init = true;
    const char *e = getenv("KFEC_WORKER_SLOTS");
    int n = e ? atoi(e) : 2;
    n = n < 1 ? 1 : (n > kMaxSlots ? kMaxSlots : n);
    for (int i = 0; i < n; ++i) {
        Slot &s = d.slots[i];
        void *p = nullptr;
        if (hipHostMalloc(&p, kSlotBytes, hipHostMallocCoherent) != hipSuccess) break;
        std::memset(p, 0, kOffShares);
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) {
            (void)hipHostFree(p);
            break;
        }
        s.h = static_cast<uint8_t *>(p);
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

int launch_worker(Slot &s)
{
    s.gen += 1;
    hipLaunchKernelGGL(kfec_worker_kernel, dim3(1), dim3(kWThreads), kLdsBytes, s.stream, s.h, s.gen, s.seq - 1,
                       idle_ticks(), getenv("KFEC_WORKER_DEBUG") ? 1 : 0);
    if (hipGetLastError() != hipSuccess) {
        s.running = false;
        return KFEC_EHIP;
    }
    s.running = true;
    return 0;
}

// post the doorbell and wait for its completion word; returns the status (0 / 1 singular) or a KFEC_E* code
int post_and_wait(Slot &s, uint32_t op, int K, int N, int B)
{
    uint32_t seq = (s.seq + 1) & kSeqMask;
    if (seq == 0) seq = 1;
    s.seq = seq;
    __atomic_store_n(reinterpret_cast<uint64_t *>(s.h + kOffDoorbell), db_pack(seq, op, (uint32_t)K, (uint32_t)N, (uint32_t)B),
                     __ATOMIC_SEQ_CST);
    if (!s.running || (uint32_t)load_acq(s.h + kOffExited) == s.gen) {
        const int rc = launch_worker(s);
        if (rc) return rc;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t it = 1;; ++it) {
        const uint64_t d = load_acq(s.h + kOffDone);
        if (db_seq(d) == seq) return (int)(d >> 32);
        if ((it & 255) == 0) {
            if ((uint32_t)load_acq(s.h + kOffExited) == s.gen) {
                // the worker left its loop (idle timeout) before it saw this doorbell: launch a new one, which
                // starts behind the old one on the slot's stream and finds the doorbell pending
                if (db_seq(load_acq(s.h + kOffDone)) == seq) continue;
                const int rc = launch_worker(s);
                if (rc) return rc;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                // no answer: report the slot's state and let the caller take the launch path from now on
                if (getenv("KFEC_WORKER_DEBUG"))
                {
                fprintf(stderr, "kfec worker: no answer; doorbell %llx done %llx exited %llx trace %llx %llx gen %u stream %d\n",
                            (unsigned long long)load_acq(s.h + kOffDoorbell), (unsigned long long)load_acq(s.h + kOffDone),
                            (unsigned long long)load_acq(s.h + kOffExited), (unsigned long long)load_acq(s.h + kOffTrace),
                            (unsigned long long)load_acq(s.h + kOffTrace + 8), s.gen, (int)hipStreamQuery(s.stream));
                for (int w = 0; w < kWThreads / 64; ++w)
                    fprintf(stderr, "  wave %d: %llx\n", w, (unsigned long long)load_acq(s.h + kOffTrace + 16 + 8 * w));
            }
                s.running = false;
                return kWorkerDead;
            }
        }
        __builtin_ia32_pause();
    }
}

bool shape_ok(int K, int N, size_t B, int mrows)
{
    const int R = N - K;
    const size_t pitch = (B + 15) & ~size_t(15);
    return B > 0 && B <= 0xFFFF && R >= 1 && R <= kMaxR && mrows <= kMaxR && (size_t)(K + R) * pitch <= kStageMax &&
           (size_t)R * K * 20 <= kTabMax;
}

}  // namespace

bool worker_enabled() { return env_enabled(); }
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
    WorkerBody *body = reinterpret_cast<WorkerBody *>(s.h + kOffBody);
    body->enc = reinterpret_cast<uint64_t>(d_enc);
    body->mat_id = mat_id;
    uint8_t *rows = s.h + kOffShares;
    if (pitch == B) {
        std::memcpy(rows, input, (size_t)K * B);
    } else {
        for (int j = 0; j < K; ++j) std::memcpy(rows + j * pitch, input + j * B, B);
    }
    const int st = post_and_wait(s, kOpEncode, K, N, (int)B);
    if (st == kWorkerDead) return worker_dead(*d);
    if (st < 0) return st;
    g_served.fetch_add(1, std::memory_order_relaxed);
    const uint8_t *out = rows + (size_t)K * pitch;
    if (pitch == B) {
        std::memcpy(parity_out, out, R * B);
    } else {
        for (size_t r = 0; r < R; ++r) std::memcpy(parity_out + r * B, out + r * pitch, B);
    }
    return 0;
}

int worker_decode(int device, const uint8_t *d_enc, uint64_t mat_id, int K, int N, size_t B,
                  const uint8_t *const *row_ptr, int m, const uint8_t *M, const uint8_t *P, uint8_t *out)
{
    if (!env_enabled() || !shape_ok(K, N, B, m)) return 1;
    DevWorkers *d = get_dev(device);
    if (!d) return env_mode() == 2 ? KFEC_EHIP : 1;
    std::unique_lock<std::mutex> lk;
    Slot &s = acquire(*d, lk);
    const size_t pitch = (B + 15) & ~size_t(15);
    WorkerBody *body = reinterpret_cast<WorkerBody *>(s.h + kOffBody);
    body->enc = reinterpret_cast<uint64_t>(d_enc);
    body->mat_id = mat_id;
    body->miss[0] = body->miss[1] = body->miss[2] = body->miss[3] = 0;
    body->m = (uint32_t)m;
    for (int t = 0; t < m; ++t) {
        body->M[t] = M[t];
        body->P[t] = P[t];
        body->miss[M[t] >> 6] |= 1ull << (M[t] & 63);
    }
    uint8_t *rows = s.h + kOffShares;
    for (int j = 0; j < K; ++j) std::memcpy(rows + j * pitch, row_ptr[j], B);
    const int st = post_and_wait(s, kOpDecode, K, N, (int)B);
    if (st == kWorkerDead) return worker_dead(*d);
    if (st < 0) return st;
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

// Stop the resident workers of a device (no coder left on it): post STOP to every running slot and wait for
// the kernel to finish.  Bounded: a worker that does not answer within 2 s is left to its idle timeout.
void worker_stop(int device)
{
    if (device < 0 || device >= 64) return;
    DevWorkers &d = g_dev[device];
    {
        std::lock_guard<std::mutex> lk(d.init_mu);
        if (!d.init || d.failed) return;
    }
    for (int i = 0; i < d.nslots; ++i) {
        Slot &s = d.slots[i];
        std::lock_guard<std::mutex> lk(s.mu);
        if (!s.running) continue;
        if ((uint32_t)load_acq(s.h + kOffExited) != s.gen) {
            uint32_t seq = (s.seq + 1) & kSeqMask;
            if (seq == 0) seq = 1;
            s.seq = seq;
            __atomic_store_n(reinterpret_cast<uint64_t *>(s.h + kOffDoorbell), db_pack(seq, kOpStop, 1, 1, 0),
                             __ATOMIC_SEQ_CST);
            const auto t0 = std::chrono::steady_clock::now();
            while ((uint32_t)load_acq(s.h + kOffExited) != s.gen &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
                __builtin_ia32_pause();
        }
        if ((uint32_t)load_acq(s.h + kOffExited) == s.gen) (void)hipStreamSynchronize(s.stream);
        s.running = false;
    }
}

}  // namespace kfec
