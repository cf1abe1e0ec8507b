// kfec_pipeline.cpp -- include/kfec_pipeline.h: kcptube's fec_maker / fec_unpack + fec_find_missings
// bookkeeping on the host, feeding batched device coding through the public C ABI (kfec.h, kfec_frame.h).
// Per-packet work here is bookkeeping and copies into staging; every byte of parity, recovered data and
// redundant packet is computed by the GPU kernels at flush time.
//
// Two flush paths, chosen per flush:
//   * the resident worker (kfec_worker.hip batch requests) for small flushes -- a doorbell, no launch and no
//     stream synchronisation -- when the staging arena lives in device memory the host writes through the PCIe
//     BAR as each datagram / shard arrives (BAR mode: large-BAR devices), so no bulk bytes cross PCIe at the
//     flush.  The reference codes a group inside fec_maker / fec_find_missings (client.cpp:797-840, 895-938):
//     at low load a flush of a few groups is the product's latency.
//   * kernel launches on the caller's stream (kfec_encode_framed_batch / kfec_decode_framed_batch + pack / seal)
//     for large flushes and for sealed queues.
// A flush that fails leaves the queue as it was (tables, staged bytes, iv counter): it can be retried.
#include "../../include/kfec_pipeline.h"

#include <hip/hip_runtime.h>

#include "kfec_internal.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

namespace {

constexpr uint32_t kFecWaits = KFEC_FEC_WAITS;

size_t round4(size_t x) { return (x + 3) & ~size_t(3); }
size_t round8(size_t x) { return (x + 7) & ~size_t(7); }
size_t round16(size_t x) { return (x + 15) & ~size_t(15); }

// KFEC_QUEUE_BAR: 1 (default where the device has a large BAR) = BAR-mode staging allowed; 0 = pinned staging
// uploaded by DMA only.  BAR mode is in effect while the queue's flushes stay small (KFEC_QUEUE_BAR_MAX groups,
// default 2048): it takes the bulk upload out of the flush (latency), but a write-combined copy through the BAR
// costs the host more per datagram than a memcpy into pinned memory that DMA uploads while the host keeps
// queueing (throughput).  KFEC_QUEUE_BAR_ALIGN: staging granule in BAR mode (default 64: whole write-combining
// lines).  KFEC_QUEUE_WORKER_MAX: the largest flush (groups) sent to the resident worker (default 64; 0 = never).
bool env_flag(const char *name, bool def)
{
    const char *e = getenv(name);
    return e ? std::string(e) != "0" : def;
}
size_t env_size(const char *name, size_t def)
{
    const char *e = getenv(name);
    return e ? (size_t)std::max(0L, atol(e)) : def;
}
size_t bar_flush_max()
{
    static const size_t v = env_size("KFEC_QUEUE_BAR_MAX", 2048);
    return v;
}
size_t bar_align()
{
    static const size_t v = [] {
        size_t a = env_size("KFEC_QUEUE_BAR_ALIGN", 64);
        return (a >= 4 && (a & (a - 1)) == 0 && a <= 4096) ? a : (size_t)64;
    }();
    return v;
}

std::atomic<long> g_worker_max{-1};  // -1: the environment not read yet
size_t worker_flush_max()
{
    long v = g_worker_max.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("KFEC_QUEUE_WORKER_MAX");
        const long x = e ? std::max(0L, atol(e)) : 64L;
        g_worker_max.compare_exchange_strong(v, x);
        v = g_worker_max.load();
    }
    return (size_t)v;
}

// Test knob: fail the n-th HIP step (copy, launch, worker request, synchronisation) of the next flush, once
// (KFEC_TEST_FAIL_FLUSH=n in the environment, or kfec_test_fail_flush(n)); the step returns KFEC_EHIP without
// running, as a failed HIP call would.
std::atomic<int> g_fail_at{-1};  // -1: the environment not read yet; 0: off
int fail_at()
{
    int v = g_fail_at.load();
    if (v < 0) {
        const char *e = getenv("KFEC_TEST_FAIL_FLUSH");
        const int x = e ? std::max(0, atoi(e)) : 0;
        g_fail_at.compare_exchange_strong(v, x);
        v = g_fail_at.load();
    }
    return v;
}
struct Steps {
    int k = 0;
    bool fail()
    {
        ++k;
        int f = fail_at();
        return f > 0 && k == f && g_fail_at.compare_exchange_strong(f, 0);
    }
};

// KFEC_QUEUE_TRACE=1: per-phase host times of the small flushes (worker paths), summed per queue and printed to
// stderr when the queue is destroyed (diagnostics)
struct Trace {
    static bool on()
    {
        static const bool v = env_flag("KFEC_QUEUE_TRACE", false);
        return v;
    }
    double us[6] = {};
    uint64_t n = 0;
    std::chrono::steady_clock::time_point t;
    int k = 0;
    void start()
    {
        if (!on()) return;
        t = std::chrono::steady_clock::now();
        k = 0;
    }
    void mark()
    {
        if (!on() || k >= 6) return;
        const auto now = std::chrono::steady_clock::now();
        us[k++] += std::chrono::duration<double, std::micro>(now - t).count();
        t = now;
    }
    void done()  // (the queue's first flush -- first launches, cold worker -- is left out)
    {
        if (!on()) return;
        if (!warm) {
            warm = true;
            for (double &u : us) u = 0;
            return;
        }
        ++n;
    }
    bool warm = false;
    void print(const char *what) const
    {
        if (!on() || !n) return;
        fprintf(stderr, "kfec %s: %llu small flushes after the first, us each: prep %.2f worker %.2f launch %.2f sync %.2f "
                        "emit %.2f\n",
                what, (unsigned long long)n, us[0] / n, us[1] / n, us[2] / n, us[3] / n, us[4] / n);
    }
};

// pinned host and device buffers, grown on demand
struct Pinned {
    void *p = nullptr;
    size_t n = 0;
    unsigned flags = hipHostMallocDefault;
    int ensure(size_t bytes)
    {
        if (bytes <= n) return KFEC_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc(&p, std::max<size_t>(bytes, 256), flags) != hipSuccess) return KFEC_ENOMEM;
        n = std::max<size_t>(bytes, 256);
        return KFEC_OK;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    ~Pinned() { if (p) (void)hipHostFree(p); }
};

// Device buffer; `uncached` (BAR mode): written by the host through the BAR and read by kernels and the resident
// worker, so no L2 line may outlive a host write.  64 bytes of readable headroom before and after the usable
// range (the worker's 16-byte granule loads reach a few bytes past a payload on either side).
constexpr size_t kDevPad = 64;
struct Device {
    void *alloc = nullptr;
    void *p = nullptr;
    size_t n = 0;
    bool uncached = false;
    int ensure(size_t bytes)
    {
        if (bytes <= n) return KFEC_OK;
        release();
        const size_t want = std::max<size_t>(bytes, 256);
        const hipError_t e = uncached ? hipExtMallocWithFlags(&alloc, want + 2 * kDevPad, hipDeviceMallocUncached)
                                      : hipMalloc(&alloc, want + 2 * kDevPad);
        if (e != hipSuccess) {
            alloc = nullptr;
            return KFEC_ENOMEM;
        }
        p = static_cast<uint8_t *>(alloc) + kDevPad;
        n = want;
        return KFEC_OK;
    }
    void release()
    {
        if (alloc) (void)hipFree(alloc);
        alloc = p = nullptr;
        n = 0;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    ~Device() { release(); }
};

// Append-only staging uploaded while the host is still filling it (pinned mode): every kUploadChunk bytes of
// finished groups go H2D on the queue's own copy stream, so the PCIe transfer overlaps the per-packet host work
// and a flush only copies the tail.  Bytes already queued for DMA are never written again before the flush has
// synchronised (the arena is append-only between flushes).
struct Upload {
    static constexpr size_t kUploadChunk = size_t(8) << 20;
    hipStream_t cs = nullptr;
    hipEvent_t ev = nullptr;
    size_t issued = 0;
    bool busy = false;  // copies were issued on cs since the last drain (a drain of an idle stream costs ~5 us)
    int init(int device)
    {
        if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
            return KFEC_EHIP;
        return KFEC_OK;
    }
    // called after the arena grew to `used` bytes: start the copy of the finished bytes once a chunk is ready
    void grow(const uint8_t *h, uint8_t *d, size_t used)
    {
        if (used - issued < kUploadChunk) return;
        busy = true;
        if (hipMemcpyAsync(d + issued, h + issued, used - issued, hipMemcpyHostToDevice, cs) == hipSuccess)
            issued = used;  // on failure the bytes are simply copied again by finish()
    }
    // copy the tail and make `s` wait for every upload
    int finish(const uint8_t *h, uint8_t *d, size_t used, hipStream_t s)
    {
        if (issued == 0)  // nothing went up early (a small flush): one copy on s, no cross-stream event
            return (used == 0 || hipMemcpyAsync(d, h, used, hipMemcpyHostToDevice, s) == hipSuccess) ? KFEC_OK : KFEC_EHIP;
        busy = true;
        if (used > issued && hipMemcpyAsync(d + issued, h + issued, used - issued, hipMemcpyHostToDevice, cs) != hipSuccess)
            return KFEC_EHIP;
        issued = 0;  // (a retried flush uploads everything again on s)
        if (hipEventRecord(ev, cs) != hipSuccess || hipStreamWaitEvent(s, ev, 0) != hipSuccess) return KFEC_EHIP;
        return KFEC_OK;
    }
    int drain()
    {
        if (!cs || !busy) return KFEC_OK;
        if (hipStreamSynchronize(cs) != hipSuccess) return KFEC_EHIP;
        busy = false;
        return KFEC_OK;
    }
    ~Upload()
    {
        (void)drain();
        if (ev) (void)hipEventDestroy(ev);
        if (cs) (void)hipStreamDestroy(cs);
    }
};

// The staging arena of a queue: the bytes in pinned host memory (the queue's own copy: compaction, deferred
// data packets) and their device image.  BAR mode: the image is uncached device memory written through the BAR
// at staging time (no upload; the worker and the kernels read it in place).  Pinned mode: uploaded (Upload).
struct Arena {
    Pinned h;
    Device d;
    size_t cap = 0;
    bool bar_ok = false;  // the device image is BAR-writable, uncached memory
    bool bar = false;     // BAR mode in effect (decided at each compaction, see set_mode)
    size_t align = 4;     // staging granule (offsets and lengths rounded up to it)
    size_t reserve = 0;   // device image bytes past cap: the sealed small flush's redundant-packet rows
    Upload up;            // (pinned mode)
    int init(int device, size_t bytes, bool use_bar, size_t max_groups, size_t extra = 0)
    {
        // until the first flush says otherwise (set_mode): BAR mode when the queue cannot hold a large flush
        bar_ok = use_bar;
        bar = use_bar && max_groups <= bar_flush_max();
        d.uncached = use_bar;
        align = use_bar ? bar_align() : 4;
        reserve = use_bar ? extra : 0;
        if (h.ensure(bytes) || d.ensure(bytes + reserve)) return KFEC_ENOMEM;
        cap = bytes;
        return up.init(device);
    }
    size_t step(size_t n) const { return (n + align - 1) & ~(align - 1); }
    // BAR mode while the flushes stay small: called between flushes (nothing staged for DMA in flight)
    void set_mode(size_t last_flush_groups) { bar = bar_ok && last_flush_groups <= bar_flush_max(); }
    uint8_t *host(size_t off = 0) const { return h.as<uint8_t>() + off; }
    // n bytes at off: the host copy and, in BAR mode, the device image
    void put(size_t off, const void *src, size_t n)
    {
        if (!n) return;
        std::memcpy(host(off), src, n);
        if (bar) kfec::copy_to_bar(d.as<uint8_t>() + off, src, n);
    }
    // bytes the host already wrote into its copy, to the device image (BAR mode)
    void mirror(size_t off, size_t n)
    {
        if (bar && n) kfec::copy_to_bar(d.as<uint8_t>() + off, host(off), n);
    }
    void staged(size_t used)
    {
        if (!bar) up.grow(host(), d.as<uint8_t>(), used);
    }
    // the device image of [0, used) complete and ordered before work on s
    int finish(size_t used, hipStream_t s)
    {
        if (bar) {
            kfec::bar_fence();
            return KFEC_OK;
        }
        return up.finish(host(), d.as<uint8_t>(), used, s);
    }
    // before the host copy is compacted: no upload may still be reading it
    int quiesce() { return up.drain(); }
    // the mode for the flushes after a compaction; true when the device image must then be rewritten whole (BAR
    // mode now, not before: the image holds only what the uploads carried).  Otherwise a compaction mirrors just
    // the ranges it moved (moved()): the unmoved live bytes are in the image since their staging.
    bool switch_mode(size_t last_flush_groups)
    {
        const bool was = bar;
        set_mode(last_flush_groups);
        return bar && !was;
    }
    void moved(size_t at, size_t n, bool whole)
    {
        if (!whole) mirror(at, n);
    }
    // after the host copy was compacted to [0, used): restart the upload (pinned) / rewrite the image if whole
    void restage(size_t used, bool whole)
    {
        up.issued = 0;
        if (whole) mirror(0, used);
    }
    // room for `need` more bytes after `used` when nothing is queued: doubles both copies, keeps [0, used)
    int grow(size_t used, size_t need)
    {
        size_t ncap = std::max<size_t>(cap, 4096);
        while (used + need > ncap) ncap *= 2;
        if (up.drain()) return KFEC_EHIP;
        Pinned nh;
        Device nd;
        nd.uncached = bar_ok;
        if (nh.ensure(ncap) || nd.ensure(ncap + reserve)) return KFEC_ENOMEM;
        if (used) std::memcpy(nh.p, h.p, used);
        std::swap(h.p, nh.p);
        std::swap(h.n, nh.n);
        std::swap(d.alloc, nd.alloc);
        std::swap(d.p, nd.p);
        std::swap(d.n, nd.n);
        up.issued = 0;
        cap = ncap;
        mirror(0, used);
        return KFEC_OK;
    }
    ~Arena() { (void)up.drain(); }  // (the copy stream is idle before the buffers go)
};

// The queue's own stream for a flush called with stream = NULL: HIP's null stream would also wait for the
// device's other streams -- a resident worker's among them, for up to its lease -- at every flush.
struct OwnStream {
    hipStream_t s = nullptr;
    int init() { return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? KFEC_OK : KFEC_EHIP; }
    void *pick(void *stream) const { return stream ? stream : static_cast<void *>(s); }
    ~OwnStream()
    {
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    }
};

// A host table written to device memory: in BAR mode straight through the BAR (no copy call), otherwise packed
// into `pack` and sent by one hipMemcpyAsync.  The sources are never moved (a failed flush can be retried).
struct TableUpload {
    bool bar;
    uint8_t *dst;   // device
    uint8_t *pack;  // pinned staging (pinned mode)
    size_t used = 0;
    void add(size_t off, const void *src, size_t n)
    {
        if (!n) return;
        if (bar) kfec::copy_to_bar(dst + off, src, n);
        else if (pack + off != src) std::memcpy(pack + off, src, n);
        used = std::max(used, off + n);
    }
    int send(hipStream_t s)
    {
        if (bar) {
            kfec::bar_fence();
            return KFEC_OK;
        }
        return (used == 0 || hipMemcpyAsync(dst, pack, used, hipMemcpyHostToDevice, s) == hipSuccess) ? KFEC_OK : KFEC_EHIP;
    }
};

inline void put_le32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
inline void put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
inline uint32_t get_be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// the AEAD iv_raw draw of sealed packet number i (kfec_txq_seal)
inline uint16_t iv_draw(uint64_t seed, uint64_t i)
{
    uint64_t x = seed + i + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return (uint16_t)((x ^ (x >> 31)) >> 48);
}

bool seal_mode_ok(int mode, const kfec_aead *aead)
{
    if (mode == KFEC_SEAL_CHECKSUM || mode == KFEC_SEAL_PLAIN_XOR) return aead == nullptr;
    if (mode == KFEC_AEAD_AES_GCM || mode == KFEC_AEAD_AES_OCB || mode == KFEC_AEAD_CHACHA20 || mode == KFEC_AEAD_XCHACHA20)
        return aead != nullptr && kfec_aead_mode(aead) == mode;
    return false;
}

size_t seal_overhead(int mode) { return mode == KFEC_SEAL_CHECKSUM || mode == KFEC_SEAL_PLAIN_XOR ? KFEC_SEAL_TRAILER : KFEC_AEAD_OVERHEAD; }

// encrypt_data / decrypt_data of P packets [off, +len) of a device arena into [P][pitch] rows
int seal_rows(int mode, const kfec_aead *aead, size_t P, const void *src, size_t src_bytes, const uint64_t *off,
              const uint32_t *len, const uint16_t *iv, void *dst, size_t pitch, uint32_t *out_len, void *stream)
{
    if (P == 0) return KFEC_OK;
    if (aead) return kfec_aead_seal_batch(aead, P, src, src_bytes, off, len, iv, dst, pitch, out_len, stream);
    return kfec_seal_batch(mode, P, src, src_bytes, off, len, dst, pitch, out_len, stream);
}

}  // namespace

// test-only hooks (not in the headers): arm the flush fault knob; override KFEC_QUEUE_WORKER_MAX (-1: env again)
extern "C" void kfec_test_fail_flush(int n) { (void)fail_at(); g_fail_at.store(n > 0 ? n : 0); }
extern "C" void kfec_test_queue_worker_max(long n) { g_worker_max.store(n < 0 ? -1 : n); }

// ---- send ------------------------------------------------------------------------------------------------
struct kfec_txq {
    const kfec_ctx *ctx = nullptr;
    int device = 0;
    size_t K = 0, N = 0, R = 0, G = 0, mtu = 0, slot = 0;  // slot: datagram stride of a kfec_tx group cache
    size_t n = 0;                                          // complete groups queued
    size_t last_n = 0;                                     // groups of the last flush (the arena's mode)
    size_t used = 0;  // staged bytes (packed back to back at Arena::step granules)
    std::vector<kfec_tx *> txs;  // the senders whose partial groups live in the arena
    // per queued group g: the K datagrams' arena offsets and lengths, sn, conv (as kfec_tx_send wrote them; a
    // flush never moves them)
    std::vector<uint64_t> off;
    std::vector<uint16_t> len;
    std::vector<uint32_t> sn, conv;
    std::vector<uint64_t> tags;
    // launch path: h_pack (pinned mode: the tables packed for one copy up), h_res (the redundant packets [n][R],
    // then their lengths, one copy back); worker path: wdesc (the batch's shard descriptors) and h_wout
    // (coherent pinned: the worker writes parity rows there, each behind a 16-byte gap for its 13-byte header)
    Pinned h_pack, h_res, h_wout;
    std::vector<uint64_t> wdesc;
    Device d_meta, d_par, d_align, d_res;
    // packet protection and deferred data packets (kfec_txq_seal)
    int seal_mode = KFEC_TXQ_SEAL_OFF;
    const kfec_aead *aead = nullptr;
    uint64_t iv_seed = 0, iv_ctr = 0;
    bool defer = false;
    struct DataPkt {
        uint64_t off;   // the whole data packet (9-byte header + datagram) in the staging arena
        uint32_t len;
        uint32_t sn;
        uint8_t sub;
        int32_t group;  // the queue slot of the group this packet completed, or -1
        uint64_t tag;
    };
    std::vector<DataPkt> dpk;  // staged since the last flush, in send order
    Pinned h_sdesc, h_sealed;  // seal descriptors (+ iv draws) up; sealed rows + lengths down
    Pinned h_done;             // the small sealed flush's completion count (coherent; launch_seal's `done`)
    uint32_t done_sum = 0;     // workgroups launched into h_done so far (never reset: a kernel left running by a
                               // failed flush still counts into it, ahead of the retry's in stream order)
    Device d_sdesc, d_sealed;
    OwnStream own;
    Trace trace;
    Arena arena;  // declared last: destroyed (and its copy stream drained) first
    ~kfec_txq() { trace.print("txq"); }
};

// test-only hook (not in the headers): the coherent completion count minus the baseline the next counted wait
// adds to (0 whenever no counted kernel is in flight, e.g. after any flush returned, failed ones included)
extern "C" int32_t kfec_test_txq_count_drift(const kfec_txq *q)
{
    return q && q->h_done.p ? (int32_t)(*q->h_done.as<volatile uint32_t>() - q->done_sum) : 0;
}

struct kfec_tx {
    kfec_txq *q = nullptr;
    uint32_t conv = 0;
    uint64_t tag = 0;
    uint32_t sn = 0;      // fec_snd_sn
    uint8_t sub_sn = 0;   // fec_snd_sub_sn
    // fec_snd_cache: the group's datagrams so far, stored once, straight into the queue's staging arena
    std::vector<uint64_t> cache_off;
    std::vector<uint16_t> cache_len;
    size_t cached = 0;
};

namespace {

// The queue's coder must still have the K / N the queue was sized for: a reset_martix on a live coder
// (client.cpp:1755, relay.cpp:947) with queues still attached would make the flush kernels overrun them.
bool kn_changed(const kfec_ctx *ctx, size_t K, size_t N) { return kfec_get_K(ctx) != K || kfec_get_N(ctx) != N; }

// Move the live bytes (datagrams of every sender's partial group) to the front of the arena, in arena order
// (every destination lies at or below its source, so memmove in that order never overwrites unread bytes).
// Called with no group queued: after a flush, and before growing a full arena, so the bytes of destroyed
// senders are reclaimed instead of doubling memory.
int tx_compact(kfec_txq *q)
{
    struct Part {
        uint64_t off;
        size_t len;
        uint64_t *rec;  // where the offset is recorded
        bool operator<(const Part &o) const { return off < o.off; }
    };
    if (q->arena.quiesce()) return KFEC_EHIP;
    std::vector<Part> part;
    for (kfec_tx *tx : q->txs)
        for (size_t i = 0; i < tx->cached; ++i) part.push_back({tx->cache_off[i], tx->cache_len[i], &tx->cache_off[i]});
    std::sort(part.begin(), part.end());
    const bool whole = q->arena.switch_mode(q->last_n);
    size_t at = 0;
    for (const Part &p : part) {
        if (p.len && at != p.off) {
            std::memmove(q->arena.host(at), q->arena.host(p.off), p.len);
            q->arena.moved(at, p.len, whole);
        }
        *p.rec = at;
        at += q->arena.step(p.len);
    }
    q->used = at;
    q->arena.restage(at, whole);
    return KFEC_OK;
}

}  // namespace

extern "C" {

size_t kfec_txq_capacity(const kfec_txq *q) { return q ? q->arena.cap : 0; }

int kfec_txq_create(const kfec_ctx *ctx, size_t max_groups, size_t max_datagram, kfec_txq **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!ctx || !max_groups || max_datagram + KFEC_FEC_CONTAINER_HEADER > 0xFFFF) return KFEC_EINVAL;
    kfec_txq *q = new (std::nothrow) kfec_txq;
    if (!q) return KFEC_ENOMEM;
    q->ctx = ctx;
    q->device = kfec_device(ctx);
    q->K = kfec_get_K(ctx);
    q->N = kfec_get_N(ctx);
    q->R = q->N - q->K;
    q->G = max_groups;
    q->mtu = max_datagram;
    const bool bar = env_flag("KFEC_QUEUE_BAR", true) && kfec::bar_writable(q->device);
    q->slot = (std::max<size_t>(max_datagram, 4) + (bar ? bar_align() : 4) - 1) & ~((bar ? bar_align() : 4) - 1);
    const size_t G = q->G, K = q->K, GK = G * K, R1 = std::max<size_t>(q->R, 1);
    const size_t pitch = round4(max_datagram + KFEC_FEC_CONTAINER_HEADER);
    const size_t pkt_pitch = round4(KFEC_PKT_REDUNDANT_HEADER + max_datagram + KFEC_FEC_CONTAINER_HEADER);
    // every buffer up front: a flush then costs copies and kernels only (pinning memory takes milliseconds)
    const size_t meta = round8(GK * 10) + G * 8, res = G * R1 * (pkt_pitch + 2);
    q->d_meta.uncached = bar;
    q->h_wout.flags = hipHostMallocCoherent;
    // the sealed small flush's seal kernel writes its rows straight into h_sealed: fine-grained (coherent) memory
    // takes those stores through to the host as they are issued, instead of an L2 write-back at the kernel's end
    if (bar && env_flag("KFEC_QUEUE_COHERENT_OUT", true)) q->h_sealed.flags = hipHostMallocCoherent;
    q->h_done.flags = hipHostMallocCoherent;
    try {
        q->off.resize(GK);
        q->len.resize(GK);
        q->sn.resize(G);
        q->conv.resize(G);
        q->tags.resize(G);
    } catch (...) {
        delete q;
        return KFEC_ENOMEM;
    }
    if (hipSetDevice(q->device) != hipSuccess) {
        delete q;
        return KFEC_EHIP;
    }
    const size_t red_rows = std::min(G, worker_flush_max()) * R1 * (16 + round16(max_datagram + KFEC_FEC_CONTAINER_HEADER));
    // (BAR mode stages at whole write-combining lines: one group's worth more, so that partial groups of small
    //  datagrams still fit beside a full queue as with 4-byte staging)
    if (q->own.init() || q->arena.init(q->device, (GK + (bar ? K : 0)) * q->slot, bar, G, red_rows + 64) || q->h_pack.ensure(meta) || q->h_res.ensure(res) ||
        q->d_meta.ensure(meta) || q->d_res.ensure(res) || q->d_par.ensure(G * R1 * pitch) || q->d_align.ensure(G * 2)) {
        delete q;
        return KFEC_ENOMEM;
    }
    *out = q;
    return KFEC_OK;
}

void kfec_txq_destroy(kfec_txq *q) { delete q; }

size_t kfec_txq_pending(const kfec_txq *q) { return q ? q->n : 0; }

int kfec_tx_create(kfec_txq *q, uint32_t conv, uint64_t tag, kfec_tx **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!q) return KFEC_EINVAL;
    kfec_tx *tx = new (std::nothrow) kfec_tx;
    if (!tx) return KFEC_ENOMEM;
    tx->q = q;
    tx->conv = conv;
    tx->tag = tag;
    try {
        tx->cache_off.resize(q->K);
        tx->cache_len.resize(q->K);
        q->txs.push_back(tx);
    } catch (...) {
        delete tx;
        return KFEC_ENOMEM;
    }
    *out = tx;
    return KFEC_OK;
}

void kfec_tx_destroy(kfec_tx *tx)
{
    if (!tx) return;
    auto &v = tx->q->txs;
    v.erase(std::remove(v.begin(), v.end(), tx), v.end());
    delete tx;
}

int kfec_tx_send(kfec_tx *tx, const uint8_t *datagram, size_t len, uint32_t timestamp, uint8_t *pkt, size_t *pkt_len)
{
    if (!tx || (len && !datagram)) return KFEC_EINVAL;
    kfec_txq *q = tx->q;
    const bool defer = q->defer;
    if (len > q->mtu || kn_changed(q->ctx, q->K, q->N) || (!defer && (!pkt || !pkt_len))) return KFEC_EINVAL;
    const bool completes = tx->conv != 0 && tx->cached + 1 == q->K;
    if (completes && q->n == q->G) return KFEC_ENOMEM;
    // staged bytes: the datagram (group cache) and, deferred, the data packet around it
    const size_t need = q->arena.step(len + (defer ? KFEC_PKT_DATA_HEADER : 0));
    if ((tx->conv != 0 || defer) && q->used + need > q->arena.cap) {
        if (q->n || !q->dpk.empty()) return KFEC_ENOMEM;  // a flush frees the queued bytes
        int rc = tx_compact(q);                            // first reclaim what no partial group holds any more
        if (!rc && q->used + need > q->arena.cap) rc = q->arena.grow(q->used, need);
        if (rc) return rc;
    }
    if (defer) {
        try {
            // geometric growth: reserve(size() + 1) reallocated -- and copied every staged packet record -- on
            // every send, quadratic in the packets between flushes (15 us per packet at 4096 groups per flush)
            if (q->dpk.size() == q->dpk.capacity()) q->dpk.reserve(std::max<size_t>(64, 2 * q->dpk.capacity()));
        } catch (...) {
            return KFEC_ENOMEM;
        }
    }
    // create_fec_data_packet (connections.cpp:395-411), sub_sn = fec_snd_sub_sn++ (client.cpp:805-806)
    const uint8_t sub = tx->sub_sn++;
    uint8_t *dst = defer ? q->arena.host(q->used) : pkt;  // deferred: staged for the flush
    put_le32(dst, timestamp);
    put_be32(dst + 4, tx->sn);
    dst[8] = sub;
    if (len) std::memcpy(dst + KFEC_PKT_DATA_HEADER, datagram, len);
    if (pkt_len) *pkt_len = defer ? 0 : KFEC_PKT_DATA_HEADER + len;
    const int32_t slot = completes ? (int32_t)q->n : -1;
    if (defer) {
        q->arena.mirror(q->used, KFEC_PKT_DATA_HEADER + len);
        q->dpk.push_back({q->used, (uint32_t)(KFEC_PKT_DATA_HEADER + len), tx->sn, sub, slot, tx->tag});
        if (tx->conv == 0) {
            q->used += need;
            q->arena.staged(q->used);
        }
    }
    if (tx->conv == 0) {  // client.cpp:811-815
        tx->sub_sn = 0;
        return KFEC_OK;
    }
    if (!defer) q->arena.put(q->used, datagram, len);
    tx->cache_off[tx->cached] = q->used + (defer ? KFEC_PKT_DATA_HEADER : 0);
    tx->cache_len[tx->cached++] = (uint16_t)len;
    q->used += need;
    q->arena.staged(q->used);
    if (!completes) return KFEC_OK;
    // the group is complete: it takes queue slot n (compact_into_container + encode run at the flush)
    const size_t g = q->n;
    for (size_t i = 0; i < q->K; ++i) {
        q->off[g * q->K + i] = tx->cache_off[i];
        q->len[g * q->K + i] = tx->cache_len[i];
    }
    q->sn[g] = tx->sn;
    q->conv[g] = tx->conv;
    q->tags[g] = tx->tag;
    q->n = g + 1;
    tx->cached = 0;  // fec_snd_cache.clear(), client.cpp:830-832
    tx->sub_sn = 0;
    tx->sn++;
    return KFEC_OK;
}

}  // extern "C"

namespace {

// Emission reads rows the GPU has just written into pinned host memory -- in DRAM, in no CPU cache -- and a
// callback typically copies each one out; requesting the rows a few packets ahead (KFEC_QUEUE_PREFETCH) keeps
// those copies from paying a DRAM round trip every few lines: the send flushes and the opener (whose packets are
// always read, by the socket send or kfec_rx_push).  Not the receive flush: most of a group's recovered rows are
// often unused, and prefetching them cost a consumer that does not read them (tools/latency_bench) 17 -> 18 /
// 95 -> 114 us per 16 / 256-group flush (profiles/r05_emit_prefetch_ab.txt).
// The small sealed flush and the opener (every mode, at most kSealCountRows packets) wait for the seal / open
// kernel's own completion count instead of the stream (KFEC_QUEUE_SEAL_COUNT, default on): the workgroups
// add themselves to a coherent pinned word once their rows are visible to the host, so the flush skips the
// runtime's completion signal and stream wait (one 20:3 group: 15-16 -> 10-11 us; kfec_seal.hip count_done).
bool seal_count_on()
{
    static const bool v = env_flag("KFEC_QUEUE_SEAL_COUNT", true);
    return v;
}

// spin until the running count *done reaches `want` (modulo 2^32).  The stream is polled only once the wait has
// lasted 2 ms (then every ms), so that a launch that failed or a kernel that faulted ends the wait with an error
// instead of spinning forever: polling it every few thousand spins put ~15 us into a 16-group flush's wait.
int wait_count(const volatile uint32_t *done, uint32_t want, hipStream_t s)
{
    auto reached = [&] { return (int32_t)(*done - want) >= 0; };
    auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(2);
    for (uint32_t spin = 1;; ++spin) {
        if (reached()) return 0;
        if ((spin & 1023u) == 0 && std::chrono::steady_clock::now() >= next) {
            const hipError_t e = hipStreamQuery(s);
            if (e != hipErrorNotReady) return e == hipSuccess && reached() ? 0 : -1;
            next = std::chrono::steady_clock::now() + std::chrono::milliseconds(1);
        }
        __builtin_ia32_pause();
    }
}

// A counted flush that fails after its launch was attempted: the launch's error code (hipGetLastError) says
// nothing certain about whether the kernel was enqueued, so the running count may or may not grow by its
// workgroups.  Drain the stream, then take the coherent count itself as the new baseline: the next counted wait
// can then neither return before its own kernel's rows are written nor spin on workgroups that never ran.
void count_resync(const Pinned &h_done, uint32_t &done_sum, hipStream_t s)
{
    (void)hipStreamSynchronize(s);
    (void)hipGetLastError();
    done_sum = *h_done.as<volatile uint32_t>();
}

bool prefetch_on()
{
    static const bool v = env_flag("KFEC_QUEUE_PREFETCH", true);
    return v;
}
constexpr size_t kPrefetchAhead = 4;  // rows
inline void prefetch_bytes(const void *p, size_t n)
{
    const char *c = static_cast<const char *>(p);
    for (size_t o = 0; o < n; o += 64) __builtin_prefetch(c + o, 0, 3);
}

// The flush's packets in emission order: the redundant ones in queue order or, with deferred data packets,
// every packet in send order with a group's redundant packets right after the data packet completing it.
template <typename Data, typename Red>
void emit(const kfec_txq *q, size_t n, Data &&data, Red &&red)
{
    if (q->defer) {
        for (size_t i = 0; i < q->dpk.size(); ++i) {
            data(i);
            if (q->dpk[i].group >= 0) red((size_t)q->dpk[i].group);
        }
    } else {
        for (size_t g = 0; g < n; ++g) red(g);
    }
}

// Small, unsealed flush through the resident worker: the groups' framed shards are read from the arena's
// device image (BAR mode), the parity rows land in h_wout behind a 16-byte gap each, and the 13-byte redundant
// headers (create_fec_redundant_packet, connections.cpp:413-430) are written into the gap here.  1: not taken.
int txq_flush_worker(kfec_txq *q, uint32_t timestamp, kfec_packet_cb cb, void *user, Steps &st)
{
    const size_t n = q->n, K = q->K, R = q->R;
    if (!q->arena.bar || R == 0 || n == 0 || n > worker_flush_max()) return 1;
    const size_t B = q->mtu + KFEC_FEC_CONTAINER_HEADER, opitch = 16 + round16(B);
    kfec::BatchSpec b;
    b.op = kfec::kBatchEncode;
    b.enc = kfec::ctx_enc(q->ctx);
    b.mat_id = kfec::ctx_mat_id(q->ctx);
    b.arena = q->arena.d.p;
    b.opitch = opitch;
    b.ooff = 16;
    b.n = (int)n;
    b.K = (int)K;
    b.N = (int)q->N;
    b.B = (int)B;
    if (!kfec::worker_batch_ok(b)) return 1;
    if (q->h_wout.ensure(n * R * opitch)) return KFEC_ENOMEM;
    try {
        q->wdesc.resize(n * K);
    } catch (...) {
        return KFEC_ENOMEM;
    }
    for (size_t i = 0; i < n * K; ++i) q->wdesc[i] = kfec::batch_desc(q->off[i], q->len[i], false);
    b.desc = q->wdesc.data();
    b.out = q->h_wout.as<uint8_t>();
    kfec::bar_fence();  // the staged datagrams before the doorbell
    if (st.fail()) return KFEC_EHIP;
    const int rc = kfec::worker_batch(q->device, b);
    if (rc) return rc;  // (1: the worker is off or gone -> the launch path)
    uint8_t *wo = q->h_wout.as<uint8_t>();
    const bool pf = prefetch_on();
    if (pf) prefetch_bytes(wo, std::min(n, kPrefetchAhead) * R * opitch);
    auto red = [&](size_t g) {
        if (pf && g + kPrefetchAhead < n) prefetch_bytes(wo + (g + kPrefetchAhead) * R * opitch, R * opitch);
        uint16_t mx = 0;  // align = max datagram length + 2 (data_operations.cpp:613-616)
        for (size_t i = 0; i < K; ++i) mx = std::max(mx, q->len[g * K + i]);
        const size_t align = (size_t)mx + KFEC_FEC_CONTAINER_HEADER;
        for (size_t r = 0; r < R; ++r) {
            uint8_t *p = wo + (g * R + r) * opitch + 16 - KFEC_PKT_REDUNDANT_HEADER;
            put_le32(p, timestamp);  // host_to_little_endian
            put_be32(p + 4, q->sn[g]);
            p[8] = (uint8_t)(K + r);
            put_be32(p + 9, q->conv[g]);
            if (cb) cb(user, q->tags[g], q->sn[g], (uint8_t)(K + r), p, KFEC_PKT_REDUNDANT_HEADER + align);
        }
    };
    auto data = [&](size_t i) {
        const kfec_txq::DataPkt &d = q->dpk[i];
        if (cb && d.len) cb(user, d.tag, d.sn, d.sub, q->arena.host(d.off), d.len);
    };
    emit(q, n, data, red);
    q->last_n = n;
    q->n = 0;
    q->dpk.clear();
    return tx_compact(q);  // keep the partial groups, at the front of the arena
}

// Small sealed flush (BAR mode): the resident worker writes the parity rows into the arena's reserve behind a
// 16-byte gap each, the host writes each redundant header into its gap through the BAR, and ONE seal launch
// protects every packet -- the staged data packets and the redundant ones, in emission order -- straight into
// pinned host rows (no pack or descriptor kernels, no copy calls).  1: not taken.
int txq_flush_sealed_small(kfec_txq *q, uint32_t timestamp, kfec_packet_cb cb, void *user, void *stream, Steps &st)
{
    const size_t n = q->n, nd = q->dpk.size(), K = q->K, R = q->R;
    if (!q->arena.bar || n > worker_flush_max() || (n && R == 0)) return 1;
    q->trace.start();
    const size_t B = q->mtu + KFEC_FEC_CONTAINER_HEADER, opitch = 16 + round16(B);
    const size_t red_base = (q->used + 63) & ~size_t(63), nr = n * R;
    if (red_base + nr * opitch > q->arena.cap + q->arena.reserve) return 1;
    uint8_t *dimg = q->arena.d.as<uint8_t>();
    kfec::BatchSpec b;
    b.op = kfec::kBatchEncode;
    b.enc = kfec::ctx_enc(q->ctx);
    b.mat_id = kfec::ctx_mat_id(q->ctx);
    b.arena = dimg;
    b.out = dimg + red_base;  // (device memory: the seal launch reads the rows in place)
    b.opitch = opitch;
    b.ooff = 16;
    b.n = (int)n;
    b.K = (int)K;
    b.N = (int)q->N;
    b.B = (int)B;
    if (n && !kfec::worker_batch_ok(b)) return 1;
    const size_t rows = nd + nr;
    const size_t spitch = round4(KFEC_PKT_REDUNDANT_HEADER + B + seal_overhead(q->seal_mode));
    const size_t dL = rows * 8, dI = round8(dL + rows * 4), dT = dI + rows * 2;
    const size_t sO = rows * spitch, sT = sO + rows * 4;
    q->d_sdesc.uncached = true;
    if (q->h_sdesc.ensure(dT) || q->d_sdesc.ensure(dT) || q->h_sealed.ensure(sT)) return KFEC_ENOMEM;
    try {
        q->wdesc.resize(n * K);
    } catch (...) {
        return KFEC_ENOMEM;
    }
    // descriptors (data rows, then redundant rows) and iv draws in emission order, built in h_sdesc and written
    // through the BAR; the redundant headers into the rows' gaps
    uint8_t *hd = q->h_sdesc.as<uint8_t>();
    uint64_t *off = reinterpret_cast<uint64_t *>(hd);
    uint32_t *len = reinterpret_cast<uint32_t *>(hd + dL);
    uint16_t *iv = reinterpret_cast<uint16_t *>(hd + dI);
    for (size_t i = 0; i < nd; ++i) {
        off[i] = q->dpk[i].off;
        len[i] = q->dpk[i].len;
    }
    uint8_t hdr[KFEC_PKT_REDUNDANT_HEADER];
    for (size_t g = 0; g < n; ++g) {
        uint16_t mx = 0;  // align = max datagram length + 2 (data_operations.cpp:613-616)
        for (size_t i = 0; i < K; ++i) mx = std::max(mx, q->len[g * K + i]);
        put_le32(hdr, timestamp);
        put_be32(hdr + 4, q->sn[g]);
        put_be32(hdr + 9, q->conv[g]);
        for (size_t r = 0; r < R; ++r) {
            const size_t row = red_base + (g * R + r) * opitch + 16 - KFEC_PKT_REDUNDANT_HEADER;
            hdr[8] = (uint8_t)(K + r);
            kfec::copy_to_bar(dimg + row, hdr, sizeof(hdr));
            off[nd + g * R + r] = row;
            len[nd + g * R + r] = (uint32_t)(KFEC_PKT_REDUNDANT_HEADER + mx + KFEC_FEC_CONTAINER_HEADER);
        }
    }
    uint64_t iv_ctr = q->iv_ctr;  // committed only when the flush succeeds
    emit(q, n, [&](size_t i) { iv[i] = iv_draw(q->iv_seed, iv_ctr++); },
         [&](size_t g) { for (size_t r = 0; r < R; ++r) iv[nd + g * R + r] = iv_draw(q->iv_seed, iv_ctr++); });
    kfec::copy_to_bar(q->d_sdesc.p, hd, dT);
    kfec::bar_fence();  // staged packets, headers and descriptors before the doorbell / the launch
    if (n) {
        for (size_t i = 0; i < n * K; ++i) q->wdesc[i] = kfec::batch_desc(q->off[i], q->len[i], false);
        b.desc = q->wdesc.data();
        q->trace.mark();
        if (st.fail()) return KFEC_EHIP;
        const int rc = kfec::worker_batch(q->device, b);
        if (rc) return rc;  // (1: the worker is off or gone -> the launch path)
        q->trace.mark();
    } else {
        q->trace.mark();
        q->trace.mark();
    }
    uint8_t *hs = q->h_sealed.as<uint8_t>();
    uint32_t *s_len = reinterpret_cast<uint32_t *>(hs + sO);
    const uint8_t *ds = q->d_sdesc.as<uint8_t>();
    if (st.fail()) return KFEC_EHIP;
    const bool count = seal_count_on() && rows <= kfec::kSealCountRows;
    uint32_t blocks = 0;
    int rc;
    if (count) {
        if (!q->h_done.p) {
            if (q->h_done.ensure(64)) return KFEC_ENOMEM;
            *q->h_done.as<volatile uint32_t>() = 0;
            q->done_sum = 0;
        }
        if (q->aead && hipSetDevice(q->aead->device) != hipSuccess) return KFEC_EHIP;  // (as kfec_aead_seal_batch)
        const hipStream_t strm = static_cast<hipStream_t>(stream);
        const size_t src_bytes = red_base + nr * opitch;
        const uint64_t *d_off = reinterpret_cast<const uint64_t *>(ds);
        const uint32_t *d_len = reinterpret_cast<const uint32_t *>(ds + dL);
        uint32_t *cnt = q->h_done.as<uint32_t>();
        (void)hipGetLastError();  // (no stale error of an earlier call may read as this launch's)
        rc = (q->aead ? kfec::launch_aead(q->aead, false, rows, dimg, src_bytes, d_off, d_len,
                                          reinterpret_cast<const uint16_t *>(ds + dI), hs, spitch, s_len, nullptr, strm, cnt,
                                          &blocks)
                      : kfec::launch_seal(false, q->seal_mode, rows, dimg, src_bytes, d_off, d_len, hs, spitch, s_len,
                                          nullptr, strm, cnt, &blocks))
                 ? KFEC_EHIP
                 : KFEC_OK;
        if (rc == KFEC_OK) q->done_sum += blocks;
    } else {
        rc = seal_rows(q->seal_mode, q->aead, rows, dimg, red_base + nr * opitch, reinterpret_cast<const uint64_t *>(ds),
                       reinterpret_cast<const uint32_t *>(ds + dL), reinterpret_cast<const uint16_t *>(ds + dI), hs, spitch,
                       s_len, stream);
    }
    const hipStream_t ss = static_cast<hipStream_t>(stream);
    auto fail = [&](int code) {
        if (count) count_resync(q->h_done, q->done_sum, ss);
        return code;
    };
    if (rc) return fail(rc);
    q->trace.mark();
    if (st.fail()) return fail(KFEC_EHIP);
    if (count ? wait_count(q->h_done.as<volatile uint32_t>(), q->done_sum, ss) != 0
              : hipStreamSynchronize(ss) != hipSuccess)
        return fail(KFEC_EHIP);
    q->trace.mark();
    const bool pf = prefetch_on();
    if (pf) {
        prefetch_bytes(hs, std::min(nd, kPrefetchAhead) * spitch);
        prefetch_bytes(hs + nd * spitch, std::min(n, (size_t)1) * R * spitch);
    }
    auto red = [&](size_t g) {
        if (pf && g + 1 < n) prefetch_bytes(hs + (nd + (g + 1) * R) * spitch, R * spitch);
        for (size_t r = 0; r < R; ++r) {
            const size_t i = nd + g * R + r;
            if (s_len[i] && cb) cb(user, q->tags[g], q->sn[g], (uint8_t)(K + r), hs + i * spitch, s_len[i]);
        }
    };
    auto data = [&](size_t i) {
        if (pf && i + kPrefetchAhead < nd) prefetch_bytes(hs + (i + kPrefetchAhead) * spitch, spitch);
        const kfec_txq::DataPkt &d = q->dpk[i];
        if (s_len[i] && cb) cb(user, d.tag, d.sn, d.sub, hs + i * spitch, s_len[i]);
    };
    emit(q, n, data, red);
    q->trace.mark();
    q->trace.done();
    q->iv_ctr = iv_ctr;
    q->last_n = n;
    q->n = 0;
    q->dpk.clear();
    return tx_compact(q);
}

}  // namespace

extern "C" {

int kfec_txq_flush(kfec_txq *q, uint32_t timestamp, kfec_packet_cb cb, void *user, void *stream)
{
    if (!q) return KFEC_EINVAL;
    const size_t n = q->n, nd = q->dpk.size();
    if (n == 0 && nd == 0) return KFEC_OK;
    if (kn_changed(q->ctx, q->K, q->N)) return KFEC_EINVAL;  // the coder was reset: recreate the queue
    const bool seal = q->seal_mode != KFEC_TXQ_SEAL_OFF;
    stream = q->own.pick(stream);
    Steps st;
    if (!seal && n) {
        const int rc = txq_flush_worker(q, timestamp, cb, user, st);
        if (rc <= 0) return rc;
    } else if (seal) {
        const int rc = txq_flush_sealed_small(q, timestamp, cb, user, stream, st);
        if (rc <= 0) return rc;
    }
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t K = q->K, R = q->R;
    const size_t B = q->mtu + KFEC_FEC_CONTAINER_HEADER, pitch = round4(B);
    const size_t pkt_pitch = round4(KFEC_PKT_REDUNDANT_HEADER + B);
    const size_t nk = n * K, nr = n * R;
    // device tables [off nk*8][len nk*2][pad][sn n*4][conv n*4], from the queue's tables (never moved)
    const size_t L = nk * 8, S = round8(L + nk * 2), C = S + n * 4;
    uint8_t *dm = q->d_meta.as<uint8_t>();
    const uint64_t *d_off = reinterpret_cast<const uint64_t *>(dm);
    const uint16_t *d_len = reinterpret_cast<const uint16_t *>(dm + L);
    // sealed rows: the nd data packets, then the n x R redundant packets; descriptors up in one copy:
    // [data off nd*8][data len nd*4][pad][iv rows*2]; down: [rows][spitch] sealed, then out_len rows*4
    const size_t rows = seal ? nd + nr : 0;
    const size_t spitch = round4(KFEC_PKT_REDUNDANT_HEADER + B + seal_overhead(q->seal_mode));
    const size_t dL = nd * 8, dI = round8(dL + nd * 4), dT = dI + rows * 2;
    const size_t sO = rows * spitch, sT = sO + rows * 4;
    uint64_t iv_ctr = q->iv_ctr;  // committed only when the flush succeeds
    if (seal) {
        q->d_sdesc.uncached = q->arena.bar_ok;
        if (q->h_sdesc.ensure(dT) || q->d_sdesc.ensure(dT + nr * 12 + 8) || q->h_sealed.ensure(sT) || q->d_sealed.ensure(sT))
            return KFEC_ENOMEM;
        uint8_t *hd = q->h_sdesc.as<uint8_t>();
        uint16_t *iv = reinterpret_cast<uint16_t *>(hd + dI);
        for (size_t i = 0; i < nd; ++i) {
            reinterpret_cast<uint64_t *>(hd)[i] = q->dpk[i].off;
            reinterpret_cast<uint32_t *>(hd + dL)[i] = q->dpk[i].len;
        }
        // iv draws in emission order: data packet i, then its group's redundant packets
        auto red_ivs = [&](size_t g) {
            for (size_t r = 0; r < R; ++r) iv[nd + g * R + r] = iv_draw(q->iv_seed, iv_ctr++);
        };
        emit(q, n, [&](size_t i) { iv[i] = iv_draw(q->iv_seed, iv_ctr++); }, red_ivs);
        if (st.fail()) return KFEC_EHIP;
        TableUpload tu{q->arena.bar, q->d_sdesc.as<uint8_t>(), hd};
        tu.add(0, hd, dT);
        if (tu.send(s)) return KFEC_EHIP;
    }
    if (st.fail() || q->arena.finish(q->used, s)) return KFEC_EHIP;
    if (n) {
        TableUpload tu{q->arena.bar, dm, q->h_pack.as<uint8_t>()};
        tu.add(0, q->off.data(), L);
        tu.add(L, q->len.data(), nk * 2);
        tu.add(S, q->sn.data(), n * 4);
        tu.add(C, q->conv.data(), n * 4);
        if (st.fail() || tu.send(s)) return KFEC_EHIP;
    }
    const size_t arena = std::max<size_t>(q->used, 4);
    const size_t P = nr * pkt_pitch;  // [n][R] compact redundant packets, then their lengths
    uint8_t *dr = q->d_res.as<uint8_t>();
    int rc = KFEC_OK;
    if (n) {
        if (st.fail()) return KFEC_EHIP;
        rc = kfec_encode_framed_batch(q->ctx, n, q->arena.d.p, arena, d_off, d_len, B, pitch, q->d_par.p,
                                      q->d_align.as<uint16_t>(), stream);
        if (rc) return rc;
        if (R) {
            if (st.fail()) return KFEC_EHIP;
            rc = kfec_pack_batch(q->ctx, n, KFEC_PACK_REDUNDANT | KFEC_PACK_COMPACT, q->arena.d.p, arena, d_off, d_len,
                                 pitch, q->d_par.p, q->d_align.as<uint16_t>(), reinterpret_cast<const uint32_t *>(dm + S),
                                 reinterpret_cast<const uint32_t *>(dm + C), timestamp, dr, pkt_pitch,
                                 reinterpret_cast<uint16_t *>(dr + P), stream);
            if (rc) return rc;
        }
    }
    if (seal) {
        uint8_t *ds = q->d_sdesc.as<uint8_t>();
        const uint16_t *d_iv = reinterpret_cast<const uint16_t *>(ds + dI);
        uint8_t *sealed = q->d_sealed.as<uint8_t>();
        uint32_t *out_len = reinterpret_cast<uint32_t *>(sealed + sO);
        const kfec_aead *a = q->aead;
        // the staged data packets, straight from the arena
        if (st.fail()) return KFEC_EHIP;
        rc = seal_rows(q->seal_mode, a, nd, q->arena.d.p, arena, reinterpret_cast<const uint64_t *>(ds),
                       reinterpret_cast<const uint32_t *>(ds + dL), d_iv, sealed, spitch, out_len, stream);
        if (rc) return rc;
        if (nr) {  // the redundant packets the pack just wrote
            uint64_t *r_off = reinterpret_cast<uint64_t *>(ds + round8(dT));
            uint32_t *r_len = reinterpret_cast<uint32_t *>(r_off + nr);
            if (st.fail() || kfec::launch_pkt_desc(nr, pkt_pitch, reinterpret_cast<const uint16_t *>(dr + P), r_off, r_len, s))
                return KFEC_EHIP;
            if (st.fail()) return KFEC_EHIP;
            rc = seal_rows(q->seal_mode, a, nr, dr, std::max<size_t>(P, 4), r_off, r_len, d_iv + nd,
                           sealed + nd * spitch, spitch, out_len + nd, stream);
            if (rc) return rc;
        }
        if (st.fail() || hipMemcpyAsync(q->h_sealed.p, sealed, sT, hipMemcpyDeviceToHost, s) != hipSuccess) return KFEC_EHIP;
    } else if (nr) {
        if (st.fail() || hipMemcpyAsync(q->h_res.p, dr, P + nr * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return KFEC_EHIP;
    }
    if (st.fail() || hipStreamSynchronize(s) != hipSuccess) return KFEC_EHIP;
    const uint8_t *pk = q->h_res.as<uint8_t>();
    const uint16_t *pk_len = reinterpret_cast<const uint16_t *>(pk + P);
    const uint8_t *hs = q->h_sealed.as<uint8_t>();
    const uint32_t *s_len = reinterpret_cast<const uint32_t *>(hs + sO);
    const bool pf = prefetch_on();
    const size_t rpitch = seal ? spitch : pkt_pitch;  // redundant rows: hs + nd * spitch, or pk
    const uint8_t *rbase = seal ? hs + nd * spitch : pk;
    if (pf) {
        if (seal) prefetch_bytes(hs, std::min(nd, kPrefetchAhead) * spitch);
        prefetch_bytes(rbase, std::min(n, (size_t)1) * R * rpitch);
    }
    auto red = [&](size_t g) {
        if (pf && g + 1 < n) prefetch_bytes(rbase + (g + 1) * R * rpitch, R * rpitch);
        for (size_t r = 0; r < R; ++r) {
            const size_t i = g * R + r;
            const uint8_t *p = seal ? hs + (nd + i) * spitch : pk + i * pkt_pitch;
            const size_t plen = seal ? s_len[nd + i] : pk_len[i];
            if (plen && cb) cb(user, q->tags[g], q->sn[g], (uint8_t)(K + r), p, plen);
        }
    };
    auto data = [&](size_t i) {
        if (pf && seal && i + kPrefetchAhead < nd) prefetch_bytes(hs + (i + kPrefetchAhead) * spitch, spitch);
        const kfec_txq::DataPkt &d = q->dpk[i];
        const uint8_t *p = seal ? hs + i * spitch : q->arena.host(d.off);
        const size_t plen = seal ? s_len[i] : d.len;
        if (plen && cb) cb(user, d.tag, d.sn, d.sub, p, plen);
    };
    emit(q, n, data, red);
    q->iv_ctr = iv_ctr;
    q->last_n = n;
    q->n = 0;
    q->dpk.clear();
    return tx_compact(q);  // keep the partial groups, at the front of the arena
}

size_t kfec_txq_staged(const kfec_txq *q) { return q ? q->dpk.size() : 0; }

int kfec_txq_seal(kfec_txq *q, int mode, const kfec_aead *aead, uint64_t iv_seed, unsigned flags)
{
    if (!q || (flags & ~KFEC_TXQ_DEFER_DATA) || q->n || !q->dpk.empty()) return KFEC_EINVAL;
    if (mode != KFEC_TXQ_SEAL_OFF) {
        if (!seal_mode_ok(mode, aead) || (aead && aead->device != q->device)) return KFEC_EINVAL;
    } else if (aead) {
        return KFEC_EINVAL;
    }
    const bool defer = (flags & KFEC_TXQ_DEFER_DATA) != 0;
    if (defer && !q->defer) {  // every data packet now takes its 9-byte header in the arena too
        const size_t slot = q->arena.step(std::max<size_t>(q->mtu + KFEC_PKT_DATA_HEADER, 4));
        if (slot * q->G * q->K > q->arena.cap && q->arena.grow(q->used, slot * q->G * q->K - q->used)) return KFEC_ENOMEM;
    }
    q->seal_mode = mode;
    q->aead = mode == KFEC_TXQ_SEAL_OFF ? nullptr : aead;
    q->iv_seed = iv_seed;
    q->iv_ctr = 0;
    q->defer = defer;
    return KFEC_OK;
}

}  // extern "C"

// ---- receive ---------------------------------------------------------------------------------------------
struct kfec_rxq {
    const kfec_ctx *ctx = nullptr;
    int device = 0;
    size_t K = 0, N = 0, R = 0, G = 0, max_shard = 0, slot = 0;
    size_t n = 0;       // groups queued for decoding
    size_t last_n = 0;  // groups of the last flush (the arena's mode)
    size_t used = 0;    // arena bytes staged (shards packed back to back at Arena::step granules)
    std::vector<kfec_rx *> rxs;  // the receivers whose cached shards live in the arena
    // per queued group g: the N shard slots' arena offsets and lengths, the present bits (never moved by a flush)
    std::vector<uint64_t> off;
    std::vector<uint16_t> len;
    std::vector<uint64_t> present;
    std::vector<uint64_t> tags;
    std::vector<uint32_t> sns;
    // launch path: h_pack (pinned mode: the tables packed for one copy up), h_res (recovered framed shards
    // [n][R], then their data indices; one copy back).  Worker path: wdesc / wrec (the batch's descriptors and
    // per-group records), wmap (batch entry -> queue group), h_wout (coherent pinned recovered rows).
    Pinned h_pack, h_res, h_wout;
    std::vector<uint64_t> wdesc;
    std::vector<uint8_t> wrec;
    std::vector<uint32_t> wmap;
    // host-solved decode coefficients by erasure pattern (m, missing ids, parity ids): live links repeat few
    // patterns (at 1% loss most groups lose one shard)
    struct Solved {
        uint8_t m = 0;
        uint8_t M[8] = {}, P[8] = {};
        std::vector<uint8_t> D;
    };
    std::vector<Solved> solved;
    Device d_meta, d_align, d_st, d_ws, d_res;
    OwnStream own;
    Arena arena;  // declared last: destroyed (and its copy stream drained) first
};

// fec_rcv_cache[sn]: the shards of one group, by sub_sn.  The bytes live in the queue's staging arena (stored
// once, at push); a restored group keeps only its membership (the reference never reads it again).
struct RxGroup {
    uint64_t off[256];
    uint16_t len[256];
    uint64_t has[4];
    uint32_t count;  // distinct sub_sn cached: fec_rcv_cache[sn].size()
    bool restored;   // sn in fec_rcv_restored (restored is always a subset of the cache's keys)
    bool test(unsigned s) const { return (has[s >> 6] >> (s & 63)) & 1; }
};

struct kfec_rx {
    kfec_rxq *q = nullptr;
    uint64_t tag = 0;
    // fec_rcv_cache + fec_rcv_restored as a flat (sn, group) list: it holds the few groups within gbv_fec_waits
    // of the newest sn, and every push scans all of it anyway (fec_find_missings), so a linear find beats the
    // map; order is irrelevant because a push can complete only its own group
    std::vector<std::pair<uint32_t, RxGroup *>> cache;
    std::vector<std::unique_ptr<RxGroup>> pool;
    std::vector<RxGroup *> free_groups;
    RxGroup *get()
    {
        if (free_groups.empty()) {
            pool.push_back(std::make_unique<RxGroup>());
            free_groups.push_back(pool.back().get());
        }
        RxGroup *x = free_groups.back();
        free_groups.pop_back();
        x->has[0] = x->has[1] = x->has[2] = x->has[3] = 0;
        x->count = 0;
        x->restored = false;
        return x;
    }
};

namespace {

bool kn_changed_rx(const kfec_rxq *q) { return kfec_get_K(q->ctx) != q->K || kfec_get_N(q->ctx) != q->N; }

// The receive side of tx_compact: the shards of every cached group that still waits for K shares move to
// the front of the arena; restored groups (kept by the reference only as membership) and evicted ones free
// their bytes.  Called with nothing queued: after a flush, and before growing a full arena -- stale-only
// traffic (groups that never reach K shares) must not grow memory without bound.
int rx_compact(kfec_rxq *q)
{
    struct Part {
        uint64_t *off;
        size_t len;
        bool operator<(const Part &o) const { return *off < *o.off; }
    };
    if (q->arena.quiesce()) return KFEC_EHIP;
    std::vector<Part> part;
    for (kfec_rx *rx : q->rxs)
        for (auto &kv : rx->cache) {
            RxGroup *x = kv.second;
            if (x->restored) continue;
            for (unsigned w = 0; w < 4; ++w)
                for (uint64_t m = x->has[w]; m; m &= m - 1) {
                    const unsigned sub = w * 64 + (unsigned)__builtin_ctzll(m);
                    part.push_back({&x->off[sub], x->len[sub]});
                }
        }
    std::sort(part.begin(), part.end());
    const bool whole = q->arena.switch_mode(q->last_n);
    size_t at = 0;
    for (const Part &p : part) {
        if (p.len && at != *p.off) {
            std::memmove(q->arena.host(at), q->arena.host(*p.off), p.len);
            q->arena.moved(at, p.len, whole);
        }
        *p.off = at;
        at += q->arena.step(p.len);
    }
    q->used = at;
    q->arena.restage(at, whole);
    return KFEC_OK;
}

// a decodable group takes queue slot q->n: its shards are already in the arena
void rx_enqueue(kfec_rxq *q, uint64_t tag, uint32_t sn, const RxGroup &grp)
{
    const size_t g = q->n;
    uint64_t *present = &q->present[g * 4];
    present[0] = present[1] = present[2] = present[3] = 0;
    // a sub_sn beyond N is cached by the reference (it counts towards size()) but never selected usefully
    for (unsigned s = 0; s < q->N; ++s) {
        if (!grp.test(s)) continue;
        const size_t e = g * q->N + s;
        q->off[e] = grp.off[s];
        q->len[e] = grp.len[s];
        present[s >> 6] |= 1ull << (s & 63);
    }
    q->tags[g] = tag;
    q->sns[g] = sn;
    q->n = g + 1;
}

}  // namespace

extern "C" {

int kfec_rxq_create(const kfec_ctx *ctx, size_t max_groups, size_t max_shard, kfec_rxq **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!ctx || !max_groups || max_shard < KFEC_FEC_CONTAINER_HEADER || max_shard > 0xFFFF) return KFEC_EINVAL;
    kfec_rxq *q = new (std::nothrow) kfec_rxq;
    if (!q) return KFEC_ENOMEM;
    q->ctx = ctx;
    q->device = kfec_device(ctx);
    q->K = kfec_get_K(ctx);
    q->N = kfec_get_N(ctx);
    q->R = q->N - q->K;
    q->G = max_groups;
    q->max_shard = max_shard;
    const bool bar = env_flag("KFEC_QUEUE_BAR", true) && kfec::bar_writable(q->device);
    q->slot = (max_shard + (bar ? bar_align() : 4) - 1) & ~((bar ? bar_align() : 4) - 1);
    const size_t G = q->G, GN = G * q->N, R1 = std::max<size_t>(q->R, 1);
    const size_t pitch = round4(max_shard);
    const size_t meta = round8(GN * 10) + G * 32, res = G * R1 * (pitch + 3);
    q->d_meta.uncached = bar;
    q->h_wout.flags = hipHostMallocCoherent;
    try {
        q->off.resize(GN);
        q->len.resize(GN);
        q->present.resize(G * 4);
        q->tags.resize(G);
        q->sns.resize(G);
        q->solved.resize(256);
    } catch (...) {
        delete q;
        return KFEC_ENOMEM;
    }
    if (hipSetDevice(q->device) != hipSuccess) {
        delete q;
        return KFEC_EHIP;
    }
    if (q->own.init() || q->arena.init(q->device, (GN + (bar ? q->N : 0)) * q->slot, bar, G) || q->h_pack.ensure(meta) || q->h_res.ensure(res) ||
        q->d_meta.ensure(meta) || q->d_res.ensure(res) || q->d_align.ensure(G * 2) || q->d_st.ensure(G) ||
        q->d_ws.ensure(kfec_decode_workspace_size(ctx, G))) {
        delete q;
        return KFEC_ENOMEM;
    }
    *out = q;
    return KFEC_OK;
}

void kfec_rxq_destroy(kfec_rxq *q) { delete q; }

size_t kfec_rxq_pending(const kfec_rxq *q) { return q ? q->n : 0; }

size_t kfec_rxq_capacity(const kfec_rxq *q) { return q ? q->arena.cap : 0; }

int kfec_rx_create(kfec_rxq *q, uint64_t tag, kfec_rx **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!q) return KFEC_EINVAL;
    kfec_rx *rx = new (std::nothrow) kfec_rx;
    if (!rx) return KFEC_ENOMEM;
    rx->q = q;
    rx->tag = tag;
    try {
        q->rxs.push_back(rx);
    } catch (...) {
        delete rx;
        return KFEC_ENOMEM;
    }
    *out = rx;
    return KFEC_OK;
}

void kfec_rx_destroy(kfec_rx *rx)
{
    if (!rx) return;
    auto &v = rx->q->rxs;
    v.erase(std::remove(v.begin(), v.end(), rx), v.end());
    delete rx;
}

size_t kfec_rx_cached(const kfec_rx *rx) { return rx ? rx->cache.size() : 0; }

int kfec_rx_push(kfec_rx *rx, const uint8_t *pkt, size_t len, const uint8_t **datagram, size_t *datagram_len)
{
    if (!rx || !pkt) return KFEC_EINVAL;
    if (datagram) *datagram = nullptr;
    if (datagram_len) *datagram_len = 0;
    kfec_rxq *q = rx->q;
    if (kn_changed_rx(q)) return KFEC_EINVAL;  // the coder was reset: recreate the queue
    // unpack_fec / unpack_fec_redundant (connections.cpp:488-511), dispatched on sub_sn as fec_unpack
    if (len < KFEC_PKT_DATA_HEADER) return KFEC_EINVAL;
    const uint8_t sub = pkt[8];
    const bool red = sub >= q->K;
    const size_t H = red ? KFEC_PKT_REDUNDANT_HEADER : KFEC_PKT_DATA_HEADER;
    if (len < H) return KFEC_EINVAL;
    const uint8_t *payload = pkt + H;
    const size_t plen = len - H;
    if (plen + (red ? 0 : KFEC_FEC_CONTAINER_HEADER) > q->max_shard) return KFEC_EINVAL;
    const uint32_t fec_sn = get_be32(pkt + 4);
    auto found = std::find_if(rx->cache.begin(), rx->cache.end(), [&](const auto &kv) { return kv.first == fec_sn; });
    // capacity: only this packet's group can become decodable on this push (every other cached group either
    // reached K shares on an earlier push, and was queued and restored then, or still lacks shares)
    const bool fresh = found == rx->cache.end();
    const bool store = fresh || !found->second->restored;
    const uint32_t have = fresh ? 0u : found->second->count + (found->second->test(sub) ? 0u : 1u);
    const bool completes = store && (fresh ? 1u : have) >= q->K;
    if (completes && q->n >= q->G) return KFEC_ENOMEM;
    const size_t need = q->arena.step(plen);
    if (store && q->used + need > q->arena.cap) {
        if (q->n) return KFEC_ENOMEM;  // a flush frees the queued groups' bytes
        int rc = rx_compact(q);        // first reclaim restored / evicted groups' bytes and overwritten duplicates
        if (!rc && q->used + need > q->arena.cap) rc = q->arena.grow(q->used, need);
        if (rc) return rc;
    }
    // fec_rcv_cache[sn][sub_sn] = ... (client.cpp:869,887): a duplicate overwrites
    RxGroup *grp;
    if (found != rx->cache.end()) {
        grp = found->second;
    } else {
        grp = rx->get();
        rx->cache.emplace_back(fec_sn, grp);
    }
    if (!grp->test(sub)) {
        grp->has[sub >> 6] |= 1ull << (sub & 63);
        grp->count++;
    }
    if (store) {
        q->arena.put(q->used, payload, plen);
        grp->off[sub] = q->used;
        grp->len[sub] = (uint16_t)plen;
        q->used += need;
        q->arena.staged(q->used);
    }
    if (!red) {
        if (datagram) *datagram = payload;
        if (datagram_len) *datagram_len = plen;
    }
    // fec_find_missings (client.cpp:895-938)
    int queued = 0;
    for (auto it = rx->cache.begin(); it != rx->cache.end();) {
        const uint32_t sn = it->first;
        RxGroup *x = it->second;
        const bool stale = (uint32_t)(fec_sn - sn) > kFecWaits;
        if (x->count < q->K || x->restored) {
            if (stale) {  // fec_rcv_restored.erase(sn) + fec_rcv_cache.erase(sn)
                rx->free_groups.push_back(x);
                it = rx->cache.erase(it);
            } else {
                ++it;
            }
            continue;
        }
        rx_enqueue(q, rx->tag, sn, *x);
        x->restored = true;
        ++queued;
        ++it;
    }
    return queued;
}

}  // extern "C"

namespace {

// The decode coefficients of one erasure pattern (host_solve of the single-group decode), cached per queue.
const uint8_t *rx_solve(kfec_rxq *q, int m, const uint8_t *M, const uint8_t *P)
{
    uint32_t h = (uint32_t)m * 0x9E3779B1u;
    for (int t = 0; t < m; ++t) h = (h ^ M[t] ^ ((uint32_t)P[t] << 8)) * 0x01000193u;
    kfec_rxq::Solved &e = q->solved[(h >> 8) & 255];
    if (e.m == m && std::memcmp(e.M, M, m) == 0 && std::memcmp(e.P, P, m) == 0) return e.D.data();
    try {
        e.D.resize((size_t)m * q->K);
    } catch (...) {
        return nullptr;
    }
    e.m = 0;
    if (!kfec::worker_solve(kfec::ctx_h_enc(q->ctx), (int)q->K, m, M, P, e.D.data())) return nullptr;
    e.m = (uint8_t)m;
    std::memcpy(e.M, M, m);
    std::memcpy(e.P, P, m);
    return e.D.data();
}

// Small flush through the resident worker.  Per queued group, on the host (bookkeeping): the reference's share
// selection (fecpp.cpp:528-548: data share i fills row i, each missing row takes the highest unused id) and the
// coefficients of the missing rows (cached by erasure pattern); on the device: the recovered framed shards,
// straight into h_wout.  Groups with fewer than K shares recover nothing (the reference's {}), groups with every
// data shard present need no device work.  1: not taken.
int rxq_flush_worker(kfec_rxq *q, kfec_datagram_cb cb, void *user, Steps &st)
{
    const size_t n = q->n, K = q->K, N = q->N, R = q->R, B = q->max_shard;
    if (!q->arena.bar || R == 0 || R > 8 || n == 0 || n > worker_flush_max()) return 1;
    const size_t G16 = (B + 15) / 16, opitch = 16 * G16, rs = round16(16 + R * K);
    try {
        q->wdesc.resize(n * K);
        q->wrec.assign(n * rs, 0);
        q->wmap.resize(n);
    } catch (...) {
        return KFEC_ENOMEM;
    }
    size_t nb = 0;
    for (size_t g = 0; g < n; ++g) {
        const uint64_t *pr = &q->present[g * 4];
        const int have = __builtin_popcountll(pr[0]) + __builtin_popcountll(pr[1]) + __builtin_popcountll(pr[2]) +
                         __builtin_popcountll(pr[3]);
        if ((size_t)have < K) continue;  // KFEC_GROUP_EMPTY: nothing recovered
        auto bit = [&](size_t s_) { return (pr[s_ >> 6] >> (s_ & 63)) & 1; };
        uint8_t M[8], P[8];
        int m = 0;
        size_t hi = N;  // parity picks: the highest present ids, descending
        uint64_t *d = &q->wdesc[nb * K];
        for (size_t i = 0; i < K; ++i) {
            if (bit(i)) {
                d[i] = kfec::batch_desc(q->off[g * N + i], q->len[g * N + i], false);
                continue;
            }
            do --hi; while (!bit(hi));
            if (m == 8) return 1;  // (R <= 8: unreachable)
            M[m] = (uint8_t)i;
            P[m] = (uint8_t)hi;
            ++m;
            d[i] = kfec::batch_desc(q->off[g * N + hi], q->len[g * N + hi], true);
        }
        if (m == 0) continue;  // every data shard present: nothing to recover
        const uint8_t *D = rx_solve(q, m, M, P);
        if (!D) return 1;  // a singular pattern (unreachable for an MDS code): the launch path reports it
        uint8_t *rec = &q->wrec[nb * rs];
        rec[0] = (uint8_t)m;
        std::memcpy(rec + 1, M, m);  // (bytes 1..8: the recovered data ids, read back here below)
        std::memcpy(rec + 16, D, (size_t)m * K);
        q->wmap[nb++] = (uint32_t)g;
    }
    if (nb) {
        kfec::BatchSpec b;
        b.op = kfec::kBatchDecode;
        b.arena = q->arena.d.p;
        b.opitch = opitch;
        b.ooff = 0;
        b.n = (int)nb;
        b.K = (int)K;
        b.N = (int)N;
        b.B = (int)B;
        b.desc = q->wdesc.data();
        b.rec = q->wrec.data();
        b.rec_stride = rs;
        if (!kfec::worker_batch_ok(b)) return 1;
        if (q->h_wout.ensure(nb * R * opitch)) return KFEC_ENOMEM;
        b.out = q->h_wout.as<uint8_t>();
        kfec::bar_fence();  // the staged shards before the doorbell
        if (st.fail()) return KFEC_EHIP;
        const int rc = kfec::worker_batch(q->device, b);
        if (rc) return rc;  // (1: the worker is off or gone -> the launch path)
    }
    const uint8_t *wo = q->h_wout.as<uint8_t>();
    for (size_t e = 0; e < nb && cb; ++e) {
        const uint8_t *rec = &q->wrec[e * rs];
        const size_t g = q->wmap[e];
        for (int u = 0; u < rec[0]; ++u) {
            const uint8_t *shard = wo + (e * R + u) * opitch;
            const size_t dlen = ((size_t)shard[0] << 8) | shard[1];  // ntohs(data_length)
            if (dlen + KFEC_FEC_CONTAINER_HEADER > B) continue;     // inconsistent group (kfec_unframe_batch's 0xFFFF)
            cb(user, q->tags[g], q->sns[g], rec[1 + u], shard + KFEC_FEC_CONTAINER_HEADER, dlen);
        }
    }
    q->last_n = n;
    q->n = 0;
    return rx_compact(q);  // keep the shards of the groups still waiting for K shares
}

}  // namespace

extern "C" {

int kfec_rxq_flush(kfec_rxq *q, kfec_datagram_cb cb, void *user, void *stream)
{
    if (!q) return KFEC_EINVAL;
    const size_t n = q->n;
    if (n == 0) return KFEC_OK;
    if (kn_changed_rx(q)) return KFEC_EINVAL;  // the coder was reset: recreate the queue
    stream = q->own.pick(stream);
    Steps st;
    {
        const int rc = rxq_flush_worker(q, cb, user, st);
        if (rc <= 0) return rc;
    }
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t N = q->N, R = q->R;
    const size_t B = q->max_shard, pitch = round4(B);
    const size_t nn = n * N;
    // device tables [off nn*8][len nn*2][pad][present n*32], from the queue's tables (never moved)
    const size_t L = nn * 8, P = round8(L + nn * 2);
    uint8_t *dm = q->d_meta.as<uint8_t>();
    if (st.fail() || q->arena.finish(q->used, s)) return KFEC_EHIP;
    {
        TableUpload tu{q->arena.bar, dm, q->h_pack.as<uint8_t>()};
        tu.add(0, q->off.data(), L);
        tu.add(L, q->len.data(), nn * 2);
        tu.add(P, q->present.data(), n * 32);
        if (st.fail() || tu.send(s)) return KFEC_EHIP;
    }
    // results: [n][R] recovered framed shards, then their data indices (one copy back).  extract_from_container
    // (data_operations.cpp:697-704) is only "skip the BE16 length": done here on the host at the callback, so
    // no unframe pass and no second copy of the recovered bytes
    const size_t D = n * R * pitch;
    uint8_t *dr = q->d_res.as<uint8_t>();
    uint8_t *d_idx = dr + D;
    // recv compact_into_container + decode fused: the chosen shares are framed on the fly from the arena
    if (st.fail()) return KFEC_EHIP;
    int rc = kfec_decode_framed_batch(q->ctx, n, q->arena.d.p, std::max<size_t>(q->used, 4),
                                      reinterpret_cast<const uint64_t *>(dm), reinterpret_cast<const uint16_t *>(dm + L),
                                      reinterpret_cast<const uint64_t *>(dm + P), B, pitch, dr, d_idx,
                                      q->d_st.as<uint8_t>(), q->d_align.as<uint16_t>(), q->d_ws.p, stream);
    if (rc) return rc;
    if (R && (st.fail() || hipMemcpyAsync(q->h_res.p, dr, D + n * R, hipMemcpyDeviceToHost, s) != hipSuccess))
        return KFEC_EHIP;
    if (st.fail() || hipStreamSynchronize(s) != hipSuccess) return KFEC_EHIP;
    const uint8_t *hr = q->h_res.as<uint8_t>();
    const uint8_t *rec_idx = hr + D;
    for (size_t g = 0; g < n && cb && R; ++g) {
        for (size_t t = 0; t < R; ++t) {
            const uint8_t idx = rec_idx[g * R + t];
            if (idx == 0xFF) continue;
            const uint8_t *shard = hr + (g * R + t) * pitch;
            const size_t dlen = ((size_t)shard[0] << 8) | shard[1];  // ntohs(data_length)
            if (dlen + KFEC_FEC_CONTAINER_HEADER > B) continue;     // inconsistent group (kfec_unframe_batch's 0xFFFF)
            cb(user, q->tags[g], q->sns[g], idx, shard + KFEC_FEC_CONTAINER_HEADER, dlen);
        }
    }
    q->last_n = n;
    q->n = 0;
    return rx_compact(q);  // keep the shards of the groups still waiting for K shares
}

}  // extern "C"

// ---- receive-side packet opening (decrypt_data on the device, ahead of kfec_rx_push) --------------------
struct kfec_opener {
    int mode = KFEC_SEAL_CHECKSUM;
    const kfec_aead *aead = nullptr;
    int device = 0;
    size_t max_packets = 0, max_packet = 0, pitch = 0;
    size_t n = 0, used = 0;
    // h_arena: the staged packets (4-byte offsets); h_desc: off u64 [n], len u32 [n] (one copy up);
    // h_out: [n][pitch] plaintext, then out_len u32 [n], then ok u8 [n] (one copy down).
    // bar (large-BAR device, at most kOpenerBarMax packets per flush): each packet is written straight into
    // d_arena through the BAR when it is added (no host copy), the descriptors likewise at the flush, and the open
    // kernel writes its rows straight into h_out: a flush is one launch and one synchronisation
    bool bar = false;
    Pinned h_arena, h_desc, h_out;
    Device d_arena, d_desc, d_out;
    Pinned h_done;          // BAR mode, checksum16 / plain_xor: the open kernel's completion count (as kfec_txq's)
    uint32_t done_sum = 0;
    std::vector<uint64_t> tags;
    OwnStream own;
};

extern "C" {

// test-only hook (not in the headers): as kfec_test_txq_count_drift
int32_t kfec_test_opener_count_drift(const kfec_opener *o)
{
    return o && o->h_done.p ? (int32_t)(*o->h_done.as<volatile uint32_t>() - o->done_sum) : 0;
}

int kfec_opener_create(int mode, const kfec_aead *aead, size_t max_packets, size_t max_packet, kfec_opener **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!max_packets || !max_packet || max_packet > 0xFFFFFF || !seal_mode_ok(mode, aead)) return KFEC_EINVAL;
    int dev = 0, count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || hipGetDevice(&dev) != hipSuccess) return KFEC_ENODEV;
    if (aead && aead->device != dev) return KFEC_EINVAL;
    kfec_opener *o = new (std::nothrow) kfec_opener;
    if (!o) return KFEC_ENOMEM;
    o->mode = mode;
    o->aead = aead;
    o->device = dev;
    o->max_packets = max_packets;
    o->max_packet = max_packet;
    o->pitch = round4(max_packet);
    const size_t arena = max_packets * round4(max_packet), desc = max_packets * 12,
                 res = max_packets * (o->pitch + 5);
    constexpr size_t kOpenerBarMax = 65536;
    o->bar = env_flag("KFEC_QUEUE_BAR", true) && max_packets <= kOpenerBarMax && kfec::bar_writable(dev);
    o->d_arena.uncached = o->d_desc.uncached = o->bar;
    if (o->bar && env_flag("KFEC_QUEUE_COHERENT_OUT", true)) o->h_out.flags = hipHostMallocCoherent;  // (as h_sealed)
    try {
        o->tags.resize(max_packets);
    } catch (...) {
        delete o;
        return KFEC_ENOMEM;
    }
    if (o->own.init() || (!o->bar && o->h_arena.ensure(arena)) || o->h_desc.ensure(desc) || o->h_out.ensure(res) ||
        o->d_arena.ensure(arena) || o->d_desc.ensure(desc) || (!o->bar && o->d_out.ensure(res))) {
        delete o;
        return KFEC_ENOMEM;
    }
    *out = o;
    return KFEC_OK;
}

void kfec_opener_destroy(kfec_opener *o)
{
    if (!o) return;
    (void)hipSetDevice(o->device);
    delete o;
}

size_t kfec_opener_pending(const kfec_opener *o) { return o ? o->n : 0; }

int kfec_opener_add(kfec_opener *o, const uint8_t *pkt, size_t len, uint64_t tag)
{
    if (!o || (len && !pkt) || len > o->max_packet) return KFEC_EINVAL;
    if (o->n == o->max_packets) return KFEC_ENOMEM;
    const size_t i = o->n++;
    if (len) {
        if (o->bar) kfec::copy_to_bar(o->d_arena.as<uint8_t>() + o->used, pkt, len);
        else std::memcpy(o->h_arena.as<uint8_t>() + o->used, pkt, len);
    }
    reinterpret_cast<uint64_t *>(o->h_desc.p)[i] = o->used;
    o->tags[i] = tag;
    // lengths follow the offsets once the batch size is known (kfec_opener_flush packs them)
    reinterpret_cast<uint32_t *>(o->h_desc.as<uint8_t>() + o->max_packets * 8)[i] = (uint32_t)len;
    o->used += round4(len);
    return KFEC_OK;
}

int kfec_opener_flush(kfec_opener *o, kfec_opened_cb cb, void *user, void *stream)
{
    if (!o) return KFEC_EINVAL;
    const size_t n = o->n;
    if (n == 0) return KFEC_OK;
    if (hipSetDevice(o->device) != hipSuccess) return KFEC_EHIP;
    stream = o->own.pick(stream);
    const hipStream_t s = static_cast<hipStream_t>(stream);
    // the host table stays as kfec_opener_add wrote it ([off max*8][len max*4]), so a flush that fails can be
    // retried: its first n offsets and first n lengths go up as two copies into [off n*8][len n*4]
    const uint8_t *hd = o->h_desc.as<uint8_t>();
    uint8_t *dd = o->d_desc.as<uint8_t>();
    // BAR mode: the kernel's rows, lengths and flags land in h_out directly
    uint8_t *dr = o->bar ? o->h_out.as<uint8_t>() : o->d_out.as<uint8_t>();
    const size_t L = n * o->pitch;
    uint32_t *out_len = reinterpret_cast<uint32_t *>(dr + L);
    uint8_t *ok = dr + L + n * 4;
    const size_t arena = std::max<size_t>(o->used, 4);
    if (o->bar) {
        kfec::copy_to_bar(dd, hd, n * 8);
        kfec::copy_to_bar(dd + n * 8, hd + o->max_packets * 8, n * 4);
        kfec::bar_fence();  // the packets (written at add) and the descriptors before the launch
    } else if (hipMemcpyAsync(o->d_arena.p, o->h_arena.p, arena, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(dd, hd, n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
               hipMemcpyAsync(dd + n * 8, hd + o->max_packets * 8, n * 4, hipMemcpyHostToDevice, s) != hipSuccess) {
        return KFEC_EHIP;
    }
    const uint64_t *d_off = reinterpret_cast<const uint64_t *>(dd);
    const uint32_t *d_len = reinterpret_cast<const uint32_t *>(dd + n * 8);
    // BAR mode, at most kSealCountRows packets: wait for the kernel's own completion count, not the stream
    const bool count = o->bar && seal_count_on() && n <= kfec::kSealCountRows;
    int rc;
    if (count) {
        if (!o->h_done.p) {
            o->h_done.flags = hipHostMallocCoherent;
            if (o->h_done.ensure(64)) return KFEC_ENOMEM;
            *o->h_done.as<volatile uint32_t>() = 0;
            o->done_sum = 0;
        }
        uint32_t blocks = 0;
        (void)hipGetLastError();  // (no stale error of an earlier call may read as this launch's)
        rc = (o->aead ? kfec::launch_aead(o->aead, true, n, o->d_arena.p, arena, d_off, d_len, nullptr, dr, o->pitch,
                                          out_len, ok, s, o->h_done.as<uint32_t>(), &blocks)
                      : kfec::launch_seal(true, o->mode, n, o->d_arena.p, arena, d_off, d_len, dr, o->pitch, out_len, ok,
                                          s, o->h_done.as<uint32_t>(), &blocks))
                 ? KFEC_EHIP
                 : KFEC_OK;
        if (rc == KFEC_OK) o->done_sum += blocks;
    } else {
        rc = o->aead ? kfec_aead_open_batch(o->aead, n, o->d_arena.p, arena, d_off, d_len, dr, o->pitch, out_len, ok, stream)
                     : kfec_open_batch(o->mode, n, o->d_arena.p, arena, d_off, d_len, dr, o->pitch, out_len, ok, stream);
    }
    if (rc) {
        if (count) count_resync(o->h_done, o->done_sum, s);
        return rc;
    }
    if (count) {
        if (wait_count(o->h_done.as<volatile uint32_t>(), o->done_sum, s) != 0) {
            count_resync(o->h_done, o->done_sum, s);
            return KFEC_EHIP;
        }
    } else if ((!o->bar && hipMemcpyAsync(o->h_out.p, dr, L + n * 5, hipMemcpyDeviceToHost, s) != hipSuccess) ||
               hipStreamSynchronize(s) != hipSuccess) {
        return KFEC_EHIP;
    }
    const uint8_t *ho = o->h_out.as<uint8_t>();
    const uint32_t *h_len = reinterpret_cast<const uint32_t *>(ho + L);
    const uint8_t *h_ok = ho + L + n * 4;
    const bool pf = prefetch_on();
    if (pf) prefetch_bytes(ho, std::min(n, kPrefetchAhead) * o->pitch);
    for (size_t i = 0; i < n && cb; ++i) {
        if (pf && i + kPrefetchAhead < n) prefetch_bytes(ho + (i + kPrefetchAhead) * o->pitch, o->pitch);
        cb(user, o->tags[i], ho + i * o->pitch, h_ok[i] ? h_len[i] : 0, h_ok[i] ? 1 : 0);
    }
    o->n = 0;
    o->used = 0;
    return KFEC_OK;
}

}  // extern "C"
