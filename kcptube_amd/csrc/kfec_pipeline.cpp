// kfec_pipeline.cpp -- include/kfec_pipeline.h: kcptube's fec_maker / fec_unpack + fec_find_missings
// bookkeeping on the host, feeding batched device coding through the public C ABI (kfec.h, kfec_frame.h).
// Per-packet work here is bookkeeping and copies into pinned staging; every byte of parity, recovered data and
// redundant packet is computed by the GPU kernels at flush time.
#include "../../include/kfec_pipeline.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

namespace {

constexpr uint32_t kFecWaits = KFEC_FEC_WAITS;

size_t round4(size_t x) { return (x + 3) & ~size_t(3); }
size_t round8(size_t x) { return (x + 7) & ~size_t(7); }

// pinned host and device buffers, grown on demand
struct Pinned {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= n) return KFEC_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc(&p, std::max<size_t>(bytes, 256), hipHostMallocDefault) != hipSuccess) return KFEC_ENOMEM;
        n = std::max<size_t>(bytes, 256);
        return KFEC_OK;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    ~Pinned() { if (p) (void)hipHostFree(p); }
};

struct Device {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes)
    {
        if (bytes <= n) return KFEC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, std::max<size_t>(bytes, 256)) != hipSuccess) return KFEC_ENOMEM;
        n = std::max<size_t>(bytes, 256);
        return KFEC_OK;
    }
    template <typename T> T *as() const { return static_cast<T *>(p); }
    ~Device() { if (p) (void)hipFree(p); }
};

// Append-only staging uploaded while the host is still filling it: every kUploadChunk bytes of finished
// groups go H2D on the queue's own copy stream, so the PCIe transfer overlaps the per-packet host work and a
// flush only copies the tail.  Bytes already queued for DMA are never written again before the flush has
// synchronised (the arena is append-only between flushes).
struct Upload {
    static constexpr size_t kUploadChunk = size_t(8) << 20;
    hipStream_t cs = nullptr;
    hipEvent_t ev = nullptr;
    size_t issued = 0;
    int init(int device)
    {
        if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
            return KFEC_EHIP;
        return KFEC_OK;
    }
    // called after the arena grew to `used` bytes: start the copy of the finished bytes once a chunk is ready
    void grow(const Pinned &h, const Device &d, size_t used)
    {
        if (used - issued < kUploadChunk) return;
        if (hipMemcpyAsync(static_cast<uint8_t *>(d.p) + issued, static_cast<const uint8_t *>(h.p) + issued,
                           used - issued, hipMemcpyHostToDevice, cs) == hipSuccess)
            issued = used;  // on failure the bytes are simply copied again by finish()
    }
    // copy the tail and make `s` wait for every upload
    int finish(const Pinned &h, const Device &d, size_t used, hipStream_t s)
    {
        if (issued == 0) {  // nothing went up early (a small flush): one copy on s, no cross-stream event
            return (used == 0 || hipMemcpyAsync(d.p, h.p, used, hipMemcpyHostToDevice, s) == hipSuccess) ? KFEC_OK
                                                                                                        : KFEC_EHIP;
        }
        if (used > issued && hipMemcpyAsync(static_cast<uint8_t *>(d.p) + issued, static_cast<const uint8_t *>(h.p) + issued,
                                            used - issued, hipMemcpyHostToDevice, cs) != hipSuccess)
            return KFEC_EHIP;
        issued = 0;
        if (hipEventRecord(ev, cs) != hipSuccess || hipStreamWaitEvent(s, ev, 0) != hipSuccess) return KFEC_EHIP;
        return KFEC_OK;
    }
    ~Upload()
    {
        if (cs) (void)hipStreamSynchronize(cs);
        if (ev) (void)hipEventDestroy(ev);
        if (cs) (void)hipStreamDestroy(cs);
    }
};

// Make room for `need` more bytes in a staging arena holding `used` bytes when nothing is queued (so a flush
// cannot free anything): the partial / waiting groups of many connections can outgrow the initial
// max_groups-sized arena.  Doubles the pinned and the device arena; the upload restarts from byte 0.
int grow_arena(Pinned &h, Device &d, Upload &up, size_t used, size_t need, size_t &cap)
{
    size_t ncap = std::max<size_t>(cap, 4096);
    while (used + need > ncap) ncap *= 2;
    if (up.cs && hipStreamSynchronize(up.cs) != hipSuccess) return KFEC_EHIP;
    Pinned nh;
    Device nd;
    if (nh.ensure(ncap) || nd.ensure(ncap)) return KFEC_ENOMEM;
    if (used) std::memcpy(nh.p, h.p, used);
    std::swap(h.p, nh.p);
    std::swap(h.n, nh.n);
    std::swap(d.p, nd.p);
    std::swap(d.n, nd.n);
    up.issued = 0;
    cap = ncap;
    return KFEC_OK;
}

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

}  // namespace

// ---- send ------------------------------------------------------------------------------------------------
struct kfec_txq {
    const kfec_ctx *ctx = nullptr;
    size_t K = 0, N = 0, R = 0, G = 0, mtu = 0, slot = 0;  // slot: datagram stride of a kfec_tx group cache
    size_t n = 0;                                          // complete groups queued
    size_t used = 0;  // staged datagram bytes (packed back to back at 4-byte offsets: one H2D of these)
    size_t cap = 0;   // staging arena bytes
    std::vector<kfec_tx *> txs;  // the senders whose partial groups live in the arena
    // h_meta: the per-group tables, filled at [0, GK*8) off, [m_len, +GK*2) len, [m_sn, +G*4) sn, [m_conv, +G*4)
    // conv; a flush packs the used parts back to back and sends them in ONE copy (small flushes are
    // latency-bound: each DMA costs microseconds to set up).  h_res: the redundant packets [n][R], then their
    // lengths, again one copy back.
    Pinned h_dg, h_meta, h_res;
    size_t m_len = 0, m_sn = 0, m_conv = 0;
    std::vector<uint64_t> tags;
    Device d_dg, d_meta, d_par, d_align, d_res;
    uint64_t *h_off() const { return h_meta.as<uint64_t>(); }
    uint16_t *h_len() const { return reinterpret_cast<uint16_t *>(h_meta.as<uint8_t>() + m_len); }
    uint32_t *h_sn() const { return reinterpret_cast<uint32_t *>(h_meta.as<uint8_t>() + m_sn); }
    uint32_t *h_conv() const { return reinterpret_cast<uint32_t *>(h_meta.as<uint8_t>() + m_conv); }
    Upload up;  // declared after the buffers: destroyed (and drained) before them
};

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
// senders are reclaimed instead of doubling memory.  Any early upload is drained and restarted.
int tx_compact(kfec_txq *q)
{
    if (q->up.cs && hipStreamSynchronize(q->up.cs) != hipSuccess) return KFEC_EHIP;
    q->up.issued = 0;
    struct Part {
        uint64_t off;
        size_t len;
        uint64_t *rec;  // where the offset is recorded
        bool operator<(const Part &o) const { return off < o.off; }
    };
    std::vector<Part> part;
    for (kfec_tx *tx : q->txs)
        for (size_t i = 0; i < tx->cached; ++i) part.push_back({tx->cache_off[i], tx->cache_len[i], &tx->cache_off[i]});
    std::sort(part.begin(), part.end());
    size_t at = 0;
    for (const Part &p : part) {
        if (p.len && at != p.off) std::memmove(q->h_dg.as<uint8_t>() + at, q->h_dg.as<uint8_t>() + p.off, p.len);
        *p.rec = at;
        at += round4(p.len);
    }
    q->used = at;
    return KFEC_OK;
}

}  // namespace

extern "C" {

size_t kfec_txq_capacity(const kfec_txq *q) { return q ? q->cap : 0; }

int kfec_txq_create(const kfec_ctx *ctx, size_t max_groups, size_t max_datagram, kfec_txq **out)
{
    if (!out) return KFEC_EINVAL;
    *out = nullptr;
    if (!ctx || !max_groups || max_datagram + KFEC_FEC_CONTAINER_HEADER > 0xFFFF) return KFEC_EINVAL;
    kfec_txq *q = new (std::nothrow) kfec_txq;
    if (!q) return KFEC_ENOMEM;
    q->ctx = ctx;
    q->K = kfec_get_K(ctx);
    q->N = kfec_get_N(ctx);
    q->R = q->N - q->K;
    q->G = max_groups;
    q->mtu = max_datagram;
    q->slot = std::max<size_t>(round4(max_datagram), 4);
    const size_t G = q->G, K = q->K, GK = G * K, R1 = std::max<size_t>(q->R, 1);
    const size_t pitch = round4(max_datagram + KFEC_FEC_CONTAINER_HEADER);
    const size_t pkt_pitch = round4(KFEC_PKT_REDUNDANT_HEADER + max_datagram + KFEC_FEC_CONTAINER_HEADER);
    // every buffer up front: a flush then costs copies and kernels only (pinning memory takes milliseconds)
    q->m_len = GK * 8;
    q->m_sn = round8(GK * 10);
    q->m_conv = q->m_sn + G * 4;
    const size_t meta = q->m_conv + G * 4, res = G * R1 * (pkt_pitch + 2);
    if (q->h_dg.ensure(GK * q->slot) || q->h_meta.ensure(meta) || q->h_res.ensure(res) ||
        q->d_dg.ensure(GK * q->slot) || q->d_meta.ensure(meta) || q->d_res.ensure(res) ||
        q->d_par.ensure(G * R1 * pitch) || q->d_align.ensure(G * 2)) {
        delete q;
        return KFEC_ENOMEM;
    }
    if (q->up.init(kfec_device(ctx))) {
        delete q;
        return KFEC_EHIP;
    }
    q->cap = GK * q->slot;
    q->tags.resize(q->G);
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
    if (!tx || !pkt || !pkt_len || (len && !datagram)) return KFEC_EINVAL;
    kfec_txq *q = tx->q;
    if (len > q->mtu || kn_changed(q->ctx, q->K, q->N)) return KFEC_EINVAL;
    const bool completes = tx->conv != 0 && tx->cached + 1 == q->K;
    if (completes && q->n == q->G) return KFEC_ENOMEM;
    if (tx->conv != 0 && q->used + round4(len) > q->cap) {
        if (q->n) return KFEC_ENOMEM;  // a flush frees the queued groups' bytes
        int rc = tx_compact(q);        // first reclaim what no partial group holds any more
        if (!rc && q->used + round4(len) > q->cap) rc = grow_arena(q->h_dg, q->d_dg, q->up, q->used, round4(len), q->cap);
        if (rc) return rc;
    }
    // create_fec_data_packet (connections.cpp:395-411), sub_sn = fec_snd_sub_sn++ (client.cpp:805-806)
    put_le32(pkt, timestamp);
    put_be32(pkt + 4, tx->sn);
    pkt[8] = tx->sub_sn++;
    if (len) std::memcpy(pkt + KFEC_PKT_DATA_HEADER, datagram, len);
    *pkt_len = KFEC_PKT_DATA_HEADER + len;
    if (tx->conv == 0) {  // client.cpp:811-815
        tx->sub_sn = 0;
        return KFEC_OK;
    }
    if (len) std::memcpy(q->h_dg.as<uint8_t>() + q->used, datagram, len);
    tx->cache_off[tx->cached] = q->used;
    tx->cache_len[tx->cached++] = (uint16_t)len;
    q->used += round4(len);
    if (!completes) return KFEC_OK;
    // the group is complete: it takes queue slot n (compact_into_container + encode run at the flush)
    const size_t g = q->n;
    for (size_t i = 0; i < q->K; ++i) {
        q->h_off()[g * q->K + i] = tx->cache_off[i];
        q->h_len()[g * q->K + i] = tx->cache_len[i];
    }
    q->up.grow(q->h_dg, q->d_dg, q->used);
    q->h_sn()[g] = tx->sn;
    q->h_conv()[g] = tx->conv;
    q->tags[g] = tx->tag;
    q->n = g + 1;
    tx->cached = 0;  // fec_snd_cache.clear(), client.cpp:830-832
    tx->sub_sn = 0;
    tx->sn++;
    return KFEC_OK;
}

int kfec_txq_flush(kfec_txq *q, uint32_t timestamp, kfec_packet_cb cb, void *user, void *stream)
{
    if (!q) return KFEC_EINVAL;
    const size_t n = q->n;
    if (n == 0) return KFEC_OK;
    if (kn_changed(q->ctx, q->K, q->N)) return KFEC_EINVAL;  // the coder was reset: recreate the queue
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t K = q->K, R = q->R;
    const size_t B = q->mtu + KFEC_FEC_CONTAINER_HEADER, pitch = round4(B);
    const size_t pkt_pitch = round4(KFEC_PKT_REDUNDANT_HEADER + B);
    const size_t nk = n * K;
    // pack the used tables back to back (each destination lies below its source, and below the sources still
    // to be moved): [off nk*8][len nk*2][pad][sn n*4][conv n*4]
    uint8_t *hm = q->h_meta.as<uint8_t>();
    const size_t L = nk * 8, S = round8(L + nk * 2), C = S + n * 4, T = C + n * 4;
    std::memmove(hm + L, hm + q->m_len, nk * 2);
    std::memmove(hm + S, hm + q->m_sn, n * 4);
    std::memmove(hm + C, hm + q->m_conv, n * 4);
    uint8_t *dm = q->d_meta.as<uint8_t>();
    const uint64_t *d_off = reinterpret_cast<const uint64_t *>(dm);
    const uint16_t *d_len = reinterpret_cast<const uint16_t *>(dm + L);
    if (q->up.finish(q->h_dg, q->d_dg, q->used, s) ||
        hipMemcpyAsync(dm, hm, T, hipMemcpyHostToDevice, s) != hipSuccess)
        return KFEC_EHIP;
    const size_t arena = std::max<size_t>(q->used, 4);
    int rc = kfec_encode_framed_batch(q->ctx, n, q->d_dg.p, arena, d_off, d_len, B, pitch, q->d_par.p,
                                      q->d_align.as<uint16_t>(), stream);
    if (rc) return rc;
    const size_t P = n * R * pkt_pitch;  // [n][R] compact redundant packets, then their lengths
    if (R) {
        uint8_t *dr = q->d_res.as<uint8_t>();
        rc = kfec_pack_batch(q->ctx, n, KFEC_PACK_REDUNDANT | KFEC_PACK_COMPACT, q->d_dg.p, arena, d_off, d_len, pitch,
                             q->d_par.p, q->d_align.as<uint16_t>(), reinterpret_cast<const uint32_t *>(dm + S),
                             reinterpret_cast<const uint32_t *>(dm + C), timestamp, dr, pkt_pitch,
                             reinterpret_cast<uint16_t *>(dr + P), stream);
        if (rc) return rc;
        if (hipMemcpyAsync(q->h_res.p, dr, P + n * R * 2, hipMemcpyDeviceToHost, s) != hipSuccess) return KFEC_EHIP;
    }
    if (hipStreamSynchronize(s) != hipSuccess) return KFEC_EHIP;
    const uint32_t *sn = reinterpret_cast<const uint32_t *>(hm + S);
    const uint8_t *pk = q->h_res.as<uint8_t>();
    const uint16_t *pk_len = reinterpret_cast<const uint16_t *>(pk + P);
    for (size_t g = 0; g < n && cb; ++g)
        for (size_t r = 0; r < R; ++r) {
            const uint16_t len = pk_len[g * R + r];
            if (len) cb(user, q->tags[g], sn[g], (uint8_t)(K + r), pk + (g * R + r) * pkt_pitch, len);
        }
    q->n = 0;
    return tx_compact(q);  // keep the partial groups, at the front of the arena
}

}  // extern "C"

// ---- receive ---------------------------------------------------------------------------------------------
struct kfec_rxq {
    const kfec_ctx *ctx = nullptr;
    size_t K = 0, N = 0, R = 0, G = 0, max_shard = 0, slot = 0;
    size_t n = 0;     // groups queued for decoding
    size_t used = 0;  // arena bytes staged (shards packed back to back at 4-byte offsets: one H2D of these)
    size_t cap = 0;   // staging arena bytes
    std::vector<kfec_rx *> rxs;  // the receivers whose cached shards live in the arena
    // h_meta: [0, GN*8) off, [m_len, +GN*2) len, [m_pres, +G*32) present, packed back to back at a flush and
    // sent in one copy; h_res: recovered framed shards [n][R], then their data indices (one copy)
    Pinned h_arena, h_meta, h_res;
    size_t m_len = 0, m_pres = 0;
    uint64_t *h_off() const { return h_meta.as<uint64_t>(); }
    uint16_t *h_len() const { return reinterpret_cast<uint16_t *>(h_meta.as<uint8_t>() + m_len); }
    uint64_t *h_present() const { return reinterpret_cast<uint64_t *>(h_meta.as<uint8_t>() + m_pres); }
    std::vector<uint64_t> tags;
    std::vector<uint32_t> sns;
    Device d_arena, d_meta, d_align, d_st, d_ws, d_res;
    Upload up;
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
    if (q->up.cs && hipStreamSynchronize(q->up.cs) != hipSuccess) return KFEC_EHIP;
    q->up.issued = 0;
    struct Part {
        uint64_t *off;
        size_t len;
        bool operator<(const Part &o) const { return *off < *o.off; }
    };
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
    size_t at = 0;
    for (const Part &p : part) {
        if (p.len && at != *p.off) std::memmove(q->h_arena.as<uint8_t>() + at, q->h_arena.as<uint8_t>() + *p.off, p.len);
        *p.off = at;
        at += round4(p.len);
    }
    q->used = at;
    return KFEC_OK;
}

// a decodable group takes queue slot q->n: its shards are already in the arena
void rx_enqueue(kfec_rxq *q, uint64_t tag, uint32_t sn, const RxGroup &grp)
{
    const size_t g = q->n;
    uint64_t *present = q->h_present() + g * 4;
    present[0] = present[1] = present[2] = present[3] = 0;
    // a sub_sn beyond N is cached by the reference (it counts towards size()) but never selected usefully
    for (unsigned s = 0; s < q->N; ++s) {
        if (!grp.test(s)) continue;
        const size_t e = g * q->N + s;
        q->h_off()[e] = grp.off[s];
        q->h_len()[e] = grp.len[s];
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
    q->K = kfec_get_K(ctx);
    q->N = kfec_get_N(ctx);
    q->R = q->N - q->K;
    q->G = max_groups;
    q->max_shard = max_shard;
    q->slot = round4(max_shard);
    const size_t G = q->G, GN = G * q->N, R1 = std::max<size_t>(q->R, 1);
    const size_t pitch = round4(max_shard);
    q->m_len = GN * 8;
    q->m_pres = round8(GN * 10);
    const size_t meta = q->m_pres + G * 32, res = G * R1 * (pitch + 3);
    if (q->h_arena.ensure(GN * q->slot) || q->h_meta.ensure(meta) || q->h_res.ensure(res) ||
        q->d_arena.ensure(GN * q->slot) || q->d_meta.ensure(meta) || q->d_res.ensure(res) ||
        q->d_align.ensure(G * 2) || q->d_st.ensure(G) ||
        q->d_ws.ensure(kfec_decode_workspace_size(ctx, G))) {
        delete q;
        return KFEC_ENOMEM;
    }
    if (q->up.init(kfec_device(ctx))) {
        delete q;
        return KFEC_EHIP;
    }
    q->cap = GN * q->slot;
    q->tags.resize(q->G);
    q->sns.resize(q->G);
    *out = q;
    return KFEC_OK;
}

void kfec_rxq_destroy(kfec_rxq *q) { delete q; }

size_t kfec_rxq_pending(const kfec_rxq *q) { return q ? q->n : 0; }

size_t kfec_rxq_capacity(const kfec_rxq *q) { return q ? q->cap : 0; }

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
    if (store && q->used + round4(plen) > q->cap) {
        if (q->n) return KFEC_ENOMEM;  // a flush frees the queued groups' bytes
        int rc = rx_compact(q);        // first reclaim restored / evicted groups' bytes and overwritten duplicates
        if (!rc && q->used + round4(plen) > q->cap)
            rc = grow_arena(q->h_arena, q->d_arena, q->up, q->used, round4(plen), q->cap);
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
        if (plen) std::memcpy(q->h_arena.as<uint8_t>() + q->used, payload, plen);
        grp->off[sub] = q->used;
        grp->len[sub] = (uint16_t)plen;
        q->used += round4(plen);
        q->up.grow(q->h_arena, q->d_arena, q->used);
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

int kfec_rxq_flush(kfec_rxq *q, kfec_datagram_cb cb, void *user, void *stream)
{
    if (!q) return KFEC_EINVAL;
    const size_t n = q->n;
    if (n == 0) return KFEC_OK;
    if (kn_changed_rx(q)) return KFEC_EINVAL;  // the coder was reset: recreate the queue
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const size_t N = q->N, R = q->R;
    const size_t B = q->max_shard, pitch = round4(B);
    const size_t nn = n * N;
    // pack the used tables back to back: [off nn*8][len nn*2][pad][present n*32]
    uint8_t *hm = q->h_meta.as<uint8_t>();
    const size_t L = nn * 8, P = round8(L + nn * 2), T = P + n * 32;
    std::memmove(hm + L, hm + q->m_len, nn * 2);
    std::memmove(hm + P, hm + q->m_pres, n * 32);
    uint8_t *dm = q->d_meta.as<uint8_t>();
    if (q->up.finish(q->h_arena, q->d_arena, q->used, s) ||
        hipMemcpyAsync(dm, hm, T, hipMemcpyHostToDevice, s) != hipSuccess)
        return KFEC_EHIP;
    // results: [n][R] recovered framed shards, then their data indices (one copy back).  extract_from_container
    // (data_operations.cpp:697-704) is only "skip the BE16 length": done here on the host at the callback, so
    // no unframe pass and no second copy of the recovered bytes
    const size_t D = n * R * pitch;
    uint8_t *dr = q->d_res.as<uint8_t>();
    uint8_t *d_idx = dr + D;
    // recv compact_into_container + decode fused: the chosen shares are framed on the fly from the arena
    int rc = kfec_decode_framed_batch(q->ctx, n, q->d_arena.p, std::max<size_t>(q->used, 4),
                                      reinterpret_cast<const uint64_t *>(dm), reinterpret_cast<const uint16_t *>(dm + L),
                                      reinterpret_cast<const uint64_t *>(dm + P), B, pitch, dr, d_idx,
                                      q->d_st.as<uint8_t>(), q->d_align.as<uint16_t>(), q->d_ws.p, stream);
    if (rc) return rc;
    if (R && hipMemcpyAsync(q->h_res.p, dr, D + n * R, hipMemcpyDeviceToHost, s) != hipSuccess) return KFEC_EHIP;
    if (hipStreamSynchronize(s) != hipSuccess) return KFEC_EHIP;
    const uint8_t *hr = q->h_res.as<uint8_t>();
    const uint8_t *rec_idx = hr + D;
    for (size_t g = 0; g < n && cb && R; ++g)
        for (size_t t = 0; t < R; ++t) {
            const uint8_t idx = rec_idx[g * R + t];
            if (idx == 0xFF) continue;
            const uint8_t *shard = hr + (g * R + t) * pitch;
            const size_t len = ((size_t)shard[0] << 8) | shard[1];  // ntohs(data_length)
            if (len + KFEC_FEC_CONTAINER_HEADER > B) continue;     // inconsistent group (kfec_unframe_batch's 0xFFFF)
            cb(user, q->tags[g], q->sns[g], idx, shard + KFEC_FEC_CONTAINER_HEADER, len);
        }
    q->n = 0;
    return rx_compact(q);  // keep the shards of the groups still waiting for K shares
}

}  // extern "C"
