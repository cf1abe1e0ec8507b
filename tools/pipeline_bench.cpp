// pipeline_bench.cpp -- host-memory end to end of the batched FEC path (include/kfec_pipeline.h):
// C connections, each sending datagrams through kfec_tx (data packets built on the host at once, complete
// groups coded on the GPU at each flush), then the packets of every group minus `loss` of them per group
// pushed through kfec_rx (receive cache + fec_find_missings scan on the host, decodable groups decoded on the
// GPU at each flush).  Reports host-side per-packet cost, GPU flush time (including the pinned H2D / D2H
// copies) and the datagram payload rate of each direction, on ONE host thread, and checks every recovered
// datagram.
// Build: g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include tools/pipeline_bench.cpp
//        -o tools/pipeline_bench -L kcptube_amd -lkfec -L /opt/rocm/lib -lamdhip64 -pthread
//        -Wl,-rpath,'$ORIGIN/../kcptube_amd'
// Usage: tools/pipeline_bench [K N mtu groups_per_flush flushes loss threads]
// PB_SEAL=none|plain_xor|chacha20|xchacha20|aes_gcm|aes_ocb: the sealed queue (kfec_txq_seal with
// KFEC_TXQ_DEFER_DATA, so every packet, data packets included, is sealed on the device and leaves at the flush)
// and, on receive, kfec_opener (decrypt_data on the device) ahead of kfec_rx_push.  Sealed runs also report
// the added send latency of deferring the data packets: per data packet, the time from its kfec_tx_send to its
// emission by the flush (the reference sends it inside the same fec_maker call, client.cpp:805-807), as
// percentiles over every data packet of the run.
// With threads > 1 every thread runs its own sender + receiver over its own queues and HIP stream (one
// context shared); all_threads_tx_plus_rx_GiBps = the payload every thread sent and received / the slowest
// thread's wall time (its data generation excluded).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "kfec_pipeline.h"

using clk = std::chrono::steady_clock;

// redundant packets land in one preallocated buffer (stride = max packet), so the flush time is the
// library's, not the allocator's
struct Sink {
    std::vector<uint8_t> buf;
    std::vector<uint16_t> len;
    size_t stride = 0, n = 0;
    const uint8_t *pkt(size_t i) const { return buf.data() + i * stride; }
};

static void on_pkt(void *u, uint64_t, uint32_t, uint8_t, const uint8_t *p, size_t len)
{
    auto *s = static_cast<Sink *>(u);
    std::memcpy(s->buf.data() + s->n * s->stride, p, len);
    s->len[s->n++] = (uint16_t)len;
}

// sealed sink: every emitted packet (data and redundant, in emission order) into one buffer, with the emission
// time of each data packet (sn * K + sub_sn indexes the send-time table)
struct SealSink {
    Sink s;
    size_t K = 0;
    const std::vector<clk::time_point> *sent = nullptr;
    std::vector<double> *delay_us = nullptr;
    std::vector<uint8_t> is_data;
};

static void on_sealed(void *u, uint64_t, uint32_t sn, uint8_t sub, const uint8_t *p, size_t len)
{
    auto *z = static_cast<SealSink *>(u);
    z->is_data.push_back(sub < z->K);
    if (sub < z->K && z->delay_us)
        z->delay_us->push_back(std::chrono::duration<double, std::micro>(clk::now() - (*z->sent)[(size_t)sn * z->K + sub]).count());
    on_pkt(&z->s, 0, sn, sub, p, len);
}

struct Rec {
    size_t n = 0, bytes = 0, bad = 0;
    const std::vector<std::vector<uint8_t>> *orig;
    size_t K;
};

static void on_dg(void *u, uint64_t tag, uint32_t sn, uint8_t idx, const uint8_t *d, size_t len)
{
    auto *r = static_cast<Rec *>(u);
    r->n++;
    r->bytes += len;
    (void)tag;
    const auto &o = (*r->orig)[(size_t)sn * r->K + idx];
    if (o.size() != len || std::memcmp(o.data(), d, len)) r->bad++;
}

struct Params {
    size_t K, N, mtu, G, loss;
    int flushes;
    int seal = KFEC_TXQ_SEAL_OFF;    // PB_SEAL: KFEC_SEAL_* or KFEC_AEAD_*
    const kfec_aead *aead = nullptr;
};

struct Result {
    double t_tx_host = 0, t_tx_flush = 0, t_rx_host = 0, t_rx_flush = 0, t_rx_open = 0, wall = 0;
    size_t recovered = 0, bad = 0;
    int rc = 0;
    std::vector<double> delay_us;  // sealed: send -> emission of every data packet
};

struct PushCtx {
    kfec_rx *rx;
    size_t own = 0, bad_open = 0;
    int rc = 0;
};

static void on_opened(void *u, uint64_t, const uint8_t *plain, size_t len, int ok)
{
    auto *c = static_cast<PushCtx *>(u);
    if (!ok) {
        c->bad_open++;
        return;
    }
    const uint8_t *d;
    size_t dn;
    if (kfec_rx_push(c->rx, plain, len, &d, &dn) < 0) c->rc = 1;
    c->own += dn;
}

// The sealed pipeline: deferred, device-sealed send; device open + receive.  Every group loses its first
// `loss` data packets.
static void run_sealed(kfec_ctx *ctx, const Params &pa, uint64_t seed, hipStream_t stream, Result &res)
{
    const size_t K = pa.K, N = pa.N, mtu = pa.mtu, G = pa.G, loss = pa.loss, R = N - K;
    const int flushes = pa.flushes;
    kfec_txq *tq;
    kfec_rxq *rq;
    if (kfec_txq_create(ctx, G, mtu, &tq) || kfec_rxq_create(ctx, G, mtu + 2, &rq)) { res.rc = 1; return; }
    if (kfec_txq_seal(tq, pa.seal, pa.aead, seed, KFEC_TXQ_DEFER_DATA)) { res.rc = 1; return; }
    const size_t max_pkt = mtu + 64;
    kfec_opener *op;
    if (kfec_opener_create(pa.seal, pa.aead, G * N, max_pkt, &op)) { res.rc = 1; return; }
    kfec_tx *tx;
    kfec_rx *rx;
    kfec_tx_create(tq, 0x4B435054, 1, &tx);
    kfec_rx_create(rq, 1, &rx);
    std::mt19937_64 rng(seed);
    const size_t total_groups = G * flushes;
    std::vector<std::vector<uint8_t>> dg(total_groups * K);
    for (auto &d : dg) {
        d.resize(mtu);
        for (size_t i = 0; i < mtu; i += 8) {
            const uint64_t v = rng();
            std::memcpy(d.data() + i, &v, std::min<size_t>(8, mtu - i));
        }
    }
    std::vector<clk::time_point> sent(total_groups * K);
    SealSink z;
    z.K = K;
    z.sent = &sent;
    z.delay_us = &res.delay_us;
    z.s.stride = max_pkt;
    z.s.buf.resize(total_groups * N * max_pkt);
    z.s.len.resize(total_groups * N);
    res.delay_us.reserve(total_groups * K);
    const auto w0 = clk::now();
    for (int f = 0; f < flushes; ++f) {
        z.delay_us = f ? &res.delay_us : nullptr;  // (flush 0 is the warm-up: first launch of every kernel)
        auto t0 = clk::now();
        for (size_t g = f * G; g < (f + 1) * G; ++g)
            for (size_t i = 0; i < K; ++i) {
                sent[g * K + i] = clk::now();
                if (kfec_tx_send(tx, dg[g * K + i].data(), mtu, 1, nullptr, nullptr)) { res.rc = 1; return; }
            }
        auto t1 = clk::now();
        if (kfec_txq_flush(tq, 1, on_sealed, &z, stream)) { res.rc = 1; return; }
        auto t2 = clk::now();
        if (f == 0) continue;
        res.t_tx_host += std::chrono::duration<double>(t1 - t0).count();
        res.t_tx_flush += std::chrono::duration<double>(t2 - t1).count();
    }
    if (z.s.n != total_groups * N) { res.rc = 4; return; }
    // receive: the emission order is per group its K data packets, then its R redundant ones
    Rec rec;
    rec.orig = &dg;
    rec.K = K;
    PushCtx pc{rx};
    for (int f = 0; f < flushes; ++f) {
        auto t0 = clk::now();
        for (size_t g = f * G; g < (f + 1) * G; ++g)
            for (size_t q = 0; q < N; ++q) {
                if (q < loss) continue;  // the group's first `loss` data packets are lost
                const size_t i = g * N + q;
                if (kfec_opener_add(op, z.s.pkt(i), z.s.len[i], 0)) { res.rc = 1; return; }
            }
        auto t1 = clk::now();
        if (kfec_opener_flush(op, on_opened, &pc, stream) || pc.rc) { res.rc = 1; return; }
        auto t2 = clk::now();
        if (kfec_rxq_flush(rq, on_dg, &rec, stream)) { res.rc = 1; return; }
        auto t3 = clk::now();
        if (f == 0) continue;
        res.t_rx_host += std::chrono::duration<double>(t1 - t0).count();
        res.t_rx_open += std::chrono::duration<double>(t2 - t1).count();
        res.t_rx_flush += std::chrono::duration<double>(t3 - t2).count();
    }
    (void)w0;  // the timed flushes only (the warm-up flush is left out of every figure)
    res.wall = res.t_tx_host + res.t_tx_flush + res.t_rx_host + res.t_rx_open + res.t_rx_flush;
    res.recovered = rec.n;
    res.bad = rec.bad + pc.bad_open;
    if (res.bad != 0 || rec.n != total_groups * loss) res.rc = 3;
    kfec_tx_destroy(tx);
    kfec_rx_destroy(rx);
    kfec_opener_destroy(op);
    kfec_txq_destroy(tq);
    kfec_rxq_destroy(rq);
}

// One host thread's sender + receiver over its own queues and HIP stream.
static void run(kfec_ctx *ctx, const Params &pa, uint64_t seed, hipStream_t stream, Result &res)
{
    const size_t K = pa.K, N = pa.N, mtu = pa.mtu, G = pa.G, loss = pa.loss, R = N - K;
    const int flushes = pa.flushes;
    kfec_txq *tq;
    kfec_rxq *rq;
    if (kfec_txq_create(ctx, G, mtu, &tq) || kfec_rxq_create(ctx, G, mtu + 2, &rq)) { res.rc = 1; return; }
    kfec_tx *tx;
    kfec_rx *rx;
    kfec_tx_create(tq, 0x4B435054, 1, &tx);
    kfec_rx_create(rq, 1, &rx);
    std::mt19937_64 rng(seed);
    const size_t total_groups = G * flushes;
    std::vector<std::vector<uint8_t>> dg(total_groups * K);
    for (auto &d : dg) {
        d.resize(mtu);
        for (size_t i = 0; i < mtu; i += 8) {
            const uint64_t v = rng();
            std::memcpy(d.data() + i, &v, std::min<size_t>(8, mtu - i));
        }
    }
    // data packets land in one preallocated buffer too (stride mtu + 16)
    const size_t dstride = mtu + 16;
    std::vector<uint8_t> data_pkts(total_groups * K * dstride);
    std::vector<uint16_t> data_len(total_groups * K);
    Sink red;
    red.stride = mtu + 16;
    red.buf.resize(total_groups * R * red.stride);
    red.len.resize(total_groups * R);
    const auto w0 = clk::now();
    for (int f = 0; f < flushes; ++f) {
        auto t0 = clk::now();
        for (size_t g = f * G; g < (f + 1) * G; ++g)
            for (size_t i = 0; i < K; ++i) {
                size_t n = 0;
                if (kfec_tx_send(tx, dg[g * K + i].data(), mtu, 1, data_pkts.data() + (g * K + i) * dstride, &n)) {
                    res.rc = 1;
                    return;
                }
                data_len[g * K + i] = (uint16_t)n;
            }
        auto t1 = clk::now();
        if (kfec_txq_flush(tq, 1, on_pkt, &red, stream)) { res.rc = 1; return; }
        auto t2 = clk::now();
        res.t_tx_host += std::chrono::duration<double>(t1 - t0).count();
        res.t_tx_flush += std::chrono::duration<double>(t2 - t1).count();
    }
    // receive: every group loses `loss` data packets (worst case for the decoder)
    Rec rec;
    rec.orig = &dg;
    rec.K = K;
    size_t own = 0;
    for (int f = 0; f < flushes; ++f) {
        auto t0 = clk::now();
        for (size_t g = f * G; g < (f + 1) * G; ++g) {
            for (size_t i = loss; i < K; ++i) {
                const uint8_t *d;
                size_t dn;
                if (kfec_rx_push(rx, data_pkts.data() + (g * K + i) * dstride, data_len[g * K + i], &d, &dn) < 0) {
                    res.rc = 1;
                    return;
                }
                own += dn;
            }
            for (size_t r = 0; r < R; ++r) {
                if (kfec_rx_push(rx, red.pkt(g * R + r), red.len[g * R + r], nullptr, nullptr) < 0) {
                    res.rc = 1;
                    return;
                }
            }
        }
        auto t1 = clk::now();
        if (kfec_rxq_flush(rq, on_dg, &rec, stream)) { res.rc = 1; return; }
        auto t2 = clk::now();
        res.t_rx_host += std::chrono::duration<double>(t1 - t0).count();
        res.t_rx_flush += std::chrono::duration<double>(t2 - t1).count();
    }
    res.wall = std::chrono::duration<double>(clk::now() - w0).count();
    res.recovered = rec.n;
    res.bad = rec.bad;
    if (rec.bad != 0 || rec.n != total_groups * loss) res.rc = 3;
    kfec_tx_destroy(tx);
    kfec_rx_destroy(rx);
    kfec_txq_destroy(tq);
    kfec_rxq_destroy(rq);
}

int main(int argc, char **argv)
{
    Params pa;
    pa.K = argc > 1 ? atoi(argv[1]) : 20;
    pa.N = argc > 2 ? atoi(argv[2]) : 23;
    pa.mtu = argc > 3 ? atoi(argv[3]) : 1440;
    pa.G = argc > 4 ? atoi(argv[4]) : 16384;
    pa.flushes = argc > 5 ? atoi(argv[5]) : 4;
    pa.loss = argc > 6 ? atoi(argv[6]) : 3;
    const int T = argc > 7 ? std::max(1, atoi(argv[7])) : 1;
    const size_t K = pa.K, R = pa.N - pa.K;
    kfec_ctx *ctx = nullptr;
    if (kfec_create(pa.K, pa.N, &ctx)) { printf("no GPU\n"); return 1; }
    const char *seal = getenv("PB_SEAL");
    std::string seal_name = seal ? seal : "off";
    kfec_aead *aead = nullptr;
    if (seal) {
        const std::string m = seal;
        const int aead_mode = m == "chacha20" ? KFEC_AEAD_CHACHA20 : m == "xchacha20" ? KFEC_AEAD_XCHACHA20
                            : m == "aes_gcm" ? KFEC_AEAD_AES_GCM : m == "aes_ocb" ? KFEC_AEAD_AES_OCB : -1;
        if (aead_mode > 0) {
            if (kfec_aead_create(aead_mode, "pipeline_bench", 14, &aead)) { printf("aead failed\n"); return 1; }
            pa.seal = aead_mode;
            pa.aead = aead;
        } else {
            pa.seal = m == "plain_xor" ? KFEC_SEAL_PLAIN_XOR : KFEC_SEAL_CHECKSUM;
        }
    }
    std::vector<Result> res(T);
    std::vector<hipStream_t> streams(T, nullptr);
    for (int t = 0; t < T; ++t)
        if (T > 1 && hipStreamCreateWithFlags(&streams[t], hipStreamNonBlocking) != hipSuccess) return 1;
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back(seal ? run_sealed : run, ctx, std::cref(pa), 7 + t, streams[t], std::ref(res[t]));
        for (auto &x : th) x.join();
    }
    Result a;  // per-thread averages of the phase times; wall = the slowest thread
    size_t recovered = 0, bad = 0;
    int rc = 0;
    std::vector<double> delay;
    for (const Result &r : res) {
        a.t_tx_host += r.t_tx_host / T; a.t_tx_flush += r.t_tx_flush / T;
        a.t_rx_host += r.t_rx_host / T; a.t_rx_flush += r.t_rx_flush / T; a.t_rx_open += r.t_rx_open / T;
        delay.insert(delay.end(), r.delay_us.begin(), r.delay_us.end());
        a.wall = std::max(a.wall, r.wall);
        recovered += r.recovered;
        bad += r.bad;
        rc = rc ? rc : r.rc;
    }
    const int timed = seal ? pa.flushes - 1 : pa.flushes;  // (sealed runs leave the warm-up flush out)
    const size_t total_groups = pa.G * timed;
    const double payload = (double)total_groups * K * pa.mtu;  // per thread and direction (timed flushes)
    const double npk_tx = (double)total_groups * K, npk_rx = (double)total_groups * (K - pa.loss + R);
    std::sort(delay.begin(), delay.end());
    auto pc = [&](double q) { return delay.empty() ? 0.0 : delay[std::min(delay.size() - 1, (size_t)(q * delay.size()))]; };
    printf("{\"seal\": \"%s\", \"rx_open_ms\": %.3f, \"data_pkt_delay_us_p50\": %.1f, \"data_pkt_delay_us_p90\": %.1f, "
           "\"data_pkt_delay_us_p99\": %.1f, \"data_pkt_delay_us_max\": %.1f, ",
           seal_name.c_str(), a.t_rx_open / std::max(1, pa.flushes - 1) * 1e3, pc(0.5), pc(0.9), pc(0.99), delay.empty() ? 0.0 : delay.back());
    printf("\"metric\": \"batched FEC pipeline, host memory in and out\", \"threads\": %d, \"fec\": \"%zu:%zu\", "
           "\"kcp_mtu\": %zu, \"groups_per_flush\": %zu, \"flushes\": %d, \"loss_per_group\": %zu, "
           "\"tx_host_ns_per_packet\": %.1f, \"tx_flush_ms\": %.3f, \"tx_GiBps\": %.3f, \"tx_flush_only_GiBps\": %.2f, "
           "\"rx_host_ns_per_packet\": %.1f, \"rx_flush_ms\": %.3f, \"rx_GiBps\": %.3f, \"rx_flush_only_GiBps\": %.2f, "
           "\"all_threads_tx_plus_rx_GiBps\": %.2f, "
           "\"recovered\": %zu, \"recovered_expected\": %zu, \"bad\": %zu}\n",
           T, K, R, pa.mtu, pa.G, pa.flushes, pa.loss, a.t_tx_host / npk_tx * 1e9, a.t_tx_flush / timed * 1e3,
           payload / (a.t_tx_host + a.t_tx_flush) / (1 << 30), payload / a.t_tx_flush / (1 << 30),
           a.t_rx_host / npk_rx * 1e9, a.t_rx_flush / timed * 1e3,
           payload / (a.t_rx_host + a.t_rx_open + a.t_rx_flush) / (1 << 30),
           payload / a.t_rx_flush / (1 << 30), 2.0 * T * payload / a.wall / (1 << 30),
           recovered, pa.G * pa.flushes * pa.loss * T, bad);
    for (hipStream_t st : streams)
        if (st) (void)hipStreamDestroy(st);
    if (aead) kfec_aead_destroy(aead);
    kfec_destroy(ctx);
    return rc;
}
