// latency_bench.cpp -- what one call costs on the latency path: the drop-in
// kfec_encode / kfec_decode on ONE fec=20:3 group from host memory (what fecpp_compat.hpp's fec_code::encode /
// decode do per call), and kfec_txq_flush / kfec_rxq_flush of small batches (1 .. 1024 groups), each timed
// over many calls on one host thread.  Prints one JSON line (microseconds per call).
// The reference leg: the reference's own coder (oracle/_ref/libfecpp_ref.so, built from /root/reference's
// fecpp*.cpp by oracle/Makefile; measurement only, loaded with dlopen at run time, never linked) times the same
// single-group encode and 3-loss decode on the same thread in the same run (ref_* keys).
// Build: g++ -O2 -std=c++17 -I include tools/latency_bench.cpp -o tools/latency_bench -L kcptube_amd -lkfec
//        -Wl,-rpath,'$ORIGIN/../kcptube_amd'
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "kfec_pipeline.h"

using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); }

// median and 90th percentile of per-call times (us) of f() over n calls
template <typename F>
static std::string pct(const std::string &name, int n, F &&f)
{
    std::vector<double> v(n);
    for (int i = 0; i < n; ++i) {
        const auto t = clk::now();
        f();
        v[i] = us_since(t);
    }
    std::sort(v.begin(), v.end());
    return ", \"" + name + "_p50_us\": " + std::to_string(v[n / 2]) + ", \"" + name + "_p90_us\": " + std::to_string(v[n * 9 / 10]);
}

static void drop_pkt(void *, uint64_t, uint32_t, uint8_t, const uint8_t *, size_t) {}
static void count_dg(void *u, uint64_t, uint32_t, uint8_t, const uint8_t *, size_t) { ++*static_cast<size_t *>(u); }

int main()
{
    const size_t K = 20, N = 23, R = 3, B = 1440;
    kfec_ctx *ctx = nullptr;
    if (kfec_create(K, N, &ctx)) { printf("no GPU\n"); return 1; }
    std::mt19937_64 rng(5);
    std::vector<uint8_t> data(K * B), par(R * B), out(R * B);
    for (auto &b : data) b = (uint8_t)rng();
    std::string js = "{\"metric\": \"latency path, fec=20:3 B=1440, one host thread (us per call)\"";
    // single group, host memory in and out
    const int reps = 2000;
    if (kfec_worker_ping(ctx) == 0) {  // the resident worker's communication floor (an empty request)
        for (int i = 0; i < 50; ++i) kfec_worker_ping(ctx);
        auto tp = clk::now();
        for (int i = 0; i < reps; ++i) kfec_worker_ping(ctx);
        js += ", \"worker_ping_us\": " + std::to_string(us_since(tp) / reps);
    }
    for (int i = 0; i < 50; ++i)
        if (int rc = kfec_encode(ctx, data.data(), K * B, B, par.data())) { printf("kfec_encode rc %d\n", rc); return 2; }
    auto t0 = clk::now();
    for (int i = 0; i < reps; ++i) kfec_encode(ctx, data.data(), K * B, B, par.data());
    js += ", \"kfec_encode_1_group_us\": " + std::to_string(us_since(t0) / reps);
    js += pct("kfec_encode_1_group", reps, [&] { kfec_encode(ctx, data.data(), K * B, B, par.data()); });
    std::vector<size_t> ids;
    std::vector<const uint8_t *> ptrs;
    for (size_t s = 3; s < K; ++s) { ids.push_back(s); ptrs.push_back(data.data() + s * B); }
    for (size_t r = 0; r < R; ++r) { ids.push_back(K + r); ptrs.push_back(par.data() + r * B); }
    size_t out_ids[3], n_out = 0;
    for (int i = 0; i < 50; ++i)
        if (int rc = kfec_decode(ctx, ids.data(), ptrs.data(), ids.size(), B, out_ids, out.data(), &n_out)) {
            printf("kfec_decode rc %d\n", rc);
            return 2;
        }
    t0 = clk::now();
    for (int i = 0; i < reps; ++i) kfec_decode(ctx, ids.data(), ptrs.data(), ids.size(), B, out_ids, out.data(), &n_out);
    js += ", \"kfec_decode_1_group_3_lost_us\": " + std::to_string(us_since(t0) / reps);
    js += pct("kfec_decode_1_group_3_lost", reps,
              [&] { kfec_decode(ctx, ids.data(), ptrs.data(), ids.size(), B, out_ids, out.data(), &n_out); });
    js += ", \"worker_requests\": " + std::to_string(kfec_worker_requests());
    // the reference coder on this thread, same group shape, same run
    {
        std::string so = "oracle/_ref/libfecpp_ref.so";
        if (const char *e = getenv("KFEC_REF_SO")) so = e;
        void *h = dlopen(so.c_str(), RTLD_NOW | RTLD_LOCAL);
        using lat_fn = int (*)(size_t, size_t, size_t, size_t, int, double *);
        lat_fn lat = h ? reinterpret_cast<lat_fn>(dlsym(h, "ref_percall_latency")) : nullptr;
        double us[6];
        if (lat && lat(K, N, B, 3, reps, us) == 0) {
            js += ", \"ref_encode_us\": " + std::to_string(us[0]) + ", \"ref_encode_p50_us\": " + std::to_string(us[1]) +
                  ", \"ref_encode_p90_us\": " + std::to_string(us[2]) + ", \"ref_decode_us\": " + std::to_string(us[3]) +
                  ", \"ref_decode_p50_us\": " + std::to_string(us[4]) + ", \"ref_decode_p90_us\": " + std::to_string(us[5]);
        } else {
            js += ", \"ref_error\": \"" + std::string(h ? "ref_percall_latency failed" : "libfecpp_ref.so not found") + "\"";
        }
    }
    bool ok = n_out == 3 && !std::memcmp(out.data(), data.data(), 3 * B);
    // per-call encode cost against K (N = K + 3, B = 1440): the slope is the per-share cost of the call
    for (size_t k : {1, 5, 10, 20}) {
        kfec_ctx *c2 = nullptr;
        if (kfec_create(k, k + 3, &c2)) break;
        for (int i = 0; i < 50; ++i) kfec_encode(c2, data.data(), k * B, B, par.data());
        auto tk = clk::now();
        for (int i = 0; i < reps / 2; ++i) kfec_encode(c2, data.data(), k * B, B, par.data());
        js += ", \"kfec_encode_" + std::to_string(k) + "_3_us\": " + std::to_string(us_since(tk) / (reps / 2));
        kfec_destroy(c2);
    }
    // small flushes of the batched queues
    for (size_t G : {1, 16, 256, 1024}) {
        kfec_txq *tq;
        kfec_rxq *rq;
        kfec_txq_create(ctx, G, B, &tq);
        kfec_rxq_create(ctx, G, B + 2, &rq);
        kfec_tx *tx;
        kfec_rx *rx;
        kfec_tx_create(tq, 7, 1, &tx);
        kfec_rx_create(rq, 1, &rx);
        std::vector<uint8_t> pkt(B + 16);
        std::vector<std::vector<uint8_t>> pk;
        double ttx = 0, trx = 0;
        size_t got = 0;
        const int rounds = G >= 256 ? 20 : 200;
        auto collect = [](void *u, uint64_t, uint32_t, uint8_t, const uint8_t *p, size_t n) {
            static_cast<std::vector<std::vector<uint8_t>> *>(u)->emplace_back(p, p + n);
        };
        for (int r = 0; r < rounds + 2; ++r) {
            pk.clear();
            std::vector<std::vector<uint8_t>> dpk;
            for (size_t g = 0; g < G; ++g)
                for (size_t i = 0; i < K; ++i) {
                    size_t n = 0;
                    kfec_tx_send(tx, data.data() + i * B, B, 1, pkt.data(), &n);
                    if (i >= 3) dpk.emplace_back(pkt.data(), pkt.data() + n);  // 3 data packets lost per group
                }
            auto a = clk::now();
            kfec_txq_flush(tq, 1, collect, &pk, nullptr);
            if (r >= 2) ttx += us_since(a);
            // receive: per group its 17 kept data packets, then its 3 redundant ones
            for (size_t g = 0; g < G; ++g) {
                for (size_t i = 0; i < K - 3; ++i) kfec_rx_push(rx, dpk[g * (K - 3) + i].data(), dpk[g * (K - 3) + i].size(), nullptr, nullptr);
                for (size_t q = 0; q < R; ++q) kfec_rx_push(rx, pk[g * R + q].data(), pk[g * R + q].size(), nullptr, nullptr);
            }
            a = clk::now();
            kfec_rxq_flush(rq, count_dg, &got, nullptr);
            if (r >= 2) trx += us_since(a);
        }
        ok = ok && got == (size_t)(rounds + 2) * G * 3;
        js += ", \"txq_flush_" + std::to_string(G) + "_groups_us\": " + std::to_string(ttx / rounds);
        js += ", \"rxq_flush_" + std::to_string(G) + "_groups_us\": " + std::to_string(trx / rounds);
        kfec_tx_destroy(tx);
        kfec_rx_destroy(rx);
        kfec_txq_destroy(tq);
        kfec_rxq_destroy(rq);
    }
    (void)drop_pkt;
    js += std::string(", \"verified\": ") + (ok ? "true" : "false") + "}";
    printf("%s\n", js.c_str());
    kfec_destroy(ctx);
    return ok ? 0 : 3;
}
