// side_effects.cpp -- what the resident per-call worker (kfec_worker.hip) does to other threads of the process.
//
// Thread A calls kfec_encode (one 20:3 group, B = 1440, from host memory) back to back for --busy-ms; thread B,
// 50 ms into that, runs ONE operation and times it.  An operation that waits for the worker's stream (HIP's
// hipFree / hipHostFree synchronise every stream of the device) would take until A stops plus the worker's idle
// exit, unless the worker bounds its own residency.  One JSON line per operation:
//   {"op": ..., "ms": duration of the operation, "a_calls": calls A made, "a_us": A's mean call time,
//    "a_ok": A's calls all correct, "rc": the operation's return code}
// Usage: tools/side_effects [busy_ms] [op ...]      ops: see kOps below (default: all)
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "kfec.h"
#include "kfec_aead.h"
#include "kfec_pipeline.h"

namespace {

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

struct Op {
    const char *name;
    std::function<int()> run;
};

}  // namespace

int main(int argc, char **argv)
{
    const double busy_ms = argc > 1 ? atof(argv[1]) : 400.0;
    std::vector<std::string> want;
    for (int i = 2; i < argc; ++i) want.push_back(argv[i]);

    const size_t K = 20, N = 23, B = 1440, R = N - K;
    kfec_ctx *ca = nullptr, *cb = nullptr;
    if (kfec_create(K, N, &ca) || kfec_create(10, 13, &cb)) {
        fprintf(stderr, "kfec_create failed\n");
        return 1;
    }
    std::vector<uint8_t> data(K * B), par(R * B), ref(R * B);
    for (size_t i = 0; i < data.size(); ++i) data[i] = (uint8_t)(i * 131 + 7);
    if (kfec_encode(ca, data.data(), K * B, B, ref.data())) return 1;  // (the answer A's calls must give)
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipStream_t own = nullptr;
    (void)hipStreamCreateWithFlags(&own, hipStreamNonBlocking);
    hipMemPool_t pool = nullptr;
    {
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        (void)hipMemPoolCreate(&pool, &props);
        uint64_t thr = ~0ull;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }

    const Op kOps[] = {
        {"kfec_reset", [&] { return kfec_reset(cb, 12, 15) | kfec_reset(cb, 10, 13); }},
        {"kfec_create_destroy", [&] {
             kfec_ctx *c = nullptr;
             const int rc = kfec_create(8, 11, &c);
             kfec_destroy(c);
             return rc;
         }},
        {"kfec_aead_create_destroy", [&] {
             kfec_aead *a = nullptr;
             const int rc = kfec_aead_create(KFEC_AEAD_CHACHA20, "pw", 2, &a);
             kfec_aead_destroy(a);
             return rc;
         }},
        {"kfec_txq_create_destroy", [&] {
             kfec_txq *q = nullptr;
             const int rc = kfec_txq_create(cb, 64, 1400, &q);
             kfec_txq_destroy(q);
             return rc;
         }},
        {"hipMalloc_hipFree", [&] {
             void *p = nullptr;
             int rc = hipMalloc(&p, 1 << 20) != hipSuccess;
             rc |= hipFree(p) != hipSuccess;
             return rc;
         }},
        {"hipHostMalloc_hipHostFree", [&] {
             void *p = nullptr;
             int rc = hipHostMalloc(&p, 1 << 20, 0) != hipSuccess;
             rc |= hipHostFree(p) != hipSuccess;
             return rc;
         }},
        {"pool_alloc_free_async", [&] {
             void *p = nullptr;
             int rc = hipMallocFromPoolAsync(&p, 1 << 20, pool, own) != hipSuccess;
             rc |= hipFreeAsync(p, own) != hipSuccess;
             rc |= hipStreamSynchronize(own) != hipSuccess;
             return rc;
         }},
        {"hipStreamCreate_Destroy", [&] {
             hipStream_t s = nullptr;
             int rc = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess;
             rc |= hipStreamDestroy(s) != hipSuccess;
             return rc;
         }},
        {"own_stream_sync", [&] { return (int)(hipStreamSynchronize(own) != hipSuccess); }},
        {"hipDeviceSynchronize", [&] { return (int)(hipDeviceSynchronize() != hipSuccess); }},
    };

    int bad = 0;
    for (const Op &op : kOps) {
        if (!want.empty()) {
            bool hit = false;
            for (auto &w : want) hit |= w == op.name;
            if (!hit) continue;
        }
        std::atomic<bool> stop{false};
        std::atomic<long> calls{0};
        std::atomic<bool> a_ok{true};
        double a_ms = 0;
        std::thread a([&] {
            std::vector<uint8_t> p(R * B);
            const auto t0 = clk::now();
            while (ms_since(t0) < busy_ms) {
                if (kfec_encode(ca, data.data(), K * B, B, p.data()) || std::memcmp(p.data(), ref.data(), p.size()))
                    a_ok = false;
                calls.fetch_add(1, std::memory_order_relaxed);
            }
            a_ms = ms_since(t0);
            stop = true;
        });
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        const bool a_running = !stop.load();
        const auto t0 = clk::now();
        const int rc = op.run();
        const double ms = ms_since(t0);
        const bool a_still = !stop.load();  // A was still calling when the operation returned
        a.join();
        printf("{\"op\": \"%s\", \"ms\": %.3f, \"rc\": %d, \"busy_ms\": %.0f, \"a_running_at_start\": %s, "
               "\"a_running_at_end\": %s, \"a_calls\": %ld, \"a_us\": %.2f, \"a_ok\": %s}\n",
               op.name, ms, rc, busy_ms, a_running ? "true" : "false", a_still ? "true" : "false", calls.load(),
               calls.load() ? a_ms * 1e3 / calls.load() : 0.0, a_ok ? "true" : "false");
        fflush(stdout);
        bad |= rc != 0 || !a_ok;
        std::this_thread::sleep_for(std::chrono::milliseconds(60));  // the worker idles out between operations
    }
    (void)hipMemPoolDestroy(pool);
    (void)hipStreamDestroy(own);
    kfec_destroy(cb);
    kfec_destroy(ca);
    return bad;
}
