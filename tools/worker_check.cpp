// worker_check.cpp -- single calls through the resident worker (kfec_worker.hip), in an order given on the
// command line: e = encode, d = decode (3 data shards lost; zero data, so zero parity, when no encode ran
// before), one line per call.  Exit status != 0 when a call fails or recovers wrong bytes.
// Build: g++ -O2 -std=c++17 -I include tools/worker_check.cpp -o tools/worker_check -L kcptube_amd -lkfec
//        -Wl,-rpath,'$ORIGIN/../kcptube_amd'
// Usage: tools/worker_check [K N B lost] [sequence, e.g. ed / de / eed]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "kfec.h"

int main(int argc, char **argv)
{
    size_t K = 2, N = 3, B = 16, lost = 1;
    std::string seq = "ed";
    if (argc >= 5) {
        K = strtoul(argv[1], nullptr, 10);
        N = strtoul(argv[2], nullptr, 10);
        B = strtoul(argv[3], nullptr, 10);
        lost = strtoul(argv[4], nullptr, 10);
    }
    if (argc == 2) seq = argv[1];
    if (argc >= 6) seq = argv[5];
    kfec_ctx *ctx = nullptr;
    if (int rc = kfec_create(K, N, &ctx)) { printf("create rc %d\n", rc); return 1; }
    const size_t R = N - K;
    std::mt19937_64 rng(K * 131 + N);
    std::vector<uint8_t> data(K * B, 0), par(R * B, 0), out(K * B);
    bool encoded = false;
    int bad = 0;
    for (char c : seq) {
        if (c == 'e') {
            if (!encoded)
                for (auto &b : data) b = (uint8_t)rng();
            const int rc = kfec_encode(ctx, data.data(), K * B, B, par.data());
            encoded = true;
            printf("encode rc %d requests %llu\n", rc, (unsigned long long)kfec_worker_requests());
            bad |= rc != 0;
        } else {
            std::vector<size_t> ids;
            std::vector<const uint8_t *> ptrs;
            for (size_t s = lost; s < K; ++s) { ids.push_back(s); ptrs.push_back(data.data() + s * B); }
            for (size_t r = 0; r < R; ++r) { ids.push_back(K + r); ptrs.push_back(par.data() + r * B); }
            size_t out_ids[256], n_out = 0;
            const int rc = kfec_decode(ctx, ids.data(), ptrs.data(), ids.size(), B, out_ids, out.data(), &n_out);
            const bool ok = rc == 0 && n_out == lost && !std::memcmp(out.data(), data.data(), lost * B);
            printf("decode rc %d n_out %zu ok %d requests %llu\n", rc, n_out, (int)ok,
                   (unsigned long long)kfec_worker_requests());
            bad |= !ok;
        }
        fflush(stdout);
        if (bad) break;
    }
    kfec_destroy(ctx);
    return bad;
}
