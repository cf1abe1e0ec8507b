// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A C wrapper around the reference coder `fecpp::fec_code`, compiled together with the reference's
// own sources where they lie (/root/reference/src/3rd_party/fecpp.cpp, fecpp_ssse3.cpp) by
// oracle/Makefile into oracle/_ref/libfecpp_ref.so.  No reference source is copied into this repo.
// Used to (1) pin the C restatement (oracle/rs_oracle.c) and generate tests/golden/ fixtures, and
// (2) serve as bench.py's cpu_baseline ("kind": "reference") on the GPU box's host cores.
//
// Reference interface wrapped: fecpp.hpp:36-81 (constructor, reset_martix, encode, decode).
#include "fecpp.hpp"

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <thread>
#include <vector>

namespace {
inline uint64_t smix(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
}  // namespace

extern "C" {

// 0 ok, -1 invalid_argument thrown
int ref_check_kn(size_t K, size_t N)
{
    try {
        fecpp::fec_code c(K, N);
        (void)c;
        return 0;
    } catch (const std::invalid_argument &) {
        return -1;
    }
}

int ref_check_reset(size_t K, size_t N)
{
    fecpp::fec_code c;
    try {
        c.reset_martix(K, N);
        return (c.get_K() == K && c.get_N() == N) ? 0 : -2;
    } catch (const std::invalid_argument &) {
        return -1;
    }
}

// encode: returns number of parity blocks written (N-K), or -1 when the reference returns {}
long ref_encode(size_t K, size_t N, const uint8_t *input, size_t data_length, size_t block_size,
                uint8_t *parity_out)
{
    fecpp::fec_code c(K, N);
    auto red = c.encode(input, data_length, block_size);
    if (red.empty() && N != K) return -1;
    for (size_t r = 0; r < red.size(); ++r) std::memcpy(parity_out + r * block_size, red[r].get(), block_size);
    return (long)red.size();
}

// enc_matrix is private in the reference; recover it by encoding unit vectors with block_size 1
int ref_enc_matrix(size_t K, size_t N, uint8_t *enc)
{
    fecpp::fec_code c(K, N);
    std::memset(enc, 0, N * K);
    for (size_t i = 0; i < K; ++i) enc[i * K + i] = 1;
    std::vector<uint8_t> unit(K);
    for (size_t j = 0; j < K; ++j) {
        std::fill(unit.begin(), unit.end(), 0);
        unit[j] = 1;
        auto red = c.encode(unit.data(), K, 1);
        for (size_t r = 0; r < red.size(); ++r) enc[(K + r) * K + j] = red[r][0];
    }
    return 0;
}

// decode: shares given as ids[n] + ptrs[n]. Returns number of recovered blocks (ascending index
// order in out / out_ids), -2 on std::invalid_argument.  An empty map returns 0.
long ref_decode(size_t K, size_t N, const size_t *ids, const uint8_t *const *ptrs, size_t n,
                size_t share_size, size_t *out_ids, uint8_t *out)
{
    fecpp::fec_code c(K, N);
    std::map<size_t, const uint8_t *> shares;
    for (size_t i = 0; i < n; ++i) shares[ids[i]] = ptrs[i];
    try {
        auto res = c.decode(shares, share_size);
        long m = 0;
        for (auto &[idx, buf] : res) {
            out_ids[m] = idx;
            std::memcpy(out + (size_t)m * share_size, buf.data(), share_size);
            ++m;
        }
        return m;
    } catch (const std::invalid_argument &) {
        return -2;
    }
}

// CPU baseline: encode + erase `erase` shards (data shards only when pool == K, else over all N)
// + decode, over G groups of distinct synthetic data, T threads, `passes` passes.
// Each thread gets a contiguous group range and its own fec_code; one instance is constructed
// before the threads start so the reference's unguarded init_fec (fecpp.cpp:150-165) cannot race.
// Returns payload bytes/s = G * passes * K * B / wall seconds.
double ref_bench_roundtrip(size_t K, size_t N, size_t B, size_t G, size_t pool, size_t erase_max,
                           int random_count, size_t threads, size_t passes, uint64_t seed,
                           double *seconds_out, size_t *recovered_out, int decode_only)
{
    fecpp::fec_code warm(K, N);
    (void)warm;
    const size_t W = (B + 7) / 8;
    std::vector<uint8_t> data(G * K * B);
    // decode-only runs read parity encoded before the timed region
    std::vector<uint8_t> parity(decode_only ? G * (N - K) * B : 0);
    // inputs are generated (and, decode-only, encoded) by the same threads over the same ranges, untimed
    auto prepare = [&](size_t t) {
        fecpp::fec_code c(K, N);
        const size_t a = G * t / threads, b = G * (t + 1) / threads;
        for (size_t g = a; g < b; ++g) {
            for (size_t s = 0; s < K; ++s) {
                uint8_t *dst = data.data() + (g * K + s) * B;
                const uint64_t base = (g * N + s) * W;
                for (size_t w = 0; w < W; ++w) {
                    uint64_t v = smix(seed ^ (base + w));
                    for (size_t k = 0; k < 8 && w * 8 + k < B; ++k) dst[w * 8 + k] = (uint8_t)(v >> (8 * k));
                }
            }
            if (decode_only) {
                auto red = c.encode(data.data() + g * K * B, K * B, B);
                for (size_t r = 0; r < N - K; ++r) std::memcpy(parity.data() + (g * (N - K) + r) * B, red[r].get(), B);
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (size_t t = 0; t < threads; ++t) th.emplace_back(prepare, t);
        for (auto &x : th) x.join();
    }
    std::vector<size_t> recovered(threads, 0);
    auto worker = [&](size_t t) {
        fecpp::fec_code c(K, N);
        const size_t a = G * t / threads, b = G * (t + 1) / threads;
        size_t rec = 0;
        for (size_t p = 0; p < passes; ++p)
            for (size_t g = a; g < b; ++g) {
                const uint8_t *d = data.data() + g * K * B;
                std::vector<std::unique_ptr<uint8_t[]>> red;
                if (!decode_only) red = c.encode(d, K * B, B);
                auto par_of = [&](size_t r) -> const uint8_t * {
                    return decode_only ? parity.data() + (g * (N - K) + r) * B : red[r].get();
                };
                // erasure draw: same definition as orc_erasure_mask / the HIP generator
                size_t cnt = erase_max;
                if (random_count == 1) cnt = 1 + (size_t)(smix(seed ^ ~(uint64_t)g) % erase_max);
                uint8_t perm[256];
                for (size_t i = 0; i < 256; ++i) perm[i] = (uint8_t)i;
                bool present[256];
                for (size_t s = 0; s < N; ++s) present[s] = true;
                if (random_count == 2) {  // i.i.d. loss, erase_max = ppm (orc_erasure_mask_iid)
                    cnt = 0;
                    for (size_t s = 0; s < N; ++s)
                        present[s] = smix(seed ^ 0xC2B2AE3D27D4EB4Full ^ ((uint64_t)g * 0x100u + s)) % 1000000u >= erase_max;
                }
                for (size_t e = 0; e < cnt && e < pool; ++e) {
                    uint64_t r = smix(seed ^ ((uint64_t)g * 0x100u + e));
                    size_t k = e + (size_t)(r % (uint64_t)(pool - e));
                    std::swap(perm[e], perm[k]);
                    present[perm[e]] = false;
                }
                std::map<size_t, const uint8_t *> shares;
                for (size_t s = 0; s < N; ++s)
                    if (present[s]) shares[s] = s < K ? d + s * B : par_of(s - K);
                auto res = c.decode(shares, B);
                rec += res.size();
            }
        recovered[t] = rec;
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (size_t t = 0; t < threads; ++t) th.emplace_back(worker, t);
    for (auto &x : th) x.join();
    auto t1 = std::chrono::steady_clock::now();
    double secs = std::chrono::duration<double>(t1 - t0).count();
    if (seconds_out) *seconds_out = secs;
    if (recovered_out) {
        size_t tot = 0;
        for (auto r : recovered) tot += r;
        *recovered_out = tot;
    }
    return (double)(G * passes) * (double)(K * B) / secs;
}

// Per-call latency of ONE group on the calling thread (tools/latency_bench.cpp's reference leg): one fec_code
// built before timing, the same group every call (warm caches, as a live KCP updater thread coding its
// connection's groups), encode, then decode with the first `lost` data shares missing (the map holds the other
// data shares and `lost` parity shares, as fec_find_missings builds it, client.cpp:895-938).
// us[0..5] = encode mean / p50 / p90, decode mean / p50 / p90 (microseconds).  Returns 0, or -1 on a wrong result.
int ref_percall_latency(size_t K, size_t N, size_t B, size_t lost, int reps, double *us)
{
    using clk = std::chrono::steady_clock;
    fecpp::fec_code c(K, N);
    std::vector<uint8_t> data(K * B);
    for (size_t i = 0; i < data.size(); ++i) data[i] = (uint8_t)smix(i);
    auto red = c.encode(data.data(), K * B, B);
    if (red.size() != N - K || lost > N - K) return -1;
    std::map<size_t, const uint8_t *> shares;
    for (size_t s = lost; s < K; ++s) shares[s] = data.data() + s * B;
    for (size_t r = 0; r < lost; ++r) shares[K + r] = red[r].get();
    auto stats = [&](std::vector<double> &v, double *o) {
        double sum = 0;
        for (double x : v) sum += x;
        std::sort(v.begin(), v.end());
        o[0] = sum / v.size();
        o[1] = v[v.size() / 2];
        o[2] = v[v.size() * 9 / 10];
    };
    std::vector<double> te(reps), td(reps);
    size_t sink = 0;
    for (int i = 0; i < 50; ++i) sink += c.encode(data.data(), K * B, B).size() + c.decode(shares, B).size();
    for (int i = 0; i < reps; ++i) {
        const auto t0 = clk::now();
        auto p = c.encode(data.data(), K * B, B);
        te[i] = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        sink += p.size();
    }
    for (int i = 0; i < reps; ++i) {
        const auto t0 = clk::now();
        auto m = c.decode(shares, B);
        td[i] = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        sink += m.size();
    }
    auto m = c.decode(shares, B);
    for (size_t t = 0; t < lost; ++t)
        if (!m.count(t) || std::memcmp(m[t].data(), data.data() + t * B, B)) return -1;
    stats(te, us);
    stats(td, us + 3);
    return sink ? 0 : -1;
}

}  // extern "C"
