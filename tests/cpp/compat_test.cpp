// compat_test.cpp -- exercises include/fecpp_compat.hpp (the fecpp::fec_code drop-in) the way kcptube's
// callers do (client.cpp:797-938): encode a group, lose shards, decode.  Run by tests/test_gpu_parity.py.
// Prints "COMPAT OK" on success, exits non-zero with a message otherwise.
#include <fecpp_compat.hpp>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c);    \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main()
{
    // ctor / reset_martix error behaviour (fecpp.cpp:431-432, 439-440)
    int throws = 0;
    for (auto kn : std::vector<std::pair<size_t, size_t>>{{0, 0}, {0, 3}, {4, 3}, {1, 257}, {257, 257}}) {
        try { fecpp::fec_code c(kn.first, kn.second); } catch (const std::invalid_argument &) { ++throws; }
    }
    CHECK(throws == 5);
    fecpp::fec_code dflt;
    CHECK(dflt.get_K() == 0 && dflt.get_N() == 0);
    try { dflt.reset_martix(5, 4); CHECK(false); } catch (const std::invalid_argument &) {}
    dflt.reset_martix(20, 23);
    CHECK(dflt.get_K() == 20 && dflt.get_N() == 23);

    // known answer: parity row 0 of the 20:23 code via unit-vector encodes, B = 1
    const uint8_t row0[20] = {0xb7, 0xae, 0x0b, 0x72, 0x0b, 0xcd, 0x29, 0x3f, 0x84, 0xa0,
                              0xe5, 0x73, 0x03, 0xdf, 0xd9, 0xba, 0xd5, 0xd0, 0x20, 0x99};
    for (size_t j = 0; j < 20; ++j) {
        uint8_t unit[20] = {0};
        unit[j] = 1;
        auto red = dflt.encode(unit, 20, 1);
        CHECK(red.size() == 3);
        CHECK(red[0][0] == row0[j]);
    }

    // a kcptube-shaped group: D = 20 datagrams of varying length framed to align = max_len + 2
    const size_t K = 20, N = 23, B = 1407;
    std::vector<uint8_t> group(K * B);
    uint32_t x = 12345;
    for (auto &b : group) { x = x * 1103515245u + 12345u; b = (uint8_t)(x >> 16); }
    auto red = dflt.encode(group.data(), group.size(), B);
    CHECK(red.size() == 3);
    CHECK(dflt.encode(group.data(), K * B - B, B).empty());  // (len/B) % K != 0 -> {}
    CHECK(dflt.encode(nullptr, K * B, B).empty());

    // lose 3 data shards, keep the parity
    std::map<size_t, const uint8_t *> shares;
    for (size_t i = 0; i < K; ++i)
        if (i != 0 && i != 7 && i != 19) shares[i] = group.data() + i * B;
    for (size_t r = 0; r < 3; ++r) shares[K + r] = red[r].get();
    auto rec = dflt.decode(shares, B);
    CHECK(rec.size() == 3);
    for (size_t i : {0u, 7u, 19u}) {
        CHECK(rec.count(i) == 1);
        CHECK(std::memcmp(rec[i].data(), group.data() + i * B, B) == 0);
    }
    // too few shares -> {}
    shares.erase(3);
    CHECK(dflt.decode(shares, B).empty());
    // nothing missing -> {}
    std::map<size_t, const uint8_t *> all;
    for (size_t i = 0; i < K; ++i) all[i] = group.data() + i * B;
    CHECK(dflt.decode(all, B).empty());
    // an id >= N among the chosen shares -> {}
    std::map<size_t, const uint8_t *> bad;
    for (size_t i = 1; i < K; ++i) bad[i] = group.data() + i * B;
    bad[40] = red[0].get();
    CHECK(dflt.decode(bad, B).empty());

    // share_size == 0: the reference still maps every missing data row to an (empty) block (fecpp.cpp:572-583)
    shares[3] = group.data() + 3 * B;  // back to 17 data + 3 parity, data 0 / 7 / 19 missing
    auto empty_blocks = dflt.decode(shares, 0);
    CHECK(empty_blocks.size() == 3);
    for (size_t i : {0u, 7u, 19u}) CHECK(empty_blocks.count(i) == 1 && empty_blocks[i].empty());
    CHECK(dflt.decode(all, 0).empty());

    // a failed reset (K > N) leaves the coder as it was
    try { dflt.reset_martix(9, 8); CHECK(false); } catch (const std::invalid_argument &) {}
    CHECK(dflt.get_K() == 20 && dflt.get_N() == 23);
    CHECK(dflt.encode(group.data(), group.size(), B).size() == 3);

    // copies keep working (fec_control_data is held by value)
    fecpp::fec_code copy = dflt;
    auto red2 = copy.encode(group.data(), group.size(), B);
    CHECK(red2.size() == 3 && std::memcmp(red2[2].get(), red[2].get(), B) == 0);
    std::printf("COMPAT OK\n");
    return 0;
}
