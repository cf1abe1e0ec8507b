// ceiling.hip -- what the encode's byte mix can reach on this box (XOR only, no GF arithmetic).
//   The encode at fec=20:3, B=1440 reads 28,800 B and writes 4,320 B per group.  These kernels move the
//   same bytes with different access shapes, to separate "HBM can't do better" from "our shape loses":
//   read_chunk<U>   : each workgroup reads one contiguous chunk of U x 4 KiB (16-B lanes), non-persistent grid
//   write_chunk<U>  : the same with stores
//   copy_chunk<U>   : read chunk + store chunk
//   enc_lin         : one workgroup per group: the group's 28,800 B read as 1,800 consecutive 16-B granules,
//                     4,320 B written (the ideal streaming form of the encode's traffic)
//   enc_cols<V,PD>  : lane = (group, V-byte column), reads the column of the 20 shards, PD shards in flight,
//                     writes 3 columns (the flattened kernel's shape), persistent grid of occ WG/CU
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ceiling tools/ceiling.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(const uint8_t *p) { return *reinterpret_cast<const u32x4 *>(p); }
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    else *reinterpret_cast<u32x4 *>(p) = v;
}

template <int U>
__global__ void __launch_bounds__(256) read_chunk(const uint8_t *a, uint8_t *sink)
{
    const uint8_t *p = a + ((size_t)blockIdx.x * U * 256 + threadIdx.x) * 16;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = ld16(p + (size_t)i * 4096);
    u32x4 acc = v[0];
#pragma unroll
    for (int i = 1; i < U; ++i) acc ^= v[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) st16(sink, acc, false);
}

template <int U>
__global__ void __launch_bounds__(256) read_chunk_nt(const uint8_t *a, uint8_t *sink)
{
    const uint8_t *p = a + ((size_t)blockIdx.x * U * 256 + threadIdx.x) * 16;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + (size_t)i * 4096));
    u32x4 acc = v[0];
#pragma unroll
    for (int i = 1; i < U; ++i) acc ^= v[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) st16(sink, acc, false);
}

template <int U>
__global__ void __launch_bounds__(256) write_chunk(uint8_t *b, bool nt)
{
    uint8_t *p = b + ((size_t)blockIdx.x * U * 256 + threadIdx.x) * 16;
    const u32x4 v = {threadIdx.x, blockIdx.x, 1u, 2u};
#pragma unroll
    for (int i = 0; i < U; ++i) st16(p + (size_t)i * 4096, v, nt);
}

template <int U>
__global__ void __launch_bounds__(256) copy_chunk(const uint8_t *a, uint8_t *b, bool nt)
{
    const size_t off = ((size_t)blockIdx.x * U * 256 + threadIdx.x) * 16;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = ld16(a + off + (size_t)i * 4096);
#pragma unroll
    for (int i = 0; i < U; ++i) st16(b + off + (size_t)i * 4096, v[i], nt);
}

// one workgroup (256 lanes) per group: 1800 granules read, 270 written
__global__ void __launch_bounds__(256) enc_lin(const uint8_t *d, uint8_t *par, bool nt)
{
    const uint8_t *p = d + (size_t)blockIdx.x * 28800;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const unsigned q = i * 256 + threadIdx.x;
        v[i] = q < 1800 ? ld16(p + q * 16) : u32x4{0, 0, 0, 0};
    }
    u32x4 acc = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) acc ^= v[i];
    uint8_t *o = par + (size_t)blockIdx.x * 4320;
    st16(o + threadIdx.x * 16, acc, nt);
    if (threadIdx.x < 14) st16(o + (256 + threadIdx.x) * 16, acc, nt);
}

// enc_lin with nontemporal loads (NTL) and optionally nt stores: the whole group is one contiguous read
template <bool NTL>
__global__ void __launch_bounds__(256) enc_lin_ntl(const uint8_t *d, uint8_t *par, bool nt)
{
    const uint8_t *p = d + (size_t)blockIdx.x * 28800;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const unsigned q = i * 256 + threadIdx.x;
        const unsigned qq = q < 1800 ? q : 1799;  // (clamped: no branch around the load)
        v[i] = NTL ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + qq * 16)) : ld16(p + qq * 16);
    }
    u32x4 acc = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) acc ^= v[i];
    uint8_t *o = par + (size_t)blockIdx.x * 4320;
    st16(o + threadIdx.x * 16, acc, nt);
    if (threadIdx.x < 14) st16(o + (256 + threadIdx.x) * 16, acc, nt);
}

// one wave per group, 4 groups per workgroup
__global__ void __launch_bounds__(256) enc_lin_wave(const uint8_t *d, uint8_t *par, unsigned G, bool nt)
{
    const unsigned g = blockIdx.x * 4 + threadIdx.x / 64, l = threadIdx.x % 64;
    if (g >= G) return;
    const uint8_t *p = d + (size_t)g * 28800;
    u32x4 acc = {0, 0, 0, 0};
    for (int i0 = 0; i0 < 29; i0 += 8) {
        u32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const unsigned q = (i0 + i) * 64 + l;
            v[i] = q < 1800 ? ld16(p + q * 16) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= v[i];
    }
    uint8_t *o = par + (size_t)g * 4320;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const unsigned q = i * 64 + l;
        if (q < 270) st16(o + q * 16, acc, nt);
    }
}

__device__ __forceinline__ u32x4 ld16nt(const uint8_t *p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p)); }

// the flattened encode's traffic with nontemporal loads: V = 32 as the shipped kernel (lane l: bytes [32l, 32l+32),
// two 16-B loads 16 B apart), V = 16 (one 16-B load per lane: every wave-instruction reads 1 KB contiguous),
// V = 32 split (lane l: 16-B columns l and l + 64 of its wave's 2 KB: two loads, each 1 KB contiguous per wave)
template <int V, int PD, bool SPLIT>
__global__ void __launch_bounds__(256) enc_cols_ntl(const uint8_t *d, uint8_t *par, unsigned total16, unsigned cols16, bool nt)
{
    constexpr int NV = V / 16;
    // item space in 16-B columns; a wave owns 64 * NV consecutive columns
    const unsigned wave0 = (blockIdx.x * 256 + (threadIdx.x & ~63u)) * NV, l = threadIdx.x & 63u;
    unsigned it[NV];
#pragma unroll
    for (int w = 0; w < NV; ++w) it[w] = SPLIT ? wave0 + w * 64 + l : wave0 + l * NV + w;
    const uint8_t *p[NV];
    bool in[NV];
#pragma unroll
    for (int w = 0; w < NV; ++w) {
        in[w] = it[w] < total16;
        const unsigned g = in[w] ? it[w] / cols16 : 0, c = in[w] ? it[w] - g * cols16 : 0;
        p[w] = d + (size_t)g * 28800 + c * 16;
    }
    u32x4 acc[NV];
#pragma unroll
    for (int w = 0; w < NV; ++w) acc[w] = u32x4{0, 0, 0, 0};
    u32x4 x[PD][NV];
#pragma unroll
    for (int u = 0; u < PD; ++u)
#pragma unroll
        for (int w = 0; w < NV; ++w) x[u][w] = ld16nt(p[w] + u * 1440);
#pragma unroll
    for (int j = 0; j < 20; ++j) {
        const int u = j % PD;
#pragma unroll
        for (int w = 0; w < NV; ++w) {
            const u32x4 cur = x[u][w];
            if (j + PD < 20) x[u][w] = ld16nt(p[w] + (j + PD) * 1440);
            acc[w] ^= cur;
        }
    }
#pragma unroll
    for (int w = 0; w < NV; ++w) {
        if (!in[w]) continue;
        const unsigned g = it[w] / cols16, c = it[w] - g * cols16;
        uint8_t *o = par + (size_t)g * 4320 + c * 16;
#pragma unroll
        for (int r = 0; r < 3; ++r) st16(o + r * 1440, acc[w] + (u32x4){(unsigned)r, 0, 0, 0}, nt);
    }
}

template <int V, int PD>
__global__ void __launch_bounds__(256) enc_cols(const uint8_t *d, uint8_t *par, unsigned total, unsigned cols, bool nt)
{
    constexpr int NV = V / 16;
    for (unsigned it = blockIdx.x * 256 + threadIdx.x; it < total; it += gridDim.x * 256) {
        const unsigned g = it / cols, c = it - g * cols;
        const uint8_t *p = d + (size_t)g * 28800 + c * V;
        u32x4 acc[NV];
#pragma unroll
        for (int w = 0; w < NV; ++w) acc[w] = u32x4{0, 0, 0, 0};
        u32x4 x[PD][NV];
#pragma unroll
        for (int u = 0; u < PD; ++u)
#pragma unroll
            for (int w = 0; w < NV; ++w) x[u][w] = ld16(p + u * 1440 + w * 16);
#pragma unroll
        for (int j = 0; j < 20; ++j) {
            const int u = j % PD;
#pragma unroll
            for (int w = 0; w < NV; ++w) {
                const u32x4 cur = x[u][w];
                if (j + PD < 20) x[u][w] = ld16(p + (j + PD) * 1440 + w * 16);
                acc[w] ^= cur;
            }
        }
        uint8_t *o = par + (size_t)g * 4320 + c * V;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int w = 0; w < NV; ++w) st16(o + r * 1440 + w * 16, acc[w] + (u32x4){(unsigned)r, 0, 0, 0}, nt);
    }
}

// shape study for any fec=K:R, B: the coder's column pattern (lane = (group, 32-B column), the K shards of
// the column read PD in flight, R columns written) against the contiguous form (one workgroup per group reading
// its K x B bytes in order, writing R x B), both XOR-only
template <int PD>
__global__ void __launch_bounds__(256) gen_cols(const uint8_t *d, uint8_t *par, unsigned total, unsigned cols, unsigned K,
                                                unsigned R, unsigned B)
{
    const unsigned it = blockIdx.x * 256 + threadIdx.x;
    if (it >= total) return;
    const unsigned g = it / cols, c = it - g * cols;
    const unsigned o = min(c * 32, ((B + 3) & ~3u) - 32);
    const uint8_t *p = d + (size_t)g * K * B + o;
    u32x4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
    u32x4 x[PD][2];
#pragma unroll
    for (int u = 0; u < PD; ++u) {
        const unsigned j = min((unsigned)u, K - 1);
        x[u][0] = ld16(p + (size_t)j * B);
        x[u][1] = ld16(p + (size_t)j * B + 16);
    }
    unsigned jb = 0;
    for (; jb + PD <= K; jb += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            a0 ^= x[u][0];
            a1 ^= x[u][1];
            const unsigned j = min(jb + u + PD, K - 1);
            x[u][0] = ld16(p + (size_t)j * B);
            x[u][1] = ld16(p + (size_t)j * B + 16);
        }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u)
        if (jb + u < K) {
            a0 ^= x[u][0];
            a1 ^= x[u][1];
        }
    uint8_t *q = par + (size_t)g * R * B + o;
    for (unsigned r = 0; r < R; ++r) {
        st16(q + (size_t)r * B, a0 + (u32x4){r, 0, 0, 0}, true);
        st16(q + (size_t)r * B + 16, a1, true);
    }
}

__global__ void __launch_bounds__(256) gen_lin(const uint8_t *d, uint8_t *par, unsigned rq, unsigned wq)
{
    const uint8_t *p = d + (size_t)blockIdx.x * rq * 16;
    u32x4 acc = {0, 0, 0, 0};
    for (unsigned q0 = 0; q0 < rq; q0 += 8 * 256) {
        u32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ld16(p + (size_t)min(q0 + i * 256 + threadIdx.x, rq - 1) * 16);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= v[i];
    }
    uint8_t *o = par + (size_t)blockIdx.x * wq * 16;
    for (unsigned q = threadIdx.x; q < wq; q += 256) st16(o + (size_t)q * 16, acc, true);
}

int main(int argc, char **argv)
{
    const size_t G = 1u << 20;
    const size_t dbytes = G * 28800, pbytes = G * 4320;
    uint8_t *a, *b, *sink;
    if (hipMalloc(&a, dbytes) != hipSuccess || hipMalloc(&b, pbytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(a, 0x5A, dbytes);
    hipMemset(b, 0, pbytes);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, double moved, auto launch) {
        std::vector<float> t;
        for (int i = 0; i < 7; ++i) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-34s %8.3f ms  %7.1f GB/s  (min %.3f)\n", name, t[3], moved / t[3] / 1e6, t[0]);
        fflush(stdout);
    };
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) printf("err %s\n", hipGetErrorString(err));
    // chunk kernels over the 30.2 GB data buffer / 4.5 GB parity buffer
    const unsigned nr4 = dbytes / (4 * 4096), nr8 = dbytes / (8 * 4096), nr16 = dbytes / (16 * 4096);
    const unsigned nw4 = pbytes / (4 * 4096), nw8 = pbytes / (8 * 4096);
    run("read_chunk<4>", nr4 * 4.0 * 4096, [&] { read_chunk<4><<<nr4, 256>>>(a, sink); });
    run("read_chunk<8>", nr8 * 8.0 * 4096, [&] { read_chunk<8><<<nr8, 256>>>(a, sink); });
    run("read_chunk<16>", nr16 * 16.0 * 4096, [&] { read_chunk<16><<<nr16, 256>>>(a, sink); });
    run("read_chunk_nt<8>", nr8 * 8.0 * 4096, [&] { read_chunk_nt<8><<<nr8, 256>>>(a, sink); });
    run("read_chunk_nt<16>", nr16 * 16.0 * 4096, [&] { read_chunk_nt<16><<<nr16, 256>>>(a, sink); });
    run("write_chunk<4>", nw4 * 4.0 * 4096, [&] { write_chunk<4><<<nw4, 256>>>(b, false); });
    run("write_chunk<8>", nw8 * 8.0 * 4096, [&] { write_chunk<8><<<nw8, 256>>>(b, false); });
    run("write_chunk<8> nt", nw8 * 8.0 * 4096, [&] { write_chunk<8><<<nw8, 256>>>(b, true); });
    run("copy_chunk<8> 4.5GB", nw8 * 16.0 * 4096, [&] { copy_chunk<8><<<nw8, 256>>>(a, b, false); });
    run("copy_chunk<8> 4.5GB nt", nw8 * 16.0 * 4096, [&] { copy_chunk<8><<<nw8, 256>>>(a, b, true); });
    run("copy_chunk<4> 4.5GB", nw4 * 8.0 * 4096, [&] { copy_chunk<4><<<nw4, 256>>>(a, b, false); });
    const double enc = (double)G * (28800 + 4320);
    run("enc_lin (WG/group)", enc, [&] { enc_lin<<<G, 256>>>(a, b, false); });
    run("enc_lin (WG/group) nt", enc, [&] { enc_lin<<<G, 256>>>(a, b, true); });
    run("enc_lin_ntl<0> nt-st", enc, [&] { enc_lin_ntl<false><<<G, 256>>>(a, b, true); });
    run("enc_lin_ntl<1> nt-st", enc, [&] { enc_lin_ntl<true><<<G, 256>>>(a, b, true); });
    run("enc_lin_ntl<1>", enc, [&] { enc_lin_ntl<true><<<G, 256>>>(a, b, false); });
    run("enc_lin_wave", enc, [&] { enc_lin_wave<<<G / 4, 256>>>(a, b, G, false); });
    run("enc_lin_wave nt", enc, [&] { enc_lin_wave<<<G / 4, 256>>>(a, b, G, true); });
    const unsigned t16 = G * 90, t32 = G * 45;
    for (int occ : {4, 8, 16}) {
        char nm[64];
        snprintf(nm, 64, "enc_cols<16,4> occ%d nt", occ);
        run(nm, enc, [&] { enc_cols<16, 4><<<cus * occ, 256>>>(a, b, t16, 90, true); });
        snprintf(nm, 64, "enc_cols<32,2> occ%d nt", occ);
        run(nm, enc, [&] { enc_cols<32, 2><<<cus * occ, 256>>>(a, b, t32, 45, true); });
        snprintf(nm, 64, "enc_cols<32,4> occ%d nt", occ);
        run(nm, enc, [&] { enc_cols<32, 4><<<cus * occ, 256>>>(a, b, t32, 45, true); });
    }
    {
        const unsigned tot16 = G * 90, nb16 = (tot16 + 255) / 256, nb32 = (tot16 + 511) / 512;
        run("enc_cols_ntl<16,4>", enc, [&] { enc_cols_ntl<16, 4, false><<<nb16, 256>>>(a, b, tot16, 90, true); });
        run("enc_cols_ntl<32,4> (as shipped)", enc, [&] { enc_cols_ntl<32, 4, false><<<nb32, 256>>>(a, b, tot16, 90, true); });
        run("enc_cols_ntl<32,4> split", enc, [&] { enc_cols_ntl<32, 4, true><<<nb32, 256>>>(a, b, tot16, 90, true); });
        run("enc_cols_ntl<16,8>", enc, [&] { enc_cols_ntl<16, 8, false><<<nb16, 256>>>(a, b, tot16, 90, true); });
        run("enc_cols_ntl<32,2> split", enc, [&] { enc_cols_ntl<32, 2, true><<<nb32, 256>>>(a, b, tot16, 90, true); });
    }
    run("enc_cols<16,4> nonpersist nt", enc, [&] { enc_cols<16, 4><<<(t16 + 255) / 256, 256>>>(a, b, t16, 90, true); });
    run("enc_cols<32,2> nonpersist nt", enc, [&] { enc_cols<32, 2><<<(t32 + 255) / 256, 256>>>(a, b, t32, 45, true); });
    run("enc_cols<32,4> nonpersist nt", enc, [&] { enc_cols<32, 4><<<(t32 + 255) / 256, 256>>>(a, b, t32, 45, true); });
    // shape study: 1M groups of fec=K:R at B (the buffers hold 30.2 GB / 4.5 GB)
    for (auto kr : {std::array<unsigned, 3>{20, 3, 1440}, {10, 3, 1400}, {10, 3, 1408}, {10, 3, 1440}, {20, 3, 1408}}) {
        const unsigned K = kr[0], R = kr[1], B = kr[2];
        const size_t Gs = std::min<size_t>(G, std::min(dbytes / ((size_t)K * B), pbytes / ((size_t)R * B)));
        const unsigned cols = (B + 31) / 32, total = (unsigned)(Gs * cols);
        const double moved = (double)Gs * (K + R) * B;
        char nm[64];
        snprintf(nm, 64, "gen_cols<4> %u:%u B=%u", K, R, B);
        run(nm, moved, [&] { gen_cols<4><<<(total + 255) / 256, 256>>>(a, b, total, cols, K, R, B); });
        if ((K * B) % 16 == 0 && (R * B) % 16 == 0) {
            snprintf(nm, 64, "gen_lin %u:%u B=%u", K, R, B);
            run(nm, moved, [&] { gen_lin<<<(unsigned)Gs, 256>>>(a, b, K * B / 16, R * B / 16); });
        }
    }
    const hipError_t e2 = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e2));
    return 0;
}
