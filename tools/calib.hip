// calib.hip -- on-box ceilings that bench.py reports its fractions against (tools/libkfec_calib.so).
// Measurement infrastructure only: never linked into libkfec.so.
//
//   calib_read(p, bytes, stream)     linear 16-B-per-lane read of [p, p + bytes), one contiguous 16 KiB chunk
//                                    per 256-lane workgroup (4 loads in flight per lane), non-persistent grid:
//                                    the HBM read ceiling of this box (6.48 TB/s on r01 boxes).
//   calib_gfmac(sink, blocks, iters, rows, stream)
//                                    the MAC kernels' inner loop with the memory taken out: 32-byte granules
//                                    (8 dwords per lane), per "shard" the three selector extractions per dword
//                                    and `rows` perm MACs per dword with the perm tables read from LDS exactly
//                                    as mac_kernel reads them (ds_read_b128 broadcast, once per 4 granules
//                                    here, so the LDS reads do not limit it).  rows = 8 is the
//                                    MT = 8 row tile of the fec=200:55 kernels; the byte-MAC rate it reaches
//                                    is the VALU ceiling those kernels are held against.
//                                    byte-MACs per launch = blocks * 256 * iters * 32 * rows.
// Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/libkfec_calib.so tools/calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../kcptube_amd/csrc/kfec_gf.hpp"

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) read_chunk4(const uint8_t *a, size_t nchunks, uint32_t *sink)
{
    if (blockIdx.x >= nchunks) return;
    const uint8_t *p = a + ((size_t)blockIdx.x * 4 * 256 + threadIdx.x) * 16;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const u32x4 *>(p + (size_t)i * 4096);
    const u32x4 acc = v[0] ^ v[1] ^ v[2] ^ v[3];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) sink[0] = acc.x;  // keeps the loads alive
}

template <int MT>
__global__ void __launch_bounds__(256) gfmac(uint32_t iters, uint32_t seed, uint32_t *sink)
{
    constexpr int TBL_DW = ((5 * MT + 3) / 4) * 4;
    constexpr int NS = 16;  // distinct "shards" of tables (wave-uniform, as the real kernels' encode tables)
    __shared__ __attribute__((aligned(16))) uint32_t s_tab[NS * TBL_DW];
    for (int e = threadIdx.x; e < NS * MT; e += 256) {
        uint32_t t[5];
        kfec::gf_perm_tables((uint32_t)(e * 37 + seed) & 0xFFu, t);
        const int s = e / MT, r = e - s * MT;
#pragma unroll
        for (int i = 0; i < 5; ++i) s_tab[s * TBL_DW + 5 * r + i] = t[i];
    }
    __syncthreads();
    uint32_t x[8], acc[MT][8];
#pragma unroll
    for (int w = 0; w < 8; ++w) x[w] = (threadIdx.x + 1) * 0x9E3779B9u ^ (seed + w * 0x85EBCA6Bu);
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) acc[r][w] = 0;
    // tables are read from LDS once per 4 granules, so the loop is the perm-MAC VALU work and nothing else
    for (uint32_t it = 0; it < iters; it += 4) {
        const uint4 *tv = reinterpret_cast<const uint4 *>(s_tab + ((it / 4) % NS) * TBL_DW);
        uint32_t t[TBL_DW];
#pragma unroll
        for (int i = 0; i < TBL_DW / 4; ++i) {
            const uint4 q = tv[i];
            t[4 * i] = q.x; t[4 * i + 1] = q.y; t[4 * i + 2] = q.z; t[4 * i + 3] = q.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                const uint32_t xv = x[w] ^ (it + k);  // a fresh granule (one XOR stands in for the load)
                const uint32_t s0 = xv & 0x07070707u, s1 = (xv >> 3) & 0x07070707u, s2 = (xv >> 6) & 0x03030303u;
#pragma unroll
                for (int r = 0; r < MT; ++r) acc[r][w] = kfec::perm_mac(acc[r][w], t + 5 * r, s0, s1, s2);
            }
        }
    }
    uint32_t v = 0;
#pragma unroll
    for (int r = 0; r < MT; ++r)
#pragma unroll
        for (int w = 0; w < 8; ++w) v ^= acc[r][w];
    if (v == 0x12345678u) sink[0] = v;
}

}  // namespace

extern "C" {

int calib_read(const void *p, size_t bytes, uint32_t *sink, void *stream)
{
    const size_t nchunks = bytes / (4 * 256 * 16);
    if (nchunks == 0 || nchunks > 0x7FFFFFFFu) return -1;
    hipLaunchKernelGGL(read_chunk4, dim3((uint32_t)nchunks), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const uint8_t *>(p), nchunks, sink);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// bytes actually read by calib_read for a buffer of `bytes`
size_t calib_read_bytes(size_t bytes) { return bytes / (4 * 256 * 16) * (4 * 256 * 16); }

int calib_gfmac(uint32_t *sink, uint32_t blocks, uint32_t iters, int rows, void *stream)
{
    const hipStream_t s = (hipStream_t)stream;
    switch (rows) {
    case 3: hipLaunchKernelGGL(gfmac<3>, dim3(blocks), dim3(256), 0, s, iters, 0x5EEDu, sink); break;
    case 8: hipLaunchKernelGGL(gfmac<8>, dim3(blocks), dim3(256), 0, s, iters, 0x5EEDu, sink); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"
