// rowcopy.hip -- what packet-row width the AEAD kernels need to move packet bytes at HBM speed.
// Copies P packets of L bytes (dword-aligned pitch, as tools/bench_aead.py lays them out) with W lanes per
// packet row, each lane moving 16 bytes per round (rounds of 16 W bytes), grid-stride over packets like the
// AEAD kernels, for W = 4, 8, 16, 32, 64; also W = 8 with 64 bytes per lane (the chacha kernel's shape).
// Prints GB/s of (read + write).  Measurement only.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/rowcopy tools/rowcopy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <int W, int Q>  // W lanes per packet, Q 16-byte pieces per lane per round (lane-contiguous)
__global__ void __launch_bounds__(256) rowcopy(const uint8_t *src, uint8_t *dst, uint64_t P, uint32_t L,
                                               uint32_t pitch)
{
    constexpr int rows = 256 / W;
    const uint32_t lane = threadIdx.x % W;
    for (uint64_t p = (uint64_t)blockIdx.x * rows + threadIdx.x / W; p < P; p += (uint64_t)gridDim.x * rows) {
        const uint8_t *s = src + p * pitch;
        uint8_t *d = dst + p * pitch;
        for (uint32_t base = 0; base < L; base += 16u * W * Q) {
            uint4 v[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const uint32_t o = base + 16u * (lane * Q + q);
                v[q] = o + 16 <= L ? *reinterpret_cast<const uint4 *>(s + o) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const uint32_t o = base + 16u * (lane * Q + q);
                if (o + 16 <= L) *reinterpret_cast<uint4 *>(d + o) = v[q];
            }
        }
    }
}

template <int W, int Q>
float run(const uint8_t *src, uint8_t *dst, uint64_t P, uint32_t L, uint32_t pitch, int cus, int wg_per_cu)
{
    const dim3 g((unsigned)cus * wg_per_cu), b(256);
    hipLaunchKernelGGL((rowcopy<W, Q>), g, b, 0, 0, src, dst, P, L, pitch);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((rowcopy<W, Q>), g, b, 0, 0, src, dst, P, L, pitch);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main()
{
    const uint64_t P = 1ull << 22;
    const uint32_t L = 1440, pitch = 1468;  // whole 16-byte pieces only
    uint8_t *src, *dst;
    if (hipMalloc(&src, P * pitch) != hipSuccess || hipMalloc(&dst, P * pitch) != hipSuccess) return 1;
    (void)hipMemset(src, 1, P * pitch);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    const int cus = prop.multiProcessorCount;
    const double bytes = 2.0 * P * L;
    for (int wg : {4, 8, 16}) {
        printf("{\"wg_per_cu\": %d, \"GBps\": {\"W4\": %.0f, \"W8\": %.0f, \"W16\": %.0f, \"W32\": %.0f, \"W64\": %.0f, "
               "\"W8x4\": %.0f}}\n",
               wg, bytes / run<4, 1>(src, dst, P, L, pitch, cus, wg) / 1e6,
               bytes / run<8, 1>(src, dst, P, L, pitch, cus, wg) / 1e6,
               bytes / run<16, 1>(src, dst, P, L, pitch, cus, wg) / 1e6,
               bytes / run<32, 1>(src, dst, P, L, pitch, cus, wg) / 1e6,
               bytes / run<64, 1>(src, dst, P, L, pitch, cus, wg) / 1e6,
               bytes / run<8, 4>(src, dst, P, L, pitch, cus, wg) / 1e6);
    }
    return 0;
}
