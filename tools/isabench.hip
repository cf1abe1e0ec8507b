// isabench.hip -- issue cost of single gfx950 VALU instructions (inline asm, so the compiler cannot fold the
// chains): 16 independent chains per lane, 8 waves per SIMD, every CU busy.  Prints SIMD-cycles per
// wave-instruction at the clock the counters report (pass the measured clock in MHz as argv[1]; default the
// device's maximum).  Used to price the AEAD kernels' ChaCha20 (add / xor / rotate) and Poly1305 (32x32->64
// multiply-add, or 24-bit / f64 alternatives) instruction mixes.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/isabench tools/isabench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kIters = 2048;

#define CHAIN16(BODY)                              \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) { BODY; }

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t seed)
{
    uint32_t v[16];
    uint64_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = seed * (threadIdx.x + 1) + i * 0x9E3779B9u;
        w[i] = v[i] * 0x100000001ull;
    }
    const uint32_t a = seed ^ threadIdx.x, b = a * 3u;
    for (int it = 0; it < kIters; ++it) {
        if constexpr (OP == 0) CHAIN16(asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(v[i])))
        if constexpr (OP == 1) CHAIN16(asm volatile("v_xor_b32 %0, %1, %0" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 2) CHAIN16(asm volatile("v_add_u32 %0, %1, %0" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 3) CHAIN16(asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 4) CHAIN16(asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(v[i]) : "v"(0x01000302u)))
        if constexpr (OP == 5) CHAIN16(asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 6) CHAIN16(asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 7) CHAIN16(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 8) CHAIN16(asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(v[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 9) CHAIN16(asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 10) CHAIN16(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(w[i]) : "v"(w[(i + 1) & 15]), "v"(w[(i + 2) & 15])))
        if constexpr (OP == 11) CHAIN16(asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 12) CHAIN16(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 13) CHAIN16(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 14) CHAIN16(asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(v[i])))
        if constexpr (OP == 15) CHAIN16(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 16) CHAIN16(asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(w[i])))
        if constexpr (OP == 17) CHAIN16(asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 18) CHAIN16(asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(v[i]) : "v"(v[(i + 1) & 15])))
        if constexpr (OP == 19) CHAIN16(asm volatile("v_lshlrev_b32_sdwa %0, 8, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "+v"(v[i])))
        if constexpr (OP == 20) CHAIN16(asm volatile("v_bfe_u32 %0, %0, 16, 8" : "+v"(v[i])))
        if constexpr (OP == 21) CHAIN16(asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b)))
        if constexpr (OP == 22) CHAIN16(asm volatile("v_or_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "+v"(v[i]) : "v"(a)))
        if constexpr (OP == 23) CHAIN16(asm volatile("v_lshl_add_u32 %0, %0, 7, %1" : "+v"(v[i]) : "v"(a)))
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r ^= v[i] ^ (uint32_t)w[i] ^ (uint32_t)(w[i] >> 32);
    if (r == 0x12345678u) out[0] = r;
}

template <int OP>
float run(uint32_t *out, int cus)
{
    const dim3 g(cus * 8), b(256);  // 8 waves per SIMD
    hipLaunchKernelGGL(k<OP>, g, b, 0, 0, out, 7u);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, g, b, 0, 0, out, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main(int argc, char **argv)
{
    uint32_t *out;
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
    const int cus = p.multiProcessorCount;
    const double clk = (argc > 1 ? atof(argv[1]) : p.clockRate * 1e-3) * 1e6;
    const char *names[] = {"v_alignbit_b32 (rotate)", "v_xor_b32", "v_add_u32", "v_add3_u32", "v_perm_b32",
                           "v_lshl_or_b32", "v_mad_u64_u32", "v_mul_lo_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                           "v_fma_f64", "v_xad_u32", "v_bitop3_b32", "v_mul_u32_u24", "v_lshrrev_b32",
                           "v_mul_hi_u32", "v_lshlrev_b64", "v_add_co_u32", "v_mov_b32_sdwa (byte 1, preserve)",
                           "v_lshlrev_b32_sdwa (byte 2)", "v_bfe_u32", "v_and_or_b32", "v_or_b32_sdwa (byte 3)",
                           "v_lshl_add_u32"};
    float ms[24];
    ms[0] = run<0>(out, cus); ms[1] = run<1>(out, cus); ms[2] = run<2>(out, cus); ms[3] = run<3>(out, cus);
    ms[4] = run<4>(out, cus); ms[5] = run<5>(out, cus); ms[6] = run<6>(out, cus); ms[7] = run<7>(out, cus);
    ms[8] = run<8>(out, cus); ms[9] = run<9>(out, cus); ms[10] = run<10>(out, cus); ms[11] = run<11>(out, cus);
    ms[12] = run<12>(out, cus); ms[13] = run<13>(out, cus); ms[14] = run<14>(out, cus); ms[15] = run<15>(out, cus);
    ms[16] = run<16>(out, cus); ms[17] = run<17>(out, cus); ms[18] = run<18>(out, cus); ms[19] = run<19>(out, cus);
    ms[20] = run<20>(out, cus); ms[21] = run<21>(out, cus); ms[22] = run<22>(out, cus); ms[23] = run<23>(out, cus);
    for (int op = 0; op < 24; ++op) {
        const double waveinst = 5.0 * cus * 8 * 4 * (double)kIters * 16;
        const double cyc = (cus * 4.0) * (ms[op] * 1e-3 * clk) / waveinst;
        printf("%-26s %8.3f ms  %.2f SIMD-cycles per wave-instruction at %.0f MHz\n", names[op], ms[op], cyc,
               clk / 1e6);
    }
    return 0;
}
