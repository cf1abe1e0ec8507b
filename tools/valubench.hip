// valubench.hip -- issue rate of the perm-MAC's VALU instructions on gfx950 (v_perm_b32, v_bitop3_b32,
// v_xor_b32): 16 independent chains per lane, 8 waves per SIMD, every CU busy.  Reports wave-instructions
// per SIMD-cycle at the measured clock (GRBM-free: cycles = elapsed * clock from hipDeviceProp).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valubench tools/valubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t seed)
{
    uint32_t v[16];
    uint64_t w[16];
    double f[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        v[i] = seed * (threadIdx.x + 1) + i * 0x9E3779B9u;
        w[i] = v[i] * 0x100000001ull;
        f[i] = (double)v[i];
    }
    uint32_t a = seed ^ threadIdx.x, b = a * 3u, c = a * 7u;
    const double fa = 1.0000001 + a * 1e-12, fb = 0.5;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (OP == 0) v[i] = __builtin_amdgcn_perm(a, b, v[i]);
            else if constexpr (OP == 1) v[i] = __builtin_amdgcn_bitop3_b32(v[i], a, b, 0x96);
            else if constexpr (OP == 2) v[i] = v[i] ^ a;
            else if constexpr (OP == 3) v[i] = __builtin_amdgcn_perm(v[i], b, c);  // table operand dependent
            else if constexpr (OP == 4) w[i] = (uint64_t)(uint32_t)w[i] * a + w[i];  // v_mad_u64_u32
            else if constexpr (OP == 5) v[i] = v[i] * a;                              // v_mul_lo_u32
            else if constexpr (OP == 6) v[i] = __umul24(v[i], a) + b;                 // v_mad_u32_u24
            else if constexpr (OP == 7) f[i] = __builtin_fma(f[i], fa, fb);           // v_fma_f64
            else if constexpr (OP == 8) v[i] = v[i] + a;                              // v_add_u32
            else if constexpr (OP == 9) v[i] = __builtin_rotateleft32(v[i] ^ a, 7);   // xor + v_alignbit
            else if constexpr (OP == 10) v[i] = __umulhi(v[i], a);                    // v_mul_hi_u32
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) r ^= v[i] ^ (uint32_t)w[i] ^ (uint32_t)(w[i] >> 32) ^ (uint32_t)(int64_t)f[i];
    if (r == 0x12345678u) out[0] = r;
}

int main()
{
    uint32_t *out;
    hipMalloc(&out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;  // Hz (max)
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"v_perm_b32 (sel dependent)", "v_bitop3_b32", "v_xor_b32", "v_perm_b32 (table dependent)",
                           "v_mad_u64_u32", "v_mul_lo_u32", "v_mad_u32_u24", "v_fma_f64", "v_add_u32",
                           "xor + rotate (2 instr)", "v_mul_hi_u32"};
    for (int op = 0; op < 11; ++op) {
        auto launch = [&] {
            const dim3 g(cus * 8), b(256);  // 8 waves per SIMD
            if (op == 0) hipLaunchKernelGGL(k<0>, g, b, 0, 0, out, 7u);
            if (op == 1) hipLaunchKernelGGL(k<1>, g, b, 0, 0, out, 7u);
            if (op == 2) hipLaunchKernelGGL(k<2>, g, b, 0, 0, out, 7u);
            if (op == 3) hipLaunchKernelGGL(k<3>, g, b, 0, 0, out, 7u);
            if (op == 4) hipLaunchKernelGGL(k<4>, g, b, 0, 0, out, 7u);
            if (op == 5) hipLaunchKernelGGL(k<5>, g, b, 0, 0, out, 7u);
            if (op == 6) hipLaunchKernelGGL(k<6>, g, b, 0, 0, out, 7u);
            if (op == 7) hipLaunchKernelGGL(k<7>, g, b, 0, 0, out, 7u);
            if (op == 8) hipLaunchKernelGGL(k<8>, g, b, 0, 0, out, 7u);
            if (op == 9) hipLaunchKernelGGL(k<9>, g, b, 0, 0, out, 7u);
            if (op == 10) hipLaunchKernelGGL(k<10>, g, b, 0, 0, out, 7u);
        };
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double waveinst = 5.0 * cus * 8 * 4 * (double)kIters * 16;  // launches x WGs x waves x ops
        const double per_simd_cycle = waveinst / (cus * 4.0) / (ms * 1e-3 * clk);
        printf("%-30s %8.3f ms  %.3f wave-instr per SIMD-cycle at %.0f MHz (%.2f cycles each)\n", names[op], ms,
               per_simd_cycle, clk / 1e6, 1.0 / per_simd_cycle);
    }
    return 0;
}
