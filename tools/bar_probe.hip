// bar_probe.hip -- can the host write device memory directly (large BAR), and what does it cost?  For the
// per-call worker (kfec_worker.hip), which today pulls each group over PCIe after seeing the doorbell.
// Allocates fine-grained device memory, writes 28 800 bytes into it from the host (SIGSEGV is caught and
// reported as "not host-accessible"), times the host copy, and has a kernel checksum the bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -mavx2 tools/bar_probe.hip -o tools/bar_probe
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <vector>

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }

__global__ void sum_kernel(const uint32_t *p, int n, uint32_t *out)
{
    uint32_t s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
    atomicAdd(out, s);
}

// copy variants into write-combined BAR memory (n a multiple of 64, both 32-byte aligned)
static void copy_stream(void *dst, const void *src, size_t n)
{
    auto *d = static_cast<__m256i *>(dst);
    auto *s = static_cast<const __m256i *>(src);
    for (size_t i = 0; i < n / 32; i += 2) {
        const __m256i a = _mm256_loadu_si256(s + i), b = _mm256_loadu_si256(s + i + 1);
        _mm256_stream_si256(d + i, a);
        _mm256_stream_si256(d + i + 1, b);
    }
    _mm_sfence();
}
static void copy_store(void *dst, const void *src, size_t n)
{
    auto *d = static_cast<__m256i *>(dst);
    auto *s = static_cast<const __m256i *>(src);
    for (size_t i = 0; i < n / 32; ++i) _mm256_storeu_si256(d + i, _mm256_loadu_si256(s + i));
    _mm_sfence();
}
__attribute__((target("avx512f"))) static void copy_store512(void *dst, const void *src, size_t n)
{
    auto *d = static_cast<__m512i *>(dst);
    auto *s = static_cast<const __m512i *>(src);
    for (size_t i = 0; i < n / 64; ++i) _mm512_storeu_si512(d + i, _mm512_loadu_si512(s + i));
    _mm_sfence();
}
__attribute__((target("avx512f"))) static void copy_stream512(void *dst, const void *src, size_t n)
{
    auto *d = static_cast<__m512i *>(dst);
    auto *s = static_cast<const __m512i *>(src);
    for (size_t i = 0; i < n / 64; ++i) _mm512_stream_si512(d + i, _mm512_loadu_si512(s + i));
    _mm_sfence();
}
static void copy_movsb(void *dst, const void *src, size_t n)
{
    asm volatile("rep movsb" : "+D"(dst), "+S"(src), "+c"(n) : : "memory");
    _mm_sfence();
}

static void time_variants(const char *name, void *p)
{
    const size_t n = 28800;
    alignas(64) static uint8_t src[28800];
    for (size_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 5 + 1);
    struct V { const char *v; void (*f)(void *, const void *, size_t); };
    const V vs[] = {{"memcpy+sfence", [](void *d, const void *s, size_t k) { std::memcpy(d, s, k); _mm_sfence(); }},
                    {"avx2 stream", copy_stream}, {"avx2 store", copy_store}, {"rep movsb", copy_movsb},
                    {"avx512 store", copy_store512}, {"avx512 stream", copy_stream512}};
    const bool avx512 = __builtin_cpu_supports("avx512f");
    for (const V &v : vs) {
        if (!avx512 && std::strncmp(v.v, "avx512", 6) == 0) {
            printf("%s: %s: no avx512f on this CPU\n", name, v.v);
            continue;
        }
        for (int i = 0; i < 50; ++i) v.f(p, src, n);
        const int reps = 4000;
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            src[i & 1023] ^= 1;
            v.f(p, src, n);
        }
        const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / reps;
        printf("%s: %s of 28800 B %.0f ns\n", name, v.v, ns);
    }
}

static void probe(const char *name, void *p)
{
    const size_t n = 28800;
    std::vector<uint8_t> src(n);
    for (size_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 7 + 3);
    struct sigaction sa = {}, old = {};
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old);
    if (sigsetjmp(g_jmp, 1)) {
        sigaction(SIGSEGV, &old, nullptr);
        printf("%s: not host-accessible (SIGSEGV)\n", name);
        return;
    }
    std::memcpy(p, src.data(), n);
    const int reps = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
        src[i & 1023] ^= 1;
        std::memcpy(p, src.data(), n);
    }
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / reps;
    std::memcpy(p, src.data(), n);
    sigaction(SIGSEGV, &old, nullptr);
    uint32_t *d_out = nullptr;
    (void)hipMalloc(&d_out, 4);
    (void)hipMemset(d_out, 0, 4);
    hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, (const uint32_t *)p, (int)(n / 4), d_out);
    uint32_t got = 0;
    (void)hipMemcpy(&got, d_out, 4, hipMemcpyDeviceToHost);
    uint32_t want = 0;
    for (size_t i = 0; i < n / 4; ++i) {
        uint32_t w;
        std::memcpy(&w, src.data() + 4 * i, 4);
        want += w;
    }
    printf("%s: host memcpy of 28800 B %.0f ns; device sees the bytes: %s\n", name, ns, got == want ? "yes" : "NO");
    if (got == want) time_variants(name, p);
    (void)hipFree(d_out);
}

int main()
{
    void *p = nullptr;
    if (hipExtMallocWithFlags(&p, 1 << 16, hipDeviceMallocFinegrained) == hipSuccess) probe("fine-grained device", p);
    else printf("fine-grained device: allocation failed\n");
    void *q = nullptr;
    if (hipExtMallocWithFlags(&q, 1 << 16, hipDeviceMallocUncached) == hipSuccess) probe("uncached device", q);
    else printf("uncached device: allocation failed\n");
    void *r = nullptr;
    if (hipMalloc(&r, 1 << 16) == hipSuccess) probe("hipMalloc", r);
    return 0;
}
