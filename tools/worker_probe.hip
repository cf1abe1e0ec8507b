// worker_probe.hip -- diagnostic for the resident-worker pattern of kfec_worker.hip: does a kernel that polls a
// word in fine-grained pinned host memory run, see the host's store, advance its wall clock and make its
// own stores visible to the host?  Prints one line per phase.  Bounded: every kernel exits on its own
// after `ticks` of the 100 MHz wall clock, and the host gives up after 2 s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/worker_probe.hip -o tools/worker_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>

__global__ void __launch_bounds__(512) probe(uint64_t *h, uint64_t ticks, int use_lds)
{
    extern __shared__ uint64_t lds[];
    __shared__ uint64_t s_v;
    if (threadIdx.x == 0) {
        const uint64_t t0 = wall_clock64();
        __hip_atomic_store(&h[1], t0 | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        uint64_t n = 0, v = 0;
        for (;;) {
            v = __hip_atomic_load(&h[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ++n;
            __hip_atomic_store(&h[2], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&h[3], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v == 42) break;
            if (wall_clock64() - t0 > ticks) break;
            __builtin_amdgcn_s_sleep(4);
        }
        s_v = v;
    }
    __syncthreads();
    if (use_lds) lds[threadIdx.x] = s_v + threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(&h[4], s_v == 42 ? 1ull : 2ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static uint64_t ld(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

static int run(const char *name, unsigned flags, int threads, size_t lds)
{
    uint64_t *h = nullptr;
    if (hipHostMalloc((void **)&h, 4096, flags) != hipSuccess) { printf("%s: hipHostMalloc failed\n", name); return 1; }
    std::memset(h, 0, 4096);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipLaunchKernelGGL(probe, dim3(1), dim3(threads), lds, s, h, (uint64_t)100000000 /* 1 s */, lds ? 1 : 0);
    const hipError_t le = hipGetLastError();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    printf("%s: launch=%d after 20ms: started=%llx polls=%llu clock=%llu query=%d\n", name, (int)le,
           (unsigned long long)ld(&h[1]), (unsigned long long)ld(&h[2]), (unsigned long long)ld(&h[3]),
           (int)hipStreamQuery(s));
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(&h[0], 42ull, __ATOMIC_SEQ_CST);
    while (ld(&h[4]) == 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) __builtin_ia32_pause();
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("%s: result=%llu after %.1f us polls=%llu clock=%llu\n", name, (unsigned long long)ld(&h[4]), us,
           (unsigned long long)ld(&h[2]), (unsigned long long)ld(&h[3]));
    for (int i = 0; i < 300 && hipStreamQuery(s) == hipErrorNotReady; ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    printf("%s: stream query at end=%d\n", name, (int)hipStreamQuery(s));
    fflush(stdout);
    return 0;
}

int main()
{
    run("coherent-1t", hipHostMallocCoherent, 64, 0);
    run("coherent-512t", hipHostMallocCoherent, 512, 0);
    run("coherent-512t-lds63k", hipHostMallocCoherent, 512, 63360 - 4096);
    run("default-512t", hipHostMallocDefault, 512, 0);
    run("mapped-512t", hipHostMallocMapped | hipHostMallocCoherent, 512, 0);
    return 0;
}
