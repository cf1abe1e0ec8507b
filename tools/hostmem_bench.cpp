// hostmem_bench.cpp -- what the per-call worker's host side costs: memcpy of one 20:3 group (28 800 B) into,
// and of its parity (4 320 B) out of, pinned host memory of each hipHostMalloc kind vs plain malloc memory.
// Prints one JSON line (ns per copy).
// Build: g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I /opt/rocm/include tools/hostmem_bench.cpp
//        -o tools/hostmem_bench -L /opt/rocm/lib -lamdhip64
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

static double ns_per(const std::chrono::steady_clock::time_point &t0, int reps)
{
    return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / reps;
}

int main()
{
    const size_t in = 28800, out = 4320;
    std::vector<uint8_t> src(in, 7), dst(out);
    struct Kind { const char *name; unsigned flags; bool pinned; };
    const Kind kinds[] = {{"malloc", 0, false},
                          {"coherent", hipHostMallocCoherent, true},
                          {"noncoherent", hipHostMallocNonCoherent, true},
                          {"default", hipHostMallocDefault, true},
                          {"writecombined", hipHostMallocWriteCombined, true}};
    std::string js = "{\"metric\": \"host memcpy ns (28800 B in, 4320 B out)\"";
    for (const Kind &k : kinds) {
        void *p = nullptr;
        if (k.pinned) {
            if (hipHostMalloc(&p, 1 << 17, k.flags) != hipSuccess) continue;
        } else {
            p = aligned_alloc(4096, 1 << 17);
        }
        uint8_t *b = static_cast<uint8_t *>(p);
        std::memset(b, 0, 1 << 17);
        const int reps = 20000;
        for (int i = 0; i < 100; ++i) std::memcpy(b, src.data(), in);
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            src[i & 1023] = (uint8_t)i;
            std::memcpy(b, src.data(), in);
        }
        const double tin = ns_per(t0, reps);
        t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < reps; ++i) {
            std::memcpy(dst.data(), b + 32768, out);
            b[32768 + (i & 1023)] ^= 1;
        }
        const double tout = ns_per(t0, reps);
        js += std::string(", \"") + k.name + "_in_ns\": " + std::to_string(tin) + ", \"" + k.name +
              "_out_ns\": " + std::to_string(tout);
        if (k.pinned) (void)hipHostFree(p);
        else free(p);
    }
    printf("%s}\n", js.c_str());
    return 0;
}
