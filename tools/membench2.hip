// membench2.hip -- variants of the kfec shard access pattern (K=20 R=3, plain XOR, no GF math) to choose the
// kernel architecture.  All: lane-level 16-B accesses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NTL, bool NTS>
__global__ void k_allk(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned total, unsigned cols, unsigned B) {
  constexpr int K = 20, R = 3;
  for (unsigned it = blockIdx.x * 256 + threadIdx.x; it < total; it += gridDim.x * 256) {
    unsigned g = it / cols, c = it - g * cols;
    const uint8_t* p = d + (size_t)g * K * B + c * 16;
    u32x4 v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) v[j] = NTL ? __builtin_nontemporal_load((const u32x4*)(p + (size_t)j * B)) : *(const u32x4*)(p + (size_t)j * B);
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < K; ++j) acc ^= v[j];
    uint8_t* o = par + (size_t)g * R * B + c * 16;
#pragma unroll
    for (int r = 0; r < R; ++r) { if (NTS) __builtin_nontemporal_store(acc, (u32x4*)(o + (size_t)r * B)); else *(u32x4*)(o + (size_t)r * B) = acc; acc.x += 1; }
  }
}

// LDS-staged: one block = one group per iteration; the group's K*B bytes (line-aligned as a whole) are read
// linearly into LDS, then 360 dword columns are XOR-reduced from LDS.
template <int TG>
__global__ void __launch_bounds__(256) k_lds(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned G, unsigned B) {
  constexpr int K = 20, R = 3;
  extern __shared__ __attribute__((aligned(16))) uint8_t s[];
  const unsigned gbytes = K * B;  // 28800
  const unsigned nv = TG * gbytes / 16;
  for (unsigned g0 = blockIdx.x * TG; g0 < G; g0 += gridDim.x * TG) {
    const uint4* src = (const uint4*)(d + (size_t)g0 * gbytes);
    __syncthreads();
    for (unsigned i = threadIdx.x; i < nv; i += 256) ((uint4*)s)[i] = src[i];
    __syncthreads();
    const unsigned ncol = TG * (B / 4);
    for (unsigned c = threadIdx.x; c < ncol; c += 256) {
      unsigned gl = c / (B / 4), cc = c - gl * (B / 4);
      const uint32_t* q = (const uint32_t*)(s + gl * gbytes) + cc;
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) acc ^= q[j * (B / 4)];
      uint32_t* o = (uint32_t*)(par + (size_t)(g0 + gl) * R * B) + cc;
#pragma unroll
      for (int r = 0; r < R; ++r) o[r * (B / 4)] = acc + r;
    }
  }
}

// LDS-DMA staged (global_load_lds_dwordx4), double-buffered per block
__global__ void __launch_bounds__(256) k_ldsdma(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned G, unsigned B) {
  constexpr int K = 20, R = 3;
  extern __shared__ __attribute__((aligned(16))) uint8_t s[];
  const unsigned gbytes = K * B;
  const unsigned nchunks = gbytes / 1024 + ((gbytes % 1024) ? 1 : 0);  // 1-KB wave chunks (last partial)
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  auto issue = [&](unsigned g, int buf) {
    const uint8_t* src = d + (size_t)g * gbytes;
    for (unsigned ch = wave; ch < nchunks; ch += 4) {
      unsigned off = ch * 1024 + lane * 16;
      if (off < gbytes)
        __builtin_amdgcn_global_load_lds((const void*)(src + off), (__attribute__((address_space(3))) void*)(s + buf * 30720 + ch * 1024), 16, 0, 0);
    }
  };
  unsigned g = blockIdx.x;
  int buf = 0;
  if (g < G) issue(g, 0);
  for (; g < G; g += gridDim.x) {
    unsigned gn = g + gridDim.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (gn < G) issue(gn, buf ^ 1);
    const unsigned ncol = B / 4;
    for (unsigned c = threadIdx.x; c < ncol; c += 256) {
      const uint32_t* q = (const uint32_t*)(s + buf * 30720) + c;
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) acc ^= q[j * (B / 4)];
      uint32_t* o = (uint32_t*)(par + (size_t)g * R * B) + c;
#pragma unroll
      for (int r = 0; r < R; ++r) o[r * (B / 4)] = acc + r;
    }
    buf ^= 1;
  }
}

__global__ void k_copy4(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
    uint4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    b[i] = v0; b[i + stride] = v1; b[i + 2 * stride] = v2; b[i + 3 * stride] = v3;
  }
}

int main() {
  const size_t bytes = 32ull << 30;
  uint8_t *a, *b; hipMalloc(&a, bytes); hipMalloc(&b, bytes / 2);
  hipMemset(a, 1, bytes); hipMemset(b, 0, bytes / 2);
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, double moved, auto launch) {
    std::vector<float> t;
    for (int i = 0; i < 7; ++i) { hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    printf("%-34s %8.3f ms  %7.1f GB/s  (err %d)\n", name, t[3], moved / t[3] / 1e6, (int)hipGetLastError());
  };
  run("copy4 16GB", bytes, [&] { k_copy4<<<cus * 8, 256>>>((const uint4*)a, (uint4*)b, bytes / 32); });
  const unsigned B = 1440, K = 20, R = 3; const size_t G = 1 << 20; const unsigned cols = B / 16; const unsigned total = G * cols;
  const double mv = (double)G * (K + R) * B;
  for (int occ : {2, 4, 8})  { char n[64]; snprintf(n, 64, "allk grid %d/CU", occ); run(n, mv, [&] { k_allk<false,false><<<cus * occ, 256>>>(a, b, total, cols, B); }); }
  run("allk ntload", mv, [&] { k_allk<true,false><<<cus * 4, 256>>>(a, b, total, cols, B); });
  run("allk ntstore", mv, [&] { k_allk<false,true><<<cus * 4, 256>>>(a, b, total, cols, B); });
  run("allk nt both", mv, [&] { k_allk<true,true><<<cus * 4, 256>>>(a, b, total, cols, B); });
  for (int occ : {4, 5}) { char n[64]; snprintf(n, 64, "lds TG1 %d/CU", occ); run(n, mv, [&] { k_lds<1><<<cus * occ, 256, 28800>>>(a, b, G, B); }); }
  run("lds TG2 2/CU", mv, [&] { k_lds<2><<<cus * 2, 256, 57600>>>(a, b, G, B); });
  for (int occ : {1, 2}) { char n[64]; snprintf(n, 64, "ldsdma dbuf %d/CU", occ); run(n, mv, [&] { k_ldsdma<<<cus * occ, 256, 61440>>>(a, b, G, B); }); }
  return 0;
}
