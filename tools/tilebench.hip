// tilebench.hip -- candidate group-tile structures for the kfec encode MAC (K=20, R=3, B=1440), real GF
// perm-MAC vs XOR-only, to pick the kernel architecture.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../kcptube_amd/csrc/kfec_gf.hpp"

using namespace kfec;
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r; asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }
__device__ __forceinline__ uint32_t pmac(uint32_t acc, const uint32_t* t, uint32_t x) {
  const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
  return xor3(acc, __builtin_amdgcn_perm(t[1], t[0], s0), __builtin_amdgcn_perm(t[3], t[2], s1)) ^ __builtin_amdgcn_perm(t[4], t[4], s2);
}
constexpr int K = 20, R = 3, B = 1440;

// A: register staging, W dwords per compute column, NT threads; tables [K][R][8] dwords in LDS
template <int W, int NT, bool GF, bool NTS>
__global__ void __launch_bounds__(NT) kA(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned G, const uint8_t* enc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s[];
  uint32_t* tb = (uint32_t*)(s + K * B);
  for (int e = threadIdx.x; e < K * R; e += NT) {
    int j = e / R, r = e % R; uint32_t t[5]; gf_perm_tables(enc[(K + r) * K + j], t);
    for (int i = 0; i < 5; ++i) tb[(j * R + r) * 8 + i] = t[i];
  }
  constexpr unsigned nv = K * B / 16, cols = B / (4 * W);
  for (unsigned g = blockIdx.x; g < G; g += gridDim.x) {
    const uint4* src = (const uint4*)(d + (size_t)g * K * B);
    __syncthreads();
#pragma unroll 8
    for (unsigned i = threadIdx.x; i < nv; i += NT) ((uint4*)s)[i] = src[i];
    __syncthreads();
    for (unsigned c = threadIdx.x; c < cols; c += NT) {
      uint32_t acc[R][W] = {};
      for (int j = 0; j < K; ++j) {
        uint32_t x[W];
        if constexpr (W == 1) x[0] = ((const uint32_t*)(s + j * B))[c];
        else if constexpr (W == 2) { uint2 v = ((const uint2*)(s + j * B))[c]; x[0] = v.x; x[1] = v.y; }
        else { uint4 v = ((const uint4*)(s + j * B))[c]; x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w; }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint4 q = *(const uint4*)(tb + (j * R + r) * 8); const uint32_t t[5] = {q.x, q.y, q.z, q.w, tb[(j * R + r) * 8 + 4]};
#pragma unroll
          for (int w = 0; w < W; ++w) acc[r][w] = GF ? pmac(acc[r][w], t, x[w]) : (acc[r][w] ^ x[w] ^ t[0]);
        }
      }
      uint8_t* o = par + (size_t)g * R * B;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if constexpr (W == 1) { if (NTS) __builtin_nontemporal_store(acc[r][0], (uint32_t*)(o + r * B) + c); else ((uint32_t*)(o + r * B))[c] = acc[r][0]; }
        else if constexpr (W == 2) ((uint2*)(o + r * B))[c] = make_uint2(acc[r][0], acc[r][1]);
        else ((uint4*)(o + r * B))[c] = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
      }
    }
  }
}

// B: tile with register prefetch of the next group (issue-early / write-late), W=2 columns, NT threads
template <int NT, bool GF, int LPT>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 5))) kB(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned G, const uint8_t* enc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s[];
  uint32_t* tb = (uint32_t*)(s + K * B);
  for (int e = threadIdx.x; e < K * R; e += NT) {
    int j = e / R, r = e % R; uint32_t t[5]; gf_perm_tables(enc[(K + r) * K + j], t);
    for (int i = 0; i < 5; ++i) tb[(j * R + r) * 8 + i] = t[i];
  }
  constexpr unsigned nv = K * B / 16, cols = B / 8;
  static_assert(LPT * NT >= nv, "prefetch covers the group");
  uint4 pf[LPT];
  unsigned g = blockIdx.x;
  {
    const uint4* src = (const uint4*)(d + (size_t)g * K * B);
#pragma unroll
    for (int k = 0; k < LPT; ++k) { const unsigned i = threadIdx.x + k * NT; if (i < nv && g < G) pf[k] = src[i]; }
  }
  for (; g < G; g += gridDim.x) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < LPT; ++k) { const unsigned i = threadIdx.x + k * NT; if (i < nv) ((uint4*)s)[i] = pf[k]; }
    __syncthreads();
    const unsigned gn = g + gridDim.x;
    if (gn < G) {
      const uint4* src = (const uint4*)(d + (size_t)gn * K * B);
#pragma unroll
      for (int k = 0; k < LPT; ++k) { const unsigned i = threadIdx.x + k * NT; if (i < nv) pf[k] = src[i]; }
    }
    const unsigned c = threadIdx.x;
    if (c < cols) {
      uint32_t acc[R][2] = {};
      for (int j = 0; j < K; ++j) {
        uint2 v = ((const uint2*)(s + j * B))[c]; uint32_t x[2] = {v.x, v.y};
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint4 q = *(const uint4*)(tb + (j * R + r) * 8); const uint32_t t[5] = {q.x, q.y, q.z, q.w, tb[(j * R + r) * 8 + 4]};
#pragma unroll
          for (int w = 0; w < 2; ++w) acc[r][w] = GF ? pmac(acc[r][w], t, x[w]) : (acc[r][w] ^ x[w] ^ t[0]);
        }
      }
      uint8_t* o = par + (size_t)g * R * B;
#pragma unroll
      for (int r = 0; r < R; ++r) ((uint2*)(o + r * B))[c] = make_uint2(acc[r][0], acc[r][1]);
    }
  }
}

int main() {
  const unsigned G = 1 << 20;
  uint8_t *d, *p, *enc; hipMalloc(&d, (size_t)G * K * B); hipMalloc(&p, (size_t)G * R * B); hipMalloc(&enc, 23 * 20);
  hipMemset(d, 0x5b, (size_t)G * K * B);
  std::vector<uint8_t> he(23 * 20, 0); for (int i = 0; i < 460; ++i) he[i] = (uint8_t)(i * 37 + 11);
  hipMemcpy(enc, he.data(), 460, hipMemcpyHostToDevice);
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double mv = (double)G * (K + R) * B;
  auto run = [&](const char* name, auto kern, int nt, int occ) {
    size_t lds = K * B + K * R * 32;
    std::vector<float> t;
    for (int i = 0; i < 6; ++i) { hipEventRecord(e0); hipLaunchKernelGGL(kern, dim3(cus * occ), dim3(nt), lds, 0, d, p, G, enc); hipEventRecord(e1); hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms); }
    std::sort(t.begin(), t.end());
    int o2 = 0; hipOccupancyMaxActiveBlocksPerMultiprocessor(&o2, (const void*)kern, nt, lds);
    printf("%-40s occ_api=%d %8.3f ms  %7.1f GB/s err=%d\n", name, o2, t[2], mv / t[2] / 1e6, (int)hipGetLastError());
  };
  run("B NT192 xor", kB<192, false, 10>, 192, 5);
  run("B NT192 gf", kB<192, true, 10>, 192, 5);
  run("B NT192 gf occ4", kB<192, true, 10>, 192, 4);
  run("B NT256 gf", kB<256, true, 8>, 256, 5);
  run("B NT384 gf", kB<384, true, 5>, 384, 5);
  run("A W1 NT256 xor", kA<1, 256, false, false>, 256, 5);
  run("A W1 NT256 gf", kA<1, 256, true, false>, 256, 5);
  run("A W1 NT256 gf ntstore", kA<1, 256, true, true>, 256, 5);
  run("A W1 NT384 gf", kA<1, 384, true, false>, 384, 5);
  run("A W1 NT512 gf", kA<1, 512, true, false>, 512, 5);
  run("A W2 NT256 gf", kA<2, 256, true, false>, 256, 5);
  run("A W2 NT192 gf", kA<2, 192, true, false>, 192, 5);
  run("A W4 NT128 gf", kA<4, 128, true, false>, 128, 5);
  run("A W1 NT256 gf occ4", kA<1, 256, true, false>, 256, 4);
  return 0;
}
