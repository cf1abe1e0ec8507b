// membench.hip -- HBM calibration on the box: what simple streams reach, to price the kfec access pattern.
//   read:   every lane sums 16-B loads over a linear buffer (grid-stride)
//   copy:   16-B load + 16-B store, linear
//   r7w1:   read 7 x 16 B, write 1 x 16 B (the encode read:write ratio at 20:3 is 6.7:1)
//   shards: the kfec pattern -- lane = (group, 16-B column), reads the column of 20 shards 1440 B apart,
//           writes 3 columns -- with plain XOR (no GF arithmetic)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ void k_read(const uint4* __restrict__ a, size_t n, uint4* __restrict__ sink) {
  uint4 acc = make_uint4(0,0,0,0);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = a[i]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = acc;
}
__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void k_r7w1(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n8) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    size_t blk = i / 64, l = i % 64;  // 8 consecutive 1-KB wave chunks: 7 read, 1 write
    const uint4* p = a + blk * 512 + l;
    uint4 acc = p[0];
#pragma unroll
    for (int k = 1; k < 7; ++k) { uint4 v = p[k * 64]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    b[blk * 64 + l] = acc;
  }
}
__global__ void k_shards(const uint8_t* __restrict__ d, uint8_t* __restrict__ par, unsigned total, unsigned cols, unsigned K, unsigned R, unsigned B) {
  for (unsigned it = blockIdx.x * 256 + threadIdx.x; it < total; it += gridDim.x * 256) {
    unsigned g = it / cols, c = it - g * cols;
    const uint8_t* p = d + (size_t)g * K * B + c * 16;
    uint4 acc = make_uint4(0,0,0,0);
    for (unsigned j = 0; j < K; ++j) { uint4 v = *(const uint4*)(p + (size_t)j * B); acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    uint8_t* o = par + (size_t)g * R * B + c * 16;
    for (unsigned r = 0; r < R; ++r) { *(uint4*)(o + (size_t)r * B) = acc; acc.x += 1; }
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
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, t[3], moved / t[3] / 1e6);
  };
  size_t n = bytes / 16;
  for (int occ : {4, 8, 16}) {
    char nm[64];
    snprintf(nm, 64, "read grid=%d/CU", occ);
    run(nm, bytes, [&] { k_read<<<cus * occ, 256>>>((const uint4*)a, n, (uint4*)b); });
  }
  run("copy 16GB->16GB", bytes, [&] { k_copy<<<cus * 8, 256>>>((const uint4*)a, (uint4*)b, n / 2); });
  run("r7w1", bytes / 8 * 7 + bytes / 8 / 7 * 1.0 * 7 / 7, [&] { k_r7w1<<<cus * 8, 256>>>((const uint4*)a, (uint4*)b, n / 8); });
  for (unsigned B : {1440u, 1408u, 1536u, 1424u}) {
    unsigned K = 20, R = 3; size_t G = (30ull << 30) / (K * B); if (G * R * B > bytes / 2) G = bytes / 2 / (R * B);
    unsigned cols = B / 16; unsigned total = (unsigned)(G * cols);
    char nm[64]; snprintf(nm, 64, "shards B=%u G=%zu", B, G);
    for (int occ : {7, 8}) {
      char nm2[80]; snprintf(nm2, 80, "%s occ%d", nm, occ);
      run(nm2, (double)G * (K + R) * B, [&] { k_shards<<<cus * occ, 256>>>(a, b, total, cols, K, R, B); });
    }
  }
  return 0;
}
