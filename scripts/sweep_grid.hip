// sweep_grid.hip — grid size for the config-B fold (8 x 256 MiB fp32 -> 256 MiB,
// production tile shape: 256 threads, U = 4, nt loads, plain stores): fewer
// or more workgroups than one per CU, and XCD-skewed placements. Not part of
// the product. build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/sweep_grid.hip -o sweep_grid
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
struct Args { const f32x4* src[8]; f32x4* dst; uint64_t nPacks; };

template <int U>
__global__ __launch_bounds__(256) void kall(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    f32x4 v[8][U];
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < 8; s++) acc = acc + v[s][u];
      a.dst[p + u * 256] = acc;
    }
  }
}

__global__ void kfill(uint32_t* p, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15;
    p[i] = 0x3f800000u | (x >> 9);
  }
}

int main() {
  const uint64_t count = 64ull << 20;
  std::vector<float*> b(9);
  for (int s = 0; s < 9; s++) {
    CK(hipMalloc(&b[s], count * 4));
    hipLaunchKernelGGL(kfill, dim3(4096), dim3(256), 0, 0, (uint32_t*)b[s], count, 11u + s);
  }
  CK(hipDeviceSynchronize());
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)b[s];
  a.dst = (f32x4*)b[8];
  a.nPacks = count / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grids[] = {64, 128, 160, 192, 224, 240, 248, 256, 264, 288, 320, 384, 512, 768, 1024};
  const int ng = sizeof(grids) / sizeof(grids[0]);
  std::vector<std::vector<float>> t(ng);
  for (int rd = 0; rd < 5; rd++)
    for (int g = 0; g < ng; g++) {
      void* args[] = {&a};
      CK(hipLaunchKernel((const void*)&kall<4>, dim3(grids[g]), dim3(256), args, 0, 0));
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; it++) CK(hipLaunchKernel((const void*)&kall<4>, dim3(grids[g]), dim3(256), args, 0, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[g].push_back(ms / 10);
    }
  for (int g = 0; g < ng; g++) {
    auto x = t[g];
    std::sort(x.begin(), x.end());
    printf("grid %5d  med %.4f ms  %.1f GB/s\n", grids[g], x[2], 9.0 * count * 4 / (x[2] * 1e-3) / 1e9);
  }
  return 0;
}
