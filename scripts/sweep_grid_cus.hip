// sweep_grid_cus.hip — does the config-B fold run faster on fewer CUs?
// The production shape (8 sources, 4 packs per lane per source, 16-B
// nontemporal loads, plain stores, 256-thread workgroups) as a grid-stride
// kernel on grids of 64 ... 512 workgroups (one per CU up to 256), rounds
// interleaved in one process, outputs checked against the first grid's.
// Config B's bytes: 8 x 256 MiB fp32 -> 256 MiB. Not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_grid_cus.hip -o scripts/sweep_grid_cus
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NSRC = 8, U = 4, BLOCK = 256;

struct Args {
  const f32x4* src[NSRC];
  f32x4* dst;
  uint64_t nPacks;
};

__global__ __launch_bounds__(BLOCK) void fold(Args a) {
  const uint64_t tile = (uint64_t)U * BLOCK;
  const uint64_t nTiles = a.nPacks / tile;
  for (uint64_t t = blockIdx.x; t < nTiles; t += gridDim.x) {
    const uint64_t p = t * tile + threadIdx.x;
    f32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * BLOCK);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc += v[s][u];
      a.dst[p + u * BLOCK] = acc;
    }
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const uint64_t count = 64ull << 20;   // fp32 per input: 256 MiB
  const uint64_t nPacks = count / 4;
  Args a{};
  std::vector<float> h(count);
  for (int s = 0; s < NSRC; s++) {
    float* p;
    CK(hipMalloc(&p, count * 4));
    for (uint64_t i = 0; i < count; i++) h[i] = (float)((i * 7 + 13 * s) % 1024) * 0.25f;
    CK(hipMemcpy(p, h.data(), count * 4, hipMemcpyHostToDevice));
    a.src[s] = (const f32x4*)p;
  }
  float *dst, *ref;
  CK(hipMalloc(&dst, count * 4));
  CK(hipMalloc(&ref, count * 4));
  a.nPacks = nPacks;
  const std::vector<int> grids = {256, 64, 128, 192, 224, 240, 320, 384, 512};
  std::vector<std::vector<float>> ms(grids.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 9.0 * (double)count * 4.0;
  for (int r = 0; r < rounds; r++) {
    for (size_t g = 0; g < grids.size(); g++) {
      a.dst = (f32x4*)(g == 0 ? ref : dst);
      hipLaunchKernelGGL(fold, dim3(grids[g]), dim3(BLOCK), 0, 0, a);   // warm
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; it++) hipLaunchKernelGGL(fold, dim3(grids[g]), dim3(BLOCK), 0, 0, a);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[g].push_back(t / 10);
      if (g > 0 && r == 0) {
        std::vector<float> x(count), y(count);
        CK(hipMemcpy(x.data(), ref, count * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(y.data(), dst, count * 4, hipMemcpyDeviceToHost));
        if (x != y) { printf("grid %d: output differs\n", grids[g]); return 3; }
      }
    }
  }
  for (size_t g = 0; g < grids.size(); g++) {
    std::sort(ms[g].begin(), ms[g].end());
    const float med = ms[g][ms[g].size() / 2], best = ms[g][0];
    printf("grid %4d  median %.4f ms (%.0f GB/s)  best %.4f ms (%.0f GB/s)\n", grids[g], med, bytes / med / 1e6,
           best, bytes / best / 1e6);
  }
  return 0;
}
