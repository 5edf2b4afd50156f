// sweep_data.hip — does the DATA change HBM throughput? The same kernels
// (1:1 copy, 2:1 and 8:1 fp32 sum; nt loads, plain stores, production tile
// shapes) over buffers holding zeros, a constant, or random bits. Not part of
// the product: it explains the zero-filled ceilings of the lowsrc sweep.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_data.hip -o sweep_data
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args { const f32x4* src[8]; f32x4* dst; uint64_t nPacks; };

template <int NSRC, int U>
__global__ __launch_bounds__(256) void kfold(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    f32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = acc + v[s][u];
      a.dst[p + u * 256] = acc;
    }
  }
}

__global__ void kfillRandom(uint32_t* p, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    p[i] = 0x3f800000u | (x >> 9);   // random float in [1, 2): random mantissa bits
  }
}

int main() {
  const uint64_t count = 64ull << 20;   // fp32 per buffer (256 MiB)
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float*> b(9);
  for (auto& p : b) CK(hipMalloc(&p, count * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* dataName[3] = {"zeros", "const 1.0", "random"};
  struct K { const char* name; const void* fn; int nsrc, u; };
  K ks[3] = {{"copy 1:1 u16", (const void*)&kfold<1, 16>, 1, 16}, {"sum 2:1 u16", (const void*)&kfold<2, 16>, 2, 16},
             {"sum 8:1 u4", (const void*)&kfold<8, 4>, 8, 4}};
  for (int rd = 0; rd < 3; rd++)
    for (int d = 0; d < 3; d++) {
      for (int s = 0; s < 9; s++) {
        if (d == 0) CK(hipMemset(b[s], 0, count * 4));
        else if (d == 1) CK(hipMemsetD32((hipDeviceptr_t)b[s], 0x3f800000, count));
        else hipLaunchKernelGGL(kfillRandom, dim3(4096), dim3(256), 0, 0, (uint32_t*)b[s], count, 77u + s);
      }
      CK(hipDeviceSynchronize());
      for (auto& k : ks) {
        Args a;
        for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)b[s];
        a.dst = (f32x4*)b[8];
        a.nPacks = count / 4;
        uint64_t tile = (uint64_t)k.u * 256;
        uint64_t grid = std::min<uint64_t>((a.nPacks + tile - 1) / tile, (uint64_t)cus);
        void* args[] = {&a};
        CK(hipLaunchKernel(k.fn, dim3((unsigned)grid), dim3(256), args, 0, 0));
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < 10; it++) CK(hipLaunchKernel(k.fn, dim3((unsigned)grid), dim3(256), args, 0, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        printf("round %d  data %-9s  %-14s  %.4f ms  %7.1f GB/s\n", rd, dataName[d], k.name, ms,
               (k.nsrc + 1.0) * count * 4 / (ms * 1e-3) / 1e9);
      }
    }
  return 0;
}
