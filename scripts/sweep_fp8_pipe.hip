// sweep_fp8_pipe.hip — is the fp8 fold (VALU-heavy: widen, add, saturate,
// narrow per step) latency-bound in a way software pipelining would fix? The
// production shape (8 sources, U packs per lane per source, nontemporal
// loads, fold, store; grid-stride over tiles) against a pipelined variant
// that issues the next tile's loads before folding the current one (double
// buffer), at several unrolls and workgroups per CU, interleaved in one
// process, outputs checked against the first variant's. The functor is the
// library's own FnSumF8<TyE4M3>. Config E's shape: 8 x 128 MiB e4m3.
// Not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_fp8_pipe.hip -o scripts/sweep_fp8_pipe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../neuronabox-nccl_amd/csrc/nbx_functors.h"

using namespace nbx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)
constexpr int NSRC = 8, BLOCK = 256;

struct Args {
  const u32x4* src[NSRC];
  u32x4* dst;
  uint64_t nPacks;
};

template <int U>
__device__ __forceinline__ void load(u32x4 (&v)[NSRC][U], const Args& a, uint64_t p) {
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * BLOCK);
}
template <int U>
__device__ __forceinline__ void foldStore(const FnSumF8<TyE4M3>& fn, const u32x4 (&v)[NSRC][U], const Args& a,
                                          uint64_t p) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 acc = v[0][u];
#pragma unroll
    for (int s = 1; s < NSRC; s++) acc = fn.redPack(acc, v[s][u]);
    a.dst[p + u * BLOCK] = acc;
  }
}

template <int U>
__global__ __launch_bounds__(BLOCK) void plain(Args a) {
  const FnSumF8<TyE4M3> fn(0);
  const uint64_t tile = (uint64_t)U * BLOCK, nT = a.nPacks / tile;
  for (uint64_t t = blockIdx.x; t < nT; t += gridDim.x) {
    const uint64_t p = t * tile + threadIdx.x;
    u32x4 v[NSRC][U];
    load<U>(v, a, p);
    __builtin_amdgcn_sched_barrier(0);
    foldStore<U>(fn, v, a, p);
  }
}

template <int U>
__global__ __launch_bounds__(BLOCK) void piped(Args a) {
  const FnSumF8<TyE4M3> fn(0);
  const uint64_t tile = (uint64_t)U * BLOCK, nT = a.nPacks / tile, G = gridDim.x;
  uint64_t t = blockIdx.x;
  u32x4 A[NSRC][U], B[NSRC][U];
  if (t < nT) load<U>(A, a, t * tile + threadIdx.x);
  while (t < nT) {
    uint64_t t1 = t + G;
    if (t1 < nT) load<U>(B, a, t1 * tile + threadIdx.x);
    __builtin_amdgcn_sched_barrier(0);
    foldStore<U>(fn, A, a, t * tile + threadIdx.x);
    t = t1;
    if (t >= nT) break;
    t1 = t + G;
    if (t1 < nT) load<U>(A, a, t1 * tile + threadIdx.x);
    __builtin_amdgcn_sched_barrier(0);
    foldStore<U>(fn, B, a, t * tile + threadIdx.x);
    t = t1;
  }
}

struct V {
  const char* name;
  void (*fn)(Args);
  int perCU;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const uint64_t bytes = 128ull << 20;   // per input
  Args a{};
  std::vector<uint8_t> h(bytes);
  for (int s = 0; s < NSRC; s++) {
    void* p;
    CK(hipMalloc(&p, bytes));
    srand(7 + s);
    for (uint64_t i = 0; i < bytes; i++) h[i] = (uint8_t)(rand() & 0x77);   // finite e4m3 codes
    CK(hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice));
    a.src[s] = (const u32x4*)p;
  }
  void *dst, *ref;
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&ref, bytes));
  a.nPacks = bytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<V> vs = {{"plain U4 x4/CU (production)", plain<4>, 4}, {"plain U4 x6/CU", plain<4>, 6},
                       {"plain U2 x8/CU", plain<2>, 8},          {"piped U2 x4/CU", piped<2>, 4},
                       {"piped U2 x6/CU", piped<2>, 6},          {"piped U1 x8/CU", piped<1>, 8},
                       {"piped U4 x2/CU", piped<4>, 2}};
  std::vector<std::vector<float>> ms(vs.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < rounds; r++) {
    for (size_t k = 0; k < vs.size(); k++) {
      a.dst = (u32x4*)(k == 0 ? ref : dst);
      const dim3 grid((unsigned)(cus * vs[k].perCU));
      hipLaunchKernelGGL(vs[k].fn, grid, dim3(BLOCK), 0, 0, a);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; it++) hipLaunchKernelGGL(vs[k].fn, grid, dim3(BLOCK), 0, 0, a);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[k].push_back(t / 10);
      if (k > 0 && r == 0) {
        std::vector<uint8_t> x(bytes), y(bytes);
        CK(hipMemcpy(x.data(), ref, bytes, hipMemcpyDeviceToHost));
        CK(hipMemcpy(y.data(), dst, bytes, hipMemcpyDeviceToHost));
        if (x != y) { printf("%s: output differs\n", vs[k].name); return 3; }
      }
    }
  }
  const double alg = 9.0 * (double)bytes;
  for (size_t k = 0; k < vs.size(); k++) {
    std::sort(ms[k].begin(), ms[k].end());
    const float med = ms[k][ms[k].size() / 2];
    printf("%-28s median %.4f ms  %.0f GB/s\n", vs[k].name, med, alg / med / 1e6);
  }
  return 0;
}
