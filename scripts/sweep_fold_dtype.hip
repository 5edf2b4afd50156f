// sweep_fold_dtype.hip — experiment, not part of the product: the 8:1 fold of
// config B's shape (8 x 256 MiB -> 256 MiB) for fp32, fp16 and bf16 with the
// library's own functors (nbx_functors.h: bf16 widens, adds in fp32 and
// rounds back per step), in-process A/B of tile shapes. The production shape
// runs one 256-thread workgroup per CU: one wave per SIMD, so a wave's fold
// (ALU) phase has no other wave's loads behind it on that SIMD — cheap for
// fp32 (7 adds per element), not for bf16 (unpack, add, round, repack per
// step). Variants put a second wave per SIMD or pipeline the next tile's
// loads behind the fold. Outputs compared bit-exact with the production shape.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_fold_dtype.hip -o scripts/sweep_fold_dtype
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../neuronabox-nccl_amd/csrc/nbx_functors.h"

using namespace nbx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

struct Args {
  const u32x4* src[8];
  u32x4* dst;
  uint64_t nPacks;
};

template <class Fn, int NSRC, int U>
__device__ __forceinline__ void fold(const Fn& fn, const u32x4 (&v)[NSRC][U], u32x4* dst, uint64_t p) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 acc = v[0][u];
#pragma unroll
    for (int s = 1; s < NSRC; s++) acc = fn.redPack(acc, v[s][u]);
    dst[p + u * 256] = acc;
  }
}

template <int NSRC, int U>
__device__ __forceinline__ void load(u32x4 (&v)[NSRC][U], const Args& a, uint64_t p) {
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
}

// plain: all loads of a tile, fold, store (production shape); MINB = waves-per-EU hint
template <class Fn, int NSRC, int U, int MINB>
__global__ __launch_bounds__(256, MINB) void kplain(Args a) {
  const Fn fn(0);
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    u32x4 v[NSRC][U];
    load<NSRC, U>(v, a, p);
    __builtin_amdgcn_sched_barrier(0);
    fold<Fn, NSRC, U>(fn, v, a.dst, p);
  }
}

// pipelined: tile j+1's loads issued before tile j is folded (two register sets)
template <class Fn, int NSRC, int U>
__global__ __launch_bounds__(256, 1) void kpipe(Args a) {
  const Fn fn(0);
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  uint64_t p = blockIdx.x * tile + threadIdx.x;
  if (p >= n) return;
  u32x4 x[NSRC][U], y[NSRC][U];
  load<NSRC, U>(x, a, p);
  for (;;) {
    const uint64_t q = p + stride;
    if (q < n) load<NSRC, U>(y, a, q);
    __builtin_amdgcn_sched_barrier(0);
    fold<Fn, NSRC, U>(fn, x, a.dst, p);
    if (q >= n) break;
    const uint64_t r = q + stride;
    if (r < n) load<NSRC, U>(x, a, r);
    __builtin_amdgcn_sched_barrier(0);
    fold<Fn, NSRC, U>(fn, y, a.dst, q);
    if (r >= n) break;
    p = r;
  }
}

struct Variant {
  std::string name;
  const void* fn;
  uint64_t tilePacks;
  int blocksPerCU;
};

template <class Fn>
std::vector<Variant> variants() {
  return {
      {"production u4 1/CU", (const void*)&kplain<Fn, 8, 4, 1>, 1024, 1},
      {"u2 2/CU", (const void*)&kplain<Fn, 8, 2, 2>, 512, 2},
      {"u4 2/CU", (const void*)&kplain<Fn, 8, 4, 2>, 1024, 2},
      {"u1 4/CU", (const void*)&kplain<Fn, 8, 1, 4>, 256, 4},
      {"u1 8/CU", (const void*)&kplain<Fn, 8, 1, 8>, 256, 8},
      {"pipelined u2 1/CU", (const void*)&kpipe<Fn, 8, 2>, 512, 1},
      {"pipelined u4 1/CU", (const void*)&kpipe<Fn, 8, 4>, 1024, 1},
      {"production u4 1/CU (again)", (const void*)&kplain<Fn, 8, 4, 1>, 1024, 1},
  };
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  const uint64_t bytes = 256ull << 20;   // per input
  const uint64_t nPacks = bytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t*> src(8);
  std::vector<uint32_t> h(bytes / 4);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], bytes));
    // finite values in every type's range: fp32 in [-1,1), halves from its bits
    for (uint64_t i = 0; i < h.size(); i++) {
      const uint32_t r = (uint32_t)((i * 2654435761ull + s * 977ull) % 200003ull);
      const float f = (float)r / 100001.0f - 1.0f;
      uint32_t b;
      memcpy(&b, &f, 4);
      const uint16_t lo = (uint16_t)(b >> 16), hi = (uint16_t)(((b >> 16) ^ 0x0100u) & 0xbfffu);   // bf16-ish
      h[i] = (uint32_t)lo | (uint32_t)hi << 16;
    }
    CK(hipMemcpy(src[s], h.data(), bytes, hipMemcpyHostToDevice));
  }
  uint32_t *dst, *ref;
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&ref, bytes));
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const u32x4*)src[s];
  a.nPacks = nPacks;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad = 0;
  auto run = [&](const char* tname, std::vector<Variant> vs) {
    auto launch = [&](const Variant& v, uint32_t* out) {
      Args b = a;
      b.dst = (u32x4*)out;
      uint64_t grid = std::min<uint64_t>((nPacks + v.tilePacks - 1) / v.tilePacks, (uint64_t)cus * v.blocksPerCU);
      void* args[] = {&b};
      CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(256), args, 0, 0));
    };
    launch(vs[0], ref);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> r(bytes / 4), o(bytes / 4);
    CK(hipMemcpy(r.data(), ref, bytes, hipMemcpyDeviceToHost));
    for (auto& v : vs) {
      CK(hipMemset(dst, 0, bytes));
      launch(v, dst);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(o.data(), dst, bytes, hipMemcpyDeviceToHost));
      if (memcmp(o.data(), r.data(), bytes) != 0) {
        printf("MISMATCH in %s %s\n", tname, v.name.c_str());
        bad++;
      }
    }
    std::vector<std::vector<float>> t(vs.size());
    for (int rd = 0; rd < rounds; rd++)
      for (size_t i = 0; i < vs.size(); i++) {
        launch(vs[i], dst);
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < iters; it++) launch(vs[i], dst);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[i].push_back(ms / iters);
      }
    printf("%s: 8 x 256 MiB -> 256 MiB sum, %d rounds x %d launches\n", tname, rounds, iters);
    for (size_t i = 0; i < vs.size(); i++) {
      auto x = t[i];
      std::sort(x.begin(), x.end());
      const double med = x[x.size() / 2];
      printf("  %-30s %8.4f ms %8.1f GB/s\n", vs[i].name.c_str(), med, 9.0 * bytes / (med * 1e-3) / 1e9);
    }
    fflush(stdout);
  };
  run("f32", variants<FnSumF<TyF32>>());
  run("f16", variants<FnSumF<TyF16>>());
  run("bf16", variants<FnSumF<TyBF16>>());
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
