// sweep_variants.hip — standalone microbenchmark of kernel shapes for the
// config-B hot loop (8 x 256 MiB fp32 -> 256 MiB, ordered left fold).
// Not part of the product: used to choose the production kernel's shape.
// Each variant is checked bit-exact against variant 0's output; timing is
// interleaved across variants (rounds x variants) in one process.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_variants.hip -o sweep
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

// LPOL: 0 plain, 1 nontemporal, 3 no load (write-only ceiling: synthesises the value)
template <int POL>
__device__ __forceinline__ f32x4 ld(const f32x4* p) {
  if constexpr (POL == 1) return __builtin_nontemporal_load(p);
  else if constexpr (POL == 3) { float x = (float)(uintptr_t)p; return (f32x4){x, x, x, x}; }
  else return *p;
}
// SPOL: 0 plain, 1 nontemporal, 2 no store (read-only ceiling; store kept live behind a never-true test)
template <int POL>
__device__ __forceinline__ void st(f32x4* p, f32x4 v) {
  if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
  else if constexpr (POL == 2) { if (v.x == 1234567.f && v.y == -7654321.f) *p = v; }
  else *p = v;
}

// MAP 0: grid-stride tiles; MAP 1: each block owns a contiguous range of tiles
template <int NSRC, int BLOCK, int U, int LPOL, int SPOL, int MAP>
__global__ __launch_bounds__(BLOCK) void kvar(Args a) {
  const uint64_t n = a.nPacks;
  constexpr uint64_t tile = (uint64_t)U * BLOCK;
  uint64_t begin, end, stride;
  if constexpr (MAP == 0) {
    begin = (uint64_t)blockIdx.x * tile;
    end = n;
    stride = (uint64_t)gridDim.x * tile;
  } else {
    uint64_t tiles = (n + tile - 1) / tile;
    uint64_t per = (tiles + gridDim.x - 1) / gridDim.x;
    begin = (uint64_t)blockIdx.x * per * tile;
    end = std::min<uint64_t>(n, begin + per * tile);
    stride = tile;
  }
  for (uint64_t p = begin + threadIdx.x; p < end; p += stride) {
    f32x4 v[NSRC][U];
    if (p + (U - 1) * BLOCK < end) {
#pragma unroll
      for (int s = 0; s < NSRC; s++)
#pragma unroll
        for (int u = 0; u < U; u++) v[s][u] = ld<LPOL>(a.src[s] + p + u * BLOCK);
#pragma unroll
      for (int u = 0; u < U; u++) {
        f32x4 acc = v[0][u];
#pragma unroll
        for (int s = 1; s < NSRC; s++) acc = acc + v[s][u];
        st<SPOL>(a.dst + p + u * BLOCK, acc);
      }
    } else {
      for (int u = 0; u < U; u++) {
        uint64_t q = p + (uint64_t)u * BLOCK;
        if (q < end) {
          f32x4 acc = ld<LPOL>(a.src[0] + q);
#pragma unroll
          for (int s = 1; s < NSRC; s++) acc = acc + ld<LPOL>(a.src[s] + q);
          st<SPOL>(a.dst + q, acc);
        }
      }
    }
  }
}

// Software-pipelined variant: the next tile's loads are issued before the
// current tile is folded and stored (loads always in flight per wave).
template <int NSRC, int U, int SPOL>
__global__ __launch_bounds__(256) void kpipe(Args a) {
  const uint64_t n = a.nPacks;
  constexpr uint64_t tile = (uint64_t)U * 256;
  const uint64_t stride = (uint64_t)gridDim.x * tile;
  uint64_t p = (uint64_t)blockIdx.x * tile + threadIdx.x;
  if (p + (U - 1) * 256 >= n) return;   // sweep sizes: every tile full
  f32x4 c[NSRC][U], x[NSRC][U];
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) c[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
  for (;;) {
    const uint64_t q = p + stride;
    const bool more = q + (U - 1) * 256 < n;
    if (more) {
#pragma unroll
      for (int s = 0; s < NSRC; s++)
#pragma unroll
        for (int u = 0; u < U; u++) x[s][u] = __builtin_nontemporal_load(a.src[s] + q + u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = c[0][u];
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = acc + c[s][u];
      st<SPOL>(a.dst + p + u * 256, acc);
    }
    if (!more) break;
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) c[s][u] = x[s][u];
    p = q;
  }
}

struct Variant {
  std::string name;
  const void* fn;
  int block, unroll, blocksPerCU;
};

#define V(NS, B, U, L, S, M, BPC) \
  Variant{#NS "src b" #B " u" #U " ld" #L " st" #S " map" #M " bpc" #BPC, (const void*)&kvar<NS, B, U, L, S, M>, B, U, BPC}

int placement(int rounds);
int lowsrc(int rounds);

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[2]) == "placement") return placement(argc > 1 ? atoi(argv[1]) : 5);
  if (argc > 2 && std::string(argv[2]) == "lowsrc") return lowsrc(argc > 1 ? atoi(argv[1]) : 5);
  const uint64_t count = 64ull << 20;   // fp32 per input
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const int iters = 10;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float*> src(8);
  std::vector<float> h(count);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], count * 4));
    srand(1234 + s);
    for (uint64_t i = 0; i < count; i++) h[i] = (float)((double)rand() / RAND_MAX * 2.0 - 1.0);
    CK(hipMemcpy(src[s], h.data(), count * 4, hipMemcpyHostToDevice));
  }
  float *dst, *ref;
  CK(hipMalloc(&dst, count * 4));
  CK(hipMalloc(&ref, count * 4));

  std::vector<Variant> vs = {
      V(8, 256, 1, 0, 0, 0, 8),  V(8, 256, 2, 1, 0, 0, 1),  V(8, 256, 2, 1, 0, 0, 2),  V(8, 256, 2, 1, 0, 0, 4),
      V(8, 256, 4, 1, 0, 0, 1),  V(8, 256, 4, 1, 0, 0, 2),  V(8, 256, 2, 1, 1, 0, 2),  V(8, 256, 4, 1, 1, 0, 1),
      V(8, 512, 2, 1, 0, 0, 1),  V(8, 512, 4, 1, 0, 0, 1),  V(8, 256, 1, 1, 1, 1, 8),  V(8, 256, 1, 1, 0, 0, 2),
      V(8, 256, 8, 1, 0, 0, 1),  V(8, 256, 2, 1, 0, 1, 2),  V(8, 256, 4, 1, 0, 1, 1),  V(8, 1024, 2, 1, 0, 0, 1),
  };
  std::vector<Variant> ro = {V(8, 256, 2, 1, 2, 0, 2), V(8, 256, 4, 1, 2, 0, 1), V(8, 256, 2, 0, 2, 0, 2),
                             V(1, 256, 4, 3, 0, 0, 2), V(1, 256, 4, 3, 1, 0, 2), V(1, 256, 8, 3, 1, 0, 1)};
  // copy ceilings: 1 source -> 1 dst (256 MiB copy), and 2 sources
  std::vector<Variant> cs = {V(1, 256, 4, 0, 0, 0, 8), V(1, 256, 4, 1, 1, 0, 8), V(2, 256, 2, 0, 0, 0, 8)};

  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.nPacks = count / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  auto launch = [&](const Variant& v, float* out) {
    Args b = a;
    b.dst = (f32x4*)out;
    uint64_t tile = (uint64_t)v.unroll * v.block;
    uint64_t tiles = (b.nPacks + tile - 1) / tile;
    uint64_t grid = std::min<uint64_t>(tiles, (uint64_t)cus * v.blocksPerCU);
    void* args[] = {&b};
    CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.block), args, 0, 0));
  };
  // reference output from variant 0
  launch(vs[0], ref);
  CK(hipDeviceSynchronize());
  std::vector<float> r(count), o(count);
  CK(hipMemcpy(r.data(), ref, count * 4, hipMemcpyDeviceToHost));
  for (size_t vi = 0; vi < 16; vi++) {
    auto& v = vs[vi];
    CK(hipMemset(dst, 0, count * 4));
    launch(v, dst);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dst, count * 4, hipMemcpyDeviceToHost));
    if (memcmp(o.data(), r.data(), count * 4) != 0) printf("MISMATCH in %s\n", v.name.c_str());
  }
  vs.insert(vs.end(), ro.begin(), ro.end());
  const size_t nCheck = vs.size() - ro.size();
  std::vector<std::vector<float>> times(vs.size() + cs.size());
  for (int rd = 0; rd < rounds; rd++) {
    for (size_t i = 0; i < vs.size() + cs.size(); i++) {
      const Variant& v = i < vs.size() ? vs[i] : cs[i - vs.size()];
      launch(v, dst);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; it++) launch(v, dst);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      times[i].push_back(ms / iters);
    }
  }
  (void)nCheck;
  printf("%-44s %10s %10s %9s\n", "variant (last 6 of 8src list: read-only x3, write-only x3)", "med_ms", "min_ms", "GB/s(med)");
  for (size_t i = 0; i < times.size(); i++) {
    const Variant& v = i < vs.size() ? vs[i] : cs[i - vs.size()];
    int nsrc = i < vs.size() ? 8 : (i - vs.size() < 2 ? 1 : 2);
    double bytes = (double)(nsrc + 1) * count * 4;
    if (i >= nCheck && i < vs.size()) {   // ceilings
      const bool writeOnly = (i - nCheck) >= 3;
      bytes = writeOnly ? (double)count * 4 : 8.0 * count * 4;
    }
    auto t = times[i];
    std::sort(t.begin(), t.end());
    double med = t[t.size() / 2];
    printf("%-44s %10.4f %10.4f %9.1f\n", v.name.c_str(), med, t[0], bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}

// Source placement experiment: one arena, sources `stride` bytes apart.
int placement(int rounds) {
  const uint64_t count = 64ull << 20;
  const uint64_t bytes = count * 4;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t extra[] = {0, 4096, 65536 + 1024, (2u << 20) + 8192, 256 * 1024 + 4096 * 3};
  const int nP = 5;
  char* arena;
  const uint64_t arenaBytes = 10 * (bytes + (4u << 20));
  CK(hipMalloc(&arena, arenaBytes));
  CK(hipMemset(arena, 0, arenaBytes));
  std::vector<float*> sep(9);
  for (int s = 0; s < 9; s++) {
    CK(hipMalloc(&sep[s], bytes));
    CK(hipMemset(sep[s], 0, bytes));
  }
  std::vector<Variant> vs = {V(8, 256, 4, 1, 0, 0, 1), V(8, 256, 2, 1, 0, 0, 2)};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // placement -1 = separate allocations
  std::vector<std::vector<float>> t((nP + 1) * vs.size());
  for (int rd = 0; rd < rounds; rd++) {
    for (int pl = -1; pl < nP; pl++) {
      Args a;
      for (int s = 0; s < 8; s++)
        a.src[s] = pl < 0 ? (const f32x4*)sep[s] : (const f32x4*)(arena + s * (bytes + extra[pl]));
      a.dst = pl < 0 ? (f32x4*)sep[8] : (f32x4*)(arena + 8 * (bytes + extra[pl]));
      a.nPacks = count / 4;
      for (size_t vi = 0; vi < vs.size(); vi++) {
        const Variant& v = vs[vi];
        uint64_t tile = (uint64_t)v.unroll * v.block;
        uint64_t grid = std::min<uint64_t>((a.nPacks + tile - 1) / tile, (uint64_t)cus * v.blocksPerCU);
        void* args[] = {&a};
        CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.block), args, 0, 0));
        CK(hipEventRecord(e0, 0));
        for (int it = 0; it < 10; it++) CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.block), args, 0, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[(pl + 1) * vs.size() + vi].push_back(ms / 10);
      }
    }
  }
  for (int pl = -1; pl < nP; pl++)
    for (size_t vi = 0; vi < vs.size(); vi++) {
      auto x = t[(pl + 1) * vs.size() + vi];
      std::sort(x.begin(), x.end());
      double med = x[x.size() / 2];
      printf("placement %-10s extra=%-8llu %-40s med %.4f ms  %.1f GB/s\n", pl < 0 ? "separate" : "arena",
             pl < 0 ? 0ull : (unsigned long long)extra[pl], vs[vi].name.c_str(), med, 9.0 * bytes / (med * 1e-3) / 1e9);
    }
  return 0;
}

// Store policy vs read:write ratio: nSrcs in {1, 2, 3, 4, 8}, plain vs nt stores.
int lowsrc(int rounds) {
  const uint64_t count = 64ull << 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float*> src(9);
  for (int s = 0; s < 9; s++) {
    CK(hipMalloc(&src[s], count * 4));
    CK(hipMemset(src[s], 0, count * 4));
  }
  struct LV { Variant v; int nsrc; };
  std::vector<LV> vs = {
      {V(1, 256, 16, 1, 0, 0, 1), 1}, {V(1, 256, 16, 1, 1, 0, 1), 1}, {V(1, 256, 8, 1, 1, 0, 2), 1}, {V(1, 256, 4, 1, 1, 0, 4), 1},
      {V(2, 256, 16, 1, 0, 0, 1), 2}, {V(2, 256, 16, 1, 1, 0, 1), 2}, {V(2, 256, 8, 1, 1, 0, 2), 2}, {V(2, 256, 4, 1, 1, 0, 4), 2},
      {V(3, 256, 8, 1, 0, 0, 1), 3},  {V(3, 256, 8, 1, 1, 0, 1), 3},  {V(3, 256, 4, 1, 1, 0, 2), 3},
      {V(4, 256, 8, 1, 0, 0, 1), 4},  {V(4, 256, 8, 1, 1, 0, 1), 4},  {V(4, 256, 4, 1, 1, 0, 2), 4},
      {V(8, 256, 4, 1, 0, 0, 1), 8},  {V(8, 256, 4, 1, 1, 0, 1), 8},
      {Variant{"8src pipelined u4 st0 bpc1", (const void*)&kpipe<8, 4, 0>, 256, 4, 1}, 8},
      {Variant{"8src pipelined u2 st0 bpc1", (const void*)&kpipe<8, 2, 0>, 256, 2, 1}, 8},
      {Variant{"8src pipelined u2 st0 bpc2", (const void*)&kpipe<8, 2, 0>, 256, 2, 2}, 8},
      {Variant{"2src pipelined u8 st1 bpc1", (const void*)&kpipe<2, 8, 1>, 256, 8, 1}, 2},
      {Variant{"2src pipelined u8 st0 bpc1", (const void*)&kpipe<2, 8, 0>, 256, 8, 1}, 2},
  };
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.dst = (f32x4*)src[8];
  a.nPacks = count / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(vs.size());
  for (int rd = 0; rd < rounds; rd++)
    for (size_t i = 0; i < vs.size(); i++) {
      const Variant& v = vs[i].v;
      uint64_t tile = (uint64_t)v.unroll * v.block;
      uint64_t grid = std::min<uint64_t>((a.nPacks + tile - 1) / tile, (uint64_t)cus * v.blocksPerCU);
      void* args[] = {&a};
      CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.block), args, 0, 0));
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; it++) CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.block), args, 0, 0));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / 10);
    }
  for (size_t i = 0; i < vs.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    double med = x[x.size() / 2];
    printf("%-44s med %.4f ms  %.1f GB/s\n", vs[i].v.name.c_str(), med, (vs[i].nsrc + 1.0) * count * 4 / (med * 1e-3) / 1e9);
  }
  return 0;
}
