// sweep_dyn_xcd.hip — experiment, not part of the product: the cost of the
// dynamic tile counter at mid sizes. The library's dynamic schedule (one
// counter per stream, every workgroup fetches once per tile) lost 20-30 % to
// the static grid stride at 4-16 MiB per input (profiles/r2/probe_mid_sizes_r4d.jsonl):
// the launch's fetches form one serialized chain of atomics on one address.
// Variants, 8 x fp32 sources -> 1, production tile (8 x 4 packs per lane, one
// 256-thread workgroup per CU):
//   static      grid stride
//   dyn1        one counter (the library's schedule)
//   dynX C      C counters, workgroup b on counter b % C: counter x hands out
//               the tiles t with t % C == x (C = 8: one per XCD under the
//               round-robin dispatch), so each chain is 1/C as long
// Every output compared bit-exact with the static schedule.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None scripts/sweep_dyn_xcd.hip -o scripts/sweep_dyn_xcd
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int U = 4, T = 256, NSRC = 8;
constexpr uint64_t kTile = (uint64_t)U * T;

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

__device__ __forceinline__ void tileFold(const Args& a, uint64_t p) {
  f32x4 v[NSRC][U];
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * T);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < U; u++) {
    f32x4 acc = v[0][u];
#pragma unroll
    for (int s = 1; s < NSRC; s++) acc = acc + v[s][u];
    a.dst[p + u * T] = acc;
  }
}

__global__ __launch_bounds__(T) void kstatic(Args a, unsigned*) {
  const uint64_t nTiles = a.nPacks / kTile;
  for (uint64_t t = blockIdx.x; t < nTiles; t += gridDim.x) tileFold(a, t * kTile + threadIdx.x);
}

// C counters at a 256-B stride; workgroup b uses counter b % C and walks the
// tiles t = x + C * l of its class x (its first is l = b / C, static)
template <int C>
__global__ __launch_bounds__(T) void kdyn(Args a, unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const uint64_t nTiles = a.nPacks / kTile;
  const unsigned x = blockIdx.x % C;
  const uint64_t nCls = nTiles > x ? (nTiles - x + C - 1) / C : 0;            // tiles of class x
  const uint64_t gCls = (gridDim.x - x + C - 1) / C;                          // workgroups of class x
  unsigned* c = ctr + 64 * x;
  uint64_t l = blockIdx.x / C;
  int par = 0;
  while (l < nCls) {
    unsigned got = 0;
    if (threadIdx.x == 0) got = atomicAdd(c, 1u);
    tileFold(a, (x + C * l) * kTile + threadIdx.x);
    if (threadIdx.x == 0) nxt[par] = got + (unsigned)gCls;
    __syncthreads();
    l = nxt[par];
    par ^= 1;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t maxCount = 64ull << 20;   // fp32 per input (256 MiB)
  std::vector<float*> src(8);
  std::vector<float> h(maxCount);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], maxCount * 4));
    for (uint64_t i = 0; i < maxCount; i++) h[i] = (float)((i * 2654435761ull + s * 977ull) % 200003ull) / 100001.0f - 1.0f;
    CK(hipMemcpy(src[s], h.data(), maxCount * 4, hipMemcpyHostToDevice));
  }
  float *dst, *ref;
  CK(hipMalloc(&dst, maxCount * 4));
  CK(hipMalloc(&ref, maxCount * 4));
  struct V { std::string name; const void* fn; };
  std::vector<V> vs = {{"static", (const void*)&kstatic},   {"dyn1", (const void*)&kdyn<1>},
                       {"dynX 2", (const void*)&kdyn<2>},   {"dynX 8", (const void*)&kdyn<8>},
                       {"dynX 32", (const void*)&kdyn<32>}, {"static (again)", (const void*)&kstatic}};
  unsigned* ctrs;
  const int kSlots = 4096, kSlotWords = 64 * 32;   // one launch's counters per slot
  CK(hipMalloc(&ctrs, (size_t)kSlots * kSlotWords * 4));
  CK(hipMemset(ctrs, 0, (size_t)kSlots * kSlotWords * 4));
  int next = 0;
  int bad = 0;
  for (uint64_t mib : {4ull, 8ull, 16ull, 32ull, 64ull, 256ull}) {
    Args a;
    for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
    a.nPacks = (mib << 20) / 16;
    const uint64_t nTiles = a.nPacks / kTile;
    const unsigned grid = (unsigned)std::min<uint64_t>(nTiles, (uint64_t)cus);
    auto launch = [&](const V& v, float* out) {
      if (next >= kSlots) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(ctrs, 0, (size_t)kSlots * kSlotWords * 4));
        next = 0;
      }
      unsigned* c = ctrs + (size_t)kSlotWords * next++;
      Args b = a;
      b.dst = (f32x4*)out;
      void* args[] = {&b, &c};
      CK(hipLaunchKernel(v.fn, dim3(grid), dim3(T), args, 0, 0));
    };
    launch(vs[0], ref);
    CK(hipDeviceSynchronize());
    const size_t bytes = (mib << 20);
    std::vector<char> r(bytes), o(bytes);
    CK(hipMemcpy(r.data(), ref, bytes, hipMemcpyDeviceToHost));
    for (auto& v : vs) {
      CK(hipMemset(dst, 0, bytes));
      launch(v, dst);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(o.data(), dst, bytes, hipMemcpyDeviceToHost));
      if (memcmp(o.data(), r.data(), bytes) != 0) {
        printf("MISMATCH %s at %llu MiB\n", v.name.c_str(), (unsigned long long)mib);
        bad++;
      }
    }
    const int iters = (int)std::max<uint64_t>(10, std::min<uint64_t>(200, (4096ull / mib)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
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
    printf("8 x %llu MiB fp32 -> 1, %llu tiles, grid %u, %d rounds x %d launches\n", (unsigned long long)mib,
           (unsigned long long)nTiles, grid, rounds, iters);
    for (size_t i = 0; i < vs.size(); i++) {
      auto x = t[i];
      std::sort(x.begin(), x.end());
      const double med = x[x.size() / 2];
      printf("  %-16s %9.2f us  %8.1f GB/s\n", vs[i].name.c_str(), med * 1e3, 9.0 * bytes / (med * 1e-3) / 1e9);
    }
    fflush(stdout);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
