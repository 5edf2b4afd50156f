// sweep_fold_defer.hip — experiment, not part of the product: deferred stores
// for the config-B fold. The production tile issues its 32 loads, folds, then
// stores its 4 results and only then issues the next tile's loads, so while a
// wave folds and stores nothing of its own is in flight. Here a wave keeps the
// previous tile's 4 results in registers (16 VGPRs) and stores them right
// after issuing the next tile's loads: the store phase overlaps the next
// tile's load latency. (Keeping the next tile's 32 loads in registers instead —
// software pipelining — lost 1-5 % to register pressure)
// Variants x {static grid stride, one dynamic tile counter}, 8 x fp32 sources
// -> 1, every output compared bit-exact with the static production shape.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None scripts/sweep_fold_defer.hip -o scripts/sweep_fold_defer
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

__device__ __forceinline__ void loadTile(const Args& a, uint64_t p, f32x4 (&v)[NSRC][U]) {
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * T);
}

__device__ __forceinline__ void fold(const f32x4 (&v)[NSRC][U], f32x4 (&acc)[U]) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    f32x4 x = v[0][u];
#pragma unroll
    for (int s = 1; s < NSRC; s++) x = x + v[s][u];
    acc[u] = x;
  }
}

__device__ __forceinline__ void storeTile(const Args& a, uint64_t p, const f32x4 (&acc)[U]) {
#pragma unroll
  for (int u = 0; u < U; u++) a.dst[p + u * T] = acc[u];
}

// DYN: tiles past the first gridDim.x from one counter (the library's schedule)
template <bool DYN, bool DEFER>
__global__ __launch_bounds__(T) void kfold(Args a, unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const uint64_t nTiles = a.nPacks / kTile;
  uint64_t t = blockIdx.x;
  int par = 0;
  f32x4 prev[U];
  uint64_t prevP = ~0ull;
  while (t < nTiles) {
    unsigned got = 0;
    if (DYN && threadIdx.x == 0) got = atomicAdd(ctr, 1u);
    const uint64_t p = t * kTile + threadIdx.x;
    f32x4 v[NSRC][U];
    loadTile(a, p, v);
    if (DEFER && prevP != ~0ull) storeTile(a, prevP, prev);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[U];
    fold(v, acc);
    if (DEFER) {
#pragma unroll
      for (int u = 0; u < U; u++) prev[u] = acc[u];
      prevP = p;
    } else {
      storeTile(a, p, acc);
    }
    if (DYN) {
      if (threadIdx.x == 0) nxt[par] = got + gridDim.x;
      __syncthreads();
      t = nxt[par];
      par ^= 1;
    } else {
      t += gridDim.x;
    }
  }
  if (DEFER && prevP != ~0ull) storeTile(a, prevP, prev);
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
  std::vector<V> vs = {{"static", (const void*)&kfold<false, false>},
                       {"static defer", (const void*)&kfold<false, true>},
                       {"dyn1", (const void*)&kfold<true, false>},
                       {"dyn1 defer", (const void*)&kfold<true, true>},
                       {"static (again)", (const void*)&kfold<false, false>},
                       {"dyn1 (again)", (const void*)&kfold<true, false>}};
  unsigned* ctrs;
  const int kSlots = 4096;
  CK(hipMalloc(&ctrs, (size_t)kSlots * 64 * 4));
  CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
  int next = 0, bad = 0;
  for (uint64_t mib : {64ull, 256ull}) {
    Args a;
    for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
    a.nPacks = (mib << 20) / 16;
    const uint64_t nTiles = a.nPacks / kTile;
    const unsigned grid = (unsigned)std::min<uint64_t>(nTiles, (uint64_t)cus);
    auto launch = [&](const V& v, float* out) {
      if (next >= kSlots) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
        next = 0;
      }
      unsigned* c = ctrs + (size_t)64 * next++;
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
    const int iters = mib >= 256 ? 10 : 40;
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
      printf("  %-16s %9.2f us (min %9.2f)  %8.1f GB/s\n", vs[i].name.c_str(), med * 1e3, x[0] * 1e3,
             9.0 * bytes / (med * 1e-3) / 1e9);
    }
    fflush(stdout);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
