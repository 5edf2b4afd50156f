// sweep_fold_phase.hip — experiment, not part of the product (VERDICT r4
// "next" item 4): chip-scale read / write phases for the config-B fold.
//
// The production tile (nbx_kernels.h kReducePacks<FnSumF<TyF32>,8,4>) issues a
// tile's 32 loads, folds and stores 4 packs per lane, so the chip's traffic is
// an interleaved 8:1 read:write stream at every instant. Its rate sits at the
// same box's mixed 8:1 stream ceiling, ~10 % under a serial read-then-write
// model of the same box's read-only and write-only ceilings.
// Per-lane store bursts of 2-4 tiles in registers lost. This
// sweep tries the one shape not measured: a workgroup folds K tiles into LDS
// (K x 16 KiB, up to 128 KiB of gfx950's 160 KiB per CU) and only then stores
// them in one burst, so each CU alternates long read-only and write-only runs;
// and, on top, a chip-wide phase barrier (one agent-scope counter, bounded
// spin) so that EVERY CU is in its read phase, then every CU in its write
// phase — long read-only and write-only runs of the whole chip.
//
// Then (clock phases, kclock) the same without any barrier: periods of the
// shared wall clock. Results: profiles/r5/sweep_fold_phase_r5a.txt and
// sweep_fold_phase_clock_r5e.txt — every shape loses to production.
// Every variant's output is compared bit-exact with the static production
// shape; times are medians of interleaved rounds in one process, same buffers.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_fold_phase.hip -o scripts/sweep_fold_phase
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int T = 256, NSRC = 8;

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

template <int U>
__device__ __forceinline__ void loadTile(const Args& a, uint64_t p, f32x4 (&v)[NSRC][U]) {
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * T);
}

template <int U>
__device__ __forceinline__ void fold(const f32x4 (&v)[NSRC][U], f32x4 (&acc)[U]) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    f32x4 x = v[0][u];
#pragma unroll
    for (int s = 1; s < NSRC; s++) x = x + v[s][u];
    acc[u] = x;
  }
}

// The production shape: static grid stride or one dynamic tile counter.
template <bool DYN>
__global__ __launch_bounds__(T) void kprod(Args a, unsigned* ctr, unsigned* err) {
  constexpr int U = 4;
  constexpr uint64_t kTile = (uint64_t)U * T;
  __shared__ unsigned nxt[2];
  const uint64_t nTiles = a.nPacks / kTile;
  uint64_t t = blockIdx.x;
  int par = 0;
  while (t < nTiles) {
    unsigned got = 0;
    if (DYN && threadIdx.x == 0) got = atomicAdd(ctr, 1u);
    const uint64_t p = t * kTile + threadIdx.x;
    f32x4 v[NSRC][U];
    loadTile<U>(a, p, v);
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[U];
    fold<U>(v, acc);
#pragma unroll
    for (int u = 0; u < U; u++) a.dst[p + u * T] = acc[u];
    if (DYN) {
      if (threadIdx.x == 0) nxt[par] = got + gridDim.x;
      __syncthreads();
      t = nxt[par];
      par ^= 1;
    } else {
      t += gridDim.x;
    }
  }
  (void)err;
}

// Chip-wide phase barrier: every workgroup adds 1 to one counter and waits
// until `target` arrivals. Bounded: after ~100 ms (wall clock at 100 MHz) the
// waiter records the timeout and goes on, so the grid always drains.
__device__ __forceinline__ void chipBarrier(unsigned* bar, unsigned target, unsigned* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > 10000000ull) {
        atomicOr(err, 1u);
        break;
      }
    }
  }
  __syncthreads();
}

// Phased fold: phase ph covers tiles [ph G K, (ph+1) G K); workgroup b folds
// tiles ph G K + k G + b (k < K: the chip stays on one window, as the grid
// stride does) into LDS, then stores them. Each lane stores back only the
// packs it folded, so LDS needs no workgroup barrier. MODE 0: no chip
// barrier (per-CU bursts); 1: chip barrier between the read and the write
// phase; 2: also between the write phase and the next read phase.
template <int U, int K, int MODE>
__global__ __launch_bounds__(T) void kphase(Args a, unsigned* bar, unsigned* err) {
  constexpr uint64_t kTile = (uint64_t)U * T;
  extern __shared__ f32x4 lds[];   // [K][U][T]
  const uint64_t nTiles = a.nPacks / kTile;
  const uint64_t G = gridDim.x;
  const uint64_t perPhase = G * (uint64_t)K;
  const uint64_t nPhases = (nTiles + perPhase - 1) / perPhase;
  unsigned arrivals = 0;
  for (uint64_t ph = 0; ph < nPhases; ph++) {
    const uint64_t base = ph * perPhase + blockIdx.x;
#pragma unroll 1
    for (int k = 0; k < K; k++) {
      const uint64_t t = base + (uint64_t)k * G;
      if (t < nTiles) {
        const uint64_t p = t * kTile + threadIdx.x;
        f32x4 v[NSRC][U];
        loadTile<U>(a, p, v);
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc[U];
        fold<U>(v, acc);
#pragma unroll
        for (int u = 0; u < U; u++) lds[((size_t)k * U + u) * T + threadIdx.x] = acc[u];
      }
    }
    if (MODE >= 1) chipBarrier(bar, (++arrivals) * (unsigned)G, err);
#pragma unroll 1
    for (int k = 0; k < K; k++) {
      const uint64_t t = base + (uint64_t)k * G;
      if (t < nTiles) {
        const uint64_t p = t * kTile + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; u++) a.dst[p + u * T] = lds[((size_t)k * U + u) * T + threadIdx.x];
      }
    }
    if (MODE == 2) chipBarrier(bar, (++arrivals) * (unsigned)G, err);
  }
}

// Clock phases (round 5, second try): no barrier at all — every CU reads the
// same 100 MHz wall clock, and time itself is cut into periods of R ticks of
// reading then W ticks of writing. In a read window a workgroup takes tiles
// from one dynamic counter (thread 0, broadcast through LDS) and folds them
// into LDS, until its K slots are full or the window closes; then it waits for
// the write window and stores what it folded. Stragglers take fewer tiles
// instead of holding everyone at a barrier. A tile is fetched only while at
// least `margin` ticks of the read window remain (its loads must land before
// the writes start).
template <int K, int R, int W>
__global__ __launch_bounds__(T) void kclock(Args a, unsigned* ctr, unsigned* err) {
  constexpr int U = 4;
  constexpr uint64_t kTile = (uint64_t)U * T;
  constexpr uint64_t P = (uint64_t)R + W, margin = 150;   // 1.5 us: a tile's loads land
  extern __shared__ f32x4 lds[];   // [K][U][T]
  __shared__ unsigned tiles[K];
  __shared__ unsigned bcast;
  const uint64_t nTiles = a.nPacks / kTile;
  bool done = false;
  while (!done) {
    // wait for a read window with room for at least one tile
    if (threadIdx.x == 0) {
      for (;;) {
        const uint64_t ph = wall_clock64() % P;
        if (ph + margin < (uint64_t)R) break;
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    int k = 0;
    for (; k < K; k++) {
      if (threadIdx.x == 0) {
        const uint64_t ph = wall_clock64() % P;
        bcast = ph + margin < (uint64_t)R ? atomicAdd(ctr, 1u) : 0xfffffffeu;   // ~0u - 1: window closed
      }
      __syncthreads();
      const unsigned t = bcast;
      __syncthreads();
      if (t == 0xfffffffeu) break;
      if ((uint64_t)t >= nTiles) {
        done = true;
        break;
      }
      if (threadIdx.x == 0) tiles[k] = t;
      const uint64_t p = (uint64_t)t * kTile + threadIdx.x;
      f32x4 v[NSRC][U];
      loadTile<U>(a, p, v);
      __builtin_amdgcn_sched_barrier(0);
      f32x4 acc[U];
      fold<U>(v, acc);
#pragma unroll
      for (int u = 0; u < U; u++) lds[((size_t)k * U + u) * T + threadIdx.x] = acc[u];
    }
    __syncthreads();
    if (k == 0) continue;
    // the write window of this period (or of the next, if it has passed)
    if (threadIdx.x == 0) {
      for (;;) {
        const uint64_t ph = wall_clock64() % P;
        if (ph >= (uint64_t)R) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    for (int j = 0; j < k; j++) {
      const uint64_t p = (uint64_t)tiles[j] * kTile + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; u++) a.dst[p + u * T] = lds[((size_t)j * U + u) * T + threadIdx.x];
    }
    __syncthreads();
  }
  (void)err;
}

struct V {
  std::string name;
  const void* fn;
  size_t lds;   // dynamic LDS bytes (0: production kernel)
};

template <int U, int K, int MODE>
V phase(const char* name) {
  return V{name, (const void*)&kphase<U, K, MODE>, (size_t)K * U * T * 16};
}

template <int K, int R, int W>
V clockv(const char* name) {
  return V{name, (const void*)&kclock<K, R, W>, (size_t)K * 4 * T * 16};
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const int only256 = argc > 2 ? atoi(argv[2]) : 0;
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
  std::vector<V> vs = {{"static (prod)", (const void*)&kprod<false>, 0},
                       {"dyn1 (prod)", (const void*)&kprod<true>, 0},
                       phase<4, 2, 0>("burst K2 (32K)"),
                       phase<4, 4, 0>("burst K4 (64K)"),
                       phase<4, 8, 0>("burst K8 (128K)"),
                       phase<2, 16, 0>("burst U2 K16"),
                       phase<1, 32, 0>("burst U1 K32"),
                       phase<4, 4, 1>("chip K4 (64K)"),
                       phase<4, 8, 1>("chip K8 (128K)"),
                       phase<2, 16, 1>("chip U2 K16"),
                       phase<4, 8, 2>("chip2 K8"),
                       clockv<8, 3600, 600>("clock K8 36/6"),
                       clockv<8, 3300, 700>("clock K8 33/7"),
                       clockv<8, 4000, 600>("clock K8 40/6"),
                       clockv<4, 1800, 300>("clock K4 18/3"),
                       clockv<4, 1600, 400>("clock K4 16/4"),
                       {"static (again)", (const void*)&kprod<false>, 0},
                       {"dyn1 (again)", (const void*)&kprod<true>, 0}};
  for (auto& v : vs)
    if (v.lds > 65536) CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
  unsigned* ctrs;
  unsigned* err;
  const int kSlots = 4096;
  CK(hipMalloc(&ctrs, (size_t)kSlots * 64 * 4));
  CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(err, 0, 4));
  int next = 0, bad = 0;
  std::vector<uint64_t> sizes = {64ull, 256ull};
  if (only256) sizes = {256ull};
  for (uint64_t mib : sizes) {
    Args a;
    for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
    a.nPacks = (mib << 20) / 16;
    // every kernel here assumes whole tiles of 1024 packs (256 MiB / 64 MiB are)
    if (a.nPacks % 1024 != 0) { printf("size not a whole number of tiles\n"); return 2; }
    const unsigned grid = (unsigned)std::min<uint64_t>(a.nPacks / 1024, (uint64_t)cus);
    auto launch = [&](const V& v, float* out) {
      if (next >= kSlots) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
        next = 0;
      }
      unsigned* c = ctrs + (size_t)64 * next++;
      Args b = a;
      b.dst = (f32x4*)out;
      void* args[] = {&b, &c, &err};
      CK(hipLaunchKernel(v.fn, dim3(grid), dim3(T), args, v.lds, 0));
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
    unsigned herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("8 x %llu MiB fp32 -> 1, grid %u, %d rounds x %d launches, barrier timeouts: %u\n",
           (unsigned long long)mib, grid, rounds, iters, herr);
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
