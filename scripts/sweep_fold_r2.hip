// sweep_fold_r2.hip — experiment for the config-B hot loop (VERDICT r1 item 6,
// second half), not part of the product: in-process A/B of work-distribution
// and store-scheduling variants of the 8:1 fp32 fold against the production
// register tile (8 sources x 4 packs per lane issued before the fold, one
// 256-thread workgroup per CU, grid-stride over 16-KiB-per-source tiles, nt
// loads, plain stores). Outputs compared bit-exact with the production shape.
//
//   burst B     : a lane folds B consecutive tiles of its workgroup and holds
//                 the results, then stores the B x U packs back to back — fewer,
//                 longer write phases per workgroup (read/write turnaround)
//   chunk       : workgroup b owns the contiguous range [b*n/G, (b+1)*n/G)
//                 instead of every G-th tile
//   xcd         : grid-stride with the tile index remapped so that the 32
//                 workgroups of one XCD (dispatch is round-robin over 8 XCDs)
//                 walk neighbouring tiles
//   w512        : 512-thread workgroups (8 waves per CU), U = 2
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-atomic-optimizer-strategy=None scripts/sweep_fold_r2.hip -o scripts/sweep_fold_r2
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

template <int NSRC, int U, int T>
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

// MODE 0: production grid stride; 1: xcd remap; sizes in the sweep are whole tiles
template <int NSRC, int U, int T, int MODE>
__global__ __launch_bounds__(T) void kstride(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * T;
  const uint64_t G = gridDim.x;
  uint64_t b = blockIdx.x;
  if constexpr (MODE == 1) b = (b % 8) * (G / 8) + b / 8;   // G is a multiple of 8
  for (uint64_t p = b * tile + threadIdx.x; p < n; p += G * tile) tileFold<NSRC, U, T>(a, p);
}

// contiguous range per workgroup
template <int NSRC, int U, int T>
__global__ __launch_bounds__(T) void kchunk(Args a) {
  const uint64_t tile = (uint64_t)U * T;
  const uint64_t nTiles = a.nPacks / tile, G = gridDim.x, b = blockIdx.x;
  const uint64_t t0 = b * nTiles / G, t1 = (b + 1) * nTiles / G;
  for (uint64_t t = t0; t < t1; t++) tileFold<NSRC, U, T>(a, t * tile + threadIdx.x);
}

// store burst: B tiles folded, results held, then all stored
template <int NSRC, int U, int B>
__global__ __launch_bounds__(256) void kburst(Args a) {
  const uint64_t tile = (uint64_t)U * 256, n = a.nPacks, G = gridDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * B; t * tile < n; t += G * B) {
    f32x4 res[B][U];
#pragma unroll
    for (int k = 0; k < B; k++) {
      const uint64_t p = (t + k) * tile + threadIdx.x;
      f32x4 v[NSRC][U];
#pragma unroll
      for (int s = 0; s < NSRC; s++)
#pragma unroll
        for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; u++) {
        f32x4 acc = v[0][u];
#pragma unroll
        for (int s = 1; s < NSRC; s++) acc = acc + v[s][u];
        res[k][u] = acc;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < B; k++)
#pragma unroll
      for (int u = 0; u < U; u++) a.dst[(t + k) * tile + threadIdx.x + u * 256] = res[k][u];
  }
}

// dynamic tiles: the first G tiles are static (one per workgroup), the rest
// are taken from a global counter, fetched one tile ahead (thread 0, into a
// double-buffered LDS word) so the atomic's latency hides behind the loads —
// CUs that stream faster take more tiles and all finish together
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kdyn(Args a, unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const uint64_t tile = (uint64_t)U * 256, nTiles = a.nPacks / tile;
  uint64_t t = blockIdx.x;
  int par = 0;
  while (t < nTiles) {
    unsigned got = 0;
    if (threadIdx.x == 0) got = atomicAdd(ctr, 1u);
    tileFold<NSRC, U, 256>(a, t * tile + threadIdx.x);
    if (threadIdx.x == 0) nxt[par] = got + gridDim.x;
    __syncthreads();
    t = nxt[par];
    par ^= 1;
  }
}

// hybrid: the first PCT % of the tiles as a static grid stride (no atomics,
// no barriers), the rest dynamic from the counter
template <int NSRC, int U, int PCT>
__global__ __launch_bounds__(256) void khyb(Args a, unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const uint64_t tile = (uint64_t)U * 256, nTiles = a.nPacks / tile, G = gridDim.x;
  const uint64_t nStatic = (nTiles * PCT / 100) / G * G;   // whole rounds
  uint64_t t = blockIdx.x;
  for (; t < nStatic; t += G) tileFold<NSRC, U, 256>(a, t * tile + threadIdx.x);
  int par = 0;
  while (t < nTiles) {
    unsigned got = 0;
    if (threadIdx.x == 0) got = atomicAdd(ctr, 1u);
    tileFold<NSRC, U, 256>(a, t * tile + threadIdx.x);
    if (threadIdx.x == 0) nxt[par] = got + (unsigned)(nStatic + G);
    __syncthreads();
    t = nxt[par];
    par ^= 1;
  }
}

// per-wave dynamic tiles: a wave owns a tile of U x 64 packs; lane 0 fetches
// the wave's next tile one ahead (readfirstlane broadcast), no LDS, no barrier
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kdynwave(Args a, unsigned* ctr) {
  const uint64_t tile = (uint64_t)U * 64, nTiles = a.nPacks / tile;
  const int lane = threadIdx.x & 63;
  const uint64_t nWaves = (uint64_t)gridDim.x * 4;
  uint64_t t = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  while (t < nTiles) {
    unsigned nx = 0;
    if (lane == 0) nx = atomicAdd(ctr, 1u) + (unsigned)nWaves;
    tileFold<NSRC, U, 64>(a, t * tile + lane);
    t = (uint64_t)__builtin_amdgcn_readfirstlane(nx);
  }
}

struct Variant {
  std::string name;
  const void* fn;
  int threads;
  uint64_t tilePacks;   // packs per workgroup per step (grid = min(tiles, cus * bpc))
  int blocksPerCU;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  const uint64_t count = 64ull << 20;   // fp32 per input (256 MiB)
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float*> src(8);
  std::vector<float> h(count);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], count * 4));
    for (uint64_t i = 0; i < count; i++) h[i] = (float)((i * 2654435761ull + s * 977ull) % 200003ull) / 100001.0f - 1.0f;
    CK(hipMemcpy(src[s], h.data(), count * 4, hipMemcpyHostToDevice));
  }
  float *dst, *ref;
  CK(hipMalloc(&dst, count * 4));
  CK(hipMalloc(&ref, count * 4));
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.nPacks = count / 4;
  std::vector<Variant> vs = {
      {"production u4 bpc1 (grid stride)", (const void*)&kstride<8, 4, 256, 0>, 256, 1024, 1},
      {"xcd-remapped stride u4 bpc1", (const void*)&kstride<8, 4, 256, 1>, 256, 1024, 1},
      {"chunk u4 bpc1", (const void*)&kchunk<8, 4, 256>, 256, 1024, 1},
      {"chunk u2 bpc2", (const void*)&kchunk<8, 2, 256>, 256, 512, 2},
      {"burst2 u4 bpc1", (const void*)&kburst<8, 4, 2>, 256, 2048, 1},
      {"burst2 u2 bpc1", (const void*)&kburst<8, 2, 2>, 256, 1024, 1},
      {"burst4 u2 bpc1", (const void*)&kburst<8, 2, 4>, 256, 2048, 1},
      {"w512 u2 bpc1", (const void*)&kstride<8, 2, 512, 0>, 512, 1024, 1},
      {"w512 u4 bpc1", (const void*)&kstride<8, 4, 512, 0>, 512, 2048, 1},
      {"dynamic u4 bpc1", (const void*)&kdyn<8, 4>, 256, 1024, 1},
      {"dynamic u2 bpc2", (const void*)&kdyn<8, 2>, 256, 512, 2},
      {"dynamic u2 bpc1", (const void*)&kdyn<8, 2>, 256, 512, 1},
      {"dynamic u8 bpc1", (const void*)&kdyn<8, 8>, 256, 2048, 1},
      {"dynamic hybrid50 u4 bpc1", (const void*)&khyb<8, 4, 50>, 256, 1024, 1},
      {"dynamic hybrid75 u4 bpc1", (const void*)&khyb<8, 4, 75>, 256, 1024, 1},
      {"dynamic hybrid90 u4 bpc1", (const void*)&khyb<8, 4, 90>, 256, 1024, 1},
      {"dynamic u4 bpc1 (again)", (const void*)&kdyn<8, 4>, 256, 1024, 1},
      {"production u4 bpc1 (again)", (const void*)&kstride<8, 4, 256, 0>, 256, 1024, 1},
  };
  // dynamic variants: one zeroed counter per launch (4096 launches' worth)
  unsigned* ctrs;
  CK(hipMalloc(&ctrs, 4096 * 64));
  CK(hipMemset(ctrs, 0, 4096 * 64));
  int ctrNext = 0;
  auto launch = [&](const Variant& v, float* out) {
    Args b = a;
    b.dst = (f32x4*)out;
    uint64_t grid = std::min<uint64_t>((b.nPacks + v.tilePacks - 1) / v.tilePacks, (uint64_t)cus * v.blocksPerCU);
    if (v.name.rfind("dynamic", 0) == 0) {
      if (ctrNext >= 4096) {
        CK(hipDeviceSynchronize());
        CK(hipMemset(ctrs, 0, 4096 * 64));
        ctrNext = 0;
      }
      unsigned* c = ctrs + 16 * ctrNext++;
      void* args[] = {&b, &c};
      CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.threads), args, 0, 0));
      return;
    }
    void* args[] = {&b};
    CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(v.threads), args, 0, 0));
  };
  launch(vs[0], ref);
  CK(hipDeviceSynchronize());
  std::vector<float> r(count), o(count);
  CK(hipMemcpy(r.data(), ref, count * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, count * 4));
    launch(v, dst);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dst, count * 4, hipMemcpyDeviceToHost));
    if (memcmp(o.data(), r.data(), count * 4) != 0) {
      printf("MISMATCH in %s\n", v.name.c_str());
      bad++;
    }
  }
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
  printf("8 x 256 MiB fp32 -> 256 MiB (config B), %d rounds x %d launches, %d CUs\n", rounds, iters, cus);
  printf("%-40s %10s %10s %9s\n", "variant", "med_ms", "min_ms", "GB/s(med)");
  for (size_t i = 0; i < vs.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    const double med = x[x.size() / 2];
    printf("%-40s %10.4f %10.4f %9.1f\n", vs[i].name.c_str(), med, x[0], 9.0 * count * 4 / (med * 1e-3) / 1e9);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
