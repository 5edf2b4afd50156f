// sweep_fold_dma.hip — experiment for the config-B hot loop (VERDICT r1
// item 6), not part of the product: the 8:1 fp32 fold with its source reads
// moved to LDS-DMA (global_load_lds_dwordx4: HBM -> LDS without VGPRs), so a
// wave can keep several tiles of loads in flight (S stages) while it folds an
// earlier tile from LDS, against the production register shape (8 sources x
// 4 packs per lane issued before the fold, one 256-thread workgroup per CU,
// nt loads, plain stores) — in one process, interleaved rounds, outputs
// compared bit-exact with the production shape.
//
// A wave owns tiles of U x 64 packs; stage buffers are private to the wave
// ([wave][stage][source][u][64 packs] in LDS), so no workgroup barrier is
// needed: the wave issues the DMA of tile j+S-1, waits (vmcnt) until tile j's
// loads have landed, reads them back (ds_read_b128), folds and stores.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_fold_dma.hip -o scripts/sweep_fold_dma
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr;

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

// production shape (nbx_kernels.h kReducePacks<FnSumF<TyF32>, 8, 4>)
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kprod(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    if (p + (U - 1) * 256 < n) {
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
        a.dst[p + u * 256] = acc;
      }
    } else {
      for (int u = 0; u < U; u++) {
        const uint64_t q = p + (uint64_t)u * 256;
        if (q < n) {
          f32x4 acc = a.src[0][q];
          for (int s = 1; s < NSRC; s++) acc = acc + a.src[s][q];
          a.dst[q] = acc;
        }
      }
    }
  }
}

#define WAIT_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

template <int N>
__device__ __forceinline__ void waitVm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  if constexpr (N == 0) WAIT_VM(0);
  else if constexpr (N == 8) WAIT_VM(8);
  else if constexpr (N == 16) WAIT_VM(16);
  else if constexpr (N == 24) WAIT_VM(24);
  else if constexpr (N == 32) WAIT_VM(32);
  else if constexpr (N == 48) WAIT_VM(48);
  else WAIT_VM(0);
}

// LDS-DMA fold: W waves per workgroup, S stages per wave, U packs per lane per
// tile, AUX the load's cache policy bits (2 = nt)
template <int NSRC, int U, int S, int W, int AUX>
__global__ __launch_bounds__(W * 64) void kdma(Args a) {
  __shared__ f32x4 sm[W][S][NSRC][U][64];
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  constexpr uint64_t kTile = (uint64_t)U * 64;
  const uint64_t n = a.nPacks;
  const uint64_t nTiles = n / kTile;   // sweep sizes: whole tiles
  const uint64_t nWaves = (uint64_t)gridDim.x * W, gw = (uint64_t)blockIdx.x * W + wave;
  auto issue = [&](uint64_t t, int st) {
    const uint64_t base = t * kTile;
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void*)(a.src[s] + base + u * 64 + lane), (lds_ptr)&sm[wave][st][s][u][0],
                                         16, 0, AUX);
  };
  // prologue: tiles 0 .. S-2 of this wave
#pragma unroll
  for (int k = 0; k < S - 1; k++) {
    const uint64_t t = gw + (uint64_t)k * nWaves;
    if (t < nTiles) issue(t, k);
  }
  int st = 0;
  for (uint64_t t = gw; t < nTiles; t += nWaves) {
    const uint64_t ahead = t + (uint64_t)(S - 1) * nWaves;
    if (ahead < nTiles) {
      issue(ahead, (st + S - 1) % S);
      waitVm<(S - 1) * NSRC * U>();   // everything but the S-1 newer tiles has landed (stores only make it stricter)
    } else {
      waitVm<0>();
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = sm[wave][st][0][u][lane];
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = acc + sm[wave][st][s][u][lane];
      a.dst[t * kTile + u * 64 + lane] = acc;
    }
    // the ds_reads of this stage retire (their values feed the stores) before
    // the stage is refilled in a later iteration
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    st = st + 1 == S ? 0 : st + 1;
  }
}

struct Variant {
  std::string name;
  const void* fn;
  int threads;
  uint64_t tilePacks;   // packs per workgroup per tile step
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
      {"production u4 bpc1 (register tile)", (const void*)&kprod<8, 4>, 256, 1024, 1},
      {"dma nt W4 U2 S2 bpc1", (const void*)&kdma<8, 2, 2, 4, 2>, 256, 512, 1},
      {"dma nt W4 U1 S4 bpc1", (const void*)&kdma<8, 1, 4, 4, 2>, 256, 256, 1},
      {"dma nt W4 U1 S3 bpc1", (const void*)&kdma<8, 1, 3, 4, 2>, 256, 256, 1},
      {"dma nt W4 U1 S2 bpc2", (const void*)&kdma<8, 1, 2, 4, 2>, 256, 256, 2},
      {"dma nt W8 U1 S2 bpc1", (const void*)&kdma<8, 1, 2, 8, 2>, 512, 512, 1},
      {"dma nt W2 U2 S2 bpc2", (const void*)&kdma<8, 2, 2, 2, 2>, 128, 256, 2},
      {"dma default W4 U2 S2 bpc1", (const void*)&kdma<8, 2, 2, 4, 0>, 256, 512, 1},
      {"dma default W4 U1 S4 bpc1", (const void*)&kdma<8, 1, 4, 4, 0>, 256, 256, 1},
  };
  auto launch = [&](const Variant& v, float* out) {
    Args b = a;
    b.dst = (f32x4*)out;
    uint64_t grid = std::min<uint64_t>((b.nPacks + v.tilePacks - 1) / v.tilePacks, (uint64_t)cus * v.blocksPerCU);
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
  printf("8 x 256 MiB fp32 -> 256 MiB (config B), %d rounds x %d launches\n", rounds, iters);
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
