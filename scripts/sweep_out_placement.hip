// sweep_out_placement.hip — experiment, not part of the product: does the
// OUTPUT buffer's placement change the config-B fold's rate? (In one
// in-process A/B, profiles/r5/ab_swar8_r5i.jsonl, byte-identical kernels ran
// 6.36 vs 6.92 TB/s on the same sources, writing to different outputs;
// DESIGN §5.2 had varied only the sources' placement.)
// Sources: 8 separate 256 MiB hipMalloc buffers, fixed. Outputs: (a) 12
// separate 256 MiB hipMalloc buffers, each timed; (b) one 1 GiB arena with
// the output at offsets 0, 4 KiB, 64 KiB, 1 MiB, 2 MiB, 16 MiB, 64 MiB, 128
// MiB, 256 MiB + 4 KiB, 512 MiB. Production tile (8 x 4 packs per lane, 256
// threads, one workgroup per CU), dynamic tiles; every output checked against
// the first. Interleaved rounds, median per placement.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_out_placement.hip -o scripts/sweep_out_placement
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int T = 256, NSRC = 8, U = 4;
constexpr uint64_t kTile = (uint64_t)U * T;

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint64_t nPacks;
};

__global__ __launch_bounds__(T) void kprod(Args a, unsigned* ctr) {
  __shared__ unsigned nxt[2];
  const uint64_t nTiles = a.nPacks / kTile;
  uint64_t t = blockIdx.x;
  int par = 0;
  while (t < nTiles) {
    unsigned got = 0;
    if (threadIdx.x == 0) got = atomicAdd(ctr, 1u);
    const uint64_t p = t * kTile + threadIdx.x;
    f32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * T);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 x = v[0][u];
#pragma unroll
      for (int s = 1; s < NSRC; s++) x = x + v[s][u];
      a.dst[p + u * T] = x;
    }
    if (threadIdx.x == 0) nxt[par] = got + gridDim.x;
    __syncthreads();
    t = nxt[par];
    par ^= 1;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t count = 64ull << 20, bytes = count * 4;
  std::vector<float*> src(8);
  std::vector<float> h(count);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], bytes));
    for (uint64_t i = 0; i < count; i++) h[i] = (float)((i * 2654435761ull + s * 977ull) % 200003ull) / 100001.0f - 1.0f;
    CK(hipMemcpy(src[s], h.data(), bytes, hipMemcpyHostToDevice));
  }
  struct P { std::string name; float* out; };
  std::vector<P> ps;
  for (int k = 0; k < 12; k++) {
    float* o;
    CK(hipMalloc(&o, bytes));
    char nm[64];
    snprintf(nm, sizeof nm, "separate #%d", k);
    ps.push_back({nm, o});
  }
  char* arena;
  CK(hipMalloc(&arena, (1ull << 30) + (8ull << 20)));
  for (uint64_t off : {0ull, 4096ull, 65536ull, 1ull << 20, 2ull << 20, 16ull << 20, 64ull << 20, 128ull << 20,
                       (256ull << 20) + 4096, 512ull << 20}) {
    char nm[64];
    snprintf(nm, sizeof nm, "arena +%llu KiB", (unsigned long long)(off >> 10));
    ps.push_back({nm, (float*)(arena + off)});
  }
  unsigned* ctrs;
  const int kSlots = 8192;
  CK(hipMalloc(&ctrs, (size_t)kSlots * 64 * 4));
  CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
  int next = 0;
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.nPacks = bytes / 16;
  const unsigned grid = (unsigned)cus;
  auto launch = [&](float* out) {
    if (next >= kSlots) {
      CK(hipDeviceSynchronize());
      CK(hipMemset(ctrs, 0, (size_t)kSlots * 64 * 4));
      next = 0;
    }
    Args b = a;
    b.dst = (f32x4*)out;
    unsigned* c = ctrs + (size_t)64 * next++;
    hipLaunchKernelGGL(kprod, dim3(grid), dim3(T), 0, 0, b, c);
  };
  // correctness: every placement's output equals the first's
  std::vector<char> r(bytes), o(bytes);
  launch(ps[0].out);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(r.data(), ps[0].out, bytes, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto& p : ps) {
    CK(hipMemset(p.out, 0, bytes));
    launch(p.out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), p.out, bytes, hipMemcpyDeviceToHost));
    if (memcmp(o.data(), r.data(), bytes) != 0) bad++;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> t(ps.size());
  for (int rd = 0; rd < rounds; rd++)
    for (size_t i = 0; i < ps.size(); i++) {
      launch(ps[i].out);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < 10; it++) launch(ps[i].out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / 10);
    }
  printf("8 x 256 MiB fp32 -> 1, grid %u, dynamic tiles, %d rounds; sources at", grid, rounds);
  for (int s = 0; s < 8; s++) printf(" %p", (void*)src[s]);
  printf("\n");
  for (size_t i = 0; i < ps.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    const double med = x[x.size() / 2];
    printf("  %-22s %p %9.2f us (min %9.2f, max %9.2f)  %8.1f GB/s\n", ps[i].name.c_str(), (void*)ps[i].out,
           med * 1e3, x[0] * 1e3, x.back() * 1e3, 9.0 * bytes / (med * 1e-3) / 1e9);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
