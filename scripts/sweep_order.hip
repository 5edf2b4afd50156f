// sweep_order.hip — source-ordering experiment for the config-B hot loop
// (8 x 256 MiB fp32 -> 256 MiB), not part of the product.
//
// The production kernel issues all NSRC x U loads of a tile at once (every
// workgroup streams 8 sources concurrently: ~2,300 concurrent sequential
// streams chip-wide). The variants here walk the sources one after another
// inside a bigger tile, with only two sources' loads in flight per lane
// (double-buffered), so each workgroup streams ~2 sources at a time and each
// stream is touched in longer runs — a test of whether fewer concurrent DRAM
// streams (better row-buffer locality) beat more bytes in flight. Outputs are
// checked bit-exact against the production shape (same left fold order).
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_order.hip -o sweep_order
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

template <int U>
__global__ __launch_bounds__(256) void kall(Args a) {   // production shape
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    f32x4 v[8][U];
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < 8; s++) acc = acc + v[s][u];
      a.dst[p + u * 256] = acc;
    }
  }
}

// Sources in sequence, DEPTH sources' loads in flight (ring of DEPTH buffers).
template <int U, int DEPTH>
__global__ __launch_bounds__(256) void kseq(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    f32x4 buf[DEPTH][U];
    f32x4 acc[U];
#pragma unroll
    for (int s = 0; s < DEPTH - 1; s++)
#pragma unroll
      for (int u = 0; u < U; u++) buf[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
#pragma unroll
    for (int s = 0; s < 8; s++) {
      const int nx = s + DEPTH - 1;
      if (nx < 8) {
#pragma unroll
        for (int u = 0; u < U; u++) buf[nx % DEPTH][u] = __builtin_nontemporal_load(a.src[nx] + p + u * 256);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; u++) acc[u] = s == 0 ? buf[0][u] : acc[u] + buf[s % DEPTH][u];
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < U; u++) a.dst[p + u * 256] = acc[u];
  }
}

struct Variant {
  std::string name;
  const void* fn;
  int unroll, blocksPerCU;
};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const uint64_t count = 64ull << 20;
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
      {"all-sources u4 bpc1 (production)", (const void*)&kall<4>, 4, 1},
      {"seq depth2 u8 bpc1", (const void*)&kseq<8, 2>, 8, 1},
      {"seq depth2 u8 bpc2", (const void*)&kseq<8, 2>, 8, 2},
      {"seq depth2 u16 bpc1", (const void*)&kseq<16, 2>, 16, 1},
      {"seq depth3 u8 bpc1", (const void*)&kseq<8, 3>, 8, 1},
      {"seq depth3 u8 bpc2", (const void*)&kseq<8, 3>, 8, 2},
      {"seq depth4 u8 bpc1", (const void*)&kseq<8, 4>, 8, 1},
      {"seq depth4 u4 bpc2", (const void*)&kseq<4, 4>, 4, 2},
      {"seq depth2 u4 bpc4", (const void*)&kseq<4, 2>, 4, 4},
      {"seq depth4 u16 bpc1", (const void*)&kseq<16, 4>, 16, 1},
  };
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.nPacks = count / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&](const Variant& v, float* out) {
    Args b = a;
    b.dst = (f32x4*)out;
    uint64_t tile = (uint64_t)v.unroll * 256;
    uint64_t grid = std::min<uint64_t>((b.nPacks + tile - 1) / tile, (uint64_t)cus * v.blocksPerCU);
    void* args[] = {&b};
    CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(256), args, 0, 0));
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
  printf("%-40s %10s %10s %9s\n", "variant (8 x 256 MiB fp32 -> 256 MiB)", "med_ms", "min_ms", "GB/s(med)");
  for (size_t i = 0; i < vs.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    double med = x[x.size() / 2];
    printf("%-40s %10.4f %10.4f %9.1f\n", vs[i].name.c_str(), med, x[0], 9.0 * count * 4 / (med * 1e-3) / 1e9);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
