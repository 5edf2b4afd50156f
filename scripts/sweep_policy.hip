// sweep_policy.hip — cache-policy sweep for the config-B hot loop
// (8 x 256 MiB fp32 -> 256 MiB, ordered left fold), not part of the product.
//
// Loads and stores go through buffer instructions whose aux operand carries
// the gfx950 cache-policy bits (sc0 = 1, nt = 2, sc1 = 16), so every
// load x store policy pair can be timed in one process, interleaved over
// rounds. The global-instruction baseline (production shape: nontemporal
// global loads, plain global stores) runs alongside. Every variant's output
// is checked bit-exact against the baseline's.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_policy.hip -o sweep_policy
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const f32x4* src[8];
  f32x4* dst;
  uint32_t nPacks;   // 16-B packs per source (< 2^28: byte offsets fit 32 bits)
};

constexpr int kRsrcWord3 = 0x00020000;   // gfx9 buffer descriptor dword3 (raw, 32-bit format)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, kRsrcWord3);
}

// Buffer variant: LAUX / SAUX = cache-policy bits on loads / stores.
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void kbuf(Args a) {
  const uint32_t n = a.nPacks, bytes = n * 16u;
  __amdgpu_buffer_rsrc_t rs[8];
#pragma unroll
  for (int s = 0; s < 8; s++) rs[s] = rsrc(a.src[s], bytes);
  const __amdgpu_buffer_rsrc_t rd = rsrc(a.dst, bytes);
  constexpr uint32_t tile = U * 256;
  const uint32_t stride = gridDim.x * tile;
  for (uint32_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {   // sweep sizes: full tiles
    u32x4 v[8][U];
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_amdgcn_raw_buffer_load_b128(rs[s], (p + u * 256) * 16u, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = __builtin_bit_cast(f32x4, v[0][u]);
#pragma unroll
      for (int s = 1; s < 8; s++) acc = acc + __builtin_bit_cast(f32x4, v[s][u]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), rd, (p + u * 256) * 16u, 0, SAUX);
    }
  }
}

// Global-instruction baseline (the production kernel's shape).
template <int U>
__global__ __launch_bounds__(256) void kglob(Args a) {
  const uint32_t n = a.nPacks;
  constexpr uint32_t tile = U * 256;
  const uint32_t stride = gridDim.x * tile;
  for (uint32_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
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

struct Variant {
  std::string name;
  const void* fn;
  int unroll, blocksPerCU;
};

static const char* pol(int aux) {
  switch (aux) {
    case 0: return "plain";
    case 1: return "sc0";
    case 2: return "nt";
    case 3: return "sc0.nt";
    case 16: return "sc1";
    case 17: return "sc0.sc1";
    case 18: return "nt.sc1";
    case 19: return "sc0.nt.sc1";
    default: return "?";
  }
}

template <int U, int L, int S>
static void add(std::vector<Variant>& vs, int bpc) {
  char b[96];
  snprintf(b, sizeof b, "buf u%d bpc%d ld=%s st=%s", U, bpc, pol(L), pol(S));
  vs.push_back({b, (const void*)&kbuf<U, L, S>, U, bpc});
}

template <int U, int L>
static void addStores(std::vector<Variant>& vs, int bpc) {
  add<U, L, 0>(vs, bpc);
  add<U, L, 2>(vs, bpc);
  add<U, L, 16>(vs, bpc);
  add<U, L, 17>(vs, bpc);
  add<U, L, 18>(vs, bpc);
}

template <int U>
static void addAll(std::vector<Variant>& vs, int bpc) {
  addStores<U, 0>(vs, bpc);
  addStores<U, 2>(vs, bpc);
  addStores<U, 16>(vs, bpc);
  addStores<U, 17>(vs, bpc);
  addStores<U, 18>(vs, bpc);
  addStores<U, 3>(vs, bpc);
  addStores<U, 19>(vs, bpc);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const uint32_t count = 64u << 20;   // fp32 per input
  const int iters = 10;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<float*> src(8);
  std::vector<float> h(count);
  for (int s = 0; s < 8; s++) {
    CK(hipMalloc(&src[s], (size_t)count * 4));
    srand(1234 + s);
    for (uint32_t i = 0; i < count; i++) h[i] = (float)((double)rand() / RAND_MAX * 2.0 - 1.0);
    CK(hipMemcpy(src[s], h.data(), (size_t)count * 4, hipMemcpyHostToDevice));
  }
  float *dst, *ref;
  CK(hipMalloc(&dst, (size_t)count * 4));
  CK(hipMalloc(&ref, (size_t)count * 4));

  std::vector<Variant> vs = {{"glob u4 bpc1 ld=nt st=plain (production)", (const void*)&kglob<4>, 4, 1},
                             {"glob u2 bpc2 ld=nt st=plain", (const void*)&kglob<2>, 2, 2}};
  addAll<4>(vs, 1);
  addAll<2>(vs, 2);

  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)src[s];
  a.nPacks = count / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&](const Variant& v, float* out) {
    Args b = a;
    b.dst = (f32x4*)out;
    uint32_t tile = (uint32_t)v.unroll * 256;
    uint32_t grid = std::min<uint32_t>((b.nPacks + tile - 1) / tile, (uint32_t)cus * v.blocksPerCU);
    void* args[] = {&b};
    CK(hipLaunchKernel(v.fn, dim3(grid), dim3(256), args, 0, 0));
  };
  launch(vs[0], ref);
  CK(hipDeviceSynchronize());
  std::vector<float> r(count), o(count);
  CK(hipMemcpy(r.data(), ref, (size_t)count * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (auto& v : vs) {
    CK(hipMemset(dst, 0, (size_t)count * 4));
    launch(v, dst);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dst, (size_t)count * 4, hipMemcpyDeviceToHost));
    if (memcmp(o.data(), r.data(), (size_t)count * 4) != 0) {
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
  printf("%-48s %10s %10s %9s\n", "variant (8 x 256 MiB fp32 -> 256 MiB)", "med_ms", "min_ms", "GB/s(med)");
  for (size_t i = 0; i < vs.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    double med = x[x.size() / 2];
    printf("%-48s %10.4f %10.4f %9.1f\n", vs[i].name.c_str(), med, x[0], 9.0 * count * 4 / (med * 1e-3) / 1e9);
  }
  printf("mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
