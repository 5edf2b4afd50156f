// nbx_stream.hip — stream ceilings measured in the same process as the
// reduction ("also report a measured stream-copy ceiling"):
// the HBM rate this box reaches for the read-only and write-only halves of
// the 8:1 fold, with the production kernel's loads (16-B nontemporal,
// kReducePacks' big tile: 8 sources x 4 packs per lane, one 256-thread
// workgroup per CU) and stores (plain 16-B). The 1:1 copy ceiling is the
// production kernel itself at one source (nbxReduceMulti, nSrcs = 1).
// Kind 2 is the mixed stream the fold actually faces: the same 8-source big
// tile, same schedule (dynamic tiles from 16 tiles per workgroup, as
// nbxReduceMulti), every load kept live but no arithmetic, and source 0's
// packs stored — 8 reads per write, so fold / mixed isolates what the fold's
// own ALU work and dependency chain cost.
// Diagnostics only: nothing in the collectives calls these.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nbx_debug.h"
#include "nbx_functors.h"
#include "nbx_internal.h"
#include "nbx_kargs.h"
#include "nbx_tiles.h"

namespace nbx {
namespace {

__device__ __forceinline__ u32x4 ldStream(const u32x4* p) { return __builtin_nontemporal_load(p); }

// 8 sources read, XOR-folded in registers; the result is stored only if it
// equals a value the host passes (never in practice), so no load is dead.
template <int NSRC, int U>
__global__ __launch_bounds__(kBlock) void kStreamRead(KArgs a) {
  const u32x4* src[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; s++) src[s] = (const u32x4*)a.src[s];
  const uint64_t n = a.nPacks;
  constexpr uint64_t kTile = (uint64_t)U * kBlock;
  u32x4 acc = {0, 0, 0, 0};
  forEachTile(a, n / kTile, [&](uint64_t t) {
    const uint64_t p = t * kTile + threadIdx.x;
    u32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = ldStream(src[s] + p + u * kBlock);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[s][u];
  });
  if (acc.x == (uint32_t)a.arg && acc.y == (uint32_t)(a.arg >> 32) && acc.z == 0x9e3779b9u)
    ((u32x4*)a.dst[0])[blockIdx.x * kBlock + threadIdx.x] = acc;
}

// 8:1 mixed stream: the fold's loads and stores without its arithmetic
template <int NSRC, int U>
__global__ __launch_bounds__(kBlock) void kStreamMixed(KArgs a) {
  const u32x4* src[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; s++) src[s] = (const u32x4*)a.src[s];
  u32x4* dst = (u32x4*)a.dst[0];
  const uint64_t n = a.nPacks;
  constexpr uint64_t kTile = (uint64_t)U * kBlock;
  forEachTile(a, n / kTile, [&](uint64_t t) {
    const uint64_t p = t * kTile + threadIdx.x;
    u32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = ldStream(src[s] + p + u * kBlock);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 1; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) asm volatile("" ::"v"(v[s][u]));   // live, not computed on
#pragma unroll
    for (int u = 0; u < U; u++) dst[p + u * kBlock] = v[0][u];
  });
}

// plain 16-B stores of a constant: the store half of the fold
template <int U>
__global__ __launch_bounds__(kBlock) void kStreamWrite(KArgs a) {
  u32x4* dst = (u32x4*)a.dst[0];
  const uint64_t n = a.nPacks;
  constexpr uint64_t kTile = (uint64_t)U * kBlock;
  const uint64_t stride = (uint64_t)gridDim.x * kTile;
  const u32x4 v = {(uint32_t)a.arg, (uint32_t)(a.arg >> 32), 0x9e3779b9u, (uint32_t)blockIdx.x};
  for (uint64_t p = (uint64_t)blockIdx.x * kTile + threadIdx.x; p < n; p += stride) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (p + (uint64_t)u * kBlock < n) dst[p + u * kBlock] = v;
  }
}

}  // namespace
}  // namespace nbx

extern "C" __attribute__((visibility("default"))) ncclResult_t nbxDebugStream(int kind, void* dst,
                                                                             const void* const* srcs, int nSrcs,
                                                                             size_t bytes, int blocksPerCU,
                                                                             ncclStream_t stream) {
  using namespace nbx;
  if (kind < 0 || kind > 2 || dst == nullptr || (bytes & 15u) != 0 || blocksPerCU < 0 || blocksPerCU > 16)
    return ncclInvalidArgument;
  if (((uintptr_t)dst & 15u) != 0) return ncclInvalidArgument;
  KArgs a{};
  a.dst[0] = dst;
  a.nPacks = bytes / 16;
  a.arg = 0x0123456789abcdefull;
  if (kind == 0 || kind == 2) {
    if (nSrcs != kMaxKSrcs || srcs == nullptr) return ncclInvalidArgument;
    for (int s = 0; s < nSrcs; s++) {
      if (srcs[s] == nullptr || ((uintptr_t)srcs[s] & 15u) != 0) return ncclInvalidArgument;
      a.src[s] = srcs[s];
    }
  }
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  // read: the production 8-source big tile (one workgroup per CU); write: the
  // production 1-source small tile (5 workgroups per CU)
  const int per = blocksPerCU > 0 ? blocksPerCU : (kind == 1 ? 5 : 1);
  const uint64_t tile = (uint64_t)(kind == 1 ? 1 : 4) * kBlock;
  uint64_t grid = (a.nPacks + tile - 1) / tile;
  if (grid > (uint64_t)cus * (uint64_t)per) grid = (uint64_t)cus * (uint64_t)per;
  if (grid == 0) return ncclSuccess;
  void* args[] = {&a};
  if (kind == 2) {   // the production schedule: dynamic tiles when each workgroup runs >= 16 tiles
    const uint64_t tiles = a.nPacks / tile;
    DynLaunch dyn;
    if (tiles >= 16 * grid) dyn.begin(dev, (hipStream_t)stream, tiles, a);
    const hipError_t e = hipLaunchKernel((const void*)&kStreamMixed<kMaxKSrcs, 4>, dim3((unsigned)grid), dim3(kBlock),
                                         args, 0, (hipStream_t)stream);
    dyn.done(e == hipSuccess);
    return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
  }
  const void* fn = kind == 0 ? (const void*)&kStreamRead<kMaxKSrcs, 4> : (const void*)&kStreamWrite<1>;
  // static tiles: for a read-only stream the grid stride is the faster
  // schedule (7.07-7.10 vs 6.61 TB/s with dynamic tiles, profiles/r2/bench_dyn_ab_r2u.jsonl),
  // so the ceiling stays the higher of the two
  const hipError_t e = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(kBlock), args, 0, (hipStream_t)stream);
  return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}
