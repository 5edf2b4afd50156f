// nbx_ll_debug.hip — a deliberately torn LL128 line against the production
// reader: the reader kernel polls one line with the
// collectives' own l128Poll / l128FoldLine while a writer kernel on another
// stream stores the line's last 32 bytes, waits, then its first 32 bytes. A
// reader that trusted one flag per line (the r1 layout: flag in the last lane)
// would accept the line after the first half and fold two stale chunks; with a
// flag in every 16-byte chunk it must wait for the second half.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/nbx_debug.h"
#include "nbx_internal.h"
#include "nbx_kernels.h"

namespace nbx {
namespace {

// one 4-lane line: lanes 2-3 (the flag half of the r1 layout) first, then,
// after `delayTicks`, lanes 0-1; stamp[0] = time the second half is issued
__global__ __launch_bounds__(64) void kL128TearWriter(uint64_t* line, const unsigned char* payload, uint32_t flag,
                                                      uint64_t delayTicks, uint64_t* stamp) {
  const int t = (int)threadIdx.x;
  if (t >= kL128Lanes) return;
  const u32x4 v = l128Chunk(payload, kL128DataBytes, 0, t, flag);
  if (t >= 2) l128StoreLine16(line, 64, 2 * t, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (t == 0) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < delayTicks) __builtin_amdgcn_s_sleep(8);
    stamp[0] = wall_clock64();
  }
  __builtin_amdgcn_wave_barrier();
  if (t < 2) l128StoreLine16(line, 64, 2 * t, v);
}

// the production poll + fold for a 2-rank line whose own contribution is zero:
// out = the received payload; stamp[1] = time the line was accepted
__global__ __launch_bounds__(64) void kL128TearReader(LLArgs a, uint32_t flag, unsigned char* out, uint64_t* stamp) {
  const int t = (int)(threadIdx.x % kL128Lanes);
  if (threadIdx.x >= (unsigned)kL128Lanes) return;
  const FnSumInt<uint32_t> fn(0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.myL128, (short)0, (int)a.l128Bytes,
                                                                      0x00020000);
  u32x4 v[kL128MaxRanks];
#pragma unroll
  for (int q = 0; q < kL128MaxRanks; q++) v[q] = (u32x4){0, 0, 0, 0};
  const bool ok = l128Poll(a, rs, v, 2u, flag, kDiagLL128Line, wall_clock64(), t, [](int) { return 0u; }, nullptr, -1);
  if (t == 0) stamp[1] = ok ? wall_clock64() : 0;
  l128FoldLine(fn, a, v, 0, t, 1, a.blockElts, [&](int, uint64_t off, uint64_t w) { llStoreBytes(out, off, kL128DataBytes, w); });
}

// Link probe (nbxDebugLinkProbe): workgroup w serves peer q = the w / wgPerPeer-th
// other rank, moving chunk j = w % wgPerPeer of this rank's part of q's Simple
// data area — pushed with the transport's system-scope stores, or pulled with
// its system-scope loads — `passes` times over. Four packs in flight per lane
// per step; a pull's loads stay live through an XOR that is stored only if it
// equals a value no real data produces.
template <bool PULL>
__global__ __launch_bounds__(kBlock) void kLinkProbe(char* const* peerStage, int me, uint64_t part,
                                                     uint64_t chunkPacks, int wgPerPeer, int passes, uint32_t* sink) {
  const int w = (int)blockIdx.x;
  int q = w / wgPerPeer;
  q += q >= me ? 1 : 0;
  const uint64_t j = (uint64_t)(w % wgPerPeer);
  const __amdgpu_buffer_rsrc_t rs = sysRsrc(peerStage[q] + (uint64_t)me * part, part);
  const uint64_t base = j * chunkPacks;
  const uint64_t step = 4ull * blockDim.x;
  u32x4 acc = {(uint32_t)me, (uint32_t)j, 0u, 0u};
  for (int pass = 0; pass < passes; pass++) {
    for (uint64_t i = threadIdx.x; i < chunkPacks; i += step) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const uint64_t k = i + (uint64_t)u * blockDim.x;
        if (k < chunkPacks) {
          if constexpr (PULL) v[u] = ldSys(rs, base + k);
          else stSys(rs, base + k, acc + (u32x4){(uint32_t)k, (uint32_t)pass, 0u, 0u});
        }
      }
      if constexpr (PULL) {
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (i + (uint64_t)u * blockDim.x < chunkPacks) acc ^= v[u];
      }
    }
  }
  if (PULL && acc[0] == 0x9e3779b9u && acc[1] == 0x7f4a7c15u && acc[2] == 0xf39cc060u) sink[threadIdx.x] = acc[3];
}

}  // namespace

ncclResult_t launchLinkProbe(char* const* peerStageDev, int me, int n, uint64_t part, uint64_t chunkPacks,
                             int wgPerPeer, int passes, bool pull, uint32_t* sink, hipStream_t stream) {
  static_assert(kLinkProbeSinkWords == kBlock, "one sink word per lane");
  const dim3 grid((unsigned)((n - 1) * wgPerPeer));
  if (pull)
    hipLaunchKernelGGL(kLinkProbe<true>, grid, dim3(kBlock), 0, stream, peerStageDev, me, part, chunkPacks, wgPerPeer,
                       passes, sink);
  else
    hipLaunchKernelGGL(kLinkProbe<false>, grid, dim3(kBlock), 0, stream, peerStageDev, me, part, chunkPacks,
                       wgPerPeer, passes, sink);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// The Simple rig's call as ONE dispatch (kSimpleFused, fp32 sum only): every
// rank's workgroups in one grid, so rocprofv3's PMC passes can count the
// call's HBM bytes (nbxDebugSimpleRun, NBX_DEBUG_SIMPLE_FUSED=1).
ncclResult_t launchSimpleFusedF32Sum(const SimpleArgs* argsDev, int n, unsigned grid, bool ring, hipStream_t stream) {
  if (ring)
    hipLaunchKernelGGL((kSimpleFused<FnSumF<TyF32>, true>), dim3((unsigned)n * grid), dim3(kBlock), 0, stream, argsDev,
                       (int)grid);
  else
    hipLaunchKernelGGL((kSimpleFused<FnSumF<TyF32>, false>), dim3((unsigned)n * grid), dim3(kBlock), 0, stream,
                       argsDev, (int)grid);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

// Workgroups of the fused Simple kernel the current device holds at once
// (occupancy x CUs): workgroup g of one rank spins on workgroup g of its
// peers, so a fused grid larger than this would wait for workgroups that are
// never scheduled; -1 on a HIP error.
int simpleFusedMaxResident(bool ring) {
  int dev = 0, cus = 0, perCu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  const void* fn = ring ? (const void*)&kSimpleFused<FnSumF<TyF32>, true> : (const void*)&kSimpleFused<FnSumF<TyF32>, false>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, fn, kBlock, 0) != hipSuccess) return -1;
  return perCu * cus;
}
}  // namespace nbx

extern "C" __attribute__((visibility("default"))) int nbxDebugLL128TearTest(int delayUs, int tear,
                                                                           long long* acceptAfterTornTicks) {
  using namespace nbx;
  unsigned char hPay[kL128DataBytes], hOut[kL128DataBytes];
  for (int b = 0; b < kL128DataBytes; b++) hPay[b] = (unsigned char)(0x11 * (b + 1) + 7);
  // stale line: every chunk from the previous call (flag 6) with other payload
  uint32_t hLine[16];
  for (int w = 0; w < 16; w++) hLine[w] = (w % 4 == 3) ? 6u : 0xdead0000u + (uint32_t)w;
  uint64_t* line = nullptr;
  unsigned char *pay = nullptr, *out = nullptr;
  uint64_t* stamp = nullptr;
  int* words = nullptr;
  hipStream_t sr = nullptr, sw = nullptr;
  int rc = -1;
  if (hipExtMallocWithFlags((void**)&line, 64, hipDeviceMallocUncached) != hipSuccess) return -1;
  if (hipMalloc((void**)&pay, kL128DataBytes) == hipSuccess && hipMalloc((void**)&out, kL128DataBytes) == hipSuccess &&
      hipMalloc((void**)&stamp, 16) == hipSuccess && hipMalloc((void**)&words, 64) == hipSuccess &&
      hipStreamCreateWithFlags(&sr, hipStreamNonBlocking) == hipSuccess &&
      hipStreamCreateWithFlags(&sw, hipStreamNonBlocking) == hipSuccess &&
      hipMemcpy(line, hLine, 64, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemcpy(pay, hPay, kL128DataBytes, hipMemcpyHostToDevice) == hipSuccess &&
      hipMemset(out, 0, kL128DataBytes) == hipSuccess && hipMemset(stamp, 0, 16) == hipSuccess &&
      hipMemset(words, 0, 64) == hipSuccess) {   // the host-words layout: a timeout's diag record lands at bytes 16-63
    LLArgs a{};
    a.myL128 = line;
    a.l128Bytes = 64;
    a.nRanks = 2;
    a.rank = 0;
    a.blockElts = 1u << 30;
    a.abortWord = words;
    a.errWord = words + 1;
    a.timeoutTicks = 10ull * 100000000ull;   // 10 s
    const uint64_t delay = (uint64_t)(delayUs > 0 ? delayUs : 0) * 100ull;   // 100 MHz ticks
    hipLaunchKernelGGL(kL128TearReader, dim3(1), dim3(64), 0, sr, a, 7u, out, stamp);
    hipLaunchKernelGGL(kL128TearWriter, dim3(1), dim3(64), 0, sw, line, (const unsigned char*)pay, 7u,
                       tear ? delay : 0ull, stamp);
    uint64_t hStamp[2] = {0, 0};
    int hWords[2] = {0, 0};
    if (hipStreamSynchronize(sw) == hipSuccess && hipStreamSynchronize(sr) == hipSuccess &&
        hipMemcpy(hOut, out, kL128DataBytes, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(hStamp, stamp, 16, hipMemcpyDeviceToHost) == hipSuccess &&
        hipMemcpy(hWords, words, 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (acceptAfterTornTicks) *acceptAfterTornTicks = (long long)(hStamp[1] - hStamp[0]);
      if (hWords[1] != 0 || hStamp[1] == 0) rc = 3;                          // the reader timed out
      else if (std::memcmp(hOut, hPay, kL128DataBytes) != 0) rc = 1;       // folded stale chunks
      else if (tear && hStamp[1] < hStamp[0]) rc = 2;                      // accepted before the second half
      else rc = 0;
    }
  }
  if (sr) (void)hipStreamDestroy(sr);
  if (sw) (void)hipStreamDestroy(sw);
  (void)hipFree(line);
  (void)hipFree(pay);
  (void)hipFree(out);
  (void)hipFree(stamp);
  (void)hipFree(words);
  return rc;
}
