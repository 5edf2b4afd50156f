// nbx_order.hip — kMpWaitDone: the wait a multi-process communicator puts on
// a stream ahead of a call when the previous call ran on another stream (see
// MpDone, nbx_ll_args.h / nbx_order.h). One wave; lane 0 polls the done word
// with s_sleep between polls, bounded like every other wait of the library
// (timeout without progress -> error word 1 and a diagnostic record, abort
// word -> 2), so a broken previous call cannot hang the stream forever.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nbx_diag.h"
#include "nbx_internal.h"

namespace nbx {
namespace {

__global__ __launch_bounds__(64) void kMpWaitDone(const uint64_t* done, uint64_t target, const volatile int* abortWord,
                                                  volatile int* errWord, uint64_t timeoutTicks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (v >= target) return;
    __builtin_amdgcn_s_sleep(2);
    if ((++spins & 255u) == 0u && (*abortWord != 0 || wall_clock64() - t0 > timeoutTicks)) {
      const bool aborted = *abortWord != 0;
      if (!aborted) diagTimeout(errWord, kDiagOrder, -1, target, v, wall_clock64() - t0);
      *errWord = aborted ? 2 : 1;
      return;
    }
  }
}

// Test hook (nbxDebugHoldStream): one wave holds its stream until the host
// sets *word (pinned, device-mapped), or timeoutTicks pass.
__global__ __launch_bounds__(64) void kHoldStream(const int* word, uint64_t timeoutTicks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         wall_clock64() - t0 < timeoutTicks)
    __builtin_amdgcn_s_sleep(8);
}

constexpr int kHoldSlots = 16;
int* g_holdWords = nullptr;   // pinned, device-mapped; never freed (test hook)
int* g_holdWordsDev = nullptr;
bool g_holdBusy[kHoldSlots] = {};
unsigned g_holdNext = 0;      // round robin: a released slot is the last one reused

}  // namespace

ncclResult_t launchMpWaitDone(const uint64_t* done, uint64_t target, const volatile int* abortWord,
                              volatile int* errWord, uint64_t timeoutTicks, hipStream_t stream) {
  hipLaunchKernelGGL(kMpWaitDone, dim3(1), dim3(64), 0, stream, done, target, abortWord, errWord, timeoutTicks);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // namespace nbx

extern "C" __attribute__((visibility("default"))) int nbxDebugHoldStream(ncclStream_t stream, int timeoutMs) {
  using namespace nbx;
  if (timeoutMs <= 0) return -1;
  if (g_holdWords == nullptr) {
    if (hipHostMalloc((void**)&g_holdWords, kHoldSlots * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&g_holdWordsDev, g_holdWords, 0) != hipSuccess)
      return -2;
  }
  int slot = -1;
  for (int k = 0; k < kHoldSlots && slot < 0; k++) {
    const int c = (int)((g_holdNext + (unsigned)k) % kHoldSlots);
    if (!g_holdBusy[c]) slot = c;
  }
  if (slot < 0) return -1;
  g_holdNext = (unsigned)slot + 1;
  __atomic_store_n(&g_holdWords[slot], 0, __ATOMIC_SEQ_CST);
  hipLaunchKernelGGL(kHoldStream, dim3(1), dim3(64), 0, (hipStream_t)stream, g_holdWordsDev + slot,
                     (uint64_t)timeoutMs * 100000ull);
  if (hipGetLastError() != hipSuccess) return -2;
  g_holdBusy[slot] = true;
  return slot;
}

extern "C" __attribute__((visibility("default"))) int nbxDebugReleaseStream(int hold) {
  using namespace nbx;
  if (hold < 0 || hold >= kHoldSlots || g_holdWords == nullptr || !g_holdBusy[hold]) return -1;
  __atomic_store_n(&g_holdWords[hold], 1, __ATOMIC_SEQ_CST);
  g_holdBusy[hold] = false;
  return 0;
}
