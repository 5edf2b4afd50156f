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

}  // namespace

ncclResult_t launchMpWaitDone(const uint64_t* done, uint64_t target, const volatile int* abortWord,
                              volatile int* errWord, uint64_t timeoutTicks, hipStream_t stream) {
  hipLaunchKernelGGL(kMpWaitDone, dim3(1), dim3(64), 0, stream, done, target, abortWord, errWord, timeoutTicks);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // namespace nbx
