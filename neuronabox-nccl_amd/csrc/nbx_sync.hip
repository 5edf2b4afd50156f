// nbx_sync.hip — cross-process / cross-device stream barrier for the
// multi-process communicator (the role of NCCL's waitPeer/postPeer step
// credits, prims_simple.h:129-185, reduced to one flag per phase).
//
// One wave: lane 0 publishes this rank's phase flag with a system-scope
// release store; lane j polls rank j's flag (IPC-mapped over xGMI) with
// relaxed system-scope loads and s_sleep backoff until it reaches `seq`, then
// a system-scope acquire fence. Every spin is bounded: the host abort word
// (ncclCommAbort) and a wall-clock timeout (s_memrealtime, 100 MHz) both end
// it and set the host error word, read by ncclCommGetAsyncError.
// Data written by earlier kernels of the stream is already released at their
// kernel boundary; the barrier orders the flag after it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nbx_diag.h"

namespace nbx {

// Advances this rank's epoch of flag `slot` (plain device memory, one counter
// per slot) to v, posts v to the flag, then waits until every rank j with bit j
// of `waitMask` has flag `slot` >= v. Every rank issues the same sequence of
// barriers on a slot, so the epochs agree without the host passing values —
// which is what lets a graph-captured collective replay.
__global__ __launch_bounds__(64) void kPeerBarrier(uint64_t* myFlags, uint64_t* const* peerFlags, int n, int slot,
                                                   uint64_t waitMask, uint64_t* epochs,
                                                   const volatile int* abortWord, volatile int* errWord,
                                                   uint64_t timeoutTicks) {
  const int lane = (int)threadIdx.x;
  __shared__ uint64_t sV;
  if (lane == 0) {
    const uint64_t v = epochs[slot] + 1;
    epochs[slot] = v;
    sV = v;
    __atomic_thread_fence(__ATOMIC_RELEASE);   // order prior work of this kernel (none) and the flag
    __hip_atomic_store(myFlags + slot, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const uint64_t seq = sV;
  if (lane < n && ((waitMask >> lane) & 1ull)) {
    const uint64_t* f = peerFlags[lane] + slot;
    const uint64_t t0 = wall_clock64();
    uint32_t spins = 0;
    uint64_t v;
    while ((v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) < seq) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 255u) == 0u) {
        if (*abortWord != 0) {
          *errWord = 2;
          break;
        }
        if (wall_clock64() - t0 > timeoutTicks) {
          diagTimeout(errWord, kDiagBarrier, lane, seq, v, wall_clock64() - t0);
          *errWord = 1;
          break;
        }
      }
    }
  }
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: drop stale cached peer data
}

hipError_t launchPeerBarrier(uint64_t* myFlags, uint64_t* const* peerFlagsDev, int n, int slot, uint64_t waitMask,
                             uint64_t* epochsDev, const int* abortWordDev, int* errWordDev, double timeoutSec,
                             hipStream_t stream) {
  if (n < 1 || n > 64) return hipErrorInvalidValue;
  const uint64_t ticks = (uint64_t)(timeoutSec * 1.0e8);   // wall_clock64 runs at 100 MHz
  hipLaunchKernelGGL(kPeerBarrier, dim3(1), dim3(64), 0, stream, myFlags, peerFlagsDev, n, slot, waitMask, epochsDev,
                     (const volatile int*)abortWordDev, (volatile int*)errWordDev, ticks);
  return hipGetLastError();
}

}  // namespace nbx
