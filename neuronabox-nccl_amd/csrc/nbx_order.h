// nbx_order.h — end-of-launch completion word of the multi-process
// communicator's kernels (MpDone, nbx_ll_args.h): how a call on another stream
// learns that the previous call of the communicator has finished without an
// event behind every call.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nbx_ll_args.h"

namespace nbx {

// Called by EVERY thread of every block as the launch's last statement (the
// early-return paths of a failed wait skip it: the communicator is broken then
// and the waiter times out). Every thread's memory operations complete, the
// block meets, thread 0 arrives at its XCD's counter (blockIdx.x % 8: the
// round-robin dispatch puts such blocks on one XCD, so the 8 counters are
// served by 8 L2s and each sees <= 32 arrivals instead of 256 on one address,
// MI355X_MICROARCH.md 'fanin'); the last block of an XCD group arrives at the
// top counter, and the last of those publishes the call's number.
__device__ __forceinline__ void mpArrive(const MpDone& d) {
  if (d.seq == 0) return;   // uniform: captured calls publish nothing
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x != 0) return;
  const unsigned g = gridDim.x, x = blockIdx.x & 7u;
  const unsigned inGroup = (g - x + 7u) >> 3;   // blocks b < g with b % 8 == x
  const unsigned groups = g < 8u ? g : 8u;
  uint32_t* const mine = d.arrive + (size_t)x * kMpArriveStride;
  uint32_t* const top = d.arrive + (size_t)8 * kMpArriveStride;
  if (__hip_atomic_fetch_add(mine, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u != inGroup) return;
  __hip_atomic_store(mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u != groups) return;
  __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(d.done, d.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace nbx
