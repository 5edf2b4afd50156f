// nbx_order.h — end-of-launch completion word of the multi-process
// communicator's kernels (MpDone, nbx_ll_args.h): how a call on another stream
// learns that the previous call of the communicator has finished without an
// event behind every call.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nbx_ll_args.h"

namespace nbx {

// Thread 0 of a block, after the whole block's memory operations completed
// (mpDrain): arrive at this block's XCD counter (blockIdx.x % 8: round-robin
// dispatch puts such blocks on one XCD, so the 8 counters sit in 8 L2s and
// each sees <= 32 arrivals instead of 256 on one address, MI355X_MICROARCH.md
// 'fanin'); the last block of an XCD group arrives at the top counter. True
// for the launch's last block, which has reset every counter for the next
// launch.
// The arrivals are RELAXED atomics, not releases: the state a later kernel of
// the communicator reads (Simple counters, LLState) is stored write-through
// (agent-scope atomic stores, `sc1`) and drained by every wave before its
// block arrives, and a later kernel's dispatch invalidates its caches — the
// guide's write-through hand-off (MI355X_MICROARCH.md, "Valid forms": `sc1`
// stores, drained, then the counter add; the adder whose add came last
// signals). Caller buffers are the caller's to order across streams, as with
// any kernel. A release here was an L2 write-back (`buffer_wbl2 sc1`) per
// block and per step of the chain — four in the last block's path.
// (A shortcut for one-block launches sped small Simple calls up but slowed the
// LL kernels, which share this function, by ~0.5 us at 2 ranks: not taken,
// profiles/r4/arrive_r4aj/.)
__device__ __forceinline__ bool mpLastBlock(uint32_t* arrive) {
  const unsigned g = gridDim.x, x = blockIdx.x & 7u;
  const unsigned inGroup = (g - x + 7u) >> 3;   // blocks b < g with b % 8 == x
  const unsigned groups = g < 8u ? g : 8u;
  uint32_t* const mine = arrive + (size_t)x * kMpArriveStride;
  uint32_t* const top = arrive + (size_t)8 * kMpArriveStride;
  if (__hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u != inGroup) return false;
  __hip_atomic_store(mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u != groups) return false;
  __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Every thread of the block: its memory operations complete, then the block meets.
__device__ __forceinline__ void mpDrain() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// The launch's last block publishes the call's number (write-through, after
// every block's arrival) — the completion word a call on another stream waits
// for. Its own stores before this point (the arrival counters' resets, and in
// llEnd the peers' done words and the LLState advance) are drained first: a
// relaxed store to another address may otherwise become visible after the
// completion word, and the next call's kernel would read the old state.
__device__ __forceinline__ void mpPublish(const MpDone& d) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (d.seq != 0) __hip_atomic_store(d.done, d.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The Simple kernels' end, called by EVERY thread of every block as the
// launch's last statement (the early-return paths of a failed wait skip it:
// the communicator is broken then and a waiter times out). Captured calls
// (seq 0) skip it.
__device__ __forceinline__ void mpArrive(const MpDone& d) {
  if (d.seq == 0) return;   // uniform
  mpDrain();
  if (threadIdx.x == 0 && mpLastBlock(d.arrive)) mpPublish(d);
}

}  // namespace nbx
