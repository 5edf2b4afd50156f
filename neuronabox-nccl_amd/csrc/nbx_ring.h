// nbx_ring.h — pipelined ring AllReduce for the multi-process communicator:
// NCCL's ring reduce-scatter as a device-side dataflow instead of one kernel
// and one barrier per step.
//
// Reference: runRing (all_reduce.h:13-95) driven by the step FIFO of
// prims_simple.h:129-185 (waitPeer / postPeer: a receiver waits for the
// sender's "tail" counter, the sender for the receiver's "head" credit).
// MI355X shape: every rank's buffers are directly addressable over xGMI (IPC
// mappings), so there is no staging FIFO to copy through — the left
// neighbour's partial is read in place from its output buffer — and the step
// FIFO reduces to one progress word per slice:
//   * chunk c (the direct schedule's block c) starts at rank c+1 and visits
//     c+2, ..., c; at step st this rank folds chunk c = me-2-st as
//     Fn(pre(local), received) — recvReduceSend's operand order — into its own
//     output (step 0 reads the left neighbour's raw input, PreOp on both; the
//     last step applies PostOp and stores into every rank's output);
//   * each chunk is cut into gridDim.x slices, slice g always handled by
//     workgroup g. Workgroup g at step st waits until the left neighbour's
//     workgroup g has posted step st-1 (progress word g of this rank, written
//     by the left neighbour with a system-scope store), folds its slice, makes
//     its stores visible (system release) and posts step st into the right
//     neighbour's word g. Slices advance independently: there is no all-rank
//     barrier between steps, so skew between ranks and slices is absorbed the
//     way NCCL's FIFO absorbs it.
// Progress values are (seq-1)*(n-1) + st + 1 with seq from RingState on the
// device (graph replays advance it), so they only grow across calls.
// Included by nbx_kernels.h after foldStore.
#pragma once
#include "nbx_diag.h"
#include "nbx_functors.h"
#include "nbx_kargs.h"
#include "nbx_ll_args.h"

namespace nbx {

__device__ __forceinline__ bool ringWait(const uint64_t* w, uint64_t target, const RingArgs& a, uint64_t t0) {
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target) return true;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0u) {
      if (*a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks) {
        const bool aborted = *a.abortWord != 0;
        if (!aborted) diagTimeout(a.errWord, kDiagRing, (a.rank + a.nRanks - 1) % a.nRanks, target, v, wall_clock64() - t0);
        *a.errWord = aborted ? 2 : 1;
        return false;
      }
    }
  }
}

template <class Fn>
__global__ __launch_bounds__(kBlock) void kRingAllReduce(RingArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // peers' data of earlier calls
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const int n = a.nRanks, me = a.rank, g = (int)blockIdx.x;
  const int left = (me + n - 1) % n;
  (void)left;
  __shared__ uint64_t sSeq;
  __shared__ int sFail;
  if (threadIdx.x == 0) {
    sSeq = __hip_atomic_load(&a.state->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    sFail = 0;
  }
  __syncthreads();
  const uint64_t base = (sSeq - 1) * (uint64_t)(n - 1);
  const uint64_t t0 = wall_clock64();
  for (int st = 0; st < n - 1; st++) {
    const int c = ((me - 2 - st) % n + n) % n;
    const uint64_t off = a.blockElts * (uint64_t)c < a.total ? a.blockElts * (uint64_t)c : a.total;
    const uint64_t len = a.total - off < a.blockElts ? a.total - off : a.blockElts;
    const uint64_t nPacks = len / EPP;
    const bool last = st == n - 2;
    if (st > 0) {   // the left neighbour's workgroup g has finished step st-1
      if (threadIdx.x == 0 && !ringWait(a.myProgress + g, base + (uint64_t)st, a, t0)) sFail = 1;
      __syncthreads();
      if (sFail) return;   // timed out / aborted: errWord is set, the host reports it
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    const E* s0 = (const E*)a.sendMe + off;
    const E* s1 = (const E*)(st == 0 ? a.sendLeft : a.recvLeft) + off;
    const u32x4* src[2] = {(const u32x4*)s0, (const u32x4*)s1};
    u32x4* dst[kMaxKDsts];
    E* dstE[kMaxKDsts];
    const int nDsts = last ? a.nOuts : 1;
#pragma unroll
    for (int d = 0; d < kMaxKDsts; d++) {
      E* b = (E*)(last ? a.outs[d < a.nOuts ? d : 0] : a.recvMe) + off;
      dstE[d] = b;
      dst[d] = (u32x4*)b;
    }
    const uint32_t preMask = st == 0 ? 3u : 1u;
    const bool doPost = Fn::kHasPost && last;
    const uint64_t lo = (uint64_t)g * a.slicePacks;
    const uint64_t hi = lo + a.slicePacks < nPacks ? lo + a.slicePacks : nPacks;
    // 4 packs per lane per source in flight (peer reads cross xGMI: latency wants depth)
    constexpr int U = 4;
    for (uint64_t q = lo + threadIdx.x; q < hi; q += (uint64_t)U * kBlock) {
      if (q + (uint64_t)(U - 1) * kBlock < hi) {
        u32x4 v[2][U];
        loadTile<2, U>(v, src, q);
        __builtin_amdgcn_sched_barrier(0);
        foldStore<Fn, 2, U>(fn, v, preMask, doPost, dst, nDsts, q);
      } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint64_t r = q + (uint64_t)u * kBlock;
          if (r < hi) {
            u32x4 v1[2][1];
            v1[0][0] = ldPack(src[0] + r);
            v1[1][0] = ldPack(src[1] + r);
            foldStore<Fn, 2, 1>(fn, v1, preMask, doPost, dst, nDsts, r);
          }
        }
      }
    }
    // elements past the last whole pack (only the message's last block has them)
    if (g == (int)gridDim.x - 1) {
      const uint64_t i = nPacks * EPP + threadIdx.x;
      if (i < len) {
        E x = s0[i];
        E y = s1[i];
        if constexpr (Fn::kHasPre) {
          x = fn.pre(x);
          if (preMask & 2u) y = fn.pre(y);
        }
        E r = fn.red(x, y);
        if constexpr (Fn::kHasPost) if (doPost) r = fn.post(r);
        for (int d = 0; d < nDsts; d++) dstE[d][i] = r;
      }
    }
    // this slice's stores (and its loads of the left neighbour's buffers) are
    // complete and visible system-wide before the right neighbour hears of them
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    // the compiler may drop the wait after the L2 write-back (MI355X guide,
    // "Compiler hazard"): wait explicitly before this wave joins the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(a.rightProgress + g, base + (uint64_t)st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    const uint64_t prev = __hip_atomic_fetch_add(&a.state->arrive, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 == (uint64_t)gridDim.x) {
      __hip_atomic_store(&a.state->arrive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.state->seq, sSeq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------
// Step-FIFO ring ReduceScatter and chain Reduce (NCCL_ALGO=Ring).
//
// Reference: ReduceScatter runRing (reduce_scatter.h:13-66) — block b enters
// the ring at rank b+1 (send), is folded by b+2, ..., (recvReduceSend) and
// finished at b (recvReduceCopy, postOp) — and Reduce runRing (reduce.h:12-68):
// the chain root+1 -> root+2 -> ... -> root. Each hop folds
// Fn(pre(local), received), recvReduceSend's operand order (prims_simple.h
// genericOp: srcs[0] = own input, srcs[1] = received). The partials travel
// through a step FIFO as NCCL's Simple protocol does (prims_simple.h:129-185):
//   * the FIFO is in the PRODUCER's HBM ([workgroup][slot][entry packs]); the
//     right neighbour reads an entry in place over xGMI, so a hop moves the
//     partial once;
//   * tail: the producer posts the count of entries it has written into the
//     consumer's tail word g (uncached, system-scope store after a system
//     release of the entry); head: the consumer posts the count it has read
//     into the producer's head word g, and the producer reuses a slot only
//     when head has passed it (kRingFifoSlots entries in flight);
//   * the first hop reads the left neighbour's raw input instead of a FIFO
//     entry (NCCL's `send` step), and the last hop writes the caller's output.
// Workgroup g owns slice g of every block and walks its slice in entries of
// kRingFifoEntryPacks packs; entry counts are cumulative per workgroup over
// all calls (RingState.produced / consumed), identical on every rank.
// Timeouts and aborts end every wait as in kRingAllReduce.
__device__ __forceinline__ bool fifoWait(const uint64_t* w, uint64_t target, const RingFifoArgs& a, uint64_t t0,
                                         int peer) {
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target) return true;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0u) {
      if (*a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks) {
        const bool aborted = *a.abortWord != 0;
        if (!aborted) diagTimeout(a.errWord, kDiagRing, peer, target, v, wall_clock64() - t0);
        *a.errWord = aborted ? 2 : 1;
        return false;
      }
    }
  }
}

// Fold `len` packs: dst[q] = Fn(pre?(a[q]), pre?(b[q])) (+ postOp), q < len;
// the message's partial last pack is stored element by element (lastElts > 0:
// valid elements of pack len-1 in `dst`; loads of a 16-B aligned pack that
// holds a byte of the buffer never leave its page).
template <class Fn>
__device__ __forceinline__ void fifoFold(const Fn& fn, const u32x4* pa, const u32x4* pb, u32x4* dst, uint64_t len,
                                         uint32_t preMask, bool doPost, int lastElts) {
  using E = typename Fn::Elt;
  constexpr int U = 4;
  u32x4* dsts[kMaxKDsts];
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++) dsts[d] = dst;
  const u32x4* src[2] = {pa, pb};
  const uint64_t full = lastElts > 0 ? len - 1 : len;
  for (uint64_t q = threadIdx.x; q < full; q += (uint64_t)U * kBlock) {
    if (q + (uint64_t)(U - 1) * kBlock < full) {
      u32x4 v[2][U];
      loadTile<2, U>(v, src, q);
      __builtin_amdgcn_sched_barrier(0);
      foldStore<Fn, 2, U>(fn, v, preMask, doPost, dsts, 1, q);
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t r = q + (uint64_t)u * kBlock;
        if (r < full) {
          u32x4 v1[2][1];
          v1[0][0] = ldPack(pa + r);
          v1[1][0] = ldPack(pb + r);
          foldStore<Fn, 2, 1>(fn, v1, preMask, doPost, dsts, 1, r);
        }
      }
    }
  }
  if (lastElts > 0 && threadIdx.x < (unsigned)lastElts) {   // the partial pack, one element per lane
    const uint64_t i = (len - 1) * (16 / sizeof(E)) + threadIdx.x;
    E x = ((const E*)pa)[i];
    E y = ((const E*)pb)[i];
    if constexpr (Fn::kHasPre) {
      if (preMask & 1u) x = fn.pre(x);
      if (preMask & 2u) y = fn.pre(y);
    }
    E r = fn.red(x, y);
    if constexpr (Fn::kHasPost) if (doPost) r = fn.post(r);
    ((E*)dst)[i] = r;
  }
}

template <class Fn>
__global__ __launch_bounds__(kBlock) void kRingFifo(RingFifoArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  constexpr uint64_t kEntry = kRingFifoEntryPacks;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // peers' data of earlier calls
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const int n = a.nRanks, me = a.rank, g = (int)blockIdx.x;
  const int left = (me + n - 1) % n, right = (me + 1) % n;
  const bool rs = a.mode == kRingFifoReduceScatter;
  // hops of this rank per entry-sized piece of its slice: RS n-1 (block
  // me-2-st at hop st; the last is block me), Reduce one (none for root+1,
  // whose input the next rank reads raw)
  const int pos = rs ? 0 : (me - a.root - 1 + 2 * n) % n;   // Reduce: position in the chain root+1, ..., root
  const int hops = rs ? n - 1 : (pos == 0 ? 0 : 1);
  const uint64_t blockPacks = (a.blockElts + EPP - 1) / EPP;
  const int tailElts = (int)(a.blockElts % EPP);   // Reduce only (RS blocks are whole packs)
  const uint64_t lo = (uint64_t)g * a.slicePacks;
  const uint64_t hi = lo + a.slicePacks < blockPacks ? lo + a.slicePacks : blockPacks;
  const uint64_t len = hi > lo ? hi - lo : 0;
  const uint64_t pieces = (len + kEntry - 1) / kEntry;
  __shared__ uint64_t sProd, sCons;
  __shared__ int sFail;
  if (threadIdx.x == 0) {
    sProd = a.state->produced[g];
    sCons = a.state->consumed[g];
    sFail = 0;
  }
  __syncthreads();
  uint64_t prod = sProd, cons = sCons;
  const uint64_t t0 = wall_clock64();
  u32x4* const myFifo = (u32x4*)a.fifoMe + (uint64_t)g * kRingFifoSlots * kEntry;
  const u32x4* const leftFifo = (const u32x4*)a.fifoLeft + (uint64_t)g * kRingFifoSlots * kEntry;
  for (uint64_t k = 0; k < pieces; k++) {
    const uint64_t pOff = lo + k * kEntry;   // packs into the block / message
    const uint64_t pLen = hi - pOff < kEntry ? hi - pOff : kEntry;
    const int lastElts = (!rs && tailElts && pOff + pLen == blockPacks) ? tailElts : 0;
    for (int st = 0; st < hops; st++) {
      // RS: block c at hop st; Reduce: the message
      const int c = rs ? ((me - 2 - st) % n + n) % n : 0;
      const uint64_t bOff = rs ? (uint64_t)c * blockPacks : 0;
      const bool first = rs ? st == 0 : pos == 1;     // the left neighbour's input, read raw
      const bool last = rs ? st == n - 2 : pos == n - 1;   // into the caller's output
      if (threadIdx.x == 0) {
        // received partial written (tail), and the slot this hop writes free (head)
        if (!first && !fifoWait(a.myTail + g, cons + 1, a, t0, left)) sFail = 1;
        if (!last && prod + 1 > kRingFifoSlots && !fifoWait(a.myHead + g, prod + 1 - kRingFifoSlots, a, t0, right))
          sFail = 1;
      }
      __syncthreads();
      if (sFail) return;   // errWord is set; the host reports it
      if (!first) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      const u32x4* pa = (const u32x4*)a.sendMe + bOff + pOff;
      const u32x4* pb = first ? (const u32x4*)a.sendLeft + bOff + pOff : leftFifo + (cons % kRingFifoSlots) * kEntry;
      u32x4* pd = last ? (u32x4*)a.recv + pOff : myFifo + (prod % kRingFifoSlots) * kEntry;
      fifoFold<Fn>(fn, pa, pb, pd, pLen, first ? 3u : 1u, Fn::kHasPost && last, last ? lastElts : 0);
      // every wave's stores done, made visible system-wide, then posted
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        if (!first)   // the entry is read: its slot may be reused
          __hip_atomic_store(a.leftHead + g, cons + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (!last) __hip_atomic_store(a.rightTail + g, prod + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (!first) cons++;
      if (!last) prod++;
    }
  }
  if (threadIdx.x == 0) {
    a.state->produced[g] = prod;
    a.state->consumed[g] = cons;
  }
}

}  // namespace nbx
