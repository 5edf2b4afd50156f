// nbx_simple.h — Simple protocol of the multi-process communicator: the
// direct schedule (kSimpleColl) and the ring schedule (kSimpleRing), one
// kernel per collective, flow control inside the kernel, peer data only
// through staging that every peer mapped once at ncclCommInitRank.
//
// Reference: the Simple protocol's step FIFO (prims_simple.h:129-185:
// waitPeer spins on the peer's tail / head, postPeer publishes after a
// system fence), driven by runRing (all_reduce.h:13-95, reduce_scatter.h:13-66,
// reduce.h:12-68) with connection buffers set up once (transport/p2p.cc:
// 290-330 p2pMap, 450-520 p2pSendConnect / p2pRecvConnect). Peers see only
// connection buffers; user pointers change every call (prims_simple.h:234-235).
//
// MI355X shape (layouts in nbx_ll_args.h SimpleArgs):
//   * staging and flag words are uncached device memory (MTYPE UC): a peer's
//     stores over xGMI land in HBM and no XCD L2 holds a stale copy. The
//     caller's coarse-grained buffers are only ever touched by their own
//     process's kernels, so dispatch-boundary coherence is all they need
//     (round 2 read and wrote peers' user buffers through IPC mappings, and
//     ranks sharing a GPU saw stale bytes and lost stores: tests/
//     test_multiprocess_churn_gpu.py reproduces that deterministically);
//   * the message is cut into n blocks (rank b owns block b); every block is
//     cut into rounds of gridDim.x slices, workgroup g owns slice g of every
//     block in every round, and waits only on workgroup g of its peers — no
//     grid-wide barrier, skew between slices is absorbed by `slots` staging
//     slots per (region, source, workgroup);
//   * direct, per round (AllReduce): A. push slice g of block j into rank j's
//     RS region (all n-1 peers, remote stores); B. fold block `me` from the
//     local input and the n-1 RS slots in the order me+1, ..., me (PreOp on
//     every source, PostOp at the end — the order NCCL's ring accumulates
//     block me), store into the output and push it into every peer's AG
//     region; C. copy the peers' AG slots into the output. Per rank 2(n-1)/n
//     of the message crosses xGMI each way, like a ring, in three hops and on
//     all n-1 links at once. ReduceScatter stops after B; Reduce pushes only
//     to the root, which alone gathers; its fold order is root+1, ..., root;
//   * ring, per round: the reference's ring schedule hop for hop through the
//     right neighbour's staging (RS region: partials, AG region: finished
//     chunks), each hop Fn(pre(local), received) (recvReduceSend's operand
//     order; PreOp on the received raw input only at the first hop).
// Every wait is bounded (timeout without progress, abort word) and records
// what it waited for (nbx_diag.h).
// Included by nbx_kernels.h after ldPack / stPack.
#pragma once
#include "nbx_diag.h"
#include "nbx_order.h"
#include "nbx_functors.h"
#include "nbx_kargs.h"
#include "nbx_ll_args.h"

namespace nbx {

// Bounded spin until *w >= target (a peer's flag word); false on timeout
// (timeoutTicks without the word reaching target) or abort.
__device__ __forceinline__ bool simpleWait(const uint64_t* w, uint64_t target, const SimpleArgs& a, int peer,
                                           uint64_t site) {
  const uint64_t t0 = wall_clock64();
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target) return true;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0u && (*a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks)) {
      const bool aborted = *a.abortWord != 0;
      if (!aborted) diagTimeout(a.errWord, site, peer, target, v, wall_clock64() - t0);
      *a.errWord = aborted ? 2 : 1;
      return false;
    }
  }
}

__device__ __forceinline__ void simplePost(uint64_t* w, uint64_t v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Staging is uncached (MTYPE UC) and written with system-scope write-through
// stores (`sc0 sc1`, as the LL128 lines): once a wave's vmcnt has drained, its
// stores are performed at the memory, so a flag stored after every wave's
// drain (workgroup barrier) publishes them without an L2 write-back fence —
// the guide's write-through hand-off (MI355X_MICROARCH.md, "Valid forms": sc0
// sc1 stores and loads both sides). Readers load staging with `sc0 sc1`
// loads too (buffer loads with the system-scope cache policy): a first
// version read it with nontemporal loads (L1 bypass only) and a chain Reduce
// folded zeros for ~1 % of a slot's elements. Round 3's
// first version used system-scope release / acquire fences per phase instead
// (buffer_wbl2 / buffer_inv of the whole XCD L2, several per round per
// workgroup): 25x slower on 1 GiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sysRsrc(const void* p, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)((bytes + 15) & ~15ull), 0x00020000);
}
// (A buffer store, not inline asm: the compiler's hazard recognizer does not
// see an asm dwordx4 store, and a VALU write to its data registers right after
// it corrupted the first dword of ~6 % of the packs.)
constexpr int kSysStoreAux = 1 | 16;  // sc0 sc1: system scope, write-through
typedef unsigned int nbxV4U __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void stSys(__amdgpu_buffer_rsrc_t rs, uint64_t pack, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(nbxV4U, v), rs, (int)(pack * 16u), 0, kSysStoreAux);
}
template <class E>
__device__ __forceinline__ void stSysElt(E* p, E v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class E>
__device__ __forceinline__ E ldElt(const E* p) { return __builtin_nontemporal_load(p); }
template <class E>
__device__ __forceinline__ E ldSysElt(const E* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int kSysLoadAux = 1 | 16;   // buffer-load cache policy sc0 sc1: system scope
__device__ __forceinline__ u32x4 ldSys(__amdgpu_buffer_rsrc_t rs, uint64_t pack) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(pack * 16u), 0, kSysLoadAux));
}

// Every wave's stores (and loads) of this phase have completed, then the
// workgroup meets: a flag posted after this publishes them.
__device__ __forceinline__ void simpleDrain() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __forceinline__ uint64_t* simpleFlag(uint64_t* base, int kind, int n, int who, int gm, int g) {
  return base + ((uint64_t)kind * n + who) * gm + g;
}

// Slot `slot` of (region, source src, workgroup g) in rank `owner`'s staging.
__device__ __forceinline__ char* simpleStage(const SimpleArgs& a, int owner, int region, uint64_t slot, int src,
                                             int g) {
  const uint64_t idx = (((uint64_t)region * a.slots + slot) * a.nRanks + src) * a.gridMax + g;
  return a.peerStage[owner] + idx * a.stageSlice;
}

// The plan header (when the communicator checks plans: SimpleArgs.planSig != 0,
// NBX_CHECK_PLANS) of slot `slot` of (region, source src, workgroup g) in rank
// `owner`'s staging (16-byte cell, the first 8 bytes used): {plan signature
// (low 32 bits), the producer's count for this slot use (high 32 bits) = the
// value its ready flag announces}, ONE 64-bit store before the drain that
// publishes the slice. Ranks that cut a call or a group run differently (or
// issue different calls) have different signatures, and the consumer fails the
// launch (kDiagSimplePlan) instead of folding data of another plan. The count
// makes a header fresh or stale without any ordering against the flag, so the
// consumer loads it in the same poll as the flag (simpleWaitSlice): no extra
// round trip per hand-off.
__device__ __forceinline__ uint64_t* simpleHdr(const SimpleArgs& a, int owner, int region, uint64_t slot, int src,
                                               int g) {
  const uint64_t idx = (((uint64_t)region * a.slots + slot) * a.nRanks + src) * a.gridMax + g;
  return (uint64_t*)(a.peerStage[owner] + a.hdrOff + idx * 16);
}
__device__ __forceinline__ void simpleStamp(uint64_t* h, const SimpleArgs& a, uint64_t count) {
  if (a.planSig == 0) return;   // plan checks off (NBX_CHECK_PLANS)
  __hip_atomic_store(h, ((uint64_t)(uint32_t)count << 32) | (uint32_t)a.planSig, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bounded spin until the ready flag *w >= target, with slice header h (of the
// slot that use `target` fills) loaded in the same poll; then the header must
// carry `target` (reloaded if that poll's copy was older — the producer stored
// it before the flag) and this launch's signature. False on timeout, abort or
// a plan mismatch.
__device__ __forceinline__ bool simpleWaitSlice(const uint64_t* w, uint64_t target, const uint64_t* h,
                                                const SimpleArgs& a, int peer, uint64_t site) {
  const uint64_t t0 = wall_clock64();
  const bool chk = a.planSig != 0;   // plan checks on (NBX_CHECK_PLANS)
  uint32_t spins = 0;
  uint64_t hv = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (chk) hv = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target) break;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255u) == 0u && (*a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks)) {
      const bool aborted = *a.abortWord != 0;
      if (!aborted) diagTimeout(a.errWord, site, peer, target, v, wall_clock64() - t0);
      *a.errWord = aborted ? 2 : 1;
      return false;
    }
  }
  if (!chk) return true;
  while ((uint32_t)(hv >> 32) != (uint32_t)target) {
    hv = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((++spins & 255u) == 0u && wall_clock64() - t0 > a.timeoutTicks) break;
  }
  if (hv == (((uint64_t)(uint32_t)target << 32) | (uint32_t)a.planSig)) return true;
  diagTimeout(a.errWord, kDiagSimplePlan, peer, (uint32_t)a.planSig, (uint32_t)hv, hv >> 32);
  *a.errWord = 1;
  return false;
}

// Slice checksums (NBX_CHECK_SLICES, SimpleArgs.checkSlices): the producer of
// a staging slice sums a hash of every element it stores there (position-mixed,
// order-free: a 32-bit sum over the workgroup, LDS atomics) and stamps {use
// count, sum} into the second word of the slice's header cell before the drain
// that publishes the slice; the consumer sums the same hash over every element
// it loads and, after its drain, compares with the header. A mismatch means the
// bytes read are not the bytes written — a stale slot, a store not yet landed,
// a misplaced copy — and fails the launch naming the peer, the slot use and both
// sums (kDiagSimpleSlice) instead of returning a silently wrong result. The hash
// is defined per element (index e within the slice, raw bits zero-extended), so
// the 16-B pack path and the element path of either side agree.
__device__ __forceinline__ uint32_t sliceMix(uint32_t lo, uint32_t hi, uint32_t e) {
  const uint32_t t = lo * 0x9E3779B1u ^ hi * 0x85EBCA77u ^ (e + 1u) * 0xC2B2AE3Du;
  return t ^ (t >> 15);
}
template <class E>
__device__ __forceinline__ uint32_t sliceEltHash(E v, uint64_t e) {
  uint64_t bits = 0;
  __builtin_memcpy(&bits, &v, sizeof(E));
  return sliceMix((uint32_t)bits, (uint32_t)(bits >> 32), (uint32_t)e);
}
// the sum of sliceEltHash over the 16 / sizeof(E) elements of pack v, the first at e0
template <class E>
__device__ __forceinline__ uint32_t slicePackHash(u32x4 v, uint64_t e0) {
  constexpr int EB = (int)sizeof(E);
  const uint32_t e = (uint32_t)e0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t h = 0;
  if constexpr (EB == 8) {
    h = sliceMix(v.x, v.y, e) + sliceMix(v.z, v.w, e + 1);
  } else if constexpr (EB == 4) {
#pragma unroll
    for (int i = 0; i < 4; i++) h += sliceMix(w[i], 0, e + i);
  } else if constexpr (EB == 2) {
#pragma unroll
    for (int i = 0; i < 4; i++) h += sliceMix(w[i] & 0xffffu, 0, e + 2 * i) + sliceMix(w[i] >> 16, 0, e + 2 * i + 1);
  } else {
#pragma unroll
    for (int i = 0; i < 16; i++) h += sliceMix((w[i / 4] >> (8 * (i % 4))) & 0xffu, 0, e + i);
  }
  return h;
}
// checkSlices == 2 (the test hook NBX_DEBUG_SLICE_FAULT=<this rank>): workgroup
// 0 stamps a wrong sum, so its consumers must fail the launch.
__device__ __forceinline__ void simpleStampSum(uint64_t* h, const SimpleArgs& a, int g, uint64_t count,
                                               uint32_t sum) {
  if (a.checkSlices == 2 && g == 0) sum ^= 1u;
  __hip_atomic_store(h + 1, ((uint64_t)(uint32_t)count << 32) | sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// After the consumer's drain: the header's {count, sum} against what was read.
__device__ __forceinline__ bool simpleCheckSum(const SimpleArgs& a, const uint64_t* h, uint64_t count, uint32_t got,
                                               int peer) {
  const uint64_t want = __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t seen = ((uint64_t)(uint32_t)count << 32) | got;
  if (want == seen) return true;
  diagTimeout(a.errWord, kDiagSimpleSlice, peer, want, seen, 0);
  *a.errWord = 1;
  return false;
}

// What workgroup g (of `grid`) moves of block b in round k: elements
// [off, off + cnt) of the message whose send / recv buffers are given (a
// group launch's segment, or the launch's one message), and that message's
// block size (ReduceScatter's output offset).
struct SimpleSpan {
  const char* send;
  char* recv;
  uint64_t off, cnt, blockElts;
};
// `segs`: the launch's segment table, read through a pointer (into the
// kernel-argument segment, or the fused rig's argument array) — never through
// the by-value argument itself: a run-time index into that copies the whole
// 824-byte argument block to scratch, and constant indices over 16 segments
// load the table into SGPRs (3,600 SGPR spills in round 4's first build).
template <class E>
__device__ __forceinline__ SimpleSpan simpleSlice(const SimpleArgs& a, const SimpleSeg* segs, int b, uint64_t k,
                                                  int g, int grid) {
  uint64_t v = k * (uint64_t)grid + (uint64_t)g;   // the launch's virtual slice of block b
  SimpleSpan sp{(const char*)a.send, (char*)a.recv, 0, 0, a.blockElts};
  uint64_t total = a.total;
  if (a.nSegs > 0) {
    int s = 0;   // the last segment starting at or before v (sliceOff ascending)
    for (int q = 1; q < a.nSegs; q++)
      if (v >= segs[q].sliceOff) s = q;
    const SimpleSeg sg = segs[s];
    sp.send = (const char*)sg.send;
    sp.recv = (char*)sg.recv;
    sp.blockElts = sg.blockElts;
    total = sg.total;
    v -= sg.sliceOff;
  }
  uint64_t lo = (uint64_t)b * sp.blockElts;
  if (lo > total) lo = total;
  const uint64_t hi = total - lo < sp.blockElts ? total : lo + sp.blockElts;
  const uint64_t sliceE = a.sliceBytes / sizeof(E);
  const uint64_t s0 = v * sliceE;
  sp.off = lo + s0;
  sp.cnt = s0 >= hi - lo ? 0 : (hi - lo - s0 < sliceE ? hi - lo - s0 : sliceE);
  return sp;
}

// Workgroup copy of nElts elements into up to two destinations (any alignment;
// 16-B packs when every pointer is 16-B aligned). sys0 / sys1: the
// destination is staging (write-through stores), else a caller buffer; sysSrc:
// the source is staging (system-scope loads).
// CHK (the NBX_CHECK_SLICES kernels): `sum` is an LDS word that receives the
// slice hash of the elements copied (the staging source read, or the staging
// destination written: the same bytes); the default kernels compile none of it.
template <class E, bool CHK = false>
__device__ __forceinline__ void simpleCopy(void* d0, bool sys0, void* d1, bool sys1, const void* src, bool sysSrc,
                                           uint64_t nElts, uint32_t* sum = nullptr) {
  constexpr int EPP = 16 / (int)sizeof(E);
  uint32_t h = 0;
  uint64_t done = 0;
  if (((((uintptr_t)d0) | ((uintptr_t)src) | (d1 ? (uintptr_t)d1 : 0)) & 15u) == 0) {
    const uint64_t nPk = nElts * sizeof(E) / 16;
    const u32x4* s = (const u32x4*)src;
    const __amdgpu_buffer_rsrc_t rs = sysRsrc(src, nElts * sizeof(E));
    const __amdgpu_buffer_rsrc_t rd0 = sysRsrc(d0, nElts * sizeof(E));
    const __amdgpu_buffer_rsrc_t rd1 = sysRsrc(d1 ? d1 : d0, nElts * sizeof(E));
    constexpr int U = 16;   // 256 B per lane in flight (a 64 KiB slice in one batch): a staging round trip is long
    for (uint64_t p = threadIdx.x; p < nPk; p += (uint64_t)U * kBlock) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++)
        if (p + (uint64_t)u * kBlock < nPk) v[u] = sysSrc ? ldSys(rs, p + (uint64_t)u * kBlock) : ldPack(s + p + (uint64_t)u * kBlock);
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (p + (uint64_t)u * kBlock < nPk) {
          const uint64_t q = p + (uint64_t)u * kBlock;
          if constexpr (CHK) h += slicePackHash<E>(v[u], q * EPP);
          if (sys0) stSys(rd0, q, v[u]);
          else stPack((u32x4*)d0 + q, v[u]);
          if (d1) {
            if (sys1) stSys(rd1, q, v[u]);
            else stPack((u32x4*)d1 + q, v[u]);
          }
        }
      }
    }
    done = nPk * 16 / sizeof(E);
  }
  for (uint64_t e = done + threadIdx.x; e < nElts; e += kBlock) {
    const E v = sysSrc ? ldSysElt((const E*)src + e) : ldElt((const E*)src + e);
    if constexpr (CHK) h += sliceEltHash(v, e);
    if (sys0) stSysElt((E*)d0 + e, v);
    else ((E*)d0)[e] = v;
    if (d1) {
      if (sys1) stSysElt((E*)d1 + e, v);
      else ((E*)d1)[e] = v;
    }
  }
  if constexpr (CHK) atomicAdd(sum, h);
}

// Workgroup fold of nElts elements: acc = pre?(src[0]); acc = Fn(acc, pre?(src[q]))
// for q = 1 .. nSrcs-1 (pre on source q iff bit q of preMask), postOp, then
// stored into every destination (bit d of sysMask: destination d is staging,
// written through). Sources and destinations come from the LDS tables
// (uniform pointers). 16-B packs when `aligned`, else element by element.
// U packs per lane per source, G = 32 / U sources' loads in flight together
// (32 packs = 512 B per lane, as the 8-source big tile): deep unrolling for
// the 2-source ring hops and small rank counts, source groups for many ranks.
// CHK (the NBX_CHECK_SLICES kernels): srcSums / dstSum are LDS words that
// receive the slice hash of each staging source read (indexed by fold
// position; nullptr: none read) and of the result stored into the staging
// destinations (nullptr: none written).
template <class Fn, int U, bool CHK>
__device__ __forceinline__ void simpleFoldU(const Fn& fn, const char* const* srcs, int nSrcs, uint64_t sysSrcMask,
                                            uint64_t preMask, bool doPost, char* const* dsts, int nDsts,
                                            uint64_t sysMask, uint64_t nElts, bool aligned, uint32_t* srcSums,
                                            uint32_t* dstSum) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  constexpr int G = 32 / U;
  uint32_t hd = 0;
  uint64_t done = 0;
  if (aligned) {
    const uint64_t nPk = nElts / EPP;
    for (uint64_t p = threadIdx.x; p < nPk; p += (uint64_t)U * kBlock) {
      u32x4 acc[U];
      for (int q0 = 0; q0 < nSrcs; q0 += G) {
        u32x4 v[G][U];
#pragma unroll
        for (int s = 0; s < G; s++) {
          if (q0 + s < nSrcs) {
            const u32x4* sp = (const u32x4*)srcs[q0 + s];
            const bool sys = (sysSrcMask >> (q0 + s)) & 1u;
            const __amdgpu_buffer_rsrc_t rs = sysRsrc(sp, nElts * sizeof(E));
#pragma unroll
            for (int u = 0; u < U; u++)
              if (p + (uint64_t)u * kBlock < nPk)
                v[s][u] = sys ? ldSys(rs, p + (uint64_t)u * kBlock) : ldPack(sp + p + (uint64_t)u * kBlock);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (CHK && srcSums) {
#pragma unroll
          for (int s = 0; s < G; s++) {
            if (q0 + s < nSrcs && ((sysSrcMask >> (q0 + s)) & 1u)) {
              uint32_t hs = 0;
#pragma unroll
              for (int u = 0; u < U; u++)
                if (p + (uint64_t)u * kBlock < nPk) hs += slicePackHash<E>(v[s][u], (p + (uint64_t)u * kBlock) * EPP);
              atomicAdd(&srcSums[q0 + s], hs);
            }
          }
        }
#pragma unroll
        for (int s = 0; s < G; s++) {
          if (q0 + s < nSrcs) {
#pragma unroll
            for (int u = 0; u < U; u++) {
              u32x4 t = v[s][u];
              if constexpr (Fn::kHasPre) if ((preMask >> (q0 + s)) & 1u) t = fn.prePack(t);
              acc[u] = (q0 + s == 0) ? t : fn.redPack(acc[u], t);
            }
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        if (p + (uint64_t)u * kBlock < nPk) {
          u32x4 r = acc[u];
          if constexpr (Fn::kHasPost) if (doPost) r = fn.postPack(r);
          if constexpr (CHK) if (dstSum) hd += slicePackHash<E>(r, (p + (uint64_t)u * kBlock) * EPP);
          for (int d = 0; d < nDsts; d++) {
            const uint64_t q = p + (uint64_t)u * kBlock;
            if ((sysMask >> d) & 1u) stSys(sysRsrc(dsts[d], nElts * sizeof(E)), q, r);
            else stPack((u32x4*)dsts[d] + q, r);
          }
        }
      }
    }
    done = nPk * EPP;
  }
  for (uint64_t e = done + threadIdx.x; e < nElts; e += kBlock) {
    E acc = (sysSrcMask & 1u) ? ldSysElt((const E*)srcs[0] + e) : ldElt((const E*)srcs[0] + e);
    if constexpr (CHK) if (srcSums && (sysSrcMask & 1u)) atomicAdd(&srcSums[0], sliceEltHash(acc, e));
    if constexpr (Fn::kHasPre) if (preMask & 1u) acc = fn.pre(acc);
    for (int q = 1; q < nSrcs; q++) {
      E x = ((sysSrcMask >> q) & 1u) ? ldSysElt((const E*)srcs[q] + e) : ldElt((const E*)srcs[q] + e);
      if constexpr (CHK) if (srcSums && ((sysSrcMask >> q) & 1u)) atomicAdd(&srcSums[q], sliceEltHash(x, e));
      if constexpr (Fn::kHasPre) if ((preMask >> q) & 1u) x = fn.pre(x);
      acc = fn.red(acc, x);
    }
    if constexpr (Fn::kHasPost) if (doPost) acc = fn.post(acc);
    if constexpr (CHK) if (dstSum) hd += sliceEltHash(acc, e);
    for (int d = 0; d < nDsts; d++) {
      if ((sysMask >> d) & 1u) stSysElt((E*)dsts[d] + e, acc);
      else ((E*)dsts[d])[e] = acc;
    }
  }
  if constexpr (CHK) if (dstSum) atomicAdd(dstSum, hd);
}

template <class Fn, bool CHK = false>
__device__ __forceinline__ void simpleFold(const Fn& fn, const char* const* srcs, int nSrcs, uint64_t sysSrcMask,
                                           uint64_t preMask, bool doPost, char* const* dsts, int nDsts,
                                           uint64_t sysMask, uint64_t nElts, bool aligned,
                                           uint32_t* srcSums = nullptr, uint32_t* dstSum = nullptr) {
  if (nSrcs <= 2)
    simpleFoldU<Fn, 16, CHK>(fn, srcs, nSrcs, sysSrcMask, preMask, doPost, dsts, nDsts, sysMask, nElts, aligned, srcSums,
                        dstSum);
  else if (nSrcs <= 4)
    simpleFoldU<Fn, 8, CHK>(fn, srcs, nSrcs, sysSrcMask, preMask, doPost, dsts, nDsts, sysMask, nElts, aligned, srcSums,
                       dstSum);
  else
    simpleFoldU<Fn, 4, CHK>(fn, srcs, nSrcs, sysSrcMask, preMask, doPost, dsts, nDsts, sysMask, nElts, aligned, srcSums,
                       dstSum);
}

__device__ __forceinline__ bool simpleAligned(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

// Per-workgroup state shared by both schedules.
struct SimpleShared {
  uint64_t cnt[4][kSimpleMaxRanks];   // SimpleCounter x peer
  const char* src[kSimpleMaxRanks];
  char* dst[kSimpleMaxRanks];
  uint32_t sumIn[kSimpleMaxRanks];    // NBX_CHECK_SLICES: hash of what was read (per source / peer)
  uint32_t sumOut[kSimpleMaxRanks];   // ... and of what was written (per target / one for all)
  int fail;
};

__device__ __forceinline__ void simpleLoadCounters(const SimpleArgs& a, SimpleShared& sh, int g) {
  const int n = a.nRanks;
  for (int i = (int)threadIdx.x; i < 4 * n; i += kBlock)
    sh.cnt[i / n][i % n] = a.counters[(uint64_t)i * a.gridMax + g];
  if (threadIdx.x == 0) sh.fail = 0;
  __syncthreads();
}

__device__ __forceinline__ void simpleStoreCounters(const SimpleArgs& a, SimpleShared& sh, int g) {
  __syncthreads();
  const int n = a.nRanks;
  // write-through (agent-scope atomic stores): the next call's kernel may run
  // on another stream and start before this one's end-of-kernel write-back
  // (nbx_order.h)
  for (int i = (int)threadIdx.x; i < 4 * n; i += kBlock)
    __hip_atomic_store(&a.counters[(uint64_t)i * a.gridMax + g], sh.cnt[i / n][i % n], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// The direct schedule as run by workgroup g of a `grid`-workgroup launch
// (kSimpleColl: the launch's own block index; kSimpleCollFused: one launch
// running every rank of a one-process rig, for the PMC passes).
template <class Fn, bool CHK>
__device__ __forceinline__ void simpleCollBody(const SimpleArgs& a, const SimpleSeg* segs, int g, int grid) {
  using E = typename Fn::Elt;
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const int n = a.nRanks, me = a.rank, gm = a.gridMax, tid = (int)threadIdx.x;
  const uint64_t slots = (uint64_t)a.slots;
  __shared__ SimpleShared sh;
  simpleLoadCounters(a, sh, g);
  uint64_t* const myFlags = a.peerFlags[me];
  const bool xport = a.mode == kSimpleTransport;   // AllReduce traffic, no fold (measurement)
  const bool ar = a.mode == kSimpleAllReduce || xport, red = a.mode == kSimpleReduce,
             rs = a.mode == kSimpleReduceScatter;
  const bool storeLocal = !red || me == a.root;        // B writes this rank's output block
  const bool gathers = ar || (red && me == a.root);    // C runs here
  const int first = ((red ? a.root : me) + 1) % n;      // fold order of block `me`
  auto pushTarget = [&](int p) { return p != me && (ar || (red && p == a.root)); };
  constexpr bool chk = CHK;                             // the NBX_CHECK_SLICES kernel

  auto phaseA = [&](uint64_t k) -> bool {
    // ---- A: slice g of block j into rank j's RS region, slot rsSent[j] % slots
    if (tid < n && tid != me) {
      const uint64_t sent = sh.cnt[kCtRsSent][tid];
      if (sent + 1 > slots &&
          !simpleWait(simpleFlag(myFlags, kFlRsCredit, n, tid, gm, g), sent + 1 - slots, a, tid, kDiagSimpleRsCredit))
        sh.fail = 1;
    }
    if (chk && tid < n) sh.sumOut[tid] = 0;
    __syncthreads();
    if (sh.fail) return false;
    for (int q = 1; q < n; q++) {
      const int j = (me + q) % n;
      const SimpleSpan sp = simpleSlice<E>(a, segs, j, k, g, grid);
      if (sp.cnt) simpleCopy<E, CHK>(simpleStage(a, j, 0, sh.cnt[kCtRsSent][j] % slots, me, g), true, nullptr, false,
                                sp.send + sp.off * sizeof(E), false, sp.cnt, chk ? &sh.sumOut[j] : nullptr);
    }
    if (chk) __syncthreads();   // every lane's hash is in
    if (tid < n && tid != me) {
      uint64_t* h = simpleHdr(a, tid, 0, sh.cnt[kCtRsSent][tid] % slots, me, g);
      simpleStamp(h, a, sh.cnt[kCtRsSent][tid] + 1);
      if (chk) simpleStampSum(h, a, g, sh.cnt[kCtRsSent][tid] + 1, sh.sumOut[tid]);
    }
    simpleDrain();
    if (tid < n && tid != me) simplePost(simpleFlag(a.peerFlags[tid], kFlRsReady, n, me, gm, g), ++sh.cnt[kCtRsSent][tid]);
    __syncthreads();
    return true;
  };
  auto phaseB = [&](uint64_t k) -> bool {
    // ---- B: fold block `me` (own input + the n-1 RS slots), store, push to the AG targets
    if (tid < n && tid != me) {
      if (!simpleWaitSlice(simpleFlag(myFlags, kFlRsReady, n, tid, gm, g), sh.cnt[kCtRsRecv][tid] + 1,
                           simpleHdr(a, me, 0, sh.cnt[kCtRsRecv][tid] % slots, tid, g), a, tid, kDiagSimpleRs))
        sh.fail = 1;
      const uint64_t sent = sh.cnt[kCtAgSent][tid];
      if (pushTarget(tid) && sent + 1 > slots &&
          !simpleWait(simpleFlag(myFlags, kFlAgCredit, n, tid, gm, g), sent + 1 - slots, a, tid, kDiagSimpleAgCredit))
        sh.fail = 1;
    }
    const SimpleSpan sp = simpleSlice<E>(a, segs, me, k, g, grid);
    const uint64_t off = sp.off, cnt = sp.cnt;
    // the output holds the whole message, except ReduceScatter's: block `me` only
    const uint64_t outOff = rs ? off - (uint64_t)me * sp.blockElts : off;
    if (tid < n) {
      const int j = (first + tid) % n;
      sh.src[tid] = j == me ? sp.send + off * sizeof(E) : simpleStage(a, me, 0, sh.cnt[kCtRsRecv][j] % slots, j, g);
      // destinations: [own output], then the push targets in the order me+1, ...
      if (tid == 0 && storeLocal) sh.dst[0] = sp.recv + outOff * sizeof(E);
      if (tid > 0) {
        const int p = (me + tid) % n;
        if (ar) sh.dst[tid] = simpleStage(a, p, 1, sh.cnt[kCtAgSent][p] % slots, me, g);
        else if (red && p == a.root) sh.dst[0] = simpleStage(a, p, 1, sh.cnt[kCtAgSent][p] % slots, me, g);
      }
      if (chk) {
        sh.sumIn[tid] = 0;
        if (tid == 0) sh.sumOut[0] = 0;
      }
    }
    __syncthreads();
    if (sh.fail) return false;
    const int nDsts = ar ? n : 1;
    if (cnt) {
      const bool aligned =
          simpleAligned(sp.send + off * sizeof(E)) && (!storeLocal || simpleAligned(sp.recv + outOff * sizeof(E)));
      // destination 0 is the caller's output unless a Reduce non-root pushes to the root
      const uint64_t sysMask = storeLocal ? ~1ull : ~0ull;
      // every source but the own input (at fold position (me - first) mod n) is staging
      const int ownPos = (me - first + n) % n;
      const uint64_t sysSrc = ~(1ull << ownPos);
      if (xport)
        simpleFold<Fn, CHK>(fn, sh.src + ownPos, 1, 0ull, ~0ull, true, sh.dst, nDsts, sysMask, cnt, aligned, nullptr,
                       chk ? &sh.sumOut[0] : nullptr);
      else
        simpleFold<Fn, CHK>(fn, sh.src, n, sysSrc, ~0ull, true, sh.dst, nDsts, sysMask, cnt, aligned,
                       chk ? sh.sumIn : nullptr, chk ? &sh.sumOut[0] : nullptr);
    }
    if (chk) {
      __syncthreads();   // every lane's hashes are in (sources read, result pushed)
      // the n-1 slots folded: what each peer stamped (a transport-only call reads none)
      if (!xport && tid < n && tid != me)
        simpleCheckSum(a, simpleHdr(a, me, 0, sh.cnt[kCtRsRecv][tid] % slots, tid, g), sh.cnt[kCtRsRecv][tid] + 1,
                       sh.sumIn[(tid - first + n) % n], tid);
    }
    if (tid < n && pushTarget(tid)) {
      uint64_t* h = simpleHdr(a, tid, 1, sh.cnt[kCtAgSent][tid] % slots, me, g);
      simpleStamp(h, a, sh.cnt[kCtAgSent][tid] + 1);
      if (chk) simpleStampSum(h, a, g, sh.cnt[kCtAgSent][tid] + 1, sh.sumOut[0]);
    }
    simpleDrain();
    if (tid < n && tid != me) {
      simplePost(simpleFlag(a.peerFlags[tid], kFlRsCredit, n, me, gm, g), ++sh.cnt[kCtRsRecv][tid]);
      if (pushTarget(tid)) simplePost(simpleFlag(a.peerFlags[tid], kFlAgReady, n, me, gm, g), ++sh.cnt[kCtAgSent][tid]);
    }
    __syncthreads();
    return true;
  };
  auto phaseC = [&](uint64_t k) -> bool {
    // ---- C: the peers' finished blocks from the AG region into the output
    if (tid < n && tid != me &&
        !simpleWaitSlice(simpleFlag(myFlags, kFlAgReady, n, tid, gm, g), sh.cnt[kCtAgRecv][tid] + 1,
                         simpleHdr(a, me, 1, sh.cnt[kCtAgRecv][tid] % slots, tid, g), a, tid, kDiagSimpleAg))
      sh.fail = 1;
    if (chk && tid < n) sh.sumIn[tid] = 0;
    __syncthreads();
    if (sh.fail) return false;
    for (int q = 1; q < n; q++) {
      const int j = (me + q) % n;
      const SimpleSpan sp = simpleSlice<E>(a, segs, j, k, g, grid);
      if (sp.cnt) simpleCopy<E, CHK>(sp.recv + sp.off * sizeof(E), false, nullptr, false,
                                simpleStage(a, me, 1, sh.cnt[kCtAgRecv][j] % slots, j, g), true, sp.cnt,
                                chk ? &sh.sumIn[j] : nullptr);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slots are read: they may be refilled
    __syncthreads();
    if (chk && tid < n && tid != me)
      simpleCheckSum(a, simpleHdr(a, me, 1, sh.cnt[kCtAgRecv][tid] % slots, tid, g), sh.cnt[kCtAgRecv][tid] + 1,
                     sh.sumIn[tid], tid);
    if (tid < n && tid != me)
      simplePost(simpleFlag(a.peerFlags[tid], kFlAgCredit, n, me, gm, g), ++sh.cnt[kCtAgRecv][tid]);
    __syncthreads();
    return true;
  };
  // With NBX_SIMPLE_PREFETCH (default on) the next round's pushes go out
  // before this round's fold waits for the peers' pushes, so the flag round
  // trip of B hides behind A(k+1); the order is local to a rank (every
  // counter sequence is unchanged), so ranks need not agree on it.
  if (a.prefetch && a.nRounds > 0 && !phaseA(0)) return;
  for (uint64_t k = 0; k < a.nRounds; k++) {
    if (a.prefetch) {
      if (k + 1 < a.nRounds && !phaseA(k + 1)) return;
    } else if (!phaseA(k)) {
      return;
    }
    if (!phaseB(k)) return;
    if (gathers && !phaseC(k)) return;
  }
  simpleStoreCounters(a, sh, g);
  mpArrive(a.order);
}

// The segment table of the launch's own kernel arguments (SimpleArgs is the
// kernel's only parameter, at offset 0 of the kernel-argument segment).
__device__ __forceinline__ const SimpleSeg* simpleKernargSegs() {
  return (const SimpleSeg*)((const char*)__builtin_amdgcn_kernarg_segment_ptr() + offsetof(SimpleArgs, seg));
}

template <class Fn, bool CHK>
__global__ __launch_bounds__(kBlock) void kSimpleColl(SimpleArgs a) {
  simpleCollBody<Fn, CHK>(a, simpleKernargSegs(), (int)blockIdx.x, (int)gridDim.x);
}

// Ring schedule through the right neighbour's staging. AllReduce /
// ReduceScatter: chunk c enters at rank c+1 (raw), is folded at c+2, ..., and
// finished (PostOp) at c; AllReduce then forwards the finished chunk around
// the ring (all_reduce.h:60-93). Reduce: the chain root+1 -> ... -> root over
// the one block of the message (reduce.h:44-67).
template <class Fn, bool CHK>
__device__ __forceinline__ void simpleRingBody(const SimpleArgs& a, const SimpleSeg* segs, int g, int grid) {
  using E = typename Fn::Elt;
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const int n = a.nRanks, me = a.rank, gm = a.gridMax, tid = (int)threadIdx.x;
  const int left = (me + n - 1) % n, right = (me + 1) % n;
  const uint64_t slots = (uint64_t)a.slots;
  __shared__ SimpleShared sh;
  simpleLoadCounters(a, sh, g);
  uint64_t* const myFlags = a.peerFlags[me];
  const bool ar = a.mode == kSimpleAllReduce, red = a.mode == kSimpleReduce;
  constexpr bool chk = CHK;   // the NBX_CHECK_SLICES kernel: per hop, sumIn[1] = read, sumOut[0] = pushed
  // thread 0 waits for what a hop needs: the left neighbour's slice (recvFrom)
  // and free slots at the right neighbour (RS region: pushRs, AG region: pushAg)
  auto hopWait = [&](int recvRegion, bool pushRs, bool pushAg) {
    if (tid == 0) {
      if (chk) sh.sumIn[1] = sh.sumOut[0] = 0;
      if (recvRegion >= 0) {
        const int fl = recvRegion == 0 ? kFlRsReady : kFlAgReady;
        const int ct = recvRegion == 0 ? kCtRsRecv : kCtAgRecv;
        if (!simpleWaitSlice(simpleFlag(myFlags, fl, n, left, gm, g), sh.cnt[ct][left] + 1,
                             simpleHdr(a, me, recvRegion, sh.cnt[ct][left] % slots, left, g), a, left,
                             recvRegion == 0 ? kDiagSimpleRs : kDiagSimpleAg))
          sh.fail = 1;
      }
      const uint64_t rsS = sh.cnt[kCtRsSent][right], agS = sh.cnt[kCtAgSent][right];
      if (pushRs && rsS + 1 > slots &&
          !simpleWait(simpleFlag(myFlags, kFlRsCredit, n, right, gm, g), rsS + 1 - slots, a, right, kDiagSimpleRsCredit))
        sh.fail = 1;
      if (pushAg && agS + 1 > slots &&
          !simpleWait(simpleFlag(myFlags, kFlAgCredit, n, right, gm, g), agS + 1 - slots, a, right, kDiagSimpleAgCredit))
        sh.fail = 1;
    }
    __syncthreads();
    return sh.fail == 0;
  };
  // the plan headers (and slice sums) of this hop's pushes, before the drain that publishes them
  auto hopStamp = [&](bool pushRs, bool pushAg) {
    if (chk) __syncthreads();   // every lane's hash is in
    if (tid == 0) {
      if (pushRs) {
        uint64_t* h = simpleHdr(a, right, 0, sh.cnt[kCtRsSent][right] % slots, me, g);
        simpleStamp(h, a, sh.cnt[kCtRsSent][right] + 1);
        if (chk) simpleStampSum(h, a, g, sh.cnt[kCtRsSent][right] + 1, sh.sumOut[0]);
      }
      if (pushAg) {
        uint64_t* h = simpleHdr(a, right, 1, sh.cnt[kCtAgSent][right] % slots, me, g);
        simpleStamp(h, a, sh.cnt[kCtAgSent][right] + 1);
        if (chk) simpleStampSum(h, a, g, sh.cnt[kCtAgSent][right] + 1, sh.sumOut[0]);
      }
    }
  };
  auto hopPost = [&](int recvRegion, bool pushRs, bool pushAg) {
    if (tid == 0) {
      if (chk && recvRegion >= 0) {   // after the drain: the slot read is what the left neighbour stamped
        const int ct = recvRegion == 0 ? kCtRsRecv : kCtAgRecv;
        simpleCheckSum(a, simpleHdr(a, me, recvRegion, sh.cnt[ct][left] % slots, left, g), sh.cnt[ct][left] + 1,
                       sh.sumIn[1], left);
      }
      if (recvRegion == 0) simplePost(simpleFlag(a.peerFlags[left], kFlRsCredit, n, me, gm, g), ++sh.cnt[kCtRsRecv][left]);
      if (recvRegion == 1) simplePost(simpleFlag(a.peerFlags[left], kFlAgCredit, n, me, gm, g), ++sh.cnt[kCtAgRecv][left]);
      if (pushRs) simplePost(simpleFlag(a.peerFlags[right], kFlRsReady, n, me, gm, g), ++sh.cnt[kCtRsSent][right]);
      if (pushAg) simplePost(simpleFlag(a.peerFlags[right], kFlAgReady, n, me, gm, g), ++sh.cnt[kCtAgSent][right]);
    }
    __syncthreads();
  };

  for (uint64_t k = 0; k < a.nRounds; k++) {
    if (red) {
      // chain position: 0 = root+1 (sends its raw input), n-1 = the root
      const int pos = (me - a.root - 1 + 2 * n) % n;
      const SimpleSpan sp = simpleSlice<E>(a, segs, 0, k, g, grid);
      const uint64_t off = sp.off, cnt = sp.cnt;
      const bool push = pos < n - 1;
      if (!hopWait(pos == 0 ? -1 : 0, push, false)) return;
      char* out = push ? simpleStage(a, right, 0, sh.cnt[kCtRsSent][right] % slots, me, g) : sp.recv + off * sizeof(E);
      if (pos == 0) {
        if (cnt) simpleCopy<E, CHK>(out, push, nullptr, false, sp.send + off * sizeof(E), false, cnt,
                               chk ? &sh.sumOut[0] : nullptr);
      } else if (cnt) {
        if (tid == 0) {
          sh.src[0] = sp.send + off * sizeof(E);
          sh.src[1] = simpleStage(a, me, 0, sh.cnt[kCtRsRecv][left] % slots, left, g);
          sh.dst[0] = out;
        }
        __syncthreads();
        const bool aligned = simpleAligned(sp.send + off * sizeof(E)) && simpleAligned(out);
        simpleFold<Fn, CHK>(fn, sh.src, 2, 2ull, pos == 1 ? 3u : 1u, !push, sh.dst, 1, push ? 1ull : 0ull, cnt, aligned,
                       chk ? sh.sumIn : nullptr, chk ? &sh.sumOut[0] : nullptr);
      }
      hopStamp(push, false);
      simpleDrain();
      hopPost(pos == 0 ? -1 : 0, push, false);
      continue;
    }
    // send step: the raw chunk me-1 into the right neighbour's RS region
    {
      const SimpleSpan sp = simpleSlice<E>(a, segs, left, k, g, grid);
      if (!hopWait(-1, true, false)) return;
      if (sp.cnt) simpleCopy<E, CHK>(simpleStage(a, right, 0, sh.cnt[kCtRsSent][right] % slots, me, g), true, nullptr,
                                false, sp.send + sp.off * sizeof(E), false, sp.cnt, chk ? &sh.sumOut[0] : nullptr);
      hopStamp(true, false);
      simpleDrain();
      hopPost(-1, true, false);
    }
    // reduce-scatter hops: chunk me-2-st, Fn(pre(local), received)
    for (int st = 0; st < n - 1; st++) {
      const int c = (me + 2 * n - 2 - st) % n;
      const bool last = st == n - 2;
      const SimpleSpan sp = simpleSlice<E>(a, segs, c, k, g, grid);
      const uint64_t off = sp.off, cnt = sp.cnt;
      if (!hopWait(0, !last, last && ar)) return;
      if (tid == 0) {
        sh.src[0] = sp.send + off * sizeof(E);
        sh.src[1] = simpleStage(a, me, 0, sh.cnt[kCtRsRecv][left] % slots, left, g);
        // the last hop's chunk is `me`; ReduceScatter's output holds that block only
        sh.dst[0] = last ? sp.recv + (ar ? off : off - (uint64_t)me * sp.blockElts) * sizeof(E)
                         : simpleStage(a, right, 0, sh.cnt[kCtRsSent][right] % slots, me, g);
        sh.dst[1] = simpleStage(a, right, 1, sh.cnt[kCtAgSent][right] % slots, me, g);
      }
      __syncthreads();
      if (cnt) {
        const bool aligned = simpleAligned(sh.src[0]) && simpleAligned(sh.dst[0]);
        // the last hop stores the caller's output (and pushes the AG start); others push the partial
        simpleFold<Fn, CHK>(fn, sh.src, 2, 2ull, st == 0 ? 3u : 1u, last, sh.dst, last && ar ? 2 : 1, last ? 2ull : 1ull,
                       cnt, aligned, chk ? sh.sumIn : nullptr, chk ? &sh.sumOut[0] : nullptr);
      }
      hopStamp(!last, last && ar);
      simpleDrain();
      hopPost(0, !last, last && ar);
    }
    if (!ar) continue;
    // all-gather hops: the finished chunk me-1-st from the left, forwarded n-2 times
    for (int st = 0; st < n - 1; st++) {
      const int c = (me + 2 * n - 1 - st) % n;
      const bool fwd = st < n - 2;
      const SimpleSpan sp = simpleSlice<E>(a, segs, c, k, g, grid);
      if (!hopWait(1, false, fwd)) return;
      if (sp.cnt)
        simpleCopy<E, CHK>(sp.recv + sp.off * sizeof(E), false,
                      fwd ? simpleStage(a, right, 1, sh.cnt[kCtAgSent][right] % slots, me, g) : nullptr, true,
                      simpleStage(a, me, 1, sh.cnt[kCtAgRecv][left] % slots, left, g), true, sp.cnt,
                      chk ? &sh.sumIn[1] : nullptr);
      if (chk) {   // the forwarded slice is the slice read
        __syncthreads();
        if (tid == 0) sh.sumOut[0] = sh.sumIn[1];
      }
      hopStamp(false, fwd);
      simpleDrain();
      hopPost(1, false, fwd);
    }
  }
  simpleStoreCounters(a, sh, g);
  mpArrive(a.order);
}

template <class Fn, bool CHK>
__global__ __launch_bounds__(kBlock) void kSimpleRing(SimpleArgs a) {
  simpleRingBody<Fn, CHK>(a, simpleKernargSegs(), (int)blockIdx.x, (int)gridDim.x);
}

// Every rank of a one-process rig in ONE launch (workgroup b runs rank
// b / grid's workgroup b % grid): the rig's call as a single dispatch, so a
// rocprofv3 PMC pass — which serializes dispatches — can count its HBM bytes
// (the per-rank launches wait for each other and cannot be serialized).
// Measurement only (nbxDebugSimpleRun with NBX_DEBUG_SIMPLE_FUSED=1).
template <class Fn, bool RING>
__global__ __launch_bounds__(kBlock) void kSimpleFused(const SimpleArgs* __restrict__ as, int grid) {
  const int r = (int)blockIdx.x / grid, g = (int)blockIdx.x % grid;
  if (RING) simpleRingBody<Fn, false>(as[r], as[r].seg, g, grid);
  else simpleCollBody<Fn, false>(as[r], as[r].seg, g, grid);
}

}  // namespace nbx
