// nbx_kernels.h — the multi-source reduce-copy kernels for gfx950.
//
// MI355X-native replacement for reduceCopy / reduceCopyPacks
// (/root/reference/src/device/common_kernel.h:28-239) and the one-rank kernel
// shell (/root/reference/src/device/onerank.cu:14-45).
//
// Design (not a translation of the warp-32 hunk loop):
//   * One wave64 instruction moves 1 KiB contiguous (64 lanes x 16-B dwordx4);
//     a 256-thread workgroup owns a tile of U x 256 packs and issues all
//     NSRC x U loads of a tile before folding, so every lane keeps
//     NSRC*U*16 B in flight — the HBM-latency cover this load-bound loop
//     needs (no LDS: an element-wise fold has no reuse to stage).
//   * NSRC is a compile-time constant (1..8): sources are folded in order,
//     acc = pre(src0); acc = Fn(acc, pre(src_s)), in registers — the
//     reference's left fold (common_kernel.h:79-131), hence bit-exact.
//   * Grid-stride over tiles with a capped grid (>= 8 workgroups per CU on
//     256 CUs), a guarded last tile, and the <16-B head/tail elements of a
//     shared misalignment done by one wave of the last workgroup.
//   * Pointers that do not share one alignment modulo 16 take the element
//     kernel (common_kernel.h:229-238's sizeof(T) packs).
#pragma once
#include <utility>
#include "nbx_functors.h"
#include "nbx_kargs.h"
#include "nbx_ll.h"
#include "nbx_tiles.h"

namespace nbx {




// Device-resident scalar: read the element's bytes while the kernel runs
// (reference: common.h:100-119 / onerank.cu:32-42 dereference by alignment;
// reading exactly sizeof(T) yields the same scalar bits).
template <class Fn>
__device__ __forceinline__ uint64_t loadArg(const KArgs& a) {
  if (a.argPtr != nullptr) return (uint64_t) * (const typename Fn::Elt*)a.argPtr;
  return a.arg;
}

// Streaming loads carry the nontemporal hint (global_load_dwordx4 ... nt):
// measured on MI355X (scripts/sweep_variants.hip, profiles/) the 8:1
// read:write fold runs ~20 % faster with nt loads, while nt STORES cost
// ~7 % (write-only ceiling 6.8 TB/s plain vs 5.3 TB/s nt), so stores stay plain.
__device__ __forceinline__ u32x4 ldPack(const u32x4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stPack(u32x4* p, u32x4 v) { *p = v; }

// One element, any source count <= kMaxKSrcs (unrolled with a uniform guard
// so the kernel-argument pointer array is never indexed dynamically).
template <class Fn>
__device__ __forceinline__ void reduceElt(const Fn& fn, const KArgs& a, int nSrcs, uint64_t i) {
  using E = typename Fn::Elt;
  E acc = ((const E*)a.src[0])[i];
  if constexpr (Fn::kHasPre) if (a.preMask & 1u) acc = fn.pre(acc);
#pragma unroll
  for (int s = 1; s < kMaxKSrcs; s++) {
    if (s < nSrcs) {
      E v = ((const E*)a.src[s])[i];
      if constexpr (Fn::kHasPre) if ((a.preMask >> s) & 1u) v = fn.pre(v);
      acc = fn.red(acc, v);
    }
  }
  if constexpr (Fn::kHasPost) if (a.postOp) acc = fn.post(acc);
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++)
    if (d < a.nDsts) ((E*)a.dst[d])[i] = acc;
}

// Fold one tile slice already in registers and store it (all U packs valid).
// Destinations beyond the first are a uniform branch per store (the direct
// schedules' push-gather writes every rank's output from one kernel).
template <class Fn, int NSRC, int U>
__device__ __forceinline__ void foldStore(const Fn& fn, const u32x4 (&v)[NSRC][U], uint32_t preMask, bool doPost,
                                          u32x4* const (&dst)[kMaxKDsts], int nDsts, uint64_t p) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 acc = v[0][u];
    if constexpr (Fn::kHasPre) if (preMask & 1u) acc = fn.prePack(acc);
#pragma unroll
    for (int s = 1; s < NSRC; s++) {
      u32x4 t = v[s][u];
      if constexpr (Fn::kHasPre) if ((preMask >> s) & 1u) t = fn.prePack(t);
      acc = fn.redPack(acc, t);
    }
    if constexpr (Fn::kHasPost) if (doPost) acc = fn.postPack(acc);
    stPack(dst[0] + p + u * kBlock, acc);
#pragma unroll
    for (int d = 1; d < kMaxKDsts; d++)
      if (d < nDsts) stPack(dst[d] + p + u * kBlock, acc);
  }
}

// Source-major issue order (all U packs of source 0, then source 1, ...). The
// unroll-major order lets the fold start after the first NSRC loads land
// (the compiler then waits vmcnt(31), (30), ... instead of near 0), which
// should help the VALU-heavy functors — measured in-process it lost for every
// dtype at the configs' shapes, fp8 included (f32 6235 -> 5979 GB/s, fp8 e4m3
// 5704 -> 5668; profiles/r2/ab_load_order_r4b.jsonl).
template <int NSRC, int U>
__device__ __forceinline__ void loadTile(u32x4 (&v)[NSRC][U], const u32x4* const (&src)[NSRC], uint64_t p) {
#pragma unroll
  for (int s = 0; s < NSRC; s++)
#pragma unroll
    for (int u = 0; u < U; u++) v[s][u] = ldPack(src[s] + p + u * kBlock);
}

// Grid-stride loop over tiles; each lane issues all NSRC x U loads of a tile
// before folding. (A software-pipelined variant — next tile's loads issued
// before the current tile is stored — measured neutral to -5 % in-process on
// MI355X, profiles/r1/sweep_lib_r1d.jsonl, and was dropped.)
// Reading another GPU's memory (the collectives' direct schedules): drop any
// line of peer memory this XCD's L2 / this CU's L1 may still hold from an
// earlier call before the first load — the peers wrote it after that, and
// ordered their writes before this launch through the flag barrier. Every
// workgroup does it (one per CU at the big tile: every XCD's L2 is covered).
__device__ __forceinline__ void acquirePeerData(const KArgs& a) {
  if (a.acquireSystem) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

template <class Fn, int NSRC, int U>
__global__ __launch_bounds__(kBlock) void kReducePacks(KArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  acquirePeerData(a);
  const Fn fn(loadArg<Fn>(a));
  const uint64_t headBytes = (uint64_t)a.headElts * sizeof(E);
  const u32x4* src[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; s++) src[s] = (const u32x4*)((const char*)a.src[s] + headBytes);
  u32x4* dst[kMaxKDsts];
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++) dst[d] = (u32x4*)((char*)a.dst[d] + headBytes);
  const int nDsts = a.nDsts;
  const bool doPost = Fn::kHasPost && a.postOp;
  const uint32_t preMask = a.preMask;
  const uint64_t n = a.nPacks;
  constexpr uint64_t kTile = (uint64_t)U * kBlock;
  forEachTile(a, (n + kTile - 1) / kTile, [&](uint64_t t) {
    const uint64_t p = t * kTile + threadIdx.x;
    if (p + (uint64_t)(U - 1) * kBlock < n) {
      // full tile: issue every load first, then fold
      u32x4 v[NSRC][U];
      loadTile<NSRC, U>(v, src, p);
      // keep every load of the tile ahead of the fold: left to itself the
      // scheduler waits on the first few loads before issuing the rest
      __builtin_amdgcn_sched_barrier(0);
      foldStore<Fn, NSRC, U>(fn, v, preMask, doPost, dst, nDsts, p);
    } else {
      // last, partial tile
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = p + (uint64_t)u * kBlock;
        if (q < n) {
          u32x4 v1[NSRC][1];
#pragma unroll
          for (int s = 0; s < NSRC; s++) v1[s][0] = ldPack(src[s] + q);
          foldStore<Fn, NSRC, 1>(fn, v1, preMask, doPost, dst, nDsts, q);
        }
      }
    }
  });

  // head (< EPP elements before the aligned body) and tail (< EPP after it)
  if (blockIdx.x == gridDim.x - 1) {
    const int head = a.headElts;
    const uint64_t tailStart = (uint64_t)head + n * EPP;
    const int tail = (int)(a.nElts - tailStart);
    const int t = (int)threadIdx.x;
    if (t < head) reduceElt(fn, a, NSRC, (uint64_t)t);
    else if (t < head + tail) reduceElt(fn, a, NSRC, tailStart + (uint64_t)(t - head));
  }
}

// Element kernel: pointers with different alignments modulo 16.
template <class Fn>
__global__ __launch_bounds__(kBlock) void kReduceElts(KArgs a) {
  acquirePeerData(a);
  const Fn fn(loadArg<Fn>(a));
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < a.nElts; i += stride)
    reduceElt(fn, a, a.nSrcs, i);
}

// ---------------------------------------------------------------------------
// Sources misaligned against the destinations (common_kernel.h:229-238 falls
// back to sizeof(T) packs there). Here the destinations (which share one
// alignment) stay 16-B packs, and each source is read as 16-B aligned packs
// and realigned: output pack q needs packs q and q+1 of the source's
// aligned-down base, funnel-shifted by the source's byte offset
// (v_alignbyte_b32; the offset is per source, so the shift case is uniform).
// Two kernels:
//  * kReduceShiftedLds<Fn, NSRC> (the default, below the fallback): the
//    sources staged through LDS by LDS-DMA, one kernel per source count;
//  * kReduceShifted<Fn>: the run-time source count fallback — each lane loads
//    q and q+1 itself with plain (temporal) loads, the second mostly an L2
//    hit (it is the next lane's first); 1 pack per lane, 8 workgroups per CU
//    (launch variant 1 or NBX_SHIFT_N=0).
// Memory safety: a 16-B aligned pack never crosses a page, and every pack
// loaded holds at least one byte of the source range (pack indices are
// clamped to the last one), so no load can touch an unmapped page.
__device__ __forceinline__ u32x4 funnel16(const u32x4& lo, const u32x4& hi, uint32_t m) {
  const uint32_t b = m & 3u;   // byte shift inside a dword (0: plain dword select)
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 r;
  switch (m >> 2) {   // uniform across the wave
    case 0:
      r = u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], b), __builtin_amdgcn_alignbyte(w[2], w[1], b),
                __builtin_amdgcn_alignbyte(w[3], w[2], b), __builtin_amdgcn_alignbyte(w[4], w[3], b)};
      break;
    case 1:
      r = u32x4{__builtin_amdgcn_alignbyte(w[2], w[1], b), __builtin_amdgcn_alignbyte(w[3], w[2], b),
                __builtin_amdgcn_alignbyte(w[4], w[3], b), __builtin_amdgcn_alignbyte(w[5], w[4], b)};
      break;
    case 2:
      r = u32x4{__builtin_amdgcn_alignbyte(w[3], w[2], b), __builtin_amdgcn_alignbyte(w[4], w[3], b),
                __builtin_amdgcn_alignbyte(w[5], w[4], b), __builtin_amdgcn_alignbyte(w[6], w[5], b)};
      break;
    default:
      r = u32x4{__builtin_amdgcn_alignbyte(w[4], w[3], b), __builtin_amdgcn_alignbyte(w[5], w[4], b),
                __builtin_amdgcn_alignbyte(w[6], w[5], b), __builtin_amdgcn_alignbyte(w[7], w[6], b)};
      break;
  }
  return r;
}

template <class Fn>
__global__ __launch_bounds__(kBlock) void kReduceShifted(KArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  acquirePeerData(a);
  const Fn fn(loadArg<Fn>(a));
  const uint64_t headBytes = (uint64_t)a.headElts * sizeof(E);
  const int nSrcs = a.nSrcs, nDsts = a.nDsts;
  const u32x4* base[kMaxKSrcs];
  uint32_t sh[kMaxKSrcs];
#pragma unroll
  for (int s = 0; s < kMaxKSrcs; s++) {
    const uintptr_t q = (uintptr_t)a.src[s < nSrcs ? s : 0] + headBytes;
    sh[s] = (uint32_t)(q & 15u);
    base[s] = (const u32x4*)(q - sh[s]);
  }
  u32x4* dst[kMaxKDsts];
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++) dst[d] = (u32x4*)((char*)a.dst[d] + headBytes);
  const bool doPost = Fn::kHasPost && a.postOp;
  const uint32_t preMask = a.preMask;
  const uint64_t n = a.nPacks;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p += stride) {
    u32x4 lo[kMaxKSrcs], hi[kMaxKSrcs];
#pragma unroll
    for (int s = 0; s < kMaxKSrcs; s++) {
      if (s < nSrcs) {   // plain (temporal) loads: the second one must find the line in L2
        lo[s] = base[s][p];
        hi[s] = sh[s] ? base[s][p + 1] : lo[s];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    u32x4 acc = funnel16(lo[0], hi[0], sh[0]);
    if constexpr (Fn::kHasPre) if (preMask & 1u) acc = fn.prePack(acc);
#pragma unroll
    for (int s = 1; s < kMaxKSrcs; s++) {
      if (s < nSrcs) {
        u32x4 t = funnel16(lo[s], hi[s], sh[s]);
        if constexpr (Fn::kHasPre) if ((preMask >> s) & 1u) t = fn.prePack(t);
        acc = fn.redPack(acc, t);
      }
    }
    if constexpr (Fn::kHasPost) if (doPost) acc = fn.postPack(acc);
    stPack(dst[0] + p, acc);
#pragma unroll
    for (int d = 1; d < kMaxKDsts; d++)
      if (d < nDsts) stPack(dst[d] + p, acc);
  }
  // head (before the destinations' 16-B boundary) and tail elements
  if (blockIdx.x == gridDim.x - 1) {
    const int head = a.headElts;
    const uint64_t tailStart = (uint64_t)head + n * EPP;
    const int tail = (int)(a.nElts - tailStart);
    const int t = (int)threadIdx.x;
    if (t < head) reduceElt(fn, a, nSrcs, (uint64_t)t);
    else if (t < head + tail) reduceElt(fn, a, nSrcs, tailStart + (uint64_t)(t - head));
  }
}

// Per-source-count realigning kernel: the sources go through LDS by LDS-DMA.
// A wave's tile is U x 64 output packs (destination side, 16-B aligned); it
// needs packs [p0, p0 + U*64] of each source's aligned-down base: U full
// global_load_lds_dwordx4 (nt; 64 lanes x 16 B straight into LDS, no VGPRs)
// plus one single-lane DMA for the extra pack, per source, into a stage
// buffer private to the wave. With kShiftLdsStages stages the wave issues
// tile j+1's DMA, waits (vmcnt) until tile j has landed, reads each output's
// 16 bytes back at byte offset 16 (q - p0) + sh (five dwords + a byte funnel
// shift), folds in source order and stores. No lane exchange, no second load
// of a pack, and several tiles in flight per wave at no register cost.
// Measured at 256 MiB per input (scripts/sweep_shift.hip,
// profiles/r2/sweep_shift_256MiB_r2f.txt): 95 % (8 sources) / 97 % (4) /
// 97 % (2) of the aligned kernel on the same buffers, against 81 / 86 / 88 %
// for the DPP / two-load register shapes it replaces. Memory safety: pack
// indices clamp to the last pack holding a byte of the source range (pack n
// when the source is shifted, n - 1 when it is not), so no load leaves it.
template <class Fn, int NSRC>
__global__ __launch_bounds__(kShiftLdsWaves * 64) void kReduceShiftedLds(KArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  constexpr int U = shiftLdsUnroll(NSRC), S = kShiftLdsStages, W = kShiftLdsWaves;
  constexpr int P = U * 64 + 1;   // packs per source per stage
  constexpr uint64_t kTile = (uint64_t)U * 64;
  __shared__ u32x4 sm[W][S][NSRC][P];
  acquirePeerData(a);
  const Fn fn(loadArg<Fn>(a));
  const uint64_t headBytes = (uint64_t)a.headElts * sizeof(E);
  const uint64_t n = a.nPacks;
  const u32x4* base[NSRC];
  uint32_t sh[NSRC];
  uint64_t lim[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; s++) {
    const uintptr_t q = (uintptr_t)a.src[s] + headBytes;
    sh[s] = (uint32_t)(q & 15u);
    base[s] = (const u32x4*)(q - sh[s]);
    lim[s] = sh[s] ? n : n - 1;
  }
  u32x4* dst[kMaxKDsts];
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++) dst[d] = (u32x4*)((char*)a.dst[d] + headBytes);
  const int nDsts = a.nDsts;
  const bool doPost = Fn::kHasPost && a.postOp;
  const uint32_t preMask = a.preMask;
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63u);
  const uint64_t nTiles = (n + kTile - 1) / kTile;
  const uint64_t nWaves = (uint64_t)gridDim.x * W, gw = (uint64_t)blockIdx.x * W + (uint64_t)wave;
  auto issue = [&](uint64_t t, int st) {
    const uint64_t p0 = t * kTile;
#pragma unroll
    for (int s = 0; s < NSRC; s++) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = p0 + (uint64_t)(u * 64 + lane);
        __builtin_amdgcn_global_load_lds((const void*)(base[s] + (q < lim[s] ? q : lim[s])),
                                         (__attribute__((address_space(3))) void*)&sm[wave][st][s][u * 64], 16, 0,
                                         2 /* nt */);
      }
      if (lane == 0) {
        const uint64_t q = p0 + kTile;
        __builtin_amdgcn_global_load_lds((const void*)(base[s] + (q < lim[s] ? q : lim[s])),
                                         (__attribute__((address_space(3))) void*)&sm[wave][st][s][kTile], 16, 0, 2);
      }
    }
  };
  // fold wave tile t from stage st (its DMA has landed) and store it
  auto foldTile = [&](uint64_t t, int st) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = t * kTile + (uint64_t)(u * 64 + lane);
      if (q < n) {
        u32x4 acc;
#pragma unroll
        for (int s = 0; s < NSRC; s++) {
          const uint32_t o = (uint32_t)(u * 64 + lane) * 16u + sh[s];
          const uint32_t* w = (const uint32_t*)&sm[wave][st][s][0] + (o >> 2);
          const uint32_t b = o & 3u;
          const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = b ? w[4] : 0u;
          u32x4 x = {__builtin_amdgcn_alignbyte(w1, w0, b), __builtin_amdgcn_alignbyte(w2, w1, b),
                     __builtin_amdgcn_alignbyte(w3, w2, b), __builtin_amdgcn_alignbyte(w4, w3, b)};
          if constexpr (Fn::kHasPre) if ((preMask >> s) & 1u) x = fn.prePack(x);
          if (s == 0) acc = x;
          else acc = fn.redPack(acc, x);
        }
        if constexpr (Fn::kHasPost) if (doPost) acc = fn.postPack(acc);
        stPack(dst[0] + q, acc);
#pragma unroll
        for (int d = 1; d < kMaxKDsts; d++)
          if (d < nDsts) stPack(dst[d] + q, acc);
      }
    }
    // this stage's LDS reads have returned before a later iteration refills it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  if (S != 2 || a.dynCtr == nullptr) {
    // static schedule: wave gw takes tiles gw, gw + nWaves, ...
#pragma unroll
    for (int k = 0; k < S - 1; k++) {
      const uint64_t t = gw + (uint64_t)k * nWaves;
      if (t < nTiles) issue(t, k);
    }
    int st = 0;
    for (uint64_t t = gw; t < nTiles; t += nWaves) {
      if (t + (uint64_t)(S - 1) * nWaves < nTiles) {
        issue(t + (uint64_t)(S - 1) * nWaves, (st + S - 1) % S);
        // everything but the newer tiles' DMA (NSRC x (U + 1) instructions each)
        // has landed; stores counted in vmcnt only make the wait stricter
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((S - 1) * NSRC * (U + 1)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      foldTile(t, st);
      st = st + 1 == S ? 0 : st + 1;
    }
  } else {
    // dynamic schedule (long eager launches): the wave tiles of class
    // x = t mod C go to the waves of class x = gw mod C; each wave runs its
    // first two tiles of the class statically (local indices l0 and l0 + gCls)
    // and takes every further one from the class counter, one fetch per tile
    // whose successor it runs, so the class's fetches number exactly
    // F = nCls - gCls and the one that returns F - 1 is the last: its wave
    // resets the counter to 0 for the next launch on this stream (no host
    // base). The fetch for tile k + 2 is issued before tile k + 1's DMA, so
    // the wait for tile k's DMA covers it and reading it never waits on
    // tile k + 1's DMA.
    constexpr uint64_t C = (uint64_t)kShiftDynClasses;
    const uint64_t x = gw % C;
    const uint64_t nCls = nTiles > x ? (nTiles - x + C - 1) / C : 0;
    const uint64_t gCls = nWaves > x ? (nWaves - x + C - 1) / C : 0;
    const uint64_t F = nCls > gCls ? nCls - gCls : 0;
    uint32_t* ctr = a.dynCtr + x * (uint64_t)kShiftDynStride;
    uint64_t lc = gw / C;
    if (lc < nCls) {
      uint64_t l1 = lc + gCls;
      int st = 0;
      issue(x + C * lc, 0);
      for (;;) {
        const bool more = l1 < nCls;
        uint32_t pend = 0;
        // the fetch as inline asm: the compiler would otherwise guard the
        // read of its result with a conservative vmcnt(0) — waiting for the
        // tile k + 1 DMA issued after it and undoing the two-stage pipeline;
        // the explicit vmcnt below covers it (it is older than that DMA)
        if (more && lane == 0)
          asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(pend) : "v"(ctr), "v"(1u) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        uint64_t l2 = nCls;
        if (more) {
          issue(x + C * l1, st ^ 1);
          // tile k's DMA and the fetch have landed (both older than tile k + 1's
          // DMA); `pend` as an operand keeps its read after the wait
          asm volatile("s_waitcnt vmcnt(%1)" : "+v"(pend) : "n"(NSRC * (U + 1)) : "memory");
          const uint32_t g = __builtin_amdgcn_readfirstlane(pend);
          if (lane == 0 && (uint64_t)g + 1 == F) atomicExch(ctr, 0u);
          l2 = (uint64_t)g + 2 * gCls;
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        foldTile(x + C * lc, st);
        st ^= 1;
        if (!more) break;
        lc = l1;
        l1 = l2;
      }
    }
  }
  // head (before the destination's 128-B boundary) and tail elements
  if (blockIdx.x == gridDim.x - 1) {
    const int head = a.headElts;
    const uint64_t tailStart = (uint64_t)head + n * EPP;
    const int tail = (int)(a.nElts - tailStart);
    const int th = (int)threadIdx.x;
    if (th < head) reduceElt(fn, a, NSRC, (uint64_t)th);
    else if (th < head + tail) reduceElt(fn, a, NSRC, tailStart + (uint64_t)(th - head));
  }
}

// ---------------------------------------------------------------------------
// Batched buckets (nbxReduceMultiBatch). The tiles of every bucket form one
// index space (bucket k owns the tiles between the previous record's tileEnd
// and its own); workgroups grid-stride over it, so a batch of small buckets
// fills the chip like one big bucket instead of one under-filled launch per
// bucket. A workgroup's tiles only move forward, so its record cursor only
// advances: a bucket's pointers are read (scalar loads from the
// kernel-argument segment) only when the cursor moves. The workgroup that
// owns a bucket's last tile also folds its < 16-B head and tail elements.
template <class Fn, int NSRC>
__device__ __forceinline__ void batchElt(const Fn& fn, const typename Fn::Elt* const (&src)[NSRC],
                                         typename Fn::Elt* const (&dst)[kMaxKDsts], int nDsts, uint32_t preMask,
                                         bool doPost, uint64_t i) {
  using E = typename Fn::Elt;
  E acc = src[0][i];
  if constexpr (Fn::kHasPre) if (preMask & 1u) acc = fn.pre(acc);
#pragma unroll
  for (int s = 1; s < NSRC; s++) {
    E v = src[s][i];
    if constexpr (Fn::kHasPre) if ((preMask >> s) & 1u) v = fn.pre(v);
    acc = fn.red(acc, v);
  }
  if constexpr (Fn::kHasPost) if (doPost) acc = fn.post(acc);
#pragma unroll
  for (int d = 0; d < kMaxKDsts; d++)
    if (d < nDsts) dst[d][i] = acc;
}

template <class Fn, int NSRC>
__global__ __launch_bounds__(kBlock) void kReduceBatch(BatchArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  if (a.acquireSystem) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const bool doPost = Fn::kHasPost && a.postOp;
  const uint32_t preMask = a.preMask;
  const uint64_t total = a.totalTiles;
  int off = 0, len = 0, nDsts = 1, head = 0;
  uint64_t tBegin = 0, tEnd = 0, nElts = 0, n = 0;
  const E* sb[NSRC];
  E* db[kMaxKDsts];
  const u32x4* src[NSRC];
  u32x4* dst[kMaxKDsts];
  for (uint64_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
    if (tile >= tEnd) {   // advance the bucket cursor (uniform across the workgroup)
      uint64_t meta;
      do {
        off += len;
        tBegin = tEnd;
        tEnd = a.w[off];
        meta = a.w[off + 1];
        nDsts = (int)(meta >> 60);
        len = 2 + NSRC + nDsts;
      } while (tile >= tEnd);
      nElts = meta & kBatchCountMask;
      head = (int)((meta >> 56) & 15u);
      n = (nElts - (uint64_t)head) / EPP;
#pragma unroll
      for (int s = 0; s < NSRC; s++) {
        sb[s] = (const E*)a.w[off + 2 + s];
        src[s] = (const u32x4*)(sb[s] + head);
      }
#pragma unroll
      for (int d = 0; d < kMaxKDsts; d++) {
        db[d] = (E*)a.w[off + 2 + NSRC + (d < nDsts ? d : 0)];
        dst[d] = (u32x4*)(db[d] + head);
      }
    }
    const uint64_t p = (tile - tBegin) * kBatchTilePacks + threadIdx.x;
    if (p < n) {
      u32x4 v[NSRC][1];
#pragma unroll
      for (int s = 0; s < NSRC; s++) v[s][0] = ldPack(src[s] + p);
      foldStore<Fn, NSRC, 1>(fn, v, preMask, doPost, dst, nDsts, p);
    }
    if (tile == tEnd - 1) {   // the bucket's last tile: its head and tail elements
      const uint64_t tailStart = (uint64_t)head + n * EPP;
      const int tail = (int)(nElts - tailStart);
      const int th = (int)threadIdx.x;
      if (th < head) batchElt<Fn, NSRC>(fn, sb, db, nDsts, preMask, doPost, (uint64_t)th);
      else if (th < head + tail)
        batchElt<Fn, NSRC>(fn, sb, db, nDsts, preMask, doPost, tailStart + (uint64_t)(th - head));
    }
  }
}

// Work-list batch (nbx_kargs.h BatchListArgs): the same per-tile work as
// kReduceBatch, records from a table in memory. Workgroups take chunks of
// `chunk` consecutive tiles round-robin over the tiles of every bucket; when a
// wave's tile leaves the current bucket it compares 64 running tile totals
// from the kernel arguments at once (one per lane) and takes the first lane
// whose total exceeds the tile (ballot) — the records are in tile order, so
// one step skips up to 64 buckets — then reads that record from the table.
// Every wave of the workgroup computes the same record independently (no LDS,
// no barrier).
template <class Fn, int NSRC>
__global__ __launch_bounds__(kBlock) void kReduceBatchList(BatchListArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPP = 16 / (int)sizeof(E);
  if (a.acquireSystem) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const Fn fn(a.argPtr != nullptr ? (uint64_t) * (const E*)a.argPtr : a.arg);
  const bool doPost = Fn::kHasPost && a.postOp;
  const uint32_t preMask = a.preMask;
  const uint64_t T = a.totalTiles, C = a.chunk, step = (uint64_t)gridDim.x * C;
  const int nRecs = a.nRecs, lane = (int)(threadIdx.x & 63u);
  int k = -1;
  uint64_t tBegin = 0, tEnd = 0, nElts = 0, n = 0;
  int nDsts = 1, head = 0;
  const E* sb[NSRC];
  E* db[kMaxKDsts];
  const u32x4* src[NSRC];
  u32x4* dst[kMaxKDsts];
  for (uint64_t c0 = (uint64_t)blockIdx.x * C; c0 < T; c0 += step) {
    const uint64_t c1 = c0 + C < T ? c0 + C : T;
    for (uint64_t tile = c0; tile < c1; tile++) {
      if (tile >= tEnd) {   // next bucket holding this tile (uniform per wave)
        for (int base = k + 1;; base += 64) {
          const int idx = base + lane;
          const uint64_t e = idx < nRecs ? (uint64_t)a.tileEnd[idx] : ~0ull;
          const uint64_t m = __ballot(e > tile);
          if (m != 0) {
            k = __builtin_amdgcn_readfirstlane(base + (int)__builtin_ctzll(m));
            break;
          }
        }
        const uint64_t* r = a.recs + (uint64_t)k * a.recWords;
        tBegin = r[0];
        tEnd = r[1];
        const uint64_t meta = r[2];
        nDsts = (int)(meta >> 60);
        nElts = meta & kBatchCountMask;
        head = (int)((meta >> 56) & 15u);
        n = (nElts - (uint64_t)head) / EPP;
#pragma unroll
        for (int s = 0; s < NSRC; s++) {
          sb[s] = (const E*)r[3 + s];
          src[s] = (const u32x4*)(sb[s] + head);
        }
#pragma unroll
        for (int d = 0; d < kMaxKDsts; d++) {
          db[d] = (E*)r[3 + NSRC + (d < nDsts ? d : 0)];
          dst[d] = (u32x4*)(db[d] + head);
        }
      }
      const uint64_t p = (tile - tBegin) * kBatchTilePacks + threadIdx.x;
      if (p < n) {
        u32x4 v[NSRC][1];
#pragma unroll
        for (int s = 0; s < NSRC; s++) v[s][0] = ldPack(src[s] + p);
        foldStore<Fn, NSRC, 1>(fn, v, preMask, doPost, dst, nDsts, p);
      }
      if (tile == tEnd - 1) {   // the bucket's last tile: its head and tail elements
        const uint64_t tailStart = (uint64_t)head + n * EPP;
        const int tail = (int)(nElts - tailStart);
        const int th = (int)threadIdx.x;
        if (th < head) batchElt<Fn, NSRC>(fn, sb, db, nDsts, preMask, doPost, (uint64_t)th);
        else if (th < head + tail)
          batchElt<Fn, NSRC>(fn, sb, db, nDsts, preMask, doPost, tailStart + (uint64_t)(th - head));
      }
    }
  }
}

}  // namespace nbx

#include "nbx_simple.h"   // uses ldPack / stPack above

namespace nbx {

// ---------------------------------------------------------------------------
// Launch table for one functor.



// Two tile shapes per source count. BIG keeps ~32 dwordx4 loads (512 B) in
// flight per lane and runs one 256-thread workgroup per CU (the best 8:1
// shape measured: 6.1-6.2 TB/s); SMALL (U = 1) gives small buckets enough
// workgroups to cover 256 CUs.
template <int NSRC, int CAP>
constexpr int bigUnroll() {
  constexpr int u = NSRC >= 5 ? 4 : (NSRC >= 3 ? 8 : 16);
  return u < CAP ? u : CAP;
}

// per-source-count realigning kernels (LDS-DMA staging)
template <class Fn, int NSRC>
inline const void* shiftedNFor() {
  return (const void*)&kReduceShiftedLds<Fn, NSRC>;
}

template <class Fn, int... I>
KernelSet makeKernelSetImpl(std::integer_sequence<int, I...>) {
  KernelSet ks{};
  const void* small[] = {(const void*)&kReducePacks<Fn, I + 1, 1>...};
  const void* big[] = {(const void*)&kReducePacks<Fn, I + 1, bigUnroll<I + 1, Fn::kUnrollCap>()>...};
  const void* batch[] = {(const void*)&kReduceBatch<Fn, I + 1>...};
  const void* batchList[] = {(const void*)&kReduceBatchList<Fn, I + 1>...};
  int un[] = {bigUnroll<I + 1, Fn::kUnrollCap>()...};
  for (int i = 0; i < kMaxKSrcs; i++) {
    ks.packs[0][i] = small[i];
    ks.packs[1][i] = big[i];
    ks.batch[i] = batch[i];
    ks.batchList[i] = batchList[i];
    ks.unroll[i] = un[i];
  }
  ks.elts = (const void*)&kReduceElts<Fn>;
  ks.shifted = (const void*)&kReduceShifted<Fn>;
  const void* sn[] = {shiftedNFor<Fn, I + 1>()...};
  for (int i = 0; i < kMaxKSrcs; i++) ks.shiftedN[i] = sn[i];
  ks.ll = (const void*)&kLLColl<Fn, false>;
  ks.ll128 = (const void*)&kLL128Coll<Fn, false>;
  ks.ll128x2 = (const void*)&kLL128AllReduce2<Fn, false>;
  ks.llChk = (const void*)&kLLColl<Fn, true>;
  ks.ll128Chk = (const void*)&kLL128Coll<Fn, true>;
  ks.ll128x2Chk = (const void*)&kLL128AllReduce2<Fn, true>;
  ks.simple = (const void*)&kSimpleColl<Fn, false>;
  ks.simpleRing = (const void*)&kSimpleRing<Fn, false>;
  ks.simpleChk = (const void*)&kSimpleColl<Fn, true>;
  ks.simpleRingChk = (const void*)&kSimpleRing<Fn, true>;
  ks.eltBytes = (int)sizeof(typename Fn::Elt);
  ks.bigBlocksPerCU = Fn::kBigBlocksPerCU;
  ks.valid = 1;
  return ks;
}

template <class Fn>
KernelSet makeKernelSet() {
  return makeKernelSetImpl<Fn>(std::make_integer_sequence<int, kMaxKSrcs>{});
}

}  // namespace nbx
