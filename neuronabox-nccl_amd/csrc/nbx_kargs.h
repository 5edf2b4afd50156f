// nbx_kargs.h — kernel argument block and launch-table entry, shared by the
// device instantiation units and the host launcher (no device code here, so
// host .cc files compile as plain C++).
#pragma once
#include <stdint.h>

namespace nbx {

constexpr int kBlock = 256;      // workgroup = 4 wave64
constexpr int kMaxKSrcs = 8;     // sources per kernel pass
// realigning kernel (kReduceShiftedLds): waves per workgroup, packs per lane
// per tile (2 from 3 sources, else 1) and workgroups per CU (1 from 3 sources,
// else 2) — profiles/r2/sweep_shift_256MiB_r2f.txt
constexpr int kShiftLdsWaves = 4;
constexpr int kShiftLdsStages = 2;
constexpr int shiftLdsUnroll(int nSrcs) { return nSrcs >= 3 ? 2 : 1; }
constexpr int shiftLdsBlocksPerCU(int nSrcs) { return nSrcs >= 3 ? 1 : 2; }
// its dynamic schedule: wave tiles in kShiftDynClasses classes (t mod C), one
// counter per class kShiftDynStride words apart (KArgs.dynCtr -> the first)
constexpr int kShiftDynClasses = 32;
constexpr int kShiftDynStride = 64;
constexpr int kMaxKDsts = 8;     // destinations: NCCL_MAX_DIRECT_ARITY + 1 (device.h:147, all_reduce.h:343-360)

struct KArgs {
  const void* src[kMaxKSrcs];
  void* dst[kMaxKDsts];
  uint64_t nElts;     // total elements
  uint64_t nPacks;    // 16-B packs in the aligned body (starts at headElts)
  uint64_t arg;       // ncclDevRedOpFull.scalarArg (by value)
  const void* argPtr; // device scalar (ncclScalarDevice) or nullptr
  uint32_t preMask;   // bit s set: apply the PreMulSum pre-op to source s
  int32_t nSrcs;
  int32_t nDsts;
  int32_t postOp;
  int32_t headElts;   // elements before the 16-B aligned body
  int32_t variant;    // 0 = small tile (U = 1), 1 = big tile
  int32_t acquireSystem;  // 1: system-scope acquire at kernel start (sources include peer GPU memory)
  // dynamic tiles (dynCtr != nullptr): tiles past the first gridDim.x come
  // from a per-stream counter that every launch on that stream advances by
  // exactly its tile count; this launch's tiles are counter - dynBase
  uint32_t* dynCtr;
  uint32_t dynBase;
  int32_t pad;
};

// Batched reduce (nbxReduceMultiBatch): several independent buckets with the
// same functor and source count in one launch — the analogue of NCCL packing
// grouped collectives into one ncclWork (enqueue.cc:67-91 appendWorkElemColl,
// up to NCCL_MAX_WORK_ELEMENTS = 9 elements, device.h:230). Every bucket's
// pointers share one alignment modulo 16. The bucket table travels in the
// kernel-argument segment (4 KiB, read with scalar loads), packed with
// variable-length records so a launch holds 46 (8 sources) to 101 (2 sources)
// single-destination buckets:
//   w[o]          tileEnd: running total of tiles through this bucket
//   w[o+1]        nElts | headElts << 56 | nDsts << 60
//   w[o+2 ..]     NSRC source pointers, then nDsts destination pointers
constexpr int kBatchTilePacks = 256;   // one 16-B pack per lane per tile (kBlock lanes)
constexpr int kBatchHeaderBytes = 40;
constexpr int kBatchWords = (4096 - kBatchHeaderBytes) / 8;
constexpr uint64_t kBatchCountMask = (1ull << 56) - 1;
// up to this many buckets of one source count (fitting one table) use the
// kernel-argument form even when work lists are on (profiles/r2/batch_list_*)
constexpr int kBatchKernargMaxBuckets = 16;

struct BatchArgs {
  uint64_t arg;
  const void* argPtr;
  uint64_t totalTiles;
  uint32_t preMask;
  int32_t postOp;
  int32_t nTasks;
  int32_t acquireSystem;
  uint64_t w[kBatchWords];
};

// Work-list form of the batch (kReduceBatchList): the bucket records live in a
// table outside the kernel arguments (NCCL's work FIFO, enqueue.cc:759
// uploadWork / common.h:146-176), so one launch takes up to kListMaxRecs
// buckets (and a call any number, in as many launches). The host writes the
// table straight into uncached device memory through the large BAR (pinned
// host memory where the BAR is small). Records of recWords = 3 + nSrcs +
// (the launch's largest nDsts) words: tileBegin, tileEnd, count | head << 56 |
// nDsts << 60, the sources, the destinations — at most kBatchRecWords; sized
// to the launch because every record crosses PCIe (a 2-source bucket's is 48 B
// instead of 160 B). The records' running tile totals also
// travel in the kernel arguments (scalar-cache hits, fresh every launch):
// workgroups take chunks of `chunk` consecutive tiles round-robin (chunk 1 =
// grid stride, the whole GPU on one window of memory, as for one bucket), and
// a wave finds the record of a tile by comparing 64 tile totals at once
// (ballot), so skipping many small buckets costs one step, not one per record.
constexpr int kBatchRecWords = 20;
constexpr int kListMaxRecs = 384;
constexpr int kBatchListSlotBytes = kListMaxRecs * kBatchRecWords * 8;   // one table per slot

struct BatchListArgs {
  const uint64_t* recs;      // recWords words per bucket
  uint64_t totalTiles;
  uint64_t arg;
  const void* argPtr;
  uint32_t preMask;
  int32_t postOp;
  int32_t acquireSystem;
  int32_t nRecs;
  uint32_t chunk;            // consecutive tiles per workgroup turn
  uint32_t recWords;         // words per record: 3 + nSrcs + max nDsts of the launch
  uint32_t tileEnd[kListMaxRecs];   // running tile totals (recs[k][1]); totals < 2^32
};

// Launch table for one functor (kernel entry points as host handles).

struct KernelSet {
  const void* packs[2][kMaxKSrcs];  // [0 = small tile, 1 = big tile][nSrcs-1]
  const void* elts;
  const void* shifted;              // sources realigned against 16-B aligned destinations (kReduceShifted, run-time source count; fallback)
  const void* shiftedN[kMaxKSrcs];   // the same per source count, [nSrcs-1] (kReduceShiftedLds: LDS-DMA staging)
  const void* ll;                   // LL-protocol collectives (nbx_ll.h)
  const void* ll128;                // LL128-protocol collectives (nbx_ll.h)
  const void* ll128x2;              // LL128 two-shot AllReduce (nbx_ll.h)
  const void* llChk;                // the same three with plan words (NBX_CHECK_PLANS)
  const void* ll128Chk;
  const void* ll128x2Chk;
  const void* simple;               // Simple protocol, direct schedule over init-mapped staging (nbx_simple.h)
  const void* simpleRing;           // Simple protocol, ring schedule over init-mapped staging (nbx_simple.h)
  const void* simpleChk;            // the same two with slice checksums (NBX_CHECK_SLICES)
  const void* simpleRingChk;
  const void* batch[kMaxKSrcs];     // batched buckets (kReduceBatch), [nSrcs-1]
  const void* batchList[kMaxKSrcs]; // batched buckets from a work-list table (kReduceBatchList), [nSrcs-1]
  int unroll[kMaxKSrcs];            // big-tile packs per lane per source
  int bigBlocksPerCU;               // Fn::kBigBlocksPerCU (at least this many big-tile workgroups per CU)
  int eltBytes;
  int valid;
};

}  // namespace nbx
