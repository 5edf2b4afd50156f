// nbx_kargs.h — kernel argument block and launch-table entry, shared by the
// device instantiation units and the host launcher (no device code here, so
// host .cc files compile as plain C++).
#pragma once
#include <stdint.h>

namespace nbx {

constexpr int kBlock = 256;      // workgroup = 4 wave64
constexpr int kMaxKSrcs = 8;     // sources per kernel pass
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
};

// Launch table for one functor (kernel entry points as host handles).

struct KernelSet {
  const void* packs[2][kMaxKSrcs];  // [0 = small tile, 1 = big tile][nSrcs-1]
  const void* elts;
  const void* ll;                   // LL-protocol collectives (nbx_ll.h)
  const void* ll128;                // LL128-protocol collectives (nbx_ll.h)
  const void* ll128x2;              // LL128 two-shot AllReduce (nbx_ll.h)
  int unroll[kMaxKSrcs];            // big-tile packs per lane per source
  int eltBytes;
  int valid;
};

}  // namespace nbx
