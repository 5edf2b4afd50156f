// nbx_ll_args.h — kernel arguments of the LL-protocol AllReduce (nbx_ll.h);
// device-free so host units can fill them.
#pragma once
#include <stdint.h>

namespace nbx {

struct LLArgs {
  const void* send;
  void* recv;
  uint64_t count;          // elements
  uint64_t nPacks;         // 8-byte packs covering count elements
  uint64_t* const* peerLL; // device table: rank -> LL buffer base
  uint64_t* myLL;
  uint64_t slotLines;      // lines per (parity, source) slot = 2 * max packs
  uint64_t blockElts;      // direct-schedule block size (elements) -> fold order
  uint64_t arg;            // functor scalar (by value)
  const void* argPtr;      // device scalar or nullptr
  const volatile int* abortWord;
  volatile int* errWord;
  uint64_t timeoutTicks;
  uint32_t flag;
  int32_t parity;
  int32_t rank;
  int32_t nRanks;
  int32_t postOp;
};

}  // namespace nbx
