// nbx_sync.h — host entry of the cross-process stream barrier (nbx_sync.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nbx {
// Advance this rank's epoch of `slot` (epochsDev: device counters, one per
// slot) to v, post v to flag `slot`; wait until every rank in `waitMask`
// (bit j = rank j) has flag `slot` >= v.
hipError_t launchPeerBarrier(uint64_t* myFlags, uint64_t* const* peerFlagsDev, int n, int slot, uint64_t waitMask,
                             uint64_t* epochsDev, const int* abortWordDev, int* errWordDev, double timeoutSec,
                             hipStream_t stream);
}  // namespace nbx
