// nbx_sync.h — host entry of the cross-process stream barrier (nbx_sync.hip).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace nbx {
hipError_t launchPeerBarrier(uint64_t* myFlags, uint64_t* const* peerFlagsDev, int n, int slot, uint64_t seq,
                             const int* abortWordDev, int* errWordDev, double timeoutSec, hipStream_t stream);
}  // namespace nbx
