// nbx_internal.h — library-internal entry points shared between host units.
#pragma once
#include <hip/hip_runtime_api.h>

#include "../../include/nbx_reduce.h"

namespace nbx {
struct LLArgs;
// Launch the LL collective kernel of (datatype, op) (nbx_ll.h); sets args.arriveTarget from *arrived and
// advances it by the grid size.
ncclResult_t launchLLColl(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, uint64_t* arrived,
                          hipStream_t stream);
// The same for the LL128 kernel (args.nLines lines of 128 bytes).
ncclResult_t launchLL128Coll(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, uint64_t* arrived,
                             hipStream_t stream);
}  // namespace nbx
