// nbx_internal.h — library-internal entry points shared between host units.
#pragma once
#include <hip/hip_runtime_api.h>

#include "../../include/nbx_reduce.h"

namespace nbx {
struct LLArgs;
// Launch the LL collective kernel of (datatype, op) (nbx_ll.h); sequencing is
// device-resident (args.state).
ncclResult_t launchLLColl(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, hipStream_t stream);
// The same for the LL128 kernel (args.nLines 64-byte lines).
ncclResult_t launchLL128Coll(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, hipStream_t stream);
// LL128 two-shot AllReduce (args.nLines = sub-slot lines; blockLines sizes the grid).
ncclResult_t launchLL128AllReduce2(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, uint64_t blockLines,
                                   hipStream_t stream);
}  // namespace nbx
