// nbx_internal.h — library-internal entry points shared between host units.
#pragma once
#include <hip/hip_runtime_api.h>

#include "../../include/nbx_reduce.h"

namespace nbx {
struct LLArgs;
// Launch the LL-protocol AllReduce kernel of (datatype, op) (nbx_ll.h).
ncclResult_t launchLLAllReduce(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, hipStream_t stream);
}  // namespace nbx
