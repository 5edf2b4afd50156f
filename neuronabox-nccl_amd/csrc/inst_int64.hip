#include "nbx_registry.h"
#include "nbx_kernels.h"
#include "inst_int.inc"
namespace nbx { NBX_FILL_INT(fillInt64, uint64_t, int64_t, 4, 5) }
