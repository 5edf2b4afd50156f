#include "nbx_registry.h"
#include "nbx_kernels.h"
#include "inst_int.inc"
namespace nbx { NBX_FILL_INT(fillInt32, uint32_t, int32_t, 2, 3) }
