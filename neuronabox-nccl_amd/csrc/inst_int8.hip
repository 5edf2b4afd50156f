#include "nbx_registry.h"
#include "nbx_kernels.h"
#include "inst_int.inc"
namespace nbx { NBX_FILL_INT(fillInt8, uint8_t, int8_t, 0, 1) }
