#include "nbx_registry.h"
#include "nbx_kernels.h"
#include "inst_float.inc"
namespace nbx { NBX_FILL_FLOAT(fillF64, TyF64, 8) }
