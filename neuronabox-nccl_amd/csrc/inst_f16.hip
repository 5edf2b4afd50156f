#include "nbx_registry.h"
#include "nbx_kernels.h"
#include "inst_float.inc"
namespace nbx { NBX_FILL_FLOAT(fillF16, TyF16, 6) }
