// nbx_registry.h — kernel table shared by the per-type instantiation units
// (inst_*.hip, compiled in parallel) and the host launcher (nbx_reduce.cc).
// Replaces the generated ncclDevFuncTable / ncclDevFuncId of the reference
// (/root/reference/src/device/generate.py:125-149, src/include/device.h:412-459):
// one KernelSet per (datatype, device op); signed integers share the
// unsigned kernels for Sum/Prod/MinMax/PreMulSum exactly as generate.py's
// equivalent_primary() maps them.
#pragma once
#include "nbx_kargs.h"

namespace nbx {
constexpr int kNumTypes = 12;   // ncclNumTypes (incl. fp8)
constexpr int kNumDevOps = 5;   // nbxNumDevRedOps
typedef KernelSet KernelTable[kNumTypes][kNumDevOps];

void fillInt8(KernelTable& t);
void fillInt32(KernelTable& t);
void fillInt64(KernelTable& t);
void fillF16(KernelTable& t);
void fillBF16(KernelTable& t);
void fillF32(KernelTable& t);
void fillF64(KernelTable& t);
void fillFp8(KernelTable& t);
}  // namespace nbx
