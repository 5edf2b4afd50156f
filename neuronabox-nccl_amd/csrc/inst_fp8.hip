#include "nbx_registry.h"
#include "nbx_kernels.h"
namespace nbx {
// fp8 (OCP e4m3fn = 10, e5m2 = 11): this build's extension, no reference functor.
void fillFp8(KernelTable& t) {
  t[10][0] = makeKernelSet<FnSumF8<TyE4M3>>();
  t[10][1] = makeKernelSet<FnProdF8<TyE4M3>>();
  t[10][2] = makeKernelSet<FnMinMaxF<TyE4M3>>();
  t[10][3] = makeKernelSet<FnPreMulSumF8<TyE4M3>>();
  t[11][0] = makeKernelSet<FnSumF8<TyE5M2>>();
  t[11][1] = makeKernelSet<FnProdF8<TyE5M2>>();
  t[11][2] = makeKernelSet<FnMinMaxF<TyE5M2>>();
  t[11][3] = makeKernelSet<FnPreMulSumF8<TyE5M2>>();
}
}  // namespace nbx
