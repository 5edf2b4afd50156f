#include <hip/hip_runtime.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
struct Args { const f32x4* src[8]; f32x4* dst; uint64_t nPacks; };
template <int U>
__global__ __launch_bounds__(256) void kall(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p = blockIdx.x * tile + threadIdx.x; p < n; p += stride) {
    f32x4 v[8][U];
#pragma unroll
    for (int s = 0; s < 8; s++)
#pragma unroll
      for (int u = 0; u < U; u++) v[s][u] = __builtin_nontemporal_load(a.src[s] + p + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) {
      f32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < 8; s++) acc = acc + v[s][u];
      a.dst[p + u * 256] = acc;
    }
  }
}
extern "C" int sa_reduce8(void* dst, void* const* srcs, uint64_t n, void* stream) {
  Args a;
  for (int s = 0; s < 8; s++) a.src[s] = (const f32x4*)srcs[s];
  a.dst = (f32x4*)dst;
  a.nPacks = n / 4;
  void* args[] = {&a};
  return (int)hipLaunchKernel((const void*)&kall<4>, dim3(256), dim3(256), args, 0, (hipStream_t)stream);
}
