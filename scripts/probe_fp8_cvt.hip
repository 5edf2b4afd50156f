// probe_fp8_cvt.hip — compares gfx950's hardware fp32->fp8 converters
// (v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32) with the software RNE narrowing of
// nbx_functors.h (f32ToSmall) over ALL 2^32 fp32 bit patterns, and reports
// the mismatch classes. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../neuronabox-nccl_amd/csrc/nbx_functors.h"

using namespace nbx;

struct Res {
  unsigned long long mism[2];
  unsigned ex[2][32][3];
  unsigned long long cls[2][5];   // nan-in, inf-in, overflow, below-min-normal, normal range
  unsigned clsEx[2][5][3];
};
__device__ int classify(float x, float maxf, float minNormal) {
  float a = fabsf(x);
  if (x != x) return 0;
  if (a == INFINITY) return 1;
  if (a > maxf) return 2;
  if (a < minNormal) return 3;
  return 4;
}

__device__ bool isNanE4(uint32_t c) { return (c & 0x7f) == 0x7f; }
__device__ bool isNanE5(uint32_t c) { return (c & 0x7c) == 0x7c && (c & 3) != 0; }

__global__ void probe(Res* r, int clamp) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
       i += (uint64_t)gridDim.x * blockDim.x) {
    float x = __uint_as_float((uint32_t)i);
    uint32_t sw4 = f32ToSmall<4, 3, true>(x), sw5 = f32ToSmall<5, 2, false>(x);
    uint32_t hw4, hw5;
    if (clamp) {
      hw4 = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(x, -448.f), 448.f), 0.f, 0, false) & 0xff;
      hw5 = (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(x, 0.f, 0, false) & 0xff;
    } else {
      hw4 = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xff;
      hw5 = (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(x, 0.f, 0, false) & 0xff;
    }
    bool ok4 = (sw4 == hw4) || (isNanE4(sw4) && isNanE4(hw4));
    bool ok5 = (sw5 == hw5) || (isNanE5(sw5) && isNanE5(hw5));
    if (!ok4) {
      int c = classify(x, 448.f, 0.015625f);
      if (atomicAdd(&r->cls[0][c], 1ull) == 0) { r->clsEx[0][c][0] = (uint32_t)i; r->clsEx[0][c][1] = sw4; r->clsEx[0][c][2] = hw4; }
      unsigned long long k = atomicAdd(&r->mism[0], 1ull);
      if (k < 32) { r->ex[0][k][0] = (uint32_t)i; r->ex[0][k][1] = sw4; r->ex[0][k][2] = hw4; }
    }
    if (!ok5) {
      int c = classify(x, 57344.f, 6.103515625e-05f);
      if (atomicAdd(&r->cls[1][c], 1ull) == 0) { r->clsEx[1][c][0] = (uint32_t)i; r->clsEx[1][c][1] = sw5; r->clsEx[1][c][2] = hw5; }
      unsigned long long k = atomicAdd(&r->mism[1], 1ull);
      if (k < 32) { r->ex[1][k][0] = (uint32_t)i; r->ex[1][k][1] = sw5; r->ex[1][k][2] = hw5; }
    }
  }
}

int main() {
  Res* d;
  Res h;
  for (int clamp = 0; clamp < 2; clamp++) {
    if (hipMalloc(&d, sizeof(Res)) != hipSuccess) return 2;
    hipMemset(d, 0, sizeof(Res));
    probe<<<4096, 256>>>(d, clamp);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    hipMemcpy(&h, d, sizeof(Res), hipMemcpyDeviceToHost);
    for (int f = 0; f < 2; f++) {
      printf("clamp=%d %s mismatches: %llu\n", clamp, f ? "e5m2" : "e4m3", h.mism[f]);
      const char* names[5] = {"nan-in", "inf-in", "overflow", "below-min-normal", "normal"};
      for (int c = 0; c < 5; c++) {
        if (!h.cls[f][c]) continue;
        uint32_t u = h.clsEx[f][c][0];
        float x;
        memcpy(&x, &u, 4);
        printf("   class %-16s count %llu  e.g. x=%08x (%g) sw=%02x hw=%02x\n", names[c], h.cls[f][c], u, x,
               h.clsEx[f][c][1], h.clsEx[f][c][2]);
      }
      for (int k = 0; k < 8 && k < (int)h.mism[f]; k++) {
        uint32_t u = h.ex[f][k][0];
        float x;
        memcpy(&x, &u, 4);
        printf("   x=%08x (%g) sw=%02x hw=%02x\n", u, x, h.ex[f][k][1], h.ex[f][k][2]);
      }
    }
    hipFree(d);
  }
  return 0;
}
