// probe_fp8_sat.hip — saturating fp32 -> fp8 narrowing on gfx950 over ALL 2^32
// fp32 bit patterns, against the software specification "SATFINITE" (HIP's
// amd_hip_fp8.h __HIP_SATFINITE, what RCCL's fp8 functors narrow with): a
// finite value beyond the largest finite code becomes that code with its sign,
// +-inf and NaN propagate (e5m2 inf, e4m3fn NaN), everything else is the RNE
// narrowing of f32ToSmall. Candidates: 0 = v_cvt_scalef32_pk_{fp8,bf8}_f32 at
// scale 1.0; 1 = HIP's form (fmed3 clamp unless the exponent is all ones, then
// v_cvt_pk_*); 2 = an unguarded fmed3 clamp, then v_cvt_pk_*; 3 = this
// build's TyE4M3::narrow / TyE5M2::narrow (satE4M3 / satE5M2, nbx_functors.h);
// 4 = its pair path, TyE*::narrow2 (satFinite2: packed fma), x in the high byte;
// 5 = v_cvt_pk_{fp8,bf8}_f32 with the VOP3 clamp bit (bit 15) set, hand-encoded:
// the assembler rejects `clamp` on these opcodes (VERDICT r5 item 5 asks whether
// the hardware honours it as SATFINITE anyway).
// The specification is nbx_functors.h f32ToSmallSat. Mismatch classes as
// probe_fp8_cvt.hip. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../neuronabox-nccl_amd/csrc/nbx_functors.h"

using namespace nbx;
typedef short v2i16 __attribute__((ext_vector_type(2)));

struct Res {
  unsigned long long mism[2];
  unsigned long long cls[2][6];   // nan-in, inf-in, overflow, f32-denormal, below-min-normal, normal range
  unsigned clsEx[2][6][3];
};
__device__ int classify(float x, float maxf, float minNormal) {
  const float a = fabsf(x);
  if (x != x) return 0;
  if (a == INFINITY) return 1;
  if (a > maxf) return 2;
  if (a != 0.f && a < 1.17549435e-38f) return 3;
  if (a < minNormal) return 4;
  return 5;
}
__device__ bool isNanE4(uint32_t c) { return (c & 0x7f) == 0x7f; }
__device__ bool isNanE5(uint32_t c) { return (c & 0x7c) == 0x7c && (c & 3) != 0; }

__global__ void probe(Res* r, int mode) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32);
       i += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)i);
    const uint32_t sw4 = f32ToSmallSat<4, 3, true>(x), sw5 = f32ToSmallSat<5, 2, false>(x);
    uint32_t hw4, hw5;
    if (mode == 0) {
      const v2i16 z = {0, 0};
      hw4 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(z, x, 0.f, 1.0f, false)) & 0xff;
      hw5 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf8_f32(z, x, 0.f, 1.0f, false)) & 0xff;
    } else if (mode == 1) {
      const bool fin = (__float_as_uint(x) & 0x7f800000u) != 0x7f800000u;
      const float c4 = fin ? __builtin_amdgcn_fmed3f(x, 448.f, -448.f) : x;
      const float c5 = fin ? __builtin_amdgcn_fmed3f(x, 57344.f, -57344.f) : x;
      hw4 = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c4, 0.f, 0, false) & 0xff;
      hw5 = (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(c5, 0.f, 0, false) & 0xff;
    } else if (mode == 3) {
      hw4 = TyE4M3::narrow(x);
      hw5 = TyE5M2::narrow(x);
    } else if (mode == 4) {   // the pair path (narrow2: packed fma), x in the high byte of the word
      hw4 = (TyE4M3::narrow2(1.0f, x, 0u, true) >> 24) & 0xff;
      hw5 = (TyE5M2::narrow2(1.0f, x, 0u, true) >> 24) & 0xff;
    } else if (mode == 5) {
      // v1 = x, v2 = 0; v_cvt_pk_fp8_f32 v1, v1, v2 clamp (0xd2a28001 0x00020501), then bf8 (0xd2a3....)
      uint32_t r4, r5;
      asm volatile(
          "v_mov_b32 v1, %2\n\tv_mov_b32 v2, 0\n\ts_nop 1\n\t.long 0xd2a28001, 0x00020501\n\ts_nop 1\n\t"
          "v_mov_b32 %0, v1\n\tv_mov_b32 v1, %2\n\ts_nop 1\n\t.long 0xd2a38001, 0x00020501\n\ts_nop 1\n\t"
          "v_mov_b32 %1, v1"
          : "=&v"(r4), "=&v"(r5)
          : "v"(x)
          : "v1", "v2");
      hw4 = r4 & 0xff;
      hw5 = r5 & 0xff;
    } else {
      hw4 = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(x, 448.f, -448.f), 0.f, 0, false) & 0xff;
      hw5 = (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(__builtin_amdgcn_fmed3f(x, 57344.f, -57344.f), 0.f, 0, false) &
            0xff;
    }
    const bool ok4 = (sw4 == hw4) || (isNanE4(sw4) && isNanE4(hw4));
    const bool ok5 = (sw5 == hw5) || (isNanE5(sw5) && isNanE5(hw5));
    if (!ok4) {
      const int c = classify(x, 448.f, 0.015625f);
      if (atomicAdd(&r->cls[0][c], 1ull) == 0) { r->clsEx[0][c][0] = (uint32_t)i; r->clsEx[0][c][1] = sw4; r->clsEx[0][c][2] = hw4; }
      atomicAdd(&r->mism[0], 1ull);
    }
    if (!ok5) {
      const int c = classify(x, 57344.f, 6.103515625e-05f);
      if (atomicAdd(&r->cls[1][c], 1ull) == 0) { r->clsEx[1][c][0] = (uint32_t)i; r->clsEx[1][c][1] = sw5; r->clsEx[1][c][2] = hw5; }
      atomicAdd(&r->mism[1], 1ull);
    }
  }
}

int main() {
  Res* d;
  Res h;
  const char* modes[6] = {"scalef32 scale 1.0", "HIP SATFINITE form (guarded fmed3)", "unguarded fmed3",
                          "this build (satE4M3 / satE5M2 + v_cvt_pk)",
                          "this build, pair path (narrow2: fmed3 x2 + v_pk_fma_f32)",
                          "v_cvt_pk with the VOP3 clamp bit (hand-encoded)"};
  const char* names[6] = {"nan-in", "inf-in", "overflow", "f32-denormal", "below-min-normal", "normal"};
  for (int mode = 0; mode < 6; mode++) {
    if (hipMalloc(&d, sizeof(Res)) != hipSuccess) return 2;
    if (hipMemset(d, 0, sizeof(Res)) != hipSuccess) return 2;
    probe<<<4096, 256>>>(d, mode);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    if (hipMemcpy(&h, d, sizeof(Res), hipMemcpyDeviceToHost) != hipSuccess) return 4;
    for (int f = 0; f < 2; f++) {
      printf("%s %s mismatches vs SATFINITE: %llu\n", modes[mode], f ? "e5m2" : "e4m3", h.mism[f]);
      for (int c = 0; c < 6; c++) {
        if (!h.cls[f][c]) continue;
        uint32_t u = h.clsEx[f][c][0];
        float x;
        memcpy(&x, &u, 4);
        printf("   class %-16s count %llu  e.g. x=%08x (%g) spec=%02x hw=%02x\n", names[c], h.cls[f][c], u, x,
               h.clsEx[f][c][1], h.clsEx[f][c][2]);
      }
    }
    (void)hipFree(d);
  }
  return 0;
}
