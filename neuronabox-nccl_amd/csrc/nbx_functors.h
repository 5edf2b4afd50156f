// nbx_functors.h — per-element reduction functors for gfx950 (CDNA4).
//
// MI355X-native restatement of the reference functors
//   FuncSum / FuncProd / FuncMinMax     /root/reference/src/device/reduce_kernel.h:34-49, 147-170
//   half/bf16 specialisations           reduce_kernel.h:236-269
//   FuncPreMulSum (+ Apply_PreOp)       reduce_kernel.h:360-484
//   FuncSumPostDiv (+ Apply_PostOp)     reduce_kernel.h:489-526
// The reference expresses them as recursive BytePack templates over PTX; here
// a functor works on one 16-byte pack held in a u32x4 (one dwordx4 per lane,
// 1 KiB per wave64 instruction) and on single elements for tails.
//
// Numerics (each is bit-identical to the reference's float round trip,
// because fp32 carries p = 24 >= 2p+2 bits for f16/bf16/fp8 — double rounding
// is innocuous and every op is correctly rounded):
//   f16  : native v_add_f16 / v_mul_f16 (RNE), packed by the compiler.
//   bf16 : widen (shift), fp32 op, v_cvt_pk_bf16_f32 (RNE, NaN stays NaN).
//   fp8  : v_cvt_pk_f32_{fp8,bf8} widen, fp32 op, saturate, v_cvt_pk_{fp8,bf8}_f32
//          narrow (RNE). Saturation is HIP's __HIP_SATFINITE (amd_hip_fp8.h),
//          what RCCL's fp8 functors narrow with: a finite result beyond the
//          largest finite code becomes that code with its sign; inf and NaN
//          go through (e5m2 inf; e4m3fn, which has none, NaN) — two
//          instructions per element (satFinite), 1.5 for a converter's pair
//          (satFinite2). The converter
//          alone was checked equal to f32ToSmall on all 2^32 fp32 inputs
//          (scripts/probe_fp8_cvt.hip, profiles/r1/probe_fp8_cvt.txt), the
//          saturated form to f32ToSmallSat (scripts/probe_fp8_sat.hip,
//          profiles/r5/probe_fp8_sat_r5t.txt), and the one-rank PreMulSum to
//          RCCL 2.26's on every code (tests/test_rccl_corroboration_gpu.py).
//          Not in the reference (NCCL 2.19 has no fp8): this build's
//          definition, aligned with the NCCL lineage's AMD port.
//   f32/f64 : native IEEE ops; denormals preserved (.amdhsa_float_denorm_mode 3);
//          build with -ffp-contract=off so x*s + acc is never fused.
//   min/max (floats): NaN operand yields the other operand, ties return the
//          second operand — the oracle's pinned fminf/fmaxf rule.
//   integers: signed Sum/Prod/PreMulSum/MinMax run on the unsigned pattern
//          (/root/reference/src/device/generate.py:125-133).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nbx {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

template <class E>
union PackU {
  u32x4 v;
  E e[16 / sizeof(E)];
};

// -------------------------------------------------------------------------
// Element-type traits: storage Elt, compute type C, widen / narrow.

struct TyF32 {
  using Elt = uint32_t; using C = float;
  __device__ static C wide(Elt e) { return __uint_as_float(e); }
  __device__ static Elt narrow(C c) { return __float_as_uint(c); }
};
struct TyF64 {
  using Elt = uint64_t; using C = double;
  __device__ static C wide(Elt e) { return __longlong_as_double((long long)e); }
  __device__ static Elt narrow(C c) { return (Elt)__double_as_longlong(c); }
};
struct TyF16 {
  using Elt = uint16_t; using C = _Float16;
  __device__ static C wide(Elt e) { return __builtin_bit_cast(_Float16, e); }
  __device__ static Elt narrow(C c) { return __builtin_bit_cast(uint16_t, c); }
};
struct TyBF16 {
  using Elt = uint16_t; using C = float;
  __device__ static C wide(Elt e) { return __uint_as_float((uint32_t)e << 16); }
  __device__ static Elt narrow(C c) { return __builtin_bit_cast(uint16_t, (__bf16)c); }
};

// fp8 narrowing, specification form: OCP e4m3fn / e5m2, round-to-nearest-even,
// overflow -> NaN (e4m3fn, which has no infinity) / -> +-inf (e5m2) — the
// hardware converter's behaviour, which equals this function bit for bit (up
// to the NaN code) on every fp32 input. Kernels narrow with SATFINITE first
// (f32ToSmallSat below, satE4M3 / satE5M2 above the types).
template <int E, int M, bool FN>
__device__ __forceinline__ uint32_t f32ToSmall(float x) {
  const uint32_t u = __float_as_uint(x);
  const uint32_t sign = (u >> 31) << (E + M);
  const uint32_t a = u & 0x7fffffffu;
  constexpr uint32_t expAllOnes = ((1u << E) - 1u) << M;
  constexpr uint32_t nanCode = FN ? (expAllOnes | ((1u << M) - 1u)) : (expAllOnes | (1u << (M - 1)));
  constexpr uint32_t infCode = expAllOnes;
  constexpr uint32_t maxFinite = FN ? (expAllOnes | ((1u << M) - 2u))
                                    : ((expAllOnes - (1u << M)) | ((1u << M) - 1u));
  constexpr int bias = (1 << (E - 1)) - 1;
  constexpr int emin = 1 - bias;
  const int e = (int)(a >> 23) - 127;
  const int et = e < emin ? emin : e;
  int shift = (23 - M) + (et - e);
  shift = shift > 31 ? 31 : shift;
  const uint32_t mant = (a & 0x7fffffu) | 0x800000u;
  uint32_t q = mant >> shift;
  const uint32_t rem = mant & ((1u << shift) - 1u);
  const uint32_t half = 1u << (shift - 1);
  q += (rem > half || (rem == half && (q & 1u))) ? 1u : 0u;
  uint32_t enc = (uint32_t)((et + bias - 1) << M) + q;
  enc = enc > maxFinite ? (FN ? nanCode : infCode) : enc;
  enc = (a >> 23) == 0 ? 0u : enc;                       // fp32 zero/denormal -> 0
  enc = a >= 0x7f800000u ? (a == 0x7f800000u && !FN ? infCode : nanCode) : enc;
  return sign | enc;
}
// ... with SATFINITE (the kernels' narrowing): a finite x beyond the largest
// finite value becomes the largest finite code with x's sign.
template <int E, int M, bool FN>
__device__ __forceinline__ uint32_t f32ToSmallSat(float x) {
  constexpr uint32_t expAllOnes = ((1u << E) - 1u) << M;
  constexpr uint32_t maxFinite = FN ? (expAllOnes | ((1u << M) - 2u))
                                    : ((expAllOnes - (1u << M)) | ((1u << M) - 1u));
  constexpr float maxf = FN ? 448.0f : 57344.0f;
  static_assert(E + M == 7 && (FN ? E == 4 : E == 5), "OCP e4m3fn / e5m2 only");
  const uint32_t u = __float_as_uint(x);
  if ((u & 0x7f800000u) != 0x7f800000u && __builtin_fabsf(x) > maxf) return ((u >> 31) << 7) | maxFinite;
  return f32ToSmall<E, M, FN>(x);
}

// SATFINITE before the converter, two instructions for either format: an
// fmed3 clamp to +-max, then fma(x, 2^-149, clamp). For a finite x the
// added x * 2^-149 is below half an ulp of the clamp (|x| < 2^128), so the
// fma returns the clamp exactly; for +-inf it returns +-inf (the clamp has
// x's sign) and for NaN NaN — the converter then narrows those as HIP's
// SATFINITE does (e5m2 inf, e4m3fn NaN). Needs f32 denormals kept (2^-149 is
// one), as every kernel here is built (.amdhsa_float_denorm_mode_32 3).
// Exhaustively equal to f32ToSmallSat (scripts/probe_fp8_sat.hip).
template <int MAXV>
__device__ __forceinline__ float satFinite(float x) {
  return __builtin_fmaf(x, 0x1p-149f, __builtin_amdgcn_fmed3f(x, (float)MAXV, -(float)MAXV));
}
__device__ __forceinline__ float satE4M3(float x) { return satFinite<448>(x); }
__device__ __forceinline__ float satE5M2(float x) { return satFinite<57344>(x); }
// the same for a pair about to share one converter: two clamps, one packed
// fma (v_pk_fma_f32) — 1.5 instructions per element
template <int MAXV>
__device__ __forceinline__ f32x2 satFinite2(float x, float y) {
  const f32x2 c = {__builtin_amdgcn_fmed3f(x, (float)MAXV, -(float)MAXV),
                   __builtin_amdgcn_fmed3f(y, (float)MAXV, -(float)MAXV)};
  const f32x2 v = {x, y};
  const f32x2 e = {0x1p-149f, 0x1p-149f};
  return __builtin_elementwise_fma(v, e, c);
}

struct TyE4M3 {
  using Elt = uint8_t; using C = float;
  __device__ static C wide(Elt e) { return __builtin_amdgcn_cvt_pk_f32_fp8((int)e, false)[0]; }
  __device__ static Elt narrow(C c) {
    const float s = satE4M3(c);
    return (Elt)(__builtin_amdgcn_cvt_pk_fp8_f32(s, s, 0, false) & 0xff);
  }
  // two results into bytes {0,1} (hi = false) or {2,3} (hi = true) of `old`
  __device__ static uint32_t narrow2(float x, float y, uint32_t old, bool hi) {
    const f32x2 s = satFinite2<448>(x, y);
    return hi ? (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(s[0], s[1], (int)old, true)
              : (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(s[0], s[1], (int)old, false);
  }
  // 4 codes in a dword <-> 4 floats
  __device__ static void wide4(uint32_t w, float (&f)[4]) {
    auto lo = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, false);
    auto hi = __builtin_amdgcn_cvt_pk_f32_fp8((int)w, true);
    f[0] = lo[0]; f[1] = lo[1]; f[2] = hi[0]; f[3] = hi[1];
  }
};
struct TyE5M2 {
  using Elt = uint8_t; using C = float;
  __device__ static C wide(Elt e) { return __builtin_amdgcn_cvt_pk_f32_bf8((int)e, false)[0]; }
  __device__ static Elt narrow(C c) {
    const float s = satE5M2(c);
    return (Elt)(__builtin_amdgcn_cvt_pk_bf8_f32(s, s, 0, false) & 0xff);
  }
  __device__ static uint32_t narrow2(float x, float y, uint32_t old, bool hi) {
    const f32x2 s = satFinite2<57344>(x, y);
    x = s[0];
    y = s[1];
    return hi ? (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(x, y, (int)old, true)
              : (uint32_t)__builtin_amdgcn_cvt_pk_bf8_f32(x, y, (int)old, false);
  }
  __device__ static void wide4(uint32_t w, float (&f)[4]) {
    auto lo = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, false);
    auto hi = __builtin_amdgcn_cvt_pk_f32_bf8((int)w, true);
    f[0] = lo[0]; f[1] = lo[1]; f[2] = hi[0]; f[3] = hi[1];
  }
};

template <class C>
__device__ __forceinline__ bool isNan(C x) { return x != x; }

// -------------------------------------------------------------------------
// Generic pack helpers built from an element functor.

template <class Fn>
__device__ __forceinline__ u32x4 packRed(const Fn& fn, u32x4 a, u32x4 b) {
  using E = typename Fn::Elt;
  PackU<E> x, y;
  x.v = a; y.v = b;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(E)); i++) x.e[i] = fn.red(x.e[i], y.e[i]);
  return x.v;
}
template <class Fn>
__device__ __forceinline__ u32x4 packPre(const Fn& fn, u32x4 a) {
  using E = typename Fn::Elt;
  PackU<E> x;
  x.v = a;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(E)); i++) x.e[i] = fn.pre(x.e[i]);
  return x.v;
}
template <class Fn>
__device__ __forceinline__ u32x4 packPost(const Fn& fn, u32x4 a) {
  using E = typename Fn::Elt;
  PackU<E> x;
  x.v = a;
#pragma unroll
  for (int i = 0; i < (int)(16 / sizeof(E)); i++) x.e[i] = fn.post(x.e[i]);
  return x.v;
}

// Base: identity pre/post, generic pack ops. Derived functors override.
template <class D, class E>
struct FnBase {
  using Elt = E;
  static constexpr bool kHasPre = false;
  static constexpr bool kHasPost = false;
  // cap on the big-tile unroll: VALU-heavy functors gain nothing from more
  // loads in flight and only grow code size
  static constexpr int kUnrollCap = 16;
  // big-tile workgroups per CU (at least): VALU-heavy functors run more, so
  // another wave per SIMD has its loads in flight while one folds — float
  // min/max two, fp8 four (profiles/r2/probe_dtypes_r3f.jsonl; fp8 e4m3 sum
  // 5.75 / 5.80 / 5.84 TB/s at 2 / 3 / 4, ab_blocks_per_cu_r4i.jsonl)
  static constexpr int kBigBlocksPerCU = 1;
  __device__ E pre(E a) const { return a; }
  __device__ E post(E a) const { return a; }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const { return packRed(*static_cast<const D*>(this), a, b); }
  __device__ u32x4 prePack(u32x4 a) const { return packPre(*static_cast<const D*>(this), a); }
  __device__ u32x4 postPack(u32x4 a) const { return packPost(*static_cast<const D*>(this), a); }
};

// -------------------------------------------------------------------------
// Integer functors (E = uint8_t / uint32_t / uint64_t storage; signed types
// share them, generate.py:125-133).

template <class E>
struct FnSumInt : FnBase<FnSumInt<E>, E> {
  __device__ explicit FnSumInt(uint64_t) {}
  __device__ E red(E a, E b) const { return (E)(a + b); }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    if constexpr (sizeof(E) == 1) {
      // bytewise modular add: carries stopped at byte boundaries (SWAR,
      // same result as reduce_kernel.h:173-183)
      const u32x4 lo7 = (u32x4)(0x7f7f7f7fu);
      const u32x4 hi1 = (u32x4)(0x80808080u);
      return ((a & lo7) + (b & lo7)) ^ ((a ^ b) & hi1);
    } else if constexpr (sizeof(E) == 4) {
      return a + b;
    } else {
      return packRed(*this, a, b);
    }
  }
};

template <class E>
struct FnProdInt : FnBase<FnProdInt<E>, E> {
  static constexpr int kUnrollCap = sizeof(E) == 1 ? 4 : 16;
  __device__ explicit FnProdInt(uint64_t) {}
  __device__ E red(E a, E b) const { return (E)(a * b); }
};

template <class E>
struct FnMinMaxInt : FnBase<FnMinMaxInt<E>, E> {
  static constexpr int kUnrollCap = sizeof(E) == 1 ? 4 : 16;
  // bytes: a second workgroup per CU hides the SWAR fold (u8 min 5.61 -> 5.92
  // TB/s, profiles/r5/ab_swar8_shared_out_r5k.jsonl)
  static constexpr int kBigBlocksPerCU = sizeof(E) == 1 ? 2 : 1;
  E xormask;  // reduce_kernel.h:43-46
  __device__ explicit FnMinMaxInt(uint64_t arg) : xormask((E)arg) {}
  __device__ E red(E a, E b) const { return ((E)(a ^ xormask) < (E)(b ^ xormask)) ? a : b; }
  // bytes: the same formula four at a time in a dword (SWAR, as the u8 sum
  // above and reduce_kernel.h:173-222's byte functors): per byte
  // x = a ^ m, y = b ^ m; (x | 0x80) - (y & 0x7f) cannot borrow across bytes
  // and its bit 7 says x & 0x7f >= y & 0x7f; with the high bits that gives
  // x >= y unsigned; a byte mask of x < y selects a, else b (a tie -> b).
  // Per-byte extract / compare / select / repack cost ~5 VALU per element
  // (4.20 TB/s at 8 x 256 MiB; this form 5.61, profiles/r5/ab_swar8_shared_out_r5k.jsonl).
  __device__ static uint32_t swarPick(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t H = 0x80808080u;
    const uint32_t x = a ^ m, y = b ^ m;
    const uint32_t d = (x | H) - (y & ~H);
    const uint32_t lt = (((x & ~y) | (~(x ^ y) & d)) & H) ^ H;   // bit 7: x < y
    const uint32_t mk = (lt - (lt >> 7)) | lt;                   // 0xff where x < y
    return (a & mk) | (b & ~mk);
  }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    if constexpr (sizeof(E) == 1) {
      const uint32_t m = (uint32_t)xormask * 0x01010101u;
      return u32x4{swarPick(a[0], b[0], m), swarPick(a[1], b[1], m), swarPick(a[2], b[2], m),
                   swarPick(a[3], b[3], m)};
    } else {
      return packRed(*this, a, b);
    }
  }
};

template <class E>
struct FnPreMulSumInt : FnBase<FnPreMulSumInt<E>, E> {
  static constexpr bool kHasPre = true;
  static constexpr int kUnrollCap = sizeof(E) == 1 ? 4 : 16;
  E scalar;  // reduce_kernel.h:360-369
  __device__ explicit FnPreMulSumInt(uint64_t arg) : scalar((E)arg) {}
  __device__ E red(E a, E b) const { return (E)(a + b); }
  __device__ E pre(E a) const { return (E)(a * scalar); }
};

// SumPostDiv: S is the signed/unsigned view used by `T / int` (reduce_kernel.h:524).
template <class E, class S>
struct FnSumPostDiv : FnBase<FnSumPostDiv<E, S>, E> {
  static constexpr bool kHasPost = true;
  static constexpr int kUnrollCap = sizeof(E) == 1 ? 4 : 16;
  int divisor;  // reduce_kernel.h:502
  __device__ explicit FnSumPostDiv(uint64_t arg) : divisor((int)arg) {}
  __device__ E red(E a, E b) const { return (E)(a + b); }
  __device__ E post(E a) const { return (E)((S)a / divisor); }
};
// unsigned 32-bit: uint32 / int converts the int to unsigned.
template <>
__device__ inline uint32_t FnSumPostDiv<uint32_t, uint32_t>::post(uint32_t a) const {
  return a / (uint32_t)divisor;
}
template <>
__device__ inline uint64_t FnSumPostDiv<uint64_t, uint64_t>::post(uint64_t a) const {
  return a / (uint64_t)(int64_t)divisor;
}
template <>
__device__ inline uint64_t FnSumPostDiv<uint64_t, int64_t>::post(uint64_t a) const {
  return (uint64_t)((int64_t)a / (int64_t)divisor);
}

// -------------------------------------------------------------------------
// Floating-point functors over a type trait Ty.

template <class Ty>
struct FnSumF : FnBase<FnSumF<Ty>, typename Ty::Elt> {
  using E = typename Ty::Elt;
  __device__ explicit FnSumF(uint64_t) {}
  __device__ E red(E a, E b) const { return Ty::narrow(Ty::wide(a) + Ty::wide(b)); }
};
template <class Ty>
struct FnProdF : FnBase<FnProdF<Ty>, typename Ty::Elt> {
  using E = typename Ty::Elt;
  __device__ explicit FnProdF(uint64_t) {}
  __device__ E red(E a, E b) const { return Ty::narrow(Ty::wide(a) * Ty::wide(b)); }
};
template <class Ty>
struct FnMinMaxF : FnBase<FnMinMaxF<Ty>, typename Ty::Elt> {
  static constexpr int kUnrollCap = sizeof(typename Ty::Elt) == 1 ? 4 : 16;
  static constexpr int kBigBlocksPerCU = 2;   // compare + NaN test + select per element
  using E = typename Ty::Elt;
  bool isMin;  // reduce_kernel.h:47: (opArg & 1) == 0
  __device__ explicit FnMinMaxF(uint64_t arg) : isMin((arg & 1ull) == 0ull) {}
  // fminf / fmaxf as pinned (a NaN operand yields the other, a tie returns the
  // second operand); bitwise | so no short-circuit turns into a branch
  template <bool MIN>
  __device__ static E pick(E a, E b) {
    const auto x = Ty::wide(a);
    const auto y = Ty::wide(b);
    const bool pickA = (MIN ? (x < y) : (x > y)) | isNan(y);
    return pickA ? a : b;   // narrowing a widened value is exact: keep the bits
  }
  __device__ E red(E a, E b) const { return isMin ? pick<true>(a, b) : pick<false>(a, b); }
  // fp8: a dword's four codes widened by two v_cvt_pk_f32_* per operand, the
  // four picks gathered into a byte mask, one select — instead of one convert
  // per code and operand and a byte insert per result (3.57 TB/s at 8 x 128
  // MiB, profiles/r5/dtype_survey_bpc_r5h.jsonl)
  template <bool MIN>
  __device__ static uint32_t pickDword8(uint32_t a, uint32_t b) {
    float fa[4], fb[4];
    Ty::wide4(a, fa);
    Ty::wide4(b, fb);
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool p = (MIN ? (fa[i] < fb[i]) : (fa[i] > fb[i])) | isNan(fb[i]);
      m |= p ? (0xffu << (8 * i)) : 0u;
    }
    return (a & m) | (b & ~m);
  }
  // the min/max choice is uniform: decided once per pack, never per element
  // (written per element it compiled into divergent branches: 5.0 vs 6.3 TB/s
  // at config B, profiles/r2/probe_dtypes_r3d.jsonl)
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    if constexpr (sizeof(E) == 1) {
      if (isMin)
        return u32x4{pickDword8<true>(a[0], b[0]), pickDword8<true>(a[1], b[1]), pickDword8<true>(a[2], b[2]),
                     pickDword8<true>(a[3], b[3])};
      return u32x4{pickDword8<false>(a[0], b[0]), pickDword8<false>(a[1], b[1]), pickDword8<false>(a[2], b[2]),
                   pickDword8<false>(a[3], b[3])};
    }
    PackU<E> x, y;
    x.v = a;
    y.v = b;
    if (isMin) {
#pragma unroll
      for (int i = 0; i < (int)(16 / sizeof(E)); i++) x.e[i] = pick<true>(x.e[i], y.e[i]);
    } else {
#pragma unroll
      for (int i = 0; i < (int)(16 / sizeof(E)); i++) x.e[i] = pick<false>(x.e[i], y.e[i]);
    }
    return x.v;
  }
};
template <class Ty>
struct FnPreMulSumF : FnBase<FnPreMulSumF<Ty>, typename Ty::Elt> {
  using E = typename Ty::Elt;
  static constexpr bool kHasPre = true;
  typename Ty::C scalar;  // reduce_kernel.h:360-413 (scalar of the element type)
  __device__ explicit FnPreMulSumF(uint64_t arg) : scalar(Ty::wide((E)arg)) {}
  __device__ E red(E a, E b) const { return Ty::narrow(Ty::wide(a) + Ty::wide(b)); }
  __device__ E pre(E a) const { return Ty::narrow(Ty::wide(a) * scalar); }
};

// fp8: 4 codes per dword — widen a dword with two v_cvt_pk_f32_* and narrow
// each lane result.
template <class Ty, class Op>
__device__ __forceinline__ u32x4 fp8PackMap2(u32x4 a, u32x4 b, Op op) {
  u32x4 r;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    float fa[4], fb[4];
    Ty::wide4(a[w], fa);
    Ty::wide4(b[w], fb);
    uint32_t o = Ty::narrow2(op(fa[0], fb[0]), op(fa[1], fb[1]), 0u, false);
    r[w] = Ty::narrow2(op(fa[2], fb[2]), op(fa[3], fb[3]), o, true);
  }
  return r;
}

template <class Ty>
struct FnSumF8 : FnBase<FnSumF8<Ty>, uint8_t> {
  static constexpr int kUnrollCap = 4;
  static constexpr int kBigBlocksPerCU = 4;   // widen, op, narrow per element (profiles/r2/ab_blocks_per_cu_r4i.jsonl)
  __device__ explicit FnSumF8(uint64_t) {}
  __device__ uint8_t red(uint8_t a, uint8_t b) const { return Ty::narrow(Ty::wide(a) + Ty::wide(b)); }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    return fp8PackMap2<Ty>(a, b, [](float x, float y) { return x + y; });
  }
};
template <class Ty>
struct FnProdF8 : FnBase<FnProdF8<Ty>, uint8_t> {
  static constexpr int kUnrollCap = 4;
  static constexpr int kBigBlocksPerCU = 4;   // widen, op, narrow per element (profiles/r2/ab_blocks_per_cu_r4i.jsonl)
  __device__ explicit FnProdF8(uint64_t) {}
  __device__ uint8_t red(uint8_t a, uint8_t b) const { return Ty::narrow(Ty::wide(a) * Ty::wide(b)); }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    return fp8PackMap2<Ty>(a, b, [](float x, float y) { return x * y; });
  }
};
template <class Ty>
struct FnPreMulSumF8 : FnBase<FnPreMulSumF8<Ty>, uint8_t> {
  static constexpr int kUnrollCap = 4;
  static constexpr int kBigBlocksPerCU = 4;   // widen, op, narrow per element (profiles/r2/ab_blocks_per_cu_r4i.jsonl)
  static constexpr bool kHasPre = true;
  float scalar;
  __device__ explicit FnPreMulSumF8(uint64_t arg) : scalar(Ty::wide((uint8_t)arg)) {}
  __device__ uint8_t red(uint8_t a, uint8_t b) const { return Ty::narrow(Ty::wide(a) + Ty::wide(b)); }
  __device__ uint8_t pre(uint8_t a) const { return Ty::narrow(Ty::wide(a) * scalar); }
  __device__ u32x4 redPack(u32x4 a, u32x4 b) const {
    return fp8PackMap2<Ty>(a, b, [](float x, float y) { return x + y; });
  }
  __device__ u32x4 prePack(u32x4 a) const {
    const float s = scalar;
    return fp8PackMap2<Ty>(a, a, [s](float x, float) { return x * s; });
  }
};

}  // namespace nbx
