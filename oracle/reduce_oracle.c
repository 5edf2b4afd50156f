/*
 * reduce_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of NCCL 2.19.4's multi-source element-wise reduction,
 * the hot path of this repo. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's shared object; the product
 * (libnbxccl.so) never links or calls it.
 *
 * Followed, line by line in meaning (not in code):
 *   - reduceCopyPacks order of operations  /root/reference/src/device/common_kernel.h:79-158
 *       acc = pre(src[0]); acc = Fn(acc, pre(src[s])) for s = 1..n-1 (left fold),
 *       then postOp, then store to every destination.
 *   - PreOp only on sources s < PreOpSrcs   common_kernel.h:79,97,119 (s < PreOpSrcs)
 *   - FuncSum/Prod base cases               /root/reference/src/device/reduce_kernel.h:153-164
 *   - FuncMinMax integer rule               reduce_kernel.h:165-170  ((a^m) < (b^m) ? a : b, unsigned)
 *   - FuncMinMax float/double               reduce_kernel.h:236-237  (fminf/fmaxf, fmin/fmax)
 *   - half / bf16 via float round trip      reduce_kernel.h:245-246, 253, 265-267
 *   - u8x4 SWAR sum/minmax/prod             reduce_kernel.h:173-222 (== per-byte modular ops)
 *   - FuncPreMulSum (scalar in elt type)    reduce_kernel.h:360-430, 435-445, 460-471
 *   - FuncSumPostDiv (int divisor, C div)   reduce_kernel.h:489-526
 *   - signed int Sum/Prod/PreMulSum/MinMax run as unsigned
 *                                           /root/reference/src/device/generate.py:125-133
 *
 * fminf semantics pinned here (the reference's float functors call fminf /
 * fmaxf): a NaN operand yields the other operand; otherwise (a < b) ? a : b
 * for min and (a > b) ? a : b for max, so an exact tie (including +0 vs -0)
 * returns the second operand — the same tie rule as the integer MinMax line
 * reduce_kernel.h:168 and glibc's x86-64 fminf/fmaxf (minss/maxss).
 * UNPINNED against the reference: what NVIDIA's fminf / min.f32 returns for
 * +0 vs -0 (IEEE 754-2008 leaves the sign of min(+0, -0) to the
 * implementation) and which NaN payload survives were never observable here;
 * only NaN-ness is compared. Because a tie returns the second operand, the
 * OPERAND ORDER of each fold step is observable for ±0 ties: the direct
 * schedules fold Fn(acc, next) (common_kernel.h:79-131 left fold), while each
 * ring / chain hop folds Fn(local input, received partial) (recvReduceSend,
 * prims_simple.h srcs[0] = own input; reduce_scatter.h:49-64, reduce.h:44-67)
 * — tests/test_multiprocess_gpu.py::test_multiprocess_float_minmax_ties checks
 * both orders against this oracle.
 *
 * fp8 (OCP e4m3fn, e5m2): NOT in the reference (NCCL 2.19 has no fp8 type) —
 * PARITY UNPINNED by the reference; this build's own definition, following the
 * half pattern: op in fp32, round-to-nearest-even to fp8 with SATFINITE as
 * HIP's amd_hip_fp8.h defines it (what RCCL 2.26's fp8 functors narrow with):
 * a finite value beyond the largest finite code becomes that code with its
 * sign; +-inf and NaN go through (e5m2 +-inf; e4m3fn, which has no infinity,
 * NaN). Corroborated against RCCL's one-rank PreMulSum on every code
 * (tests/test_rccl_corroboration_gpu.py).
 *
 * PIN STATUS: the reference cannot be built here (its device headers need
 * cuda_runtime.h / cuda_fp16.h / PTX; writing stand-ins is not permitted), and
 * it ships no tests or golden vectors. This oracle is
 * therefore pinned PARTIALLY: against the known-answer values recorded in
 * SURVEY.md §8c, which were produced by the reference's own functors, and by
 * independent cross-checks (numpy IEEE arithmetic, torch dtype casts) in
 * tests/test_oracle_*.py.
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off; no FMA contraction, so
 * a*s + b is two roundings as in the reference).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ncclDataType_t values (nccl.h.in:199-214) + this build's fp8 (10, 11). */
enum { T_I8 = 0, T_U8, T_I32, T_U32, T_I64, T_U64, T_F16, T_F32, T_F64, T_BF16, T_E4M3, T_E5M2, T_NUM };
/* ncclDevRedOp_t values (src/include/device.h:26-30). */
enum { OP_SUM = 0, OP_PROD, OP_MINMAX, OP_PREMULSUM, OP_SUMPOSTDIV, OP_NUM };

int oracle_type_size(int t) {
  switch (t) {
    case T_I8: case T_U8: case T_E4M3: case T_E5M2: return 1;
    case T_F16: case T_BF16: return 2;
    case T_I32: case T_U32: case T_F32: return 4;
    case T_I64: case T_U64: case T_F64: return 8;
    default: return -1;
  }
}

/* ------------------------------------------------------------------------ */
/* Small-float codecs (float round trip of reduce_kernel.h:245-267).          */

static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* Decode a small IEEE-like float (E exponent bits, M mantissa bits) to fp32.
 * fn = 1: OCP "fn" flavour (no inf; only all-ones exponent+mantissa is NaN). */
static float small_to_f32(uint32_t code, int E, int M, int fn) {
  uint32_t sign = (code >> (E + M)) & 1u;
  uint32_t ef = (code >> M) & ((1u << E) - 1u);
  uint32_t mf = code & ((1u << M) - 1u);
  int bias = (1 << (E - 1)) - 1;
  float v;
  if (ef == (1u << E) - 1u && (!fn || mf == (1u << M) - 1u)) {
    v = (mf == 0 && !fn) ? INFINITY : NAN;
  } else if (ef == 0) {
    v = ldexpf((float)mf, 1 - bias - M);  /* subnormal, exact */
  } else {
    v = u2f(((uint32_t)((int)ef - bias + 127) << 23) | (mf << (23 - M)));
  }
  return sign ? -v : v;
}

/* Round fp32 to a small float, round-to-nearest-even. Overflow: +-inf for
 * IEEE-like formats, NaN for the fn flavour. NaN in -> quiet NaN out. */
static uint32_t f32_to_small(float x, int E, int M, int fn) {
  uint32_t u = f2u(x);
  uint32_t sign = (u >> 31) << (E + M);
  uint32_t a = u & 0x7fffffffu;
  uint32_t expAllOnes = ((1u << E) - 1u) << M;
  uint32_t nanCode = fn ? (expAllOnes | ((1u << M) - 1u)) : (expAllOnes | (1u << (M - 1)));
  uint32_t infCode = expAllOnes;                        /* IEEE only */
  uint32_t maxFinite = fn ? (expAllOnes | ((1u << M) - 2u)) : (expAllOnes - (1u << M)) | ((1u << M) - 1u);
  if (a > 0x7f800000u) return sign | nanCode;
  if (a == 0x7f800000u) return sign | (fn ? nanCode : infCode);
  if ((a >> 23) == 0) return sign;                      /* fp32 zero/subnormal -> +-0 */
  int bias = (1 << (E - 1)) - 1;
  int e = (int)(a >> 23) - 127;
  uint64_t mant = (a & 0x7fffffu) | 0x800000u;
  int emin = 1 - bias;
  int et = e < emin ? emin : e;
  int shift = (23 - M) + (et - e);
  if (shift > 40) return sign;
  uint64_t q = mant >> shift;
  uint64_t rem = mant & ((1ull << shift) - 1ull);
  uint64_t half = 1ull << (shift - 1);
  if (rem > half || (rem == half && (q & 1ull))) q++;
  uint64_t enc = ((uint64_t)(et + bias - 1) << M) + q;
  if (enc > maxFinite) return sign | (fn ? nanCode : infCode);
  return sign | (uint32_t)enc;
}

float oracle_f16_to_f32(uint16_t h) { return small_to_f32(h, 5, 10, 0); }
uint16_t oracle_f32_to_f16(float f) { return (uint16_t)f32_to_small(f, 5, 10, 0); }
float oracle_bf16_to_f32(uint16_t b) { return u2f((uint32_t)b << 16); }
uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  /* quiet NaN */
  u += 0x7fffu + ((u >> 16) & 1u);                                              /* RNE */
  return (uint16_t)(u >> 16);
}
/* fp8 narrowing with SATFINITE (header): finite |x| above the largest finite
 * value (448 e4m3fn, 57344 e5m2) -> the largest finite code with x's sign. */
static uint32_t f32_to_fp8_sat(float x, int E, int M, int fn) {
  uint32_t u = f2u(x);
  float maxv = fn ? 448.0f : 57344.0f;
  if ((u & 0x7f800000u) != 0x7f800000u && fabsf(x) > maxv) {
    uint32_t expAllOnes = ((1u << E) - 1u) << M;
    uint32_t maxFinite = fn ? (expAllOnes | ((1u << M) - 2u)) : (expAllOnes - (1u << M)) | ((1u << M) - 1u);
    return ((u >> 31) << (E + M)) | maxFinite;
  }
  return f32_to_small(x, E, M, fn);
}

float oracle_e4m3_to_f32(uint8_t c) { return small_to_f32(c, 4, 3, 1); }
uint8_t oracle_f32_to_e4m3(float f) { return (uint8_t)f32_to_fp8_sat(f, 4, 3, 1); }
float oracle_e5m2_to_f32(uint8_t c) { return small_to_f32(c, 5, 2, 0); }
uint8_t oracle_f32_to_e5m2(float f) { return (uint8_t)f32_to_fp8_sat(f, 5, 2, 0); }

/* ------------------------------------------------------------------------ */
/* Element functors. fminf/fmaxf restated (see header).                       */

static inline float fmin_ref(float a, float b) { return (a < b || isnan(b)) ? a : b; }
static inline float fmax_ref(float a, float b) { return (a > b || isnan(b)) ? a : b; }
static inline double dmin_ref(double a, double b) { return (a < b || isnan(b)) ? a : b; }
static inline double dmax_ref(double a, double b) { return (a > b || isnan(b)) ? a : b; }

typedef struct {
  int op;
  uint64_t arg;   /* MinMax xormask / PreMulSum scalar bits / SumPostDiv divisor */
  int isMin;      /* float MinMax: (opArg & 1) == 0, reduce_kernel.h:47 */
} fnstate;

/* Reduce two elements of a 1/2/4/8-byte integer or float type given as raw bits. */
static inline uint64_t red_elem(int t, const fnstate* fs, uint64_t a, uint64_t b) {
  int op = fs->op;
  if (op == OP_PREMULSUM || op == OP_SUMPOSTDIV) op = OP_SUM;  /* reduce_kernel.h:415-421, 511-518 */
  switch (t) {
    case T_I8: case T_U8: case T_I32: case T_U32: case T_I64: case T_U64: {
      int nb = 8 * oracle_type_size(t);
      uint64_t mask = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
      if (op == OP_SUM) return (a + b) & mask;                    /* unsigned wrap, generate.py:127 */
      if (op == OP_PROD) return (a * b) & mask;
      /* OP_MINMAX: (a ^ m) < (b ^ m) ? a : b on the unsigned pattern */
      uint64_t m = fs->arg & mask;
      return ((a ^ m) < (b ^ m)) ? a : b;
    }
    case T_F32: {
      float x = u2f((uint32_t)a), y = u2f((uint32_t)b), r;
      if (op == OP_SUM) r = x + y;
      else if (op == OP_PROD) r = x * y;
      else r = fs->isMin ? fmin_ref(x, y) : fmax_ref(x, y);
      return f2u(r);
    }
    case T_F64: {
      double x, y, r;
      memcpy(&x, &a, 8); memcpy(&y, &b, 8);
      if (op == OP_SUM) r = x + y;
      else if (op == OP_PROD) r = x * y;
      else r = fs->isMin ? dmin_ref(x, y) : dmax_ref(x, y);
      uint64_t o; memcpy(&o, &r, 8);
      return o;
    }
    default: {  /* f16 / bf16 / fp8: float round trip */
      float x, y;
      switch (t) {
        case T_F16: x = oracle_f16_to_f32((uint16_t)a); y = oracle_f16_to_f32((uint16_t)b); break;
        case T_BF16: x = oracle_bf16_to_f32((uint16_t)a); y = oracle_bf16_to_f32((uint16_t)b); break;
        case T_E4M3: x = oracle_e4m3_to_f32((uint8_t)a); y = oracle_e4m3_to_f32((uint8_t)b); break;
        default: x = oracle_e5m2_to_f32((uint8_t)a); y = oracle_e5m2_to_f32((uint8_t)b); break;
      }
      if (op == OP_MINMAX) {
        /* fminf on the widened values; narrowing back is exact, so the result is
         * the selected operand's own bits (reduce_kernel.h:253, 267). */
        int pickA = fs->isMin ? (x < y || isnan(y)) : (x > y || isnan(y));
        return pickA ? a : b;
      }
      float r = (op == OP_SUM) ? x + y : x * y;
      switch (t) {
        case T_F16: return oracle_f32_to_f16(r);
        case T_BF16: return oracle_f32_to_bf16(r);
        case T_E4M3: return oracle_f32_to_e4m3(r);
        default: return oracle_f32_to_e5m2(r);
      }
    }
  }
}

/* PreMulSum pre-op: x * scalar in the element type (reduce_kernel.h:424-430;
 * half/bf16 through float, :442, :469). */
static inline uint64_t pre_elem(int t, const fnstate* fs, uint64_t x) {
  uint64_t s = fs->arg;
  switch (t) {
    case T_I8: case T_U8: return (x * s) & 0xffull;
    case T_I32: case T_U32: return (x * s) & 0xffffffffull;
    case T_I64: case T_U64: return x * s;
    case T_F32: return f2u(u2f((uint32_t)x) * u2f((uint32_t)s));
    case T_F64: { double a, b; memcpy(&a, &x, 8); memcpy(&b, &s, 8); a *= b; uint64_t o; memcpy(&o, &a, 8); return o; }
    case T_F16: return oracle_f32_to_f16(oracle_f16_to_f32((uint16_t)x) * oracle_f16_to_f32((uint16_t)s));
    case T_BF16: return oracle_f32_to_bf16(oracle_bf16_to_f32((uint16_t)x) * oracle_bf16_to_f32((uint16_t)s));
    case T_E4M3: return oracle_f32_to_e4m3(oracle_e4m3_to_f32((uint8_t)x) * oracle_e4m3_to_f32((uint8_t)s));
    default: return oracle_f32_to_e5m2(oracle_e5m2_to_f32((uint8_t)x) * oracle_e5m2_to_f32((uint8_t)s));
  }
}

/* SumPostDiv post-op: C division by `int divisor` with the usual arithmetic
 * conversions of `T / int` (reduce_kernel.h:502-503, 524). */
static inline uint64_t post_elem(int t, const fnstate* fs, uint64_t x) {
  int d = (int)(int64_t)fs->arg;
  switch (t) {
    case T_I8: return (uint8_t)(int8_t)((int)(int8_t)(uint8_t)x / d);
    case T_U8: return (uint8_t)((int)(uint8_t)x / d);
    case T_I32: return (uint32_t)((int32_t)(uint32_t)x / d);
    case T_U32: return (uint32_t)((uint32_t)x / (uint32_t)d);
    case T_I64: return (uint64_t)((int64_t)x / (int64_t)d);
    case T_U64: return x / (uint64_t)(int64_t)d;
    default: return x;
  }
}

static inline uint64_t load_elem(const void* p, size_t i, int sz) {
  const uint8_t* b = (const uint8_t*)p + i * (size_t)sz;
  switch (sz) {
    case 1: return *b;
    case 2: { uint16_t v; memcpy(&v, b, 2); return v; }
    case 4: { uint32_t v; memcpy(&v, b, 4); return v; }
    default: { uint64_t v; memcpy(&v, b, 8); return v; }
  }
}
static inline void store_elem(void* p, size_t i, int sz, uint64_t v) {
  uint8_t* b = (uint8_t*)p + i * (size_t)sz;
  switch (sz) {
    case 1: *b = (uint8_t)v; break;
    case 2: { uint16_t x = (uint16_t)v; memcpy(b, &x, 2); break; }
    case 4: { uint32_t x = (uint32_t)v; memcpy(b, &x, 4); break; }
    default: memcpy(b, &v, 8); break;
  }
}

/* ------------------------------------------------------------------------ */
/* Specialised fp32 Sum loop: same arithmetic as the generic path (one IEEE
 * add per source, left fold); kept separate only so the CPU baseline is a
 * fair, vectorisable C loop rather than a per-element switch. */
static void sum_f32_range(float* const* dsts, int nDsts, const float* const* srcs, int nSrcs,
                          size_t lo, size_t hi) {
  const size_t B = 4096;
  float acc[4096];
  for (size_t base = lo; base < hi; base += B) {
    size_t n = hi - base < B ? hi - base : B;
    const float* s0 = srcs[0] + base;
    for (size_t i = 0; i < n; i++) acc[i] = s0[i];
    for (int s = 1; s < nSrcs; s++) {
      const float* ss = srcs[s] + base;
      for (size_t i = 0; i < n; i++) acc[i] = acc[i] + ss[i];
    }
    for (int d = 0; d < nDsts; d++) memcpy(dsts[d] + base, acc, n * sizeof(float));
  }
}

typedef struct {
  void* const* dsts; int nDsts;
  const void* const* srcs; int nSrcs;
  size_t lo, hi; int t; fnstate fs; int nPreOpSrcs; int postOp;
} job;

static void run_range(const job* j) {
  int sz = oracle_type_size(j->t);
  if (j->t == T_F32 && j->fs.op == OP_SUM && !j->postOp) {
    sum_f32_range((float* const*)j->dsts, j->nDsts, (const float* const*)j->srcs, j->nSrcs, j->lo, j->hi);
    return;
  }
  int isPre = j->fs.op == OP_PREMULSUM;
  for (size_t i = j->lo; i < j->hi; i++) {
    uint64_t acc = load_elem(j->srcs[0], i, sz);
    if (isPre && 0 < j->nPreOpSrcs) acc = pre_elem(j->t, &j->fs, acc);
    for (int s = 1; s < j->nSrcs; s++) {
      uint64_t v = load_elem(j->srcs[s], i, sz);
      if (isPre && s < j->nPreOpSrcs) v = pre_elem(j->t, &j->fs, v);
      acc = red_elem(j->t, &j->fs, acc, v);
    }
    if (j->postOp && j->fs.op == OP_SUMPOSTDIV) acc = post_elem(j->t, &j->fs, acc);
    for (int d = 0; d < j->nDsts; d++) store_elem(j->dsts[d], i, sz, acc);
  }
}

static void* thread_main(void* p) { run_range((const job*)p); return NULL; }

/* Returns 0 on success, -1 on a bad argument.
 * dtype: ncclDataType_t; op: ncclDevRedOp_t; arg: ncclDevRedOpFull.scalarArg
 * (by value; the oracle never dereferences device scalars). */
int oracle_reduce_multi(void* const* dsts, int nDsts, const void* const* srcs, int nSrcs,
                        size_t count, int dtype, int op, uint64_t arg,
                        int nPreOpSrcs, int postOp, int nThreads) {
  if (dtype < 0 || dtype >= T_NUM || op < 0 || op >= OP_NUM) return -1;
  if (nSrcs < 1 || nDsts < 1) return -1;
  int isFloat = dtype == T_F16 || dtype == T_F32 || dtype == T_F64 || dtype == T_BF16 ||
                dtype == T_E4M3 || dtype == T_E5M2;
  if (op == OP_SUMPOSTDIV && (isFloat || (int)(int64_t)arg == 0)) return -1;
  if (count == 0) return 0;
  fnstate fs;
  fs.op = op;
  fs.arg = arg;
  fs.isMin = (arg & 1ull) == 0ull;
  if (nThreads < 1) nThreads = 1;
  if ((size_t)nThreads > count / 4096 + 1) nThreads = (int)(count / 4096 + 1);
  job jobs[256];
  pthread_t th[256];
  if (nThreads > 256) nThreads = 256;
  size_t per = (count + nThreads - 1) / nThreads;
  per = (per + 1023) & ~(size_t)1023;
  int n = 0;
  for (size_t lo = 0; lo < count && n < nThreads; lo += per, n++) {
    jobs[n] = (job){dsts, nDsts, srcs, nSrcs, lo, lo + per < count ? lo + per : count,
                    dtype, fs, nPreOpSrcs, postOp};
  }
  for (int k = 1; k < n; k++) pthread_create(&th[k], NULL, thread_main, &jobs[k]);
  run_range(&jobs[0]);
  for (int k = 1; k < n; k++) pthread_join(th[k], NULL);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* hostToDevRedOp restatement — /root/reference/src/enqueue.cc:1436-1512.     */
/* Returns 0 and fills (devOp, scalarArg), or -1 for an invalid combination.  */
int oracle_host_to_dev_redop(int op, int dtype, int nRanks, int* devOp, uint64_t* scalarArg) {
  int sz = oracle_type_size(dtype);
  if (sz < 0) return -1;
  int nbits = 8 * sz;
  uint64_t allBits = ~0ull >> (64 - nbits);
  uint64_t signBit = allBits ^ (allBits >> 1);
  *scalarArg = 0;
  switch (op) {
    case 0: *devOp = OP_SUM; return 0;
    case 1: *devOp = OP_PROD; return 0;
    case 2: case 3:   /* ncclMax = 2, ncclMin = 3 */
      *devOp = OP_MINMAX;
      if (dtype == T_I8 || dtype == T_I32 || dtype == T_I64) *scalarArg ^= signBit;
      *scalarArg ^= (op == 2) ? allBits : 0;
      return 0;
    case 4:           /* ncclAvg */
      switch (dtype) {
        case T_I8: case T_I32: case T_I64: case T_U8: case T_U32: case T_U64:
          *devOp = OP_SUMPOSTDIV; *scalarArg = (uint64_t)nRanks; return 0;
        case T_F16: *devOp = OP_PREMULSUM; *scalarArg = oracle_f32_to_f16((float)(1.0 / nRanks)); return 0;
        case T_BF16: *devOp = OP_PREMULSUM; *scalarArg = oracle_f32_to_bf16((float)(1.0 / nRanks)); return 0;
        case T_F32: *devOp = OP_PREMULSUM; *scalarArg = f2u((float)(1.0 / nRanks)); return 0;
        case T_F64: { double v = 1.0 / nRanks; *devOp = OP_PREMULSUM; memcpy(scalarArg, &v, 8); return 0; }
        case T_E4M3: *devOp = OP_PREMULSUM; *scalarArg = oracle_f32_to_e4m3((float)(1.0 / nRanks)); return 0;
        case T_E5M2: *devOp = OP_PREMULSUM; *scalarArg = oracle_f32_to_e5m2((float)(1.0 / nRanks)); return 0;
      }
      return -1;
    default: return -1;
  }
}
