/* nbx_perf.c — an nccl-tests style driver (all_reduce_perf / reduce_scatter_perf /
 * reduce_perf) written against the NCCL C API only: include "nccl.h", link
 * -lnbxccl (plus the HIP runtime for buffers and streams). One process drives
 * every rank through ncclCommInitAll + ncclGroupStart/End, as nccl-tests' -g
 * mode does.
 *
 *   nbx_perf [-c allreduce|reducescatter|reduce] [-d dev,dev,...] [-b minbytes]
 *            [-e maxbytes] [-f factor] [-n iters] [-w warmup] [-t float|half|bfloat16|int32|int64|double]
 *            [-o sum|prod|max|min|avg] [-p 0|1] [-m agg]
 *
 * -d lists the device of each rank (a device may repeat: ranks sharing one GPU).
 * -p 1 runs one process per rank instead (fork after ncclGetUniqueId, each
 * child ncclCommInitRank on its device — the multi-process communicator with
 * its LL / LL128 / Simple protocols); times and #wrong are reduced over the
 * ranks with the library's own ncclAllReduce (max / sum), as nccl-tests does
 * with MPI.
 * Sizes are the per-rank send size in bytes (nccl-tests' convention for
 * all_reduce; reduce_scatter sends nranks x recvcount). Each size is checked:
 * rank r's input element i is ((i * 7 + r * 13) % 61) - 30 (exact in every
 * type for sum/max/min/prod with few ranks), the output is compared on the
 * host with the exact expected value, and #wrong counts differing elements.
 * Out-of-place then in-place, like nccl-tests. -m aggregates agg operations per
 * iteration in one ncclGroupStart/End (nccl-tests' -m), each on its own slice
 * of the buffers so they are independent; time is per operation, every
 * slice is checked. Exit status 1 if any wrong. */
#define _POSIX_C_SOURCE 200809L
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <sys/wait.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nccl.h"

#define HIPT(x)                                                                     \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)
#define NCCLT(x)                                                                    \
  do {                                                                              \
    ncclResult_t r_ = (x);                                                          \
    if (r_ != ncclSuccess) {                                                        \
      fprintf(stderr, "NCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

enum { kAllReduce, kReduceScatter, kReduce };
#define MAXR 16

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int tsize(ncclDataType_t t) {
  switch (t) {
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt64: case ncclFloat64: return 8;
    default: return 4;
  }
}

/* value -> element bits (values are small integers: exact in every type) */
static void put(void* p, size_t i, ncclDataType_t t, double v) {
  switch (t) {
    case ncclInt32: ((int32_t*)p)[i] = (int32_t)v; break;
    case ncclInt64: ((int64_t*)p)[i] = (int64_t)v; break;
    case ncclFloat32: ((float*)p)[i] = (float)v; break;
    case ncclFloat64: ((double*)p)[i] = v; break;
    case ncclFloat16: {   /* small integers |v| <= 2048 are exact halves */
      float f = (float)v;
      uint32_t u;
      memcpy(&u, &f, 4);
      uint16_t s = (uint16_t)((u >> 16) & 0x8000u);
      if (f == 0.0f) { ((uint16_t*)p)[i] = s; break; }
      int e = (int)((u >> 23) & 0xff) - 127;
      uint16_t h = (uint16_t)(s | (uint16_t)((e + 15) << 10) | (uint16_t)((u >> 13) & 0x3ffu));
      ((uint16_t*)p)[i] = h;
      break;
    }
    case ncclBfloat16: {   /* small integers |v| <= 256 are exact bf16 */
      float f = (float)v;
      uint32_t u;
      memcpy(&u, &f, 4);
      ((uint16_t*)p)[i] = (uint16_t)(u >> 16);
      break;
    }
    default: break;
  }
}

static double get(const void* p, size_t i, ncclDataType_t t) {
  switch (t) {
    case ncclInt32: return ((const int32_t*)p)[i];
    case ncclInt64: return (double)((const int64_t*)p)[i];
    case ncclFloat32: return ((const float*)p)[i];
    case ncclFloat64: return ((const double*)p)[i];
    case ncclFloat16: {
      uint16_t h = ((const uint16_t*)p)[i];
      int e = (h >> 10) & 0x1f, m = h & 0x3ff;
      double v = e == 0 ? ldexp(m, -24) : ldexp(1024 + m, e - 25);
      return (h & 0x8000) ? -v : v;
    }
    case ncclBfloat16: {
      uint32_t u = (uint32_t)((const uint16_t*)p)[i] << 16;
      float f;
      memcpy(&f, &u, 4);
      return f;
    }
    default: return 0;
  }
}

static double input(size_t i, int r) { return (double)((long)((i * 7 + (size_t)r * 13) % 61) - 30); }

static double expect(size_t i, int n, ncclRedOp_t op, ncclDataType_t t) {
  double acc = input(i, 0);
  for (int r = 1; r < n; r++) {
    double x = input(i, r);
    switch (op) {
      case ncclSum: case ncclAvg: acc += x; break;
      case ncclProd: acc *= x; break;
      case ncclMax: acc = x > acc ? x : acc; break;
      case ncclMin: acc = x < acc ? x : acc; break;
      default: break;
    }
  }
  if (op == ncclAvg) {
    if (t == ncclInt32 || t == ncclInt64) acc = (double)((long)acc / n);   /* C truncation (SumPostDiv) */
    else acc = acc / n;
  }
  return acc;
}

/* max over ranks of a double and sum of an int64 through ncclAllReduce (process mode) */
static void reduceStats(ncclComm_t comm, hipStream_t st, double* t, long* wrong) {
  double* dt;
  int64_t* dw;
  HIPT(hipMalloc((void**)&dt, sizeof(double)));
  HIPT(hipMalloc((void**)&dw, sizeof(int64_t)));
  int64_t w = *wrong;
  HIPT(hipMemcpy(dt, t, sizeof(double), hipMemcpyHostToDevice));
  HIPT(hipMemcpy(dw, &w, sizeof(int64_t), hipMemcpyHostToDevice));
  NCCLT(ncclAllReduce(dt, dt, 1, ncclFloat64, ncclMax, comm, st));
  NCCLT(ncclAllReduce(dw, dw, 1, ncclInt64, ncclSum, comm, st));
  HIPT(hipStreamSynchronize(st));
  HIPT(hipMemcpy(t, dt, sizeof(double), hipMemcpyDeviceToHost));
  HIPT(hipMemcpy(&w, dw, sizeof(int64_t), hipMemcpyDeviceToHost));
  *wrong = (long)w;
  HIPT(hipFree(dt));
  HIPT(hipFree(dw));
}

int main(int argc, char** argv) {
  int coll = kAllReduce, n = 0, devs[MAXR], iters = 20, warm = 5, procMode = 0, agg = 1;
  size_t minB = 4096, maxB = 16u << 20;
  double factor = 4.0;
  ncclDataType_t type = ncclFloat32;
  ncclRedOp_t op = ncclSum;
  const char* cname = "allreduce";
  for (int a = 1; a + 1 < argc; a += 2) {
    const char* k = argv[a];
    const char* v = argv[a + 1];
    if (!strcmp(k, "-c")) {
      cname = v;
      coll = !strcmp(v, "reducescatter") ? kReduceScatter : !strcmp(v, "reduce") ? kReduce : kAllReduce;
    } else if (!strcmp(k, "-d")) {
      char buf[256];
      snprintf(buf, sizeof buf, "%s", v);
      for (char* tok = strtok(buf, ","); tok && n < MAXR; tok = strtok(NULL, ",")) devs[n++] = atoi(tok);
    } else if (!strcmp(k, "-b")) minB = strtoull(v, NULL, 10);
    else if (!strcmp(k, "-e")) maxB = strtoull(v, NULL, 10);
    else if (!strcmp(k, "-f")) factor = atof(v);
    else if (!strcmp(k, "-n")) iters = atoi(v);
    else if (!strcmp(k, "-w")) warm = atoi(v);
    else if (!strcmp(k, "-t")) {
      type = !strcmp(v, "half") ? ncclFloat16 : !strcmp(v, "bfloat16") ? ncclBfloat16 : !strcmp(v, "int32") ? ncclInt32
             : !strcmp(v, "int64") ? ncclInt64 : !strcmp(v, "double") ? ncclFloat64 : ncclFloat32;
    } else if (!strcmp(k, "-o")) {
      op = !strcmp(v, "prod") ? ncclProd : !strcmp(v, "max") ? ncclMax : !strcmp(v, "min") ? ncclMin
           : !strcmp(v, "avg") ? ncclAvg : ncclSum;
    } else if (!strcmp(k, "-p")) procMode = atoi(v);
    else if (!strcmp(k, "-m")) agg = atoi(v) < 1 ? 1 : atoi(v);
  }
  if (n == 0) {
    int cnt = 0;
    HIPT(hipGetDeviceCount(&cnt));
    for (n = 0; n < cnt && n < MAXR; n++) devs[n] = n;
  }
  const int eb = tsize(type);
  ncclComm_t comms[MAXR];
  /* local ranks [lo, hi): every rank in clique mode, this process's rank in process mode */
  int lo = 0, hi = n;
  if (procMode) {
    ncclUniqueId id;
    NCCLT(ncclGetUniqueId(&id));   /* bootstrap root thread in this (parent) process; no HIP yet */
    fflush(stdout);
    int me = -1;
    pid_t pids[MAXR];
    for (int r = 0; r < n; r++) {
      pids[r] = fork();
      if (pids[r] < 0) return 2;
      if (pids[r] == 0) {
        me = r;
        break;
      }
    }
    if (me < 0) {   /* parent: wait for every rank, exit with the worst status */
      int worst = 0;
      for (int r = 0; r < n; r++) {
        int status = 0;
        waitpid(pids[r], &status, 0);
        const int rc = WIFEXITED(status) ? WEXITSTATUS(status) : 3;
        if (rc > worst) worst = rc;
      }
      return worst;
    }
    lo = me;
    hi = me + 1;
    HIPT(hipSetDevice(devs[me]));
    NCCLT(ncclCommInitRank(&comms[me], n, id, me));
  } else {
    NCCLT(ncclCommInitAll(comms, n, devs));
  }
  const int printer = lo == 0;
  hipStream_t st[MAXR];
  void *sb[MAXR], *rb[MAXR];
  const size_t sendMax = maxB, recvMax = coll == kReduceScatter ? maxB / (size_t)n + 16 : maxB;
  /* per-operation slices (-m): 256-byte aligned strides */
  const size_t sStride = (sendMax + 255) / 256 * 256;
  const size_t rStride = ((recvMax > sendMax ? recvMax : sendMax) + 255) / 256 * 256;
  for (int r = lo; r < hi; r++) {
    HIPT(hipSetDevice(devs[r]));
    HIPT(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
    HIPT(hipMalloc(&sb[r], sStride * (size_t)agg));
    HIPT(hipMalloc(&rb[r], rStride * (size_t)agg));
  }
  void* host = malloc(sendMax);
  if (printer) {
    printf("# nbx_perf: %s, %d ranks (%s), %d op(s) per group, devices", cname, n,
           procMode ? "one process per rank" : "one process, ncclCommInitAll", agg);
    for (int r = 0; r < n; r++) printf(" %d", devs[r]);
    printf("\n#\n# %12s %12s %8s %6s   %9s %8s %8s %6s   %9s %8s %8s %6s\n", "size", "count", "type", "redop",
           "time(us)", "algbw", "busbw", "#wrong", "time(us)", "algbw", "busbw", "#wrong");
  }
  long totalWrong = 0;
  for (size_t bytes = minB; bytes <= maxB; bytes = (size_t)((double)bytes * factor) > bytes ? (size_t)((double)bytes * factor) : bytes + 1) {
    size_t sendCount = bytes / (size_t)eb;
    if (coll == kReduceScatter) sendCount -= sendCount % (size_t)n;
    const size_t count = coll == kReduceScatter ? sendCount / (size_t)n : sendCount;   /* API count */
    if (count == 0) continue;
    const size_t outCount = count;
    double us[2];
    long wrong[2];
    for (int inplace = 0; inplace < 2; inplace++) {
      for (int r = lo; r < hi; r++) {   /* inputs */
        for (size_t i = 0; i < sendCount; i++) put(host, i, type, input(i, r));
        HIPT(hipSetDevice(devs[r]));
        for (int k = 0; k < agg; k++) {
          char* dst = inplace ? (char*)rb[r] + (size_t)k * rStride : (char*)sb[r] + (size_t)k * sStride;
          /* on the rank's own (non-blocking) stream: a null-stream hipMemset would not be
           * ordered before the collective */
          HIPT(hipMemcpyAsync(dst, host, sendCount * (size_t)eb, hipMemcpyHostToDevice, st[r]));
          if (!inplace) HIPT(hipMemsetAsync((char*)rb[r] + (size_t)k * rStride, 0, outCount * (size_t)eb, st[r]));
        }
        HIPT(hipStreamSynchronize(st[r]));
      }
      const int root = 0;
      /* in place: AllReduce / Reduce send == recv; ReduceScatter recv = send + rank * recvcount */
      for (int it = -1; it < warm + iters; it++) {
        if (it == warm) {
          for (int r = lo; r < hi; r++) {
            HIPT(hipSetDevice(devs[r]));
            HIPT(hipStreamSynchronize(st[r]));
          }
          us[inplace] = now_s();
        }
        NCCLT(ncclGroupStart());
        for (int k = 0; k < agg; k++)
          for (int r = lo; r < hi; r++) {
            char* rk = (char*)rb[r] + (size_t)k * rStride;
            const void* s = inplace ? (const void*)rk : (const void*)((char*)sb[r] + (size_t)k * sStride);
            void* d = rk;
            if (coll == kReduceScatter && inplace) d = rk + (size_t)r * count * (size_t)eb;
            if (coll == kAllReduce) NCCLT(ncclAllReduce(s, d, count, type, op, comms[r], st[r]));
            else if (coll == kReduceScatter) NCCLT(ncclReduceScatter(s, d, count, type, op, comms[r], st[r]));
            else NCCLT(ncclReduce(s, d, count, type, op, root, comms[r], st[r]));
          }
        NCCLT(ncclGroupEnd());
        if (it == -1) {   /* check the first call's result (later calls re-reduce in-place data) */
          wrong[inplace] = 0;
          for (int r = lo; r < hi; r++) {
            HIPT(hipSetDevice(devs[r]));
            HIPT(hipStreamSynchronize(st[r]));
          }
          for (int k = 0; k < agg; k++)
          for (int r = lo; r < hi; r++) {
            if (coll == kReduce && r != root) continue;
            HIPT(hipSetDevice(devs[r]));
            const char* d = (const char*)rb[r] + (size_t)k * rStride +
                            ((coll == kReduceScatter && inplace) ? (size_t)r * count * (size_t)eb : 0);
            HIPT(hipMemcpyAsync(host, d, outCount * (size_t)eb, hipMemcpyDeviceToHost, st[r]));
            HIPT(hipStreamSynchronize(st[r]));
            const size_t base = coll == kReduceScatter ? (size_t)r * count : 0;
            /* exact, except ncclAvg on floats: a PreMulSum by a rounded 1/n and a
             * rounded sum of rounded products — bounded relative to sum_r |x_r| / n
             * (a few ulps of the element type: bf16 2^-8, half 2^-11, float 2^-24) */
            const int fl = type != ncclInt32 && type != ncclInt64;
            const double ulp = type == ncclBfloat16 ? 0x1p-8 : type == ncclFloat16 ? 0x1p-11
                               : type == ncclFloat32 ? 0x1p-24 : 0x1p-53;
            const double tol = (op == ncclAvg && fl) ? 2.0 * (n + 1) * ulp : 0.0;
            for (size_t i = 0; i < outCount; i++) {
              const double e = expect(base + i, n, op, type);
              double mag = 0;
              for (int q = 0; q < n; q++) mag += fabs(input(base + i, q));
              if (fabs(get(host, i, type) - e) > tol * (mag / n)) wrong[inplace]++;
            }
          }
          /* restore in-place inputs consumed by the checked call */
          if (inplace) {
            for (int r = lo; r < hi; r++) {
              for (size_t i = 0; i < sendCount; i++) put(host, i, type, input(i, r));
              HIPT(hipSetDevice(devs[r]));
              for (int k = 0; k < agg; k++)
                HIPT(hipMemcpyAsync((char*)rb[r] + (size_t)k * rStride, host, sendCount * (size_t)eb,
                                    hipMemcpyHostToDevice, st[r]));
              HIPT(hipStreamSynchronize(st[r]));
            }
          }
        }
      }
      for (int r = lo; r < hi; r++) {
        HIPT(hipSetDevice(devs[r]));
        HIPT(hipStreamSynchronize(st[r]));
      }
      us[inplace] = (now_s() - us[inplace]) * 1e6 / iters / agg;   /* per operation */
      if (procMode) reduceStats(comms[lo], st[lo], &us[inplace], &wrong[inplace]);
      totalWrong += wrong[inplace];
    }
    const double algFactor = coll == kReduceScatter ? (double)n : 1.0;   /* bytes = recv x nranks for RS */
    const double sz = (double)count * eb * algFactor;
    const double bus = coll == kAllReduce ? 2.0 * (n - 1) / n : coll == kReduceScatter ? (double)(n - 1) / n : 1.0;
    const char* tn = type == ncclFloat16 ? "half" : type == ncclBfloat16 ? "bfloat16" : type == ncclInt32 ? "int32"
                     : type == ncclInt64 ? "int64" : type == ncclFloat64 ? "double" : "float";
    const char* on = op == ncclProd ? "prod" : op == ncclMax ? "max" : op == ncclMin ? "min" : op == ncclAvg ? "avg" : "sum";
    if (printer) {
      printf("  %12zu %12zu %8s %6s", (size_t)sz, count, tn, on);
      for (int k = 0; k < 2; k++) {
        const double alg = sz / (us[k] * 1e-6) / 1e9;
        printf("   %9.2f %8.2f %8.2f %6ld", us[k], alg, alg * bus, wrong[k]);
      }
      printf("\n");
      fflush(stdout);
    }
  }
  if (printer) printf("# Out of bounds values : %ld %s\n", totalWrong, totalWrong ? "FAILED" : "OK");
  for (int r = lo; r < hi; r++) {
    HIPT(hipSetDevice(devs[r]));
    HIPT(hipFree(sb[r]));
    HIPT(hipFree(rb[r]));
    HIPT(hipStreamDestroy(st[r]));
    NCCLT(ncclCommDestroy(comms[r]));
  }
  free(host);
  return totalWrong ? 1 : 0;
}
