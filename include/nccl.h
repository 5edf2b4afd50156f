/*
 * nccl.h — NCCL-compatible public C ABI of the MI355X-native reduction library
 * (libnbxccl.so).
 *
 * Every declaration below replaces the same-named entry point of the reference
 * NCCL 2.19.4 public header, /root/reference/src/nccl.h.in (cited per item), so
 * that a harness linked against NCCL (the NeuronaBox emulator) links against
 * this library unchanged. Enum VALUES are identical to the reference
 * (nccl.h.in:37-45 results, :181-197 ops, :199-214 types); the only additions
 * are the two OCP fp8 types, numbered as later NCCL releases number them.
 *
 * Streams are HIP streams (hipStream_t is an opaque pointer, as cudaStream_t
 * is). No torch types, no C++ types: plain pointers and sizes only.
 *
 * Every function also exists with a `p` prefix (pncclAllReduce, ...), the
 * profiling alias the reference exports via NCCL_API (src/include/core.h:17-32).
 */
#ifndef NBX_NCCL_H_
#define NBX_NCCL_H_

#include <stddef.h>
#include <stdint.h>
#include <limits.h>

#define NCCL_MAJOR 2
#define NCCL_MINOR 19
#define NCCL_PATCH 4
#define NCCL_SUFFIX ""
#define NCCL_VERSION_CODE 21904
#define NCCL_VERSION(X, Y, Z) \
  (((X) <= 2 && (Y) <= 8) ? (X)*1000 + (Y)*100 + (Z) : (X)*10000 + (Y)*100 + (Z))

#ifdef __cplusplus
extern "C" {
#endif

/* hipStream_t without pulling in the HIP headers (same opaque-pointer type). */
typedef struct ihipStream_t* ncclStream_t;

/* Opaque communicator handle — nccl.h.in:29 */
typedef struct ncclComm* ncclComm_t;
#define NCCL_COMM_NULL NULL

/* nccl.h.in:32-33 */
#define NCCL_UNIQUE_ID_BYTES 128
typedef struct { char internal[NCCL_UNIQUE_ID_BYTES]; } ncclUniqueId;

/* nccl.h.in:37-45 */
typedef enum {
  ncclSuccess = 0,
  ncclUnhandledCudaError = 1,
  ncclSystemError = 2,
  ncclInternalError = 3,
  ncclInvalidArgument = 4,
  ncclInvalidUsage = 5,
  ncclRemoteError = 6,
  ncclInProgress = 7,
  ncclNumResults = 8
} ncclResult_t;

#define NCCL_CONFIG_UNDEF_INT INT_MIN
#define NCCL_CONFIG_UNDEF_PTR NULL
#define NCCL_SPLIT_NOCOLOR -1

/* nccl.h.in:53-79 (layout identical) */
typedef struct ncclConfig_v21700 {
  size_t size;
  unsigned int magic;
  unsigned int version;
  int blocking;
  int cgaClusterSize;
  int minCTAs;
  int maxCTAs;
  const char* netName;
  int splitShare;
} ncclConfig_t;

#define NCCL_CONFIG_INITIALIZER {                               \
  sizeof(ncclConfig_t), 0xcafebeef,                             \
  NCCL_VERSION(NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH),             \
  NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,                 \
  NCCL_CONFIG_UNDEF_INT, NCCL_CONFIG_UNDEF_INT,                 \
  NCCL_CONFIG_UNDEF_PTR, NCCL_CONFIG_UNDEF_INT }

/* nccl.h.in:181-197 */
typedef enum { ncclNumOps_dummy = 5 } ncclRedOp_dummy_t;
typedef enum {
  ncclSum = 0,
  ncclProd = 1,
  ncclMax = 2,
  ncclMin = 3,
  ncclAvg = 4,
  ncclNumOps = 5,
  ncclMaxRedOp = 0x7fffffff >> (32 - 8 * sizeof(ncclRedOp_dummy_t))
} ncclRedOp_t;

/* nccl.h.in:199-214; fp8 (OCP e4m3fn / e5m2) are this build's additions,
 * numbered 10/11 as NCCL >= 2.24 numbers them. */
typedef enum {
  ncclInt8 = 0, ncclChar = 0,
  ncclUint8 = 1,
  ncclInt32 = 2, ncclInt = 2,
  ncclUint32 = 3,
  ncclInt64 = 4,
  ncclUint64 = 5,
  ncclFloat16 = 6, ncclHalf = 6,
  ncclFloat32 = 7, ncclFloat = 7,
  ncclFloat64 = 8, ncclDouble = 8,
  ncclBfloat16 = 9,
  ncclFloat8e4m3 = 10,
  ncclFloat8e5m2 = 11,
  ncclNumTypes = 12
} ncclDataType_t;

/* nccl.h.in:217-225 */
typedef enum {
  ncclScalarDevice = 0,
  ncclScalarHostImmediate = 1
} ncclScalarResidence_t;

/* ---- library / communicator lifecycle (nccl.h.in:94-177) ---- */
ncclResult_t  ncclGetVersion(int* version);                          /* :94  */
ncclResult_t pncclGetVersion(int* version);
ncclResult_t  ncclGetUniqueId(ncclUniqueId* uniqueId);               /* :100 */
ncclResult_t pncclGetUniqueId(ncclUniqueId* uniqueId);
ncclResult_t  ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId,
                                     int rank, ncclConfig_t* config); /* :105 */
ncclResult_t pncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId commId,
                                     int rank, ncclConfig_t* config);
ncclResult_t  ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank); /* :114 */
ncclResult_t pncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId commId, int rank);
ncclResult_t  ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist); /* :123 */
ncclResult_t pncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist);
ncclResult_t  ncclCommFinalize(ncclComm_t comm);                      /* :131 */
ncclResult_t pncclCommFinalize(ncclComm_t comm);
ncclResult_t  ncclCommDestroy(ncclComm_t comm);                       /* :135 */
ncclResult_t pncclCommDestroy(ncclComm_t comm);
ncclResult_t  ncclCommAbort(ncclComm_t comm);                         /* :140 */
ncclResult_t pncclCommAbort(ncclComm_t comm);
const char*   ncclGetErrorString(ncclResult_t result);                /* :154 */
const char*  pncclGetErrorString(ncclResult_t result);
const char*   ncclGetLastError(ncclComm_t comm);                      /* :160 */
const char*  pncclGetLastError(ncclComm_t comm);
ncclResult_t  ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError); /* :164 */
ncclResult_t pncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* asyncError);
ncclResult_t  ncclCommCount(const ncclComm_t comm, int* count);       /* :168 */
ncclResult_t pncclCommCount(const ncclComm_t comm, int* count);
ncclResult_t  ncclCommCuDevice(const ncclComm_t comm, int* device);   /* :172 */
ncclResult_t pncclCommCuDevice(const ncclComm_t comm, int* device);
ncclResult_t  ncclCommUserRank(const ncclComm_t comm, int* rank);     /* :176 */
ncclResult_t pncclCommUserRank(const ncclComm_t comm, int* rank);
ncclResult_t  ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm,
                            ncclConfig_t* config);                     /* :150 */
ncclResult_t pncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t* newcomm,
                            ncclConfig_t* config);
ncclResult_t  ncclMemAlloc(void** ptr, size_t size);                  /* :84  */
ncclResult_t pncclMemAlloc(void** ptr, size_t size);
ncclResult_t  ncclMemFree(void* ptr);                                 /* :87  */
ncclResult_t pncclMemFree(void* ptr);
ncclResult_t  ncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle); /* :430 */
ncclResult_t pncclCommRegister(const ncclComm_t comm, void* buff, size_t size, void** handle);
ncclResult_t  ncclCommDeregister(const ncclComm_t comm, void* handle); /* :434 */
ncclResult_t pncclCommDeregister(const ncclComm_t comm, void* handle);

/* ---- user reduction operators (nccl.h.in:237-248) ---- */
ncclResult_t  ncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                       ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t pncclRedOpCreatePreMulSum(ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
                                       ncclScalarResidence_t residence, ncclComm_t comm);
ncclResult_t  ncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);
ncclResult_t pncclRedOpDestroy(ncclRedOp_t op, ncclComm_t comm);

/* ---- reducing collectives: the hot path's callers ---- */
/* nccl.h.in:274-277 */
ncclResult_t  ncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                         ncclRedOp_t op, int root, ncclComm_t comm, ncclStream_t stream);
ncclResult_t pncclReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                         ncclRedOp_t op, int root, ncclComm_t comm, ncclStream_t stream);
/* nccl.h.in:315-318 */
ncclResult_t  ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                            ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                            ncclStream_t stream);
ncclResult_t pncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                            ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                            ncclStream_t stream);
/* nccl.h.in:331-336 */
ncclResult_t  ncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                                ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                                ncclStream_t stream);
ncclResult_t pncclReduceScatter(const void* sendbuff, void* recvbuff, size_t recvcount,
                                ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                                ncclStream_t stream);

/* ---- group semantics (nccl.h.in:416-427) ---- */
ncclResult_t  ncclGroupStart(void);
ncclResult_t pncclGroupStart(void);
ncclResult_t  ncclGroupEnd(void);
ncclResult_t pncclGroupEnd(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* NBX_NCCL_H_ */
