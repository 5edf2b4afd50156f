/*
 * nbx_reduce.h — internal C ABI of the MI355X reduction core.
 *
 * This is the hot path the library is built around: NCCL's device-side
 * multi-source element-wise reduction ("ReduceOrCopyMulti"),
 *   reduceCopy / reduceCopyPacks   /root/reference/src/device/common_kernel.h:28-239
 *   functors                       /root/reference/src/device/reduce_kernel.h:34-526
 *   one-rank launch                /root/reference/src/device/onerank.cu:48-79
 *   host op encoding               /root/reference/src/enqueue.cc:1436-1512
 * exposed as plain C so that the NCCL API layer, a multi-GPU sharder, a test
 * harness or an emulator can call it with raw device pointers.
 *
 * Semantics of nbxReduceMulti (identical to reduceCopy, common_kernel.h:79-158):
 *   for every element i in [0, count):
 *     acc = pre_0(srcs[0][i])
 *     for s = 1 .. nSrcs-1:  acc = Fn(acc, pre_s(srcs[s][i]))    (ordered left fold)
 *     if postOp:             acc = post(acc)
 *     for d in dsts:         dsts[d][i] = acc
 *   where pre_s is the PreMulSum pre-multiply for s < nPreOpSrcs (identity
 *   otherwise) and post is the SumPostDiv integer divide.
 */
#ifndef NBX_REDUCE_H_
#define NBX_REDUCE_H_

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device reduction opcode — /root/reference/src/include/device.h:26-30 (same order). */
typedef enum {
  nbxDevSum = 0,
  nbxDevProd = 1,
  nbxDevMinMax = 2,
  nbxDevPreMulSum = 3,
  nbxDevSumPostDiv = 4,
  nbxNumDevRedOps = 5
} nbxDevRedOp_t;

/* Full device op — /root/reference/src/include/device.h:31-36 (ncclDevRedOpFull).
 * scalarArg: MinMax xormask, PreMulSum scalar bits (element type, low bytes),
 * SumPostDiv divisor. If scalarArgIsPtr, scalarArg is a device address of the
 * PreMulSum scalar, dereferenced by the kernel while it runs (ncclScalarDevice,
 * common.h:100-119 / onerank.cu:32-42). */
typedef struct {
  int32_t op;             /* nbxDevRedOp_t */
  int32_t scalarArgIsPtr; /* bool */
  uint64_t scalarArg;
} nbxDevRedOpFull;

#define NBX_MAX_SRCS 64   /* > 8 sources run as ordered multi-pass folds (one source per rank up to 64) */
#define NBX_MAX_DSTS 8    /* NCCL_MAX_DIRECT_ARITY + 1 (device.h:147): local output + 7 peers */

/* Host-side op encoding: replaces hostToDevRedOp, enqueue.cc:1436-1512, for
 * the built-in ops (Sum/Prod/Max/Min/Avg). nRanks feeds ncclAvg. */
ncclResult_t nbxHostToDevRedOp(nbxDevRedOpFull* out, ncclRedOp_t op,
                               ncclDataType_t datatype, int nRanks);

/* The reduction core: replaces reduceCopy<...>(...) (common_kernel.h:183-239)
 * plus its kernel shell (onerank.cu:14-45, common.h:121-210).
 * Stream-ordered and asynchronous; returns once the kernel is enqueued.
 * count == 0 is a no-op. Any pointer alignment is accepted (16-B packs when
 * the pointers share one alignment, element packs otherwise — common_kernel.h:209-238).
 * Errors: ncclInvalidArgument for nSrcs outside [1, NBX_MAX_SRCS], nDsts
 * outside [1, NBX_MAX_DSTS], a NULL pointer with count > 0, a bad datatype,
 * op or op/type combination (SumPostDiv on floats: reduce_kernel.h:506-509);
 * ncclUnhandledCudaError if the launch fails. */
ncclResult_t nbxReduceMulti(void* const* dsts, int nDsts,
                            const void* const* srcs, int nSrcs,
                            size_t count, ncclDataType_t datatype,
                            nbxDevRedOpFull op, int nPreOpSrcs, int postOp,
                            ncclStream_t stream);

/* One bucket of a batched reduction (same meaning as nbxReduceMulti's arguments). */
typedef struct {
  void* const* dsts;
  int nDsts;
  const void* const* srcs;
  int nSrcs;
  size_t count;
} nbxReduceTask;

/* Batched form: nTasks independent buckets with one datatype and op, as if
 * nbxReduceMulti were called for each — the analogue of NCCL packing grouped
 * collectives into one kernel's work list (enqueue.cc:67-91
 * appendWorkElemColl, NCCL_MAX_WORK_ELEMENTS, device.h:230). Buckets with the
 * same source count (<= 8) and one shared pointer alignment run together
 * (46 to 101 single-destination buckets per launch, from 8 down to 2
 * sources), their tiles in one index space, so many small buckets fill the
 * GPU like one large one; large buckets of 3+ sources, > 8 sources or mixed
 * alignments run as single-bucket launches. Buckets must be independent: no bucket's destinations
 * may overlap another bucket's sources or destinations (they may run
 * concurrently, in any order). Every bucket is checked before anything is
 * enqueued; errors as nbxReduceMulti (nTasks < 0 or tasks == NULL with
 * nTasks > 0: ncclInvalidArgument). nTasks == 0 is a no-op. */
ncclResult_t nbxReduceMultiBatch(const nbxReduceTask* tasks, int nTasks,
                                 ncclDataType_t datatype, nbxDevRedOpFull op,
                                 int nPreOpSrcs, int postOp, ncclStream_t stream);

/* Host-staged form of nbxReduceMulti: sources and destinations in HOST memory
 * (pinned for full speed; pageable works), the path NCCL's NET/SHM transports
 * stage through (host-pinned proxy FIFOs net.cc:735/883, /dev/shm buffers
 * shm.cc:86-114) — where an emulator's proxy/net buffers live. Data is chunked
 * (NBX_HOST_CHUNK_BYTES per source, default 16 MiB) through a two-slot device
 * staging ring so H2D, the reduction and D2H of consecutive chunks overlap.
 * When every buffer is pinned and device-mapped (hipHostMalloc /
 * hipHostRegister), the kernel instead reads and writes them in place over
 * PCIe (zero-copy; env NBX_HOST_MODE=auto|staged|zerocopy, zerocopy on
 * pageable memory: ncclInvalidArgument).
 * Ordered after prior work on `stream`; BLOCKING: returns when every host
 * destination holds the result. Same semantics and errors as nbxReduceMulti. */
ncclResult_t nbxReduceMultiHost(void* const* hostDsts, int nDsts,
                                const void* const* hostSrcs, int nSrcs,
                                size_t count, ncclDataType_t datatype,
                                nbxDevRedOpFull op, int nPreOpSrcs, int postOp,
                                ncclStream_t stream);

/* Launch knobs (NCCL_NTHREADS / NCCL_MAX_NCHANNELS analogues, tuning.cc:12,
 * connect.cc:314): blocksPerCU caps the grid at CUs x blocksPerCU workgroups
 * (0 = default: 1 for big tiles, 3-5 for small; env NBX_BLOCKS_PER_CU);
 * variant 0 = auto tile choice, 1 = force small tiles (and, for sources
 * misaligned against the destinations, the 1-pack run-time-source-count
 * realigning kernel), 2 = force big tiles. */
ncclResult_t nbxSetLaunchConfig(int blocksPerCU, int variant);
ncclResult_t nbxGetLaunchConfig(int* blocksPerCU, int* variant);

/* Number of (datatype, device op) kernel sets compiled in (for the ABI test). */
int nbxKernelCount(void);

/* Version of the core ABI (bumped on incompatible changes). */
int nbxAbiVersion(void);

#ifdef __cplusplus
}
#endif

#endif /* NBX_REDUCE_H_ */
