/*
 * nbx_debug.h — test hooks of libnbxccl.so (no GPU needed).
 */
#ifndef NBX_DEBUG_H_
#define NBX_DEBUG_H_

#include <stdint.h>

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Connects rank `rank` of `nranks` to the bootstrap root named by `id` (from
 * ncclGetUniqueId) and runs `rounds` allgathers of rank-stamped payloads of
 * varying length, verifying every contribution. Exercises the host bootstrap
 * that multi-process ncclCommInitRank uses (the role of src/bootstrap.cc). */
ncclResult_t nbxBootstrapSelfTest(const ncclUniqueId* id, int rank, int nranks, int rounds);

/* The Simple protocol's kernels (direct schedule, or ring when `ring`) for n
 * "ranks" driven from ONE process on the current device: staging, flag words and
 * counters laid out as ncclCommInitRank lays them out, every rank's kernel on
 * its own stream, all n launches of a call running together (n x gridMax
 * workgroups must fit the GPU at once). kind 0 AllReduce, 1 ReduceScatter
 * (count = recvcount), 2 Reduce (to `root`); sends[r] / recvs[r] are rank r's
 * device buffers (recvs[r] may be NULL on Reduce non-roots). Runs one untimed
 * and `iters` timed calls; *msPerCall = mean device time per call. Returns an
 * ncclResult_t (ncclRemoteError if a device wait timed out). Tuning and tests
 * only: the multi-process communicator's data path without its processes. */
int nbxDebugSimpleRun(int n, int kind, int ring, size_t count, int datatype, int op, const void* const* sends,
                      void* const* recvs, int root, int gridMax, size_t sliceBytes, int slots, int prefetch,
                      int iters, float* msPerCall);

/* NCCL_PROTO parsing (tuning.cc:254-259 list syntax: "LL,LL128", "^Simple",
 * case-insensitive; NULL or "" = all): bit 0 LL, bit 1 LL128, bit 2 Simple. */
int nbxDebugProtoMask(const char* ncclProto);

/* The multi-process communicator's per-message protocol choice: 0 LL, 1 LL128
 * (one-shot), 2 Simple, 3 LL128 two-shot, for a message of slotBytes (per-rank
 * block for ReduceScatter) whose direct-schedule block is blockBytes;
 * twoShotKind = 1 for AllReduce / Reduce, 0 for ReduceScatter. */
int nbxDebugChooseProto(int protoMask, int twoShotKind, uint64_t slotBytes, uint64_t blockBytes, int nRanks,
                        uint64_t llMaxBytes, uint64_t ll128MaxBytes, uint64_t ll128OneShotMax);

/* The protocol set a communicator starts from for NCCL_PROTO = ncclProto
 * (NULL: unset) when its ranks span more than one GPU (multiGpu = 1) or share
 * one: across GPUs LL128 is left out unless NCCL_PROTO names it (not in a
 * "^list") or NBX_LL128_ACROSS_GPUS=1 — the reference enables LL128 by default
 * only on validated fabrics (tuning.cc:287-297). NBX_DEBUG_ASSUME_MULTI_GPU=1
 * (test hook) applies the gate to ranks sharing a GPU. */
int nbxDebugGatedProtoMask(const char* ncclProto, int multiGpu);

/* The protocol set a communicator runs with (bits as nbxDebugProtoMask): its
 * NCCL_PROTO at creation gated as nbxDebugGatedProtoMask, minus LL128 if the
 * creation-time LL128 self-test failed (multi-rank communicators and clique
 * ranks; -1 for others or a bad handle). NBX_LL128_SELFTEST_FAIL=1 makes that
 * self-test report a failure (test hook). */
int nbxDebugCommProtoMask(ncclComm_t comm);

/* The transport settings a communicator runs with (after NCCL_BUFFSIZE /
 * NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE / NCCL_MAX_NCHANNELS /
 * NCCL_MIN_NCHANNELS and the NBX_* overrides are applied at creation):
 * out[0] LL max bytes, [1] LL128 max bytes, [2] Simple slice bytes, [3] Simple
 * slots, [4] Simple grid, [5] LL grid cap, [6] LL128 grid cap, [7] group
 * batching, [8] connection buffers re-exported at creation because a peer's
 * IPC mapping of them showed other memory (verified before first use), [9]
 * plan checks on (NBX_CHECK_PLANS / NCCL_CHECK_POINTERS), [10] Simple slice
 * checksums on (NBX_CHECK_SLICES). Writes min(nOut, 11) values and returns that
 * count; -1 for a bad handle or a communicator without a multi-rank transport. */
int nbxDebugCommSettings(ncclComm_t comm, int64_t* out, int nOut);

/* Config D's xGMI transport alone, on a multi-process
 * communicator: an AllReduce-shaped call of the direct Simple schedule (forced
 * for any size and NCCL_ALGO) that moves every byte an AllReduce of `count`
 * elements moves between the ranks, with the fold reduced to a copy of the
 * own input; recvbuff receives junk. Collective (every rank, same count and
 * datatype), stream-ordered like ncclAllReduce. Measurement only. */
ncclResult_t nbxDebugTransportAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                                        ncclComm_t comm, ncclStream_t stream);

/* Per-link fabric rate of a multi-process communicator (the roofline config
 * D is priced against): each rank pushes (pull = 0, the Simple transport's
 * system-scope stores) or pulls (pull = 1, its system-scope loads)
 * bytesPerPeer to / from every peer's staging at once, in its own part of
 * each peer's slice area, on workgroupsPerPeer workgroups per peer (0: 32).
 * One kernel on `stream`; *bytesMovedPerPeer = the bytes one launch moves per
 * peer (bytesPerPeer rounded up to whole passes). Not ordered against
 * collectives and it overwrites the peers' staging: the caller keeps every
 * rank's communicator quiet around it. ncclInvalidArgument without a
 * multi-process transport. Measurement only. */
ncclResult_t nbxDebugLinkProbe(ncclComm_t comm, size_t bytesPerPeer, int pull, int workgroupsPerPeer,
                               ncclStream_t stream, size_t* bytesMovedPerPeer);

/* Stream ceilings in the caller's process (SURVEY §8(d) "a measured stream
 * ceiling"): kind 0 reads nSrcs == 8 buffers of `bytes` each with the hot
 * kernel's loads and tile (16-B nontemporal, 8 x 4 packs per lane, one
 * workgroup per CU) and stores nothing; kind 1 writes `bytes` to dst with its
 * stores (plain 16-B); kind 2 is the 8:1 mixed stream: the read kernel's
 * tile and the fold's schedule (dynamic tiles from 16 tiles per workgroup),
 * every load kept live without arithmetic, source 0 stored to dst (bytes per
 * source). Buffers 16-B aligned, bytes a multiple of 16;
 * blocksPerCU 0 = the production shape. Asynchronous on `stream` (a
 * hipStream_t). The 1:1 copy ceiling is nbxReduceMulti with one source. */
ncclResult_t nbxDebugStream(int kind, void* dst, const void* const* srcs, int nSrcs, size_t bytes, int blocksPerCU,
                            ncclStream_t stream);

/* A deliberately torn LL128 line against the collectives' own line reader
 * (nbx_ll.h l128Poll + l128FoldLine), one GPU: a writer kernel stores the
 * line's last 32 bytes, waits delayUs, then its first 32 bytes (tear = 1; 0
 * stores it whole); a reader kernel on another stream polls it. Returns 0 if
 * the reader folded exactly the new payload and (tear = 1) accepted the line
 * only after its second half was issued; 1 stale payload folded; 2 accepted
 * early; 3 the reader timed out; < 0 HIP error. *acceptAfterTornTicks =
 * acceptance time minus second-half issue time (100 MHz ticks). */
int nbxDebugLL128TearTest(int delayUs, int tear, long long* acceptAfterTornTicks);

/* Batched-reduce launch form (nbxReduceMultiBatch): 1 = work-list kernels
 * (bucket records in a table in device memory, or pinned host memory without
 * a large BAR, up to 384 buckets per launch; the default, env NBX_BATCH_LIST;
 * sets of <= 16 buckets that fit one kernel-argument table still use it),
 * 2 = work lists for every set, 0 = kernel-argument tables only; any other
 * value only queries. Returns the mode in force before the call. */
int nbxDebugSetBatchMode(int mode);

/* Work-list table slots of `device` in `state` (0 free, 1 read by an eager
 * launch that may still run, 2 owned by a captured graph); state 3: launches
 * so far that found no free slot and fell back to kernel-argument tables;
 * -1 bad device. */
int nbxDebugBatchListSlots(int device, int state);

/* Dynamic tile scheduling threshold of the big-tile reduce kernel: launches
 * with at least this many tiles per workgroup take tiles from the stream's
 * counter, shorter ones run the static grid stride (default 16, env
 * NBX_DYN_MIN_TILES_PER_WG; 1 makes every big-tile launch dynamic). Values < 1
 * only query. Returns the threshold in force before the call. */
int nbxDebugSetDynMinTiles(int tilesPerWorkgroup);

/* Per-stream counters allocated so far on `device` by the dynamic schedules
 * (which: 0 = big-tile reduce's tile counters, 1 = realigning kernel's class
 * counters); keyed by stream handle (nbx_reduce.cc). -1 bad device. */
int nbxDebugDynStreamSlots(int device, int which);

/* Holds `stream` with a one-wave kernel until nbxDebugReleaseStream(hold) or
 * timeoutMs pass, so a test can queue work behind it deterministically
 * (instead of racing a sleep against the host). Returns the hold (>= 0), -1
 * no free hold (16 at once) or bad timeout, -2 HIP error. Test hook. */
int nbxDebugHoldStream(ncclStream_t stream, int timeoutMs);
int nbxDebugReleaseStream(int hold);

#ifdef __cplusplus
}
#endif

#endif /* NBX_DEBUG_H_ */
