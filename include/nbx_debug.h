/*
 * nbx_debug.h — test hooks of libnbxccl.so (no GPU needed).
 */
#ifndef NBX_DEBUG_H_
#define NBX_DEBUG_H_

#include "nccl.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Connects rank `rank` of `nranks` to the bootstrap root named by `id` (from
 * ncclGetUniqueId) and runs `rounds` allgathers of rank-stamped payloads of
 * varying length, verifying every contribution. Exercises the host bootstrap
 * that multi-process ncclCommInitRank uses (the role of src/bootstrap.cc). */
ncclResult_t nbxBootstrapSelfTest(const ncclUniqueId* id, int rank, int nranks, int rounds);

#ifdef __cplusplus
}
#endif

#endif /* NBX_DEBUG_H_ */
