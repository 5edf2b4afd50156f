// nbx_bootstrap.h — minimal single-node TCP bootstrap for multi-process
// communicators (replaces the role of src/bootstrap.cc: unique-id root,
// allgather of per-rank blobs). A root thread, started by ncclGetUniqueId in
// the calling process, relays fixed-size allgather rounds between the ranks
// (star topology over loopback / the interface in NBX_BOOTSTRAP_ADDR).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/nccl.h"

namespace nbx {

// Fills `id` (magic, random key, IPv4 address, port) and starts the root
// thread. Returns ncclSystemError on socket failure.
ncclResult_t bootstrapCreateRoot(ncclUniqueId* id);

// True if `id` carries a bootstrap root address (multi-process capable).
bool bootstrapIdHasRoot(const ncclUniqueId& id);

struct Bootstrap;

// Connect rank `rank` of `nranks` to the root named by `id`.
ncclResult_t bootstrapConnect(const ncclUniqueId& id, int rank, int nranks, Bootstrap** out);

// All ranks contribute `len` bytes; `all` receives nranks * len bytes in rank order.
ncclResult_t bootstrapAllGather(Bootstrap* b, const void* mine, size_t len, void* all);

void bootstrapClose(Bootstrap* b);

// The calling thread's bootstrap waits (connect, every send / receive) also
// end, with ncclRemoteError, once *flag != 0 — how ncclCommAbort stops a
// non-blocking communicator's initialisation thread. nullptr: no flag.
void bootstrapSetAbortFlag(const int* flag);

}  // namespace nbx
