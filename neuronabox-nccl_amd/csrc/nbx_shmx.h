// nbx_shmx.h — host-side per-call exchange through POSIX shared memory for the
// multi-process communicator (all ranks on one node). Replaces the TCP
// bootstrap round trip of the Simple path's per-call allgather of buffer
// handles (NCCL's collectives "may perform inter-CPU synchronization",
// nccl.h.in:253-261) with a few cache-line writes and polls.
//
// Layout: header | ack[n] (cache line each) | slot[n] (cache line aligned)
//   slot[r] = {atomic u64 seq, u64 len, payload}
// Exchange s by rank r: wait until every ack[j] >= the previous exchange's
// seq (nobody still reads r's old payload), write the payload, publish
// slot[r].seq = s (release); wait until every slot[j].seq == s (acquire), copy
// the payloads, publish ack[r] = s. Every wait is bounded (timeout, abort word).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/nccl.h"

namespace nbx {

struct ShmExchange;

// Rank 0 creates (`create`), the others attach to, the segment `name` for n
// ranks and payloads up to maxLen bytes. nullptr on failure.
ShmExchange* shmxOpen(const char* name, int rank, int n, size_t maxLen, bool create);
// Removes the name (the mappings stay valid); call once every rank attached.
void shmxUnlink(const char* name);
// All ranks contribute len (<= maxLen) bytes for exchange number `seq`
// (strictly increasing, identical on every rank); `all` gets n * len bytes.
ncclResult_t shmxAllGather(ShmExchange* x, uint64_t seq, const void* mine, size_t len, void* all, double timeoutSec,
                           const volatile int* abortWord);
void shmxClose(ShmExchange* x);

}  // namespace nbx
