// comm_lifecycle.cc — communicator lifecycle beyond creation: ncclCommSplit
// (init.cc:2027-2085), ncclMemAlloc / ncclCommRegister, ncclCommFinalize /
// Destroy / Abort (init.cc:1986-2060), ncclCommGetAsyncError and the queries
// (init.cc:2091-2180).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include "nbx_comm.h"


using namespace nbxcomm;

// ncclCommSplit (init.cc:2027-2085, commGetSplitInfo init.cc:1303-1340): a
// collective over the parent. Every rank's (color, key) travels over the
// parent's bootstrap; the members of a color are ordered by key, ties by
// parent rank; the color's first member starts the child's bootstrap root
// and its unique id reaches the others in a second allgather; every member
// then initialises the child like ncclCommInitRankConfig (the parent's
// blocking mode unless `config` says otherwise). NCCL_SPLIT_NOCOLOR ranks take
// part in the allgathers and get NULL. Multi-process (and one-rank)
// communicators only: the ranks of an ncclCommInitAll clique are driven by
// one thread, which cannot join a collective rank by rank.
NBX_API(ncclResult_t, ncclCommSplit, ncclComm_t comm, int color, int key, ncclComm_t* newcomm, ncclConfig_t* config) {
  NCCLCHECK(commCheck(comm, "CommSplit"));
  if (newcomm == nullptr) {
    warn("CommSplit : newcomm argument is NULL");
    return ncclInvalidArgument;
  }
  NCCLCHECK(commEnsureReady(comm));
  *newcomm = nullptr;
  if (color < 0 && color != NCCL_SPLIT_NOCOLOR) {
    warn("CommSplit : invalid color %d", color);
    return ncclInvalidArgument;
  }
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  if (config == nullptr) {   // the parent's config (copyCommConfig, init.cc:1506-1510)
    cfg.blocking = comm->blocking;
    cfg.cgaClusterSize = comm->cgaClusterSize;
    cfg.splitShare = comm->splitShare;
    // min / max CTAs as a pair (a lone minCTAs would fail the reference's
    // config check in the child; an env-set one is read again there anyway)
    if (comm->maxCTAs != NCCL_CONFIG_UNDEF_INT) {
      cfg.maxCTAs = comm->maxCTAs;
      if (comm->minCTAs != NCCL_CONFIG_UNDEF_INT) cfg.minCTAs = comm->minCTAs;
    }
    config = &cfg;
  }
  DevGuard g(comm->device);
  if (comm->nRanks == 1) {
    if (color == NCCL_SPLIT_NOCOLOR) return ncclSuccess;
    ncclUniqueId id;
    NCCLCHECK(ncclGetUniqueId(&id));
    return ncclCommInitRankConfig(newcomm, 1, id, 0, config);
  }
  if (comm->mp == nullptr) {
    warn("CommSplit : communicators from ncclCommInitAll cannot be split here (one thread drives every rank)");
    return ncclInvalidUsage;
  }
  const int n = comm->nRanks, me = comm->rank;
  struct ColorKey {
    int32_t color, key;
  };
  const ColorKey mine{color, key};
  std::vector<ColorKey> ck(n);
  NCCLCHECK(nbx::bootstrapAllGather(comm->mp->bs, &mine, sizeof(mine), ck.data()));
  std::vector<int> members;   // parent ranks of my color, in child rank order
  if (color != NCCL_SPLIT_NOCOLOR) {
    for (int i = 0; i < n; i++) {
      if (ck[i].color != color) continue;
      size_t at = 0;
      while (at < members.size() && ck[members[at]].key <= ck[i].key) at++;
      members.insert(members.begin() + (long)at, i);
    }
  }
  struct IdMsg {
    int32_t color, leader;
    ncclUniqueId id;
  };
  IdMsg msg{};
  msg.color = color;
  msg.leader = !members.empty() && members[0] == me;
  if (msg.leader) NCCLCHECK(ncclGetUniqueId(&msg.id));
  std::vector<IdMsg> ids(n);
  NCCLCHECK(nbx::bootstrapAllGather(comm->mp->bs, &msg, sizeof(msg), ids.data()));
  if (color == NCCL_SPLIT_NOCOLOR) return ncclSuccess;
  const int myNew = (int)(std::find(members.begin(), members.end(), me) - members.begin());
  return ncclCommInitRankConfig(newcomm, (int)members.size(), ids[members[0]].id, myNew, config);
}

// ncclMemAlloc / ncclMemFree (nccl.h.in:84-87): device memory for
// communication buffers. NCCL uses cuMem allocations there so that NVLS and
// user-buffer registration can map them; plain device memory is what every
// path of this library uses.
NBX_API(ncclResult_t, ncclMemAlloc, void** ptr, size_t size) {
  if (ptr == nullptr) return ncclInvalidArgument;
  *ptr = nullptr;
  if (size == 0) return ncclSuccess;
  HIPCHECK(hipMalloc(ptr, size));
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclMemFree, void* ptr) {
  if (ptr != nullptr) HIPCHECK(hipFree(ptr));
  return ncclSuccess;
}

// ncclCommRegister / ncclCommDeregister (nccl.h.in:430-434): user-buffer
// registration is a zero-copy optimisation in NCCL; no path here needs it
// (peers only ever touch the connection buffers mapped at init), so a
// registration is a checked, owned handle and nothing else.
namespace {
struct RegHandle {
  uint64_t magic;
  ncclComm* comm;
  void* buff;
  size_t size;
};
constexpr uint64_t kRegMagic = 0x4e42585245474831ull;   // "NBXREGH1"
}  // namespace

NBX_API(ncclResult_t, ncclCommRegister, const ncclComm_t comm, void* buff, size_t size, void** handle) {
  NCCLCHECK(commCheck(comm, "CommRegister"));
  NCCLCHECK(commEnsureReady(comm));
  if (handle == nullptr || (buff == nullptr && size != 0)) {
    warn("CommRegister : invalid buffer %p / handle %p", buff, (void*)handle);
    return ncclInvalidArgument;
  }
  RegHandle* h = new (std::nothrow) RegHandle{kRegMagic, comm, buff, size};
  if (h == nullptr) return ncclSystemError;
  *handle = h;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommDeregister, const ncclComm_t comm, void* handle) {
  NCCLCHECK(commCheck(comm, "CommDeregister"));
  RegHandle* h = (RegHandle*)handle;
  if (h == nullptr || h->magic != kRegMagic || h->comm != comm) {
    warn("CommDeregister : %p is not a registration of comm %p", handle, (void*)comm);
    return ncclInvalidArgument;
  }
  h->magic = 0;
  delete h;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommFinalize, ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclCommFinalize"));
  NCCLCHECK(commEnsureReady(comm));
  return flushPending();
}

namespace {
ncclResult_t commFree(ncclComm* comm) {
  std::shared_ptr<Clique> c = comm->clique;
  comm->magic = 0;
  // calls still queued in this thread's open group die with the communicator
  t_groupMpComms.erase(std::remove(t_groupMpComms.begin(), t_groupMpComms.end(), comm), t_groupMpComms.end());
  mpFree(comm);
  if (comm->preScratch || !comm->preScratchOld.empty()) {
    DevGuard dg(comm->device);
    (void)hipDeviceSynchronize();
    if (comm->preScratch) (void)hipFree(comm->preScratch);
    for (void* p : comm->preScratchOld) (void)hipFree(p);
  }
  if (comm->preScratchFree) {
    DevGuard dg(comm->device);
    (void)hipEventDestroy(comm->preScratchFree);
  }
  if (c) {
    std::lock_guard<std::mutex> gp(g_pendMu);
    std::lock_guard<std::mutex> g(c->mu);
    int r = comm->rank;
    if (r >= 0 && r < c->n) c->pending[r].clear();
    if (r >= 0 && r < c->n) {
      c->comms[r] = nullptr;
      DevGuard dg(c->devs[r]);
      (void)hipEventDestroy(c->evEnter[r]);
      (void)hipEventDestroy(c->evReduced[r]);
      (void)hipEventDestroy(c->evDone[r]);
    }
  }
  delete comm;
  return ncclSuccess;
}
}  // namespace

NBX_API(ncclResult_t, ncclCommDestroy, ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;   // init.cc: NULL comm is a no-op
  NCCLCHECK(commCheck(comm, "ncclCommDestroy"));
  NCCLCHECK(commEnsureReady(comm));   // init.cc:1986-1987: the init thread must have finished
  return commFree(comm);
}

NBX_API(ncclResult_t, ncclCommAbort, ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  NCCLCHECK(commCheck(comm, "ncclCommAbort"));
  // every device wait of this rank polls the abort word; set first, so a
  // pending initialisation's kernels (the LL128 self-test) end too, not only
  // its bootstrap waits (the flag), before the init thread is joined
  if (comm->hostWords) __atomic_store_n(&comm->hostWords[0], 1, __ATOMIC_SEQ_CST);
  if (comm->initThread.joinable()) {
    __atomic_store_n(&comm->initAbort, 1, __ATOMIC_RELAXED);
    comm->initThread.join();
  }
  return commFree(comm);
}

NBX_API(ncclResult_t, ncclCommGetAsyncError, ncclComm_t comm, ncclResult_t* asyncError) {
  NCCLCHECK(commCheck(comm, "ncclGetAsyncError"));
  if (asyncError == nullptr) return ncclInvalidArgument;
  *asyncError = (ncclResult_t)comm->asyncError.load();
  // the transport pointer only after a finished initialisation: the init
  // thread's final asyncError store orders its assignment before this load
  if (*asyncError != ncclSuccess) return ncclSuccess;
  const MpState* mp = mpOf(comm);
  if (mp && mp->hostWords && mp->hostWords[1] != 0) {
    *asyncError = ncclRemoteError;   // a peer barrier timed out or was aborted
    mpReportDeviceError(comm);
  }
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommCount, const ncclComm_t comm, int* count) {
  NCCLCHECK(commCheck(comm, "CommCount"));
  NCCLCHECK(commEnsureReady(comm));
  if (count == nullptr) return ncclInvalidArgument;
  *count = comm->nRanks;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommCuDevice, const ncclComm_t comm, int* devid) {
  NCCLCHECK(commCheck(comm, "CommCuDevice"));
  NCCLCHECK(commEnsureReady(comm));
  if (devid == nullptr) return ncclInvalidArgument;
  *devid = comm->device;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommUserRank, const ncclComm_t comm, int* rank) {
  NCCLCHECK(commCheck(comm, "CommUserRank"));
  NCCLCHECK(commEnsureReady(comm));
  if (rank == nullptr) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}
