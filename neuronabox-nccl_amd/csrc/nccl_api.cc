// nccl_api.cc — the NCCL-compatible C ABI (include/nccl.h) over the MI355X
// reduction core (include/nbx_reduce.h): argument checks, op encoding, the
// one-rank path and the enqueue of the reducing collectives, plus their entry
// points, groups, user redops and error strings. The multi-rank transports
// live in comm_mp_init.cc / comm_mp_launch.cc (one process per GPU) and
// comm_clique.cc (ncclCommInitAll); the rest of the lifecycle in
// comm_lifecycle.cc (nbx_comm.h maps the units).
//
// Mirrors the reference's host path for the reducing collectives:
//   ncclAllReduce / ncclReduceScatter / ncclReduce   src/collectives.cc:29-124
//   ncclEnqueueCheck / ArgsCheck / PtrCheck           src/enqueue.cc:1613-1646, src/misc/argcheck.cc:28-75
//   hostToDevRedOp (op -> device op + scalar)         src/enqueue.cc:1436-1512
//   taskAppend nRanks==1 -> ncclLaunchOneRank          src/enqueue.cc:1564-1566, src/device/onerank.cu:48-79
//   ncclRedOpCreatePreMulSum / ncclRedOpDestroy       src/enqueue.cc:1648-1717
//   ncclUserRedOpMangle                               src/include/comm.h:456-467
//   ncclGetErrorString / ncclGetLastError             src/init.cc:2091-2112
//   ncclGroupStart / ncclGroupEnd                     src/group.cc:82-103
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include "nbx_comm.h"

namespace nbxcomm {

char g_lastError[1024] = "";
std::mutex g_errMu;

int debugLevel() {
  static int lvl = [] {
    const char* v = std::getenv("NCCL_DEBUG");
    if (!v) return 0;
    if (!strcasecmp(v, "VERSION")) return 1;
    if (!strcasecmp(v, "WARN")) return 2;
    if (!strcasecmp(v, "INFO")) return 3;
    if (!strcasecmp(v, "TRACE")) return 4;
    return 0;
  }();
  return lvl;
}

void warn(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  {
    std::lock_guard<std::mutex> g(g_errMu);
    std::snprintf(g_lastError, sizeof(g_lastError), "%s", buf);
  }
  if (debugLevel() >= 2) std::fprintf(stderr, "NCCL WARN %s\n", buf);
}

bool traceOn() {
  static bool on = [] { const char* v = std::getenv("NBX_TRACE"); return v && *v && *v != '0'; }();
  return on;
}

void info(const char* fmt, ...) {
  if (debugLevel() < 3) return;
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "NCCL INFO ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
}


int typeSize(ncclDataType_t t) {
  switch ((int)t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return -1;
  }
}


ncclResult_t commCheck(ncclComm* comm, const char* opName) {
  // PtrCheck(comm) — argcheck.cc:28-34
  if (comm == nullptr) {
    warn("%s : comm argument is NULL", opName);
    return ncclInvalidArgument;
  }
  if (comm->magic != kCommMagic) {
    warn("%s : comm %p is not a valid communicator", opName, (void*)comm);
    return ncclInvalidArgument;
  }
  return ncclSuccess;
}

// ncclCommEnsureReady (init.cc:287-305): an operation on a communicator needs
// its (non-blocking) initialisation finished and no asynchronous error; an
// initialisation still running is ncclInvalidArgument, any other error is
// returned as it is. A finished background initialisation is joined here.
ncclResult_t commEnsureReady(ncclComm* comm) {
  const ncclResult_t r = (ncclResult_t)comm->asyncError.load();
  if (r != ncclInProgress && comm->initThread.joinable()) comm->initThread.join();
  if (r == ncclSuccess) return ncclSuccess;
  warn("Attempt to use communicator before the previous operation returned ncclSuccess");
  return r == ncclInProgress ? ncclInvalidArgument : r;
}

// comm.h:456-467
ncclRedOp_t userRedOpMangle(ncclComm* comm, ncclRedOp_t op) {
  if ((int)op < (int)ncclNumOps) return op;
  uint64_t h = reinterpret_cast<uint64_t>(comm);
  h ^= h >> 32;
  h *= 0x9e3779b97f4a7c13ull;
  h >>= 32;
  h &= (uint64_t)ncclMaxRedOp;
  int op1 = (int)h ^ (int)op;
  // builtin values are preserved, so their preimage is too
  return op1 < (int)ncclNumOps ? op : (ncclRedOp_t)op1;
}


// hostToDevRedOp — enqueue.cc:1436-1512, including the user-op branch.
ncclResult_t hostToDevRedOp(nbxDevRedOpFull* opFull, ncclRedOp_t op, ncclDataType_t dt, ncclComm* comm) {
  if ((int)op < (int)ncclNumOps) return nbxHostToDevRedOp(opFull, op, dt, comm->nRanks);
  int ix = (int)userRedOpMangle(comm, op) - (int)ncclNumOps;
  std::lock_guard<std::mutex> g(comm->opsMu);
  if (ix < 0 || ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1) {
    warn("reduction operation %d unknown to this communicator", (int)op);
    return ncclInvalidArgument;
  }
  const UserRedOp& u = comm->userOps[ix];
  if (dt != u.datatype) {
    warn("Data type supplied to user-created ncclRedOp_t does not match type given to reduction operation");
    return ncclInvalidArgument;
  }
  *opFull = u.opFull;
  return ncclSuccess;
}

// ArgsCheck — argcheck.cc:36-75 (pointer checks only under NCCL_CHECK_POINTERS=1,
// as in the reference; NULL buffers with count > 0 are always rejected here).
ncclResult_t argsCheck(ncclComm* comm, const char* opName, const void* sendbuff, const void* recvbuff,
                       size_t count, ncclDataType_t dt, ncclRedOp_t op, int root, bool isReduce) {
  if (root < 0 || root >= comm->nRanks) {
    warn("%s : invalid root %d (root should be in the 0..%d range)", opName, root, comm->nRanks);
    return ncclInvalidArgument;
  }
  if ((int)dt < 0 || (int)dt >= (int)ncclNumTypes) {
    warn("%s : invalid type %d", opName, (int)dt);
    return ncclInvalidArgument;
  }
  if ((int)op < 0 || (int)ncclMaxRedOp < (int)op) {
    warn("%s : invalid reduction operation %d", opName, (int)op);
    return ncclInvalidArgument;
  }
  if ((int)op >= (int)ncclNumOps) {
    int ix = (int)userRedOpMangle(comm, op) - (int)ncclNumOps;
    std::lock_guard<std::mutex> g(comm->opsMu);
    if (ix < 0 || ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1) {
      warn("%s : reduction operation %d unknown to this communicator", opName, (int)op);
      return ncclInvalidArgument;
    }
  }
  if (count > 0) {
    if (sendbuff == nullptr) {
      warn("%s : sendbuff argument is NULL", opName);
      return ncclInvalidArgument;
    }
    if (recvbuff == nullptr && (!isReduce || comm->rank == root)) {
      warn("%s : recvbuff argument is NULL", opName);
      return ncclInvalidArgument;
    }
  }
  if (comm->checkPointers && count > 0) {
    const void* ptrs[2] = {sendbuff, recvbuff};
    const char* names[2] = {"sendbuff", "recvbuff"};
    for (int i = 0; i < 2; i++) {
      if (i == 1 && isReduce && comm->rank != root) continue;
      hipPointerAttribute_t attr;
      if (hipPointerGetAttributes(&attr, ptrs[i]) != hipSuccess || attr.devicePointer == nullptr) {
        warn("%s : %s %p is not a valid pointer", opName, names[i], ptrs[i]);
        return ncclInvalidArgument;
      }
      if (attr.type == hipMemoryTypeDevice && attr.device != comm->device) {
        warn("%s : %s allocated on device %d mismatchs with NCCL device %d", opName, names[i], attr.device,
             comm->device);
        return ncclInvalidArgument;
      }
    }
  }
  return ncclSuccess;
}

// ncclLaunchOneRank — onerank.cu:48-79: PreMulSum -> kernel (pre-op on the one
// source, postOp=true); every other op -> D2D copy, or nothing when in place.
ncclResult_t launchOneRank(void* dst, const void* src, size_t count, const nbxDevRedOpFull& op,
                           ncclDataType_t dt, hipStream_t stream) {
  if (count == 0) return ncclSuccess;
  if (op.op != nbxDevPreMulSum) {
    if (dst != src) HIPCHECK(hipMemcpyAsync(dst, src, count * (size_t)typeSize(dt), hipMemcpyDeviceToDevice, stream));
    return ncclSuccess;
  }
  void* dsts[1] = {dst};
  const void* srcs[1] = {src};
  return nbxReduceMulti(dsts, 1, srcs, 1, count, dt, op, /*nPreOpSrcs=*/1, /*postOp=*/1, (ncclStream_t)stream);
}


// localPre (PendingColl): scratch = x * s on c->stream, then the collective
// sums the scratch. Scratch grows by doubling (the exact size when the doubled
// allocation fails) and superseded buffers are kept while the communicator
// lives (an earlier call, possibly on another stream, may still read the old
// buffer); growing is refused inside a stream capture — one eager call of the
// size first, as graph capture of NCCL calls expects anyway. The pre-pass
// first waits for the event recorded behind the last call that read the
// scratch (preScratchDone): peers' folds of the previous PreMulSum may still
// read it, on any stream. A captured pre-pass does not wait on that eager
// event (the graph's own edges order captured calls): a graph holding a
// PreMulSum must not be replayed while an eager PreMulSum of the same
// communicator runs (the one scratch buffer is shared).
ncclResult_t localPreOp(ncclComm* comm, int device, PendingColl* c, int nRanks) {
  const size_t eb = (size_t)typeSize(c->dt);
  const size_t elts = c->kind == kReduceScatter ? c->count * (size_t)nRanks : c->count;
  const size_t bytes = elts * eb;
  DevGuard g(device);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(c->stream, &cap));
  if (comm->preScratchBytes < bytes) {
    if (cap != hipStreamCaptureStatusNone) {
      warn("user PreMulSum of %zu bytes inside a stream capture needs its scratch first: run one eager call of "
           "that size on this communicator before capturing", bytes);
      return ncclInvalidUsage;
    }
    size_t want = std::max<size_t>(bytes, std::max<size_t>(2 * comm->preScratchBytes, 1u << 20));
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
      (void)hipGetLastError();
      want = bytes;   // the doubled size does not fit: the exact one may
      HIPCHECK(hipMalloc(&p, want));
    }
    if (comm->preScratch) comm->preScratchOld.push_back(comm->preScratch);
    comm->preScratch = p;
    comm->preScratchBytes = want;
  } else if (comm->preScratchPending && cap == hipStreamCaptureStatusNone) {
    HIPCHECK(hipStreamWaitEvent(c->stream, comm->preScratchFree, 0));
  }
  void* dsts[1] = {comm->preScratch};
  const void* srcs[1] = {c->send};
  NCCLCHECK(nbxReduceMulti(dsts, 1, srcs, 1, elts, c->dt, c->op, /*nPreOpSrcs=*/1, /*postOp=*/0,
                           (ncclStream_t)c->stream));
  c->send = comm->preScratch;
  c->op = nbxDevRedOpFull{nbxDevSum, 0, 0};
  c->localPre = false;
  return ncclSuccess;
}

// Behind the last reader of the scratch a pre-pass filled (the collective's
// own kernel, and on a clique every peer's fold: called after the leave step),
// on that call's stream; eager calls only.
ncclResult_t preScratchDone(ncclComm* comm, int device, hipStream_t stream) {
  DevGuard g(device);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(stream, &cap));
  if (cap != hipStreamCaptureStatusNone) return ncclSuccess;
  if (comm->preScratchFree == nullptr) HIPCHECK(hipEventCreateWithFlags(&comm->preScratchFree, hipEventDisableTiming));
  HIPCHECK(hipEventRecord(comm->preScratchFree, stream));
  comm->preScratchPending = true;
  return ncclSuccess;
}

// ---------------------------------------------------------------------------
// Group semantics (group.cc:82-103 depth is thread-local). One-rank
// collectives launch at enqueue, as in the reference (taskAppend returns after
// ncclLaunchOneRank); in-process multi-rank collectives are queued and run
// when every rank has enqueued its part and the outermost group ends.

thread_local int t_groupDepth = 0;


// Element range of block b when `count` is split over n ranks, aligned so
// every block starts on a 16-byte boundary relative to the buffer.
void blockRange(size_t count, int eb, int n, int b, size_t* off, size_t* len) {
  const size_t epp = (size_t)(16 / eb);
  size_t per = (count + (size_t)n - 1) / (size_t)n;
  per = (per + epp - 1) / epp * epp;
  size_t lo = per * (size_t)b;
  if (lo > count) lo = count;
  size_t hi = lo + per;
  if (hi > count) hi = count;
  *off = lo;
  *len = hi - lo;
}


// ncclEnqueueCheck + taskAppend for the reducing collectives.
ncclResult_t enqueueColl(CollKind kind, const char* opName, const void* sendbuff, void* recvbuff, size_t count,
                         ncclDataType_t dt, ncclRedOp_t op, int root, ncclComm* comm, hipStream_t stream) {
  NCCLCHECK(commCheck(comm, opName));
  NCCLCHECK(commEnsureReady(comm));
  NCCLCHECK(argsCheck(comm, opName, sendbuff, recvbuff, count, dt, op, root, kind == kReduce));
  info("%s: sendbuff %p recvbuff %p count %zu datatype %d op %d root %d comm %p [nranks=%d] stream %p", opName,
       sendbuff, (void*)recvbuff, count, (int)dt, (int)op, root, (void*)comm, comm->nRanks, (void*)stream);
  nbxDevRedOpFull opFull;
  NCCLCHECK(hostToDevRedOp(&opFull, op, dt, comm));   // op state copied at enqueue (enqueue.cc:1557-1562)
  if (comm->nRanks == 1) {
    DevGuard g(comm->device);
    ncclResult_t r = launchOneRank(recvbuff, sendbuff, count, opFull, dt, stream);
    if (r != ncclSuccess) comm->asyncError.store(r);
    return r;
  }
  // a user PreMulSum: the scalar is this rank's alone (PendingColl::localPre)
  const bool localPre = (int)op >= (int)ncclNumOps && opFull.op == nbxDevPreMulSum;
  if (comm->mp) {
    MpCall call{kind, sendbuff, recvbuff, count, dt, opFull, root, stream};
    call.localPre = localPre;
    if (t_groupDepth > 0) {   // run at the outermost ncclGroupEnd
      if (comm->mp->group.empty()) t_groupMpComms.push_back(comm);
      comm->mp->group.push_back(call);
      return ncclSuccess;
    }
    DevGuard g(comm->device);
    ncclResult_t r;
    try {
      r = runMpColl(comm, call);
    } catch (const std::exception& e) {
      warn("internal exception: %s", e.what());
      r = ncclInternalError;
    }
    if (r != ncclSuccess) comm->asyncError.store(r);
    return r;
  }
  {
    std::lock_guard<std::mutex> g(g_pendMu);
    PendingColl pc{kind, sendbuff, recvbuff, count, dt, opFull, root, stream};
    pc.localPre = localPre;
    comm->clique->pending[comm->rank].push_back(pc);
  }
  if (t_groupDepth == 0) return flushPending();
  return ncclSuccess;
}

ncclResult_t parseConfig(const ncclConfig_t* config, ncclConfig_t* out) {
  const ncclConfig_t dflt = NCCL_CONFIG_INITIALIZER;
  *out = dflt;
  if (config == nullptr) return ncclSuccess;
  size_t realSize = 0;
  std::memcpy(&realSize, config, sizeof(size_t));
  if (realSize > sizeof(ncclConfig_t)) realSize = sizeof(ncclConfig_t);
  std::memcpy((void*)out, config, realSize);
  if (out->magic != 0xcafebeef) {
    warn("ncclConfig_t argument not initialized via NCCL_CONFIG_INITIALIZER");
    return ncclInvalidArgument;
  }
  if (out->version < NCCL_VERSION(2, 14, 0)) out->blocking = dflt.blocking;
  if (out->version < NCCL_VERSION(2, 17, 0)) {
    out->cgaClusterSize = dflt.cgaClusterSize;
    out->minCTAs = dflt.minCTAs;
    out->maxCTAs = dflt.maxCTAs;
    out->netName = dflt.netName;
  }
  if (out->blocking != NCCL_CONFIG_UNDEF_INT && out->blocking != 0 && out->blocking != 1) {
    warn("Invalid config blocking attribute value %d", out->blocking);
    return ncclInvalidArgument;
  }
  if (out->cgaClusterSize != NCCL_CONFIG_UNDEF_INT && out->cgaClusterSize < 0) {
    warn("Invalid config cgaClusterSize attribute value %d", out->cgaClusterSize);
    return ncclInvalidArgument;
  }
  // as the reference: an unset maxCTAs is INT_MIN here, so minCTAs alone fails
  // this check too (init.cc:1555-1563)
  if ((out->minCTAs != NCCL_CONFIG_UNDEF_INT && out->minCTAs <= 0) ||
      (out->maxCTAs != NCCL_CONFIG_UNDEF_INT && out->maxCTAs <= 0) || out->minCTAs > out->maxCTAs) {
    warn("Invalid config min/max channels attribute value %d/%d", out->minCTAs, out->maxCTAs);
    return ncclInvalidArgument;
  }
  if (out->splitShare != NCCL_CONFIG_UNDEF_INT && out->splitShare != 0 && out->splitShare != 1) {
    warn("Invalid config splitShare attribute value %d", out->splitShare);
    return ncclInvalidArgument;
  }
  return ncclSuccess;
}

ncclResult_t newComm(ncclComm** out, int nRanks, int rank, int dev, const ncclConfig_t* config) {
  ncclComm* c = new (std::nothrow) ncclComm();
  if (c == nullptr) return ncclSystemError;
  c->nRanks = nRanks;
  c->rank = rank;
  c->device = dev;
  const char* cp = std::getenv("NCCL_CHECK_POINTERS");
  c->checkPointers = cp && std::atoi(cp) != 0;
  if (nRanks > 1) {
    DevGuard g(dev);
    if (hipHostMalloc((void**)&c->hostWords, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->hostWordsDev, c->hostWords, 0) != hipSuccess) {
      warn("cannot allocate the communicator's pinned wait words");
      delete c;
      return ncclUnhandledCudaError;
    }
    std::memset(c->hostWords, 0, 64);
  }
  if (config) {   // checked by parseConfig already
    if (config->blocking != NCCL_CONFIG_UNDEF_INT) c->blocking = config->blocking;
    c->minCTAs = config->minCTAs;
    c->maxCTAs = config->maxCTAs;
    c->cgaClusterSize = config->cgaClusterSize;
    c->splitShare = config->splitShare;
  }
  // envConfigOverride (init.cc:1437-1494): the environment overrides the config
  if (const char* be = std::getenv("NCCL_COMM_BLOCKING")) {   // init.cc:1444-1446
    char* end = nullptr;
    const long v = std::strtol(be, &end, 10);
    if (end != be && *end == '\0' && (v == 0 || v == 1)) c->blocking = (int)v;
  }
  auto envInt = [](const char* name, int* field) {
    const char* v = std::getenv(name);
    if (v == nullptr || *v == 0) return;
    char* end = nullptr;
    const long x = std::strtol(v, &end, 10);
    if (end != v && *end == '\0') *field = (int)x;
  };
  envInt("NCCL_MIN_CTAS", &c->minCTAs);
  envInt("NCCL_MAX_CTAS", &c->maxCTAs);
  if (c->minCTAs != NCCL_CONFIG_UNDEF_INT && c->maxCTAs != NCCL_CONFIG_UNDEF_INT && c->minCTAs > c->maxCTAs) {
    warn("minCTAs %d is larger than maxCTAs %d, set both to %d", c->minCTAs, c->maxCTAs, c->maxCTAs);
    c->minCTAs = c->maxCTAs;
  }
  *out = c;
  return ncclSuccess;
}

}  // namespace nbxcomm

using namespace nbxcomm;

// ===========================================================================
// Public C ABI

NBX_API(ncclResult_t, ncclGetVersion, int* version) {
  if (version == nullptr) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

NBX_API(const char*, ncclGetErrorString, ncclResult_t code) {
  switch (code) {   // init.cc:2091-2104
    case ncclSuccess: return "no error";
    case ncclUnhandledCudaError: return "unhandled cuda error (run with NCCL_DEBUG=INFO for details)";
    case ncclSystemError: return "unhandled system error (run with NCCL_DEBUG=INFO for details)";
    case ncclInternalError: return "internal error - please report this issue to the NCCL developers";
    case ncclInvalidArgument: return "invalid argument (run with NCCL_DEBUG=WARN for details)";
    case ncclInvalidUsage: return "invalid usage (run with NCCL_DEBUG=WARN for details)";
    case ncclRemoteError: return "remote process exited or there was a network error";
    case ncclInProgress: return "NCCL operation in progress";
    default: return "unknown result code";
  }
}

NBX_API(const char*, ncclGetLastError, ncclComm_t comm) {
  (void)comm;
  return g_lastError;
}

NBX_API(ncclResult_t, ncclRedOpCreatePreMulSum, ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
        ncclScalarResidence_t residence, ncclComm_t comm) {
  // enqueue.cc:1648-1685
  NCCLCHECK(commCheck(comm, "ncclRedOpCreatePreMulSum"));
  NCCLCHECK(commEnsureReady(comm));
  if (op == nullptr || scalar == nullptr) return ncclInvalidArgument;
  const int sz = typeSize(datatype);
  if (sz < 0) return ncclInvalidArgument;
  std::lock_guard<std::mutex> g(comm->opsMu);
  if (comm->freeHead == (int)comm->userOps.size()) {
    int cap = 2 * (int)comm->userOps.size();
    if (cap < 4) cap = 4;
    int old = (int)comm->userOps.size();
    comm->userOps.resize(cap);
    for (int ix = old; ix < cap; ix++) comm->userOps[ix].freeNext = ix + 1;
  }
  int ix = comm->freeHead;
  UserRedOp& u = comm->userOps[ix];
  comm->freeHead = u.freeNext;
  u.freeNext = -1;
  u.datatype = datatype;
  u.opFull.op = nbxDevPreMulSum;
  if (residence == ncclScalarHostImmediate) {
    u.opFull.scalarArgIsPtr = 0;
    u.opFull.scalarArg = 0;
    std::memcpy(&u.opFull.scalarArg, scalar, (size_t)sz);
  } else {
    u.opFull.scalarArgIsPtr = 1;
    u.opFull.scalarArg = reinterpret_cast<uint64_t>(scalar);
  }
  *op = userRedOpMangle(comm, (ncclRedOp_t)((int)ncclNumOps + ix));
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclRedOpDestroy, ncclRedOp_t op, ncclComm_t comm) {
  // enqueue.cc:1687-1717
  if (0 <= (int)op && (int)op < (int)ncclNumOps) {
    warn("ncclRedOpDestroy : operator is a NCCL builtin.");
    return ncclInvalidArgument;
  }
  if ((int)op < 0 || (int)ncclMaxRedOp < (int)op) {
    warn("ncclRedOpDestroy :  operator is garbage.");
    return ncclInvalidArgument;
  }
  if (comm == nullptr) {
    warn("ncclRedOpDestroy : invalid communicator passed.");
    return ncclInvalidArgument;
  }
  NCCLCHECK(commCheck(comm, "ncclRedOpDestroy"));
  int ix = (int)userRedOpMangle(comm, op) - (int)ncclNumOps;
  std::lock_guard<std::mutex> g(comm->opsMu);
  if (ix < 0 || ix >= (int)comm->userOps.size() || comm->userOps[ix].freeNext != -1) {
    warn("ncclRedOpDestroy : operator unknown to this communicator.");
    return ncclInvalidArgument;
  }
  comm->userOps[ix].freeNext = comm->freeHead;
  comm->freeHead = ix;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclAllReduce, const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
        ncclRedOp_t op, ncclComm_t comm, ncclStream_t stream) {
  return enqueueColl(kAllReduce, "AllReduce", sendbuff, recvbuff, count, datatype, op, 0, comm,
                     (hipStream_t)stream);
}

NBX_API(ncclResult_t, ncclReduceScatter, const void* sendbuff, void* recvbuff, size_t recvcount,
        ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm, ncclStream_t stream) {
  return enqueueColl(kReduceScatter, "ReduceScatter", sendbuff, recvbuff, recvcount, datatype, op, 0, comm,
                     (hipStream_t)stream);
}

NBX_API(ncclResult_t, ncclReduce, const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
        ncclRedOp_t op, int root, ncclComm_t comm, ncclStream_t stream) {
  return enqueueColl(kReduce, "Reduce", sendbuff, recvbuff, count, datatype, op, root, comm,
                     (hipStream_t)stream);
}

NBX_API(ncclResult_t, ncclGroupStart) {
  t_groupDepth++;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclGroupEnd) {
  if (t_groupDepth == 0) {
    warn("ncclGroupEnd: not in a group call.");
    return ncclInvalidUsage;
  }
  if (--t_groupDepth > 0) return ncclSuccess;
  ncclResult_t r = flushPending();
  ncclResult_t r2 = flushMpGroups();
  return r != ncclSuccess ? r : r2;
}
