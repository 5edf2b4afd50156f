// nccl_api.cc — the NCCL-compatible C ABI (include/nccl.h) over the MI355X
// reduction core (include/nbx_reduce.h).
//
// Mirrors the reference's host path for the reducing collectives:
//   ncclAllReduce / ncclReduceScatter / ncclReduce   src/collectives.cc:29-124
//   ncclEnqueueCheck / ArgsCheck / PtrCheck           src/enqueue.cc:1613-1646, src/misc/argcheck.cc:28-75
//   hostToDevRedOp (op -> device op + scalar)         src/enqueue.cc:1436-1512
//   taskAppend nRanks==1 -> ncclLaunchOneRank          src/enqueue.cc:1564-1566, src/device/onerank.cu:48-79
//   ncclRedOpCreatePreMulSum / ncclRedOpDestroy       src/enqueue.cc:1648-1717
//   ncclUserRedOpMangle                               src/include/comm.h:456-467
//   ncclGetErrorString / ncclGetLastError             src/init.cc:2091-2112
// and, for nRanks > 1 inside one process (ncclCommInitAll, init.cc:1678-1734),
// replaces NCCL's ring schedule (all_reduce.h:13-95, reduce_scatter.h:13-66)
// with a direct one-shot exchange over xGMI peer access: rank r's kernel reads
// block r of every rank's send buffer (nSrcs = nRanks, the CollNet-direct
// shape all_reduce.h:318-327), folding in ring order r+1, r+2, ..., r — the
// order in which NCCL's ring reduce-scatter accumulates block r — and, for
// AllReduce, storing the finished block into every rank's output from the
// same kernel (push-gather, all_reduce.h:343-360). Cross-device ordering is by
// HIP events (stream-ordered, asynchronous, graph-capturable), not spin flags.
// One process per GPU (ncclCommInitRank, nranks > 1) runs the same schedules
// over hipIpc-mapped peer buffers with device flag barriers, plus the LL /
// LL128 protocols for small / medium messages (nbx_ll.h).
#include <hip/hip_runtime_api.h>

#include <array>
#include <atomic>
#include <exception>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <unistd.h>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../include/nbx_debug.h"
#include "../../include/nbx_reduce.h"
#include "nbx_bootstrap.h"
#include "nbx_internal.h"
#include "nbx_ll_args.h"
#include "nbx_diag.h"

#define NBX_EXPORT extern "C" __attribute__((visibility("default")))
// NCCL_API (src/include/core.h:17-32): every entry point plus a p-prefixed alias.
#define NBX_API(ret, func, ...)                                                     \
  NBX_EXPORT ret func(__VA_ARGS__);                                                 \
  NBX_EXPORT __attribute__((alias(#func))) ret p##func(__VA_ARGS__);                \
  NBX_EXPORT ret func(__VA_ARGS__)

namespace {

// ---------------------------------------------------------------------------
// Logging (NCCL_DEBUG=WARN|INFO, debug.cc:26-147) and last-error string.

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
#define NBX_TRACE(...)                                   \
  do {                                                   \
    if (traceOn()) {                                     \
      std::fprintf(stderr, "[nbx] " __VA_ARGS__);        \
      std::fprintf(stderr, "\n");                        \
      std::fflush(stderr);                               \
    }                                                    \
  } while (0)

void info(const char* fmt, ...) {
  if (debugLevel() < 3) return;
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "NCCL INFO ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
}

#define HIPCHECK(cmd)                                                         \
  do {                                                                        \
    hipError_t e_ = (cmd);                                                    \
    if (e_ != hipSuccess) {                                                   \
      warn("HIP failure '%s' at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
      return ncclUnhandledCudaError;                                          \
    }                                                                         \
  } while (0)
#define NCCLCHECK(cmd)                          \
  do {                                          \
    ncclResult_t r_ = (cmd);                    \
    if (r_ != ncclSuccess) return r_;           \
  } while (0)

int typeSize(ncclDataType_t t) {
  switch ((int)t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return -1;
  }
}

// ---------------------------------------------------------------------------
// Communicator.

constexpr uint64_t kCommMagic = 0x4e42584343434f4dull;  // "NBXCCCOM"
constexpr char kIdMagic[8] = {'N', 'B', 'X', 'U', 'I', 'D', '0', '1'};

struct UserRedOp {   // comm.h ncclUserRedOp
  int freeNext;      // -1 = allocated
  ncclDataType_t datatype;
  nbxDevRedOpFull opFull;
};

struct Clique;
struct MpState;

}  // namespace

struct ncclComm {
  uint64_t magic = kCommMagic;
  int nRanks = 1;
  int rank = 0;
  int device = 0;
  int blocking = 1;
  bool checkPointers = false;
  std::atomic<int> asyncError{ncclSuccess};
  std::mutex opsMu;
  std::vector<UserRedOp> userOps;
  int freeHead = 0;
  std::shared_ptr<Clique> clique;  // nRanks > 1 (single process)
  MpState* mp = nullptr;           // nRanks > 1 (one process per rank)
  MpState* lt = nullptr;           // clique rank: in-process LL / LL128 transport (cliqueInitTransport)
  std::thread initThread;         // non-blocking ncclCommInitRankConfig: mpInit in the background
  int initAbort = 0;               // set by ncclCommAbort: the init thread's bootstrap waits end
  // pinned, device-mapped words every device wait of this rank polls: [0]
  // abort, [1] error, diag record at byte 16 (nbx_diag.h). Owned here, not by
  // the transport state, so ncclCommAbort can end a wait of a background
  // initialisation (the LL128 self-test's kernels) before it joins that thread.
  int* hostWords = nullptr;
  int* hostWordsDev = nullptr;
  ~ncclComm() {
    if (hostWords) (void)hipHostFree(hostWords);
  }
};

namespace {

// In-process clique (ncclCommInitAll): per-rank streams are the caller's; the
// clique owns the events used to order the exchange across devices.
enum CollKind { kAllReduce, kReduceScatter, kReduce };

struct PendingColl {
  CollKind kind;
  const void* send;
  void* recv;
  size_t count;   // AllReduce/Reduce: count; ReduceScatter: recvcount
  ncclDataType_t dt;
  nbxDevRedOpFull op;
  int root;
  hipStream_t stream;
};

struct Clique {
  int n = 0;
  bool ll = false;       // LL / LL128-sized calls run in-kernel (every rank has comm->lt)
  bool simple = false;   // and Simple-sized calls too (every rank's lt has Simple staging) ...
  uint64_t simpleMaxBytes = 0;   // ... up to this many bytes per rank's send buffer (NBX_CLIQUE_SIMPLE_MAX_BYTES)
  std::vector<ncclComm*> comms;
  std::vector<int> devs;
  std::vector<hipEvent_t> evEnter, evReduced, evDone;   // one per rank
  std::vector<std::deque<PendingColl>> pending;         // per-rank FIFO of enqueued parts
  std::mutex mu;
};

// Live cliques (weak: a clique dies with its last communicator). Guarded by
// g_pendMu together with every clique's pending queues.
std::mutex g_pendMu;
std::vector<std::weak_ptr<Clique>> g_cliques;

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

class DevGuard {
 public:
  explicit DevGuard(int dev) {
    if (hipGetDevice(&old_) != hipSuccess) old_ = -1;
    if (old_ != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (old_ >= 0) (void)hipSetDevice(old_);
  }

 private:
  int old_ = -1;
};

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

// Every rank of the clique enqueued the same collective.
bool sameCollective(const std::vector<PendingColl>& parts) {
  const PendingColl& p0 = parts[0];
  for (size_t r = 1; r < parts.size(); r++)
    if (parts[r].kind != p0.kind || parts[r].count != p0.count || parts[r].dt != p0.dt ||
        parts[r].root != p0.root || parts[r].op.op != p0.op.op)
      return false;
  return true;
}

// Rank r's share of one collective: block r of every send buffer, in fold
// order, and where the folded block goes (both communicator kinds).
struct RankBlock {
  std::vector<const void*> srcs;
  std::vector<void*> dsts;
  size_t len = 0;
};

RankBlock cliqueBlock(const std::vector<PendingColl>& parts, int n, int r) {
  const PendingColl& p0 = parts[0];
  const int eb = typeSize(p0.dt);
  const size_t total = p0.kind == kReduceScatter ? p0.count * (size_t)n : p0.count;
  RankBlock cb;
  size_t off;
  if (p0.kind == kReduceScatter) {
    off = (size_t)r * p0.count;
    cb.len = p0.count;
  } else {
    blockRange(total, eb, n, r, &off, &cb.len);
  }
  if (cb.len == 0) return cb;
  // fold order: AllReduce / ReduceScatter block r as NCCL's ring accumulates it
  // (r+1, ..., r); Reduce as NCCL's chain toward the root (root+1, ..., root,
  // reduce.h:44-67) for every block.
  const int first = (p0.kind == kReduce ? p0.root : r) + 1;
  cb.srcs.resize(n);
  for (int k = 0; k < n; k++) cb.srcs[k] = (const char*)parts[(first + k) % n].send + off * (size_t)eb;
  // AllReduce with n <= NBX_MAX_DSTS: push-gather — the fold stores block r
  // into every rank's output at once (all peer links busy in one kernel,
  // the CollNet-direct scatter shape, all_reduce.h:343-360)
  if (p0.kind == kReduceScatter) cb.dsts.push_back(parts[r].recv);
  else if (p0.kind == kReduce) cb.dsts.push_back((char*)parts[p0.root].recv + off * (size_t)eb);
  else if (n > NBX_MAX_DSTS) cb.dsts.push_back((char*)parts[r].recv + off * (size_t)eb);
  else
    for (int k = 0; k < n; k++) cb.dsts.push_back((char*)parts[(r + k) % n].recv + off * (size_t)eb);
  return cb;
}

// Fold this rank's blocks of several independent collectives: one batched
// launch (nbxReduceMultiBatch) per run of consecutive collectives with the
// same (datatype, op); PreOp on every source and PostOp, as one pass does.
ncclResult_t foldBlocksBatched(const std::vector<const PendingColl*>& colls, const std::vector<RankBlock>& blocks,
                               int n, hipStream_t stream) {
  size_t i = 0;
  while (i < blocks.size()) {
    const PendingColl& pi = *colls[i];
    std::vector<nbxReduceTask> tasks;
    size_t j = i;
    for (; j < blocks.size(); j++) {
      const PendingColl& pj = *colls[j];
      if (pj.dt != pi.dt || pj.op.op != pi.op.op || pj.op.scalarArg != pi.op.scalarArg ||
          pj.op.scalarArgIsPtr != pi.op.scalarArgIsPtr)
        break;
      const RankBlock& b = blocks[j];
      if (b.len == 0) continue;
      tasks.push_back({b.dsts.data(), (int)b.dsts.size(), b.srcs.data(), n, b.len});
    }
    NCCLCHECK(nbx::reduceMultiBatchEx(tasks.data(), (int)tasks.size(), pi.dt, pi.op, /*nPreOpSrcs=*/n,
                                      /*postOp=*/1, (ncclStream_t)stream, nbx::kReduceAcquireSystem));
    i = j;
  }
  return ncclSuccess;
}

// The in-process LL transport of a clique (defined with the multi-process code it shares).
enum MpProto : int;
bool cliqueInKernel(Clique* c, const std::vector<PendingColl>& parts);
ncclResult_t cliqueRunLL(Clique* c, const std::vector<std::vector<PendingColl>>& rounds, size_t lo, size_t hi);
ncclResult_t cliqueOrderBefore(Clique* c, int r, hipStream_t s);
ncclResult_t cliqueOrderAfter(Clique* c, int r, hipStream_t s);

// Run one collective across every rank of an in-process clique.
ncclResult_t runCliqueColl(Clique* c, const std::vector<PendingColl>& parts) {
  const int n = c->n;
  const PendingColl& p0 = parts[0];
  if (!sameCollective(parts)) {
    warn("collective mismatch across ranks of the clique");
    return ncclInvalidUsage;
  }
  const int eb = typeSize(p0.dt);
  NBX_TRACE("clique coll kind=%d n=%d count=%zu dt=%d op=%d", (int)p0.kind, n, p0.count, (int)p0.dt, p0.op.op);
  // 1. enter: every rank's stream reaches the collective (after the previous
  //    call of the rank when that ran on another stream)
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    NCCLCHECK(cliqueOrderBefore(c, r, parts[r].stream));
    HIPCHECK(hipEventRecord(c->evEnter[r], parts[r].stream));
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    for (int j = 0; j < n; j++)
      if (j != r) HIPCHECK(hipStreamWaitEvent(parts[r].stream, c->evEnter[j], 0));
  }
  NBX_TRACE("clique enter events done");
  // 2. reduce: rank r folds block r of every send buffer (postOp here: the fold
  //    is complete in one pass)
  const size_t total = p0.kind == kReduceScatter ? p0.count * (size_t)n : p0.count;
  const bool push = n <= NBX_MAX_DSTS;
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    RankBlock cb = cliqueBlock(parts, n, r);
    if (cb.len == 0) continue;
    NBX_TRACE("clique reduce rank %d len=%zu dst=%p src0=%p", r, cb.len, cb.dsts[0], cb.srcs[0]);
    NCCLCHECK(nbx::reduceMultiEx(cb.dsts.data(), (int)cb.dsts.size(), cb.srcs.data(), n, cb.len, p0.dt, parts[r].op,
                                 /*nPreOpSrcs=*/n, /*postOp=*/1, (ncclStream_t)parts[r].stream,
                                 nbx::kReduceAcquireSystem));
  }
  // evReduced only orders the pull gather (n > 8); each marker costs ~5 us of
  // device time per stream (scripts/probe_order_cost.hip)
  if (p0.kind == kAllReduce && !push) {
    for (int r = 0; r < n; r++) {
      DevGuard g(c->devs[r]);
      HIPCHECK(hipEventRecord(c->evReduced[r], parts[r].stream));
    }
  }
  NBX_TRACE("clique reduce launched");
  // 3. gather (AllReduce with n > NBX_MAX_DSTS only): rank r pulls block j from rank j's recv buffer
  if (p0.kind == kAllReduce && !push) {
    for (int r = 0; r < n; r++) {
      DevGuard g(c->devs[r]);
      for (int j = 0; j < n; j++)
        if (j != r) HIPCHECK(hipStreamWaitEvent(parts[r].stream, c->evReduced[j], 0));
      for (int j = 0; j < n; j++) {
        if (j == r) continue;
        size_t off, len;
        blockRange(total, eb, n, j, &off, &len);
        if (len == 0) continue;
        char* d = (char*)parts[r].recv + off * (size_t)eb;
        const char* s = (const char*)parts[j].recv + off * (size_t)eb;
        if (c->devs[j] == c->devs[r])
          HIPCHECK(hipMemcpyAsync(d, s, len * (size_t)eb, hipMemcpyDeviceToDevice, parts[r].stream));
        else
          HIPCHECK(hipMemcpyPeerAsync(d, c->devs[r], s, c->devs[j], len * (size_t)eb, parts[r].stream));
      }
      HIPCHECK(hipEventRecord(c->evDone[r], parts[r].stream));
    }
  } else {
    for (int r = 0; r < n; r++) {
      DevGuard g(c->devs[r]);
      HIPCHECK(hipEventRecord(c->evDone[r], parts[r].stream));
    }
  }
  NBX_TRACE("clique gather enqueued");
  // 4. leave: no rank reuses its buffers before every peer is done with them
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    for (int j = 0; j < n; j++)
      if (j != r) HIPCHECK(hipStreamWaitEvent(parts[r].stream, c->evDone[j], 0));
    NCCLCHECK(cliqueOrderAfter(c, r, parts[r].stream));
  }
  return ncclSuccess;
}

// Byte ranges one clique collective reads and writes (every rank's buffers).
struct Span {
  uintptr_t lo, hi;
  bool write;
};

void collSpans(const std::vector<PendingColl>& parts, std::vector<Span>* out) {
  const size_t n = parts.size();
  for (const PendingColl& p : parts) {
    const size_t eb = (size_t)typeSize(p.dt);
    const size_t sendBytes = (p.kind == kReduceScatter ? p.count * n : p.count) * eb;
    const size_t recvBytes = p.count * eb;
    out->push_back({(uintptr_t)p.send, (uintptr_t)p.send + sendBytes, false});
    if (p.recv != nullptr) out->push_back({(uintptr_t)p.recv, (uintptr_t)p.recv + recvBytes, true});
  }
}

bool spansConflict(const std::vector<Span>& a, const std::vector<Span>& b) {
  for (const Span& x : a)
    for (const Span& y : b)
      if ((x.write || y.write) && x.lo < y.hi && y.lo < x.hi) return true;
  return false;
}

// Several collectives of one group as ONE exchange: a single enter / leave
// event exchange, and per rank one batched launch (nbxReduceMultiBatch) for
// the blocks of every collective — NCCL likewise packs a group's collectives
// into one kernel's work list (enqueue.cc:67-91 appendWorkElemColl). Only
// for independent collectives on one stream per rank that need no gather step.
ncclResult_t runCliqueBatch(Clique* c, const std::vector<std::vector<PendingColl>>& rounds, size_t lo, size_t hi) {
  const int n = c->n;
  NBX_TRACE("clique batch of %zu collectives", hi - lo);
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    NCCLCHECK(cliqueOrderBefore(c, r, rounds[lo][r].stream));
    HIPCHECK(hipEventRecord(c->evEnter[r], rounds[lo][r].stream));
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    for (int j = 0; j < n; j++)
      if (j != r) HIPCHECK(hipStreamWaitEvent(rounds[lo][r].stream, c->evEnter[j], 0));
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    std::vector<RankBlock> blocks;
    std::vector<const PendingColl*> colls;
    for (size_t k = lo; k < hi; k++) {
      blocks.push_back(cliqueBlock(rounds[k], n, r));
      colls.push_back(&rounds[k][r]);
    }
    NCCLCHECK(foldBlocksBatched(colls, blocks, n, rounds[lo][r].stream));
    HIPCHECK(hipEventRecord(c->evDone[r], rounds[lo][r].stream));
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    for (int j = 0; j < n; j++)
      if (j != r) HIPCHECK(hipStreamWaitEvent(rounds[lo][r].stream, c->evDone[j], 0));
    NCCLCHECK(cliqueOrderAfter(c, r, rounds[lo][r].stream));
  }
  return ncclSuccess;
}

// Run a group's queued collectives in order: maximal runs of batchable ones
// (same collective on every rank, same per-rank streams, no gather step, no
// buffer dependency on an earlier member of the run, at most kMaxCliqueBatch)
// as one batch, the rest one by one.
constexpr size_t kMaxCliqueBatch = 64;

ncclResult_t runCliqueRounds(Clique* c, const std::vector<std::vector<PendingColl>>& rounds) {
  const int n = c->n;
  auto batchable = [&](const std::vector<PendingColl>& parts) {
    return sameCollective(parts) && !(parts[0].kind == kAllReduce && n > NBX_MAX_DSTS);
  };
  size_t i = 0;
  while (i < rounds.size()) {
    size_t j = i;
    std::vector<Span> spans;
    if (cliqueInKernel(c, rounds[i])) {   // a run of in-kernel collectives, independent of each other
      collSpans(rounds[i], &spans);
      for (j = i + 1; j < rounds.size() && cliqueInKernel(c, rounds[j]); j++) {
        std::vector<Span> sj;
        collSpans(rounds[j], &sj);
        if (spansConflict(spans, sj)) break;
        spans.insert(spans.end(), sj.begin(), sj.end());
      }
      NCCLCHECK(cliqueRunLL(c, rounds, i, j));
      i = j;
      continue;
    }
    if (batchable(rounds[i])) {
      collSpans(rounds[i], &spans);
      for (j = i + 1; j < rounds.size() && j - i < kMaxCliqueBatch; j++) {
        if (!batchable(rounds[j]) || cliqueInKernel(c, rounds[j])) break;
        bool sameStreams = true;
        for (int r = 0; r < n; r++) sameStreams &= rounds[j][r].stream == rounds[i][r].stream;
        if (!sameStreams) break;
        std::vector<Span> sj;
        collSpans(rounds[j], &sj);
        if (spansConflict(spans, sj)) break;
        spans.insert(spans.end(), sj.begin(), sj.end());
      }
    }
    if (j <= i + 1) {
      NCCLCHECK(runCliqueColl(c, rounds[i]));
      i++;
    } else {
      NCCLCHECK(runCliqueBatch(c, rounds, i, j));
      i = j;
    }
  }
  return ncclSuccess;
}

// Launch every complete collective queued for every clique (called when the
// outermost group ends, or immediately outside a group).
ncclResult_t flushPendingImpl();
ncclResult_t flushPending() {
  try {
    return flushPendingImpl();
  } catch (const std::exception& e) {
    warn("internal exception: %s", e.what());
    return ncclInternalError;
  } catch (...) {
    warn("internal exception");
    return ncclInternalError;
  }
}
ncclResult_t flushPendingImpl() {
  std::lock_guard<std::mutex> g(g_pendMu);
  for (size_t i = 0; i < g_cliques.size();) {
    std::shared_ptr<Clique> c = g_cliques[i].lock();
    if (!c) {   // every communicator of this clique was destroyed
      g_cliques.erase(g_cliques.begin() + (long)i);
      continue;
    }
    auto& pr = c->pending;
    std::vector<std::vector<PendingColl>> rounds;
    for (;;) {
      bool ready = true;
      for (int r = 0; r < c->n; r++) ready &= !pr[r].empty();
      if (!ready) break;
      std::vector<PendingColl> parts;
      parts.reserve(c->n);
      for (int r = 0; r < c->n; r++) {
        parts.push_back(pr[r].front());
        pr[r].pop_front();
      }
      rounds.push_back(std::move(parts));
    }
    NCCLCHECK(runCliqueRounds(c.get(), rounds));
    i++;
  }
  return ncclSuccess;
}


// ---------------------------------------------------------------------------
// Multi-process communicator (ncclCommInitRank with nranks > 1, one process
// per rank on one node). Replaces NCCL's bootstrap + P2P transport setup
// (bootstrap.cc, transport/p2p.cc:190-381) with a TCP bootstrap for the
// init-time allgathers and connection buffers that the library allocates and
// every peer IPC-maps ONCE, at init (p2pMap / p2pSendConnect / p2pRecvConnect,
// p2p.cc:290-330,450-520):
//   * LL / LL128 line buffers (nbx_ll.h) for small and medium messages;
//   * the Simple protocol's staging and flag words (nbx_simple.h) for the rest,
//     direct or ring schedule (NCCL_ALGO=Ring).
// Peers never touch the caller's buffers and no call exchanges anything on
// the host: a collective is one kernel on the caller's stream whose flow
// control (the reference's waitPeer / postPeer, prims_simple.h:129-185)
// runs inside it. All sequencing state is device-resident, so graph capture
// and replay need nothing special.

constexpr int kMaxMpRanks = nbx::kSimpleMaxRanks;   // one staging source region per rank

// One reducing collective as enqueued on a multi-process communicator (the
// same record the in-process clique queues).
using MpCall = PendingColl;

struct MpState {
  nbx::Bootstrap* bs = nullptr;
  int* hostWords = nullptr;            // the communicator's (ncclComm::hostWords), not owned
  int* hostWordsDev = nullptr;
  double timeoutSec = 300.0;
  std::vector<void*> peerMaps;         // every IPC mapping this communicator opened (closed at destroy)
  // LL protocol (nbx_ll.h): own buffer [2][n][slotLines] lines + [n] done words
  uint64_t* ll = nullptr;
  uint64_t** peerLLDev = nullptr;
  uint64_t llMaxBytes = 0;
  uint64_t llSlotLines = 0;
  uint64_t llDoneOff = 0;
  uint64_t llPlanOff = 0;   // plan words [parity 2][source n] (nbx_ll.h)
  nbx::LLState* llState = nullptr;  // device-resident LL-family sequencing (nbx_ll_args.h)
  // LL128 protocol (nbx_ll.h kLL128Coll): own buffer [2][n][l128SlotLines] 64-B lines;
  // shares the LL buffer's done words and parity credits
  uint64_t* l128 = nullptr;
  uint64_t** peerL128Dev = nullptr;
  uint64_t l128MaxBytes = 0;        // 0: LL128 unavailable (n > 8)
  uint64_t l128OneShotMax = 0;      // AllReduce, n > 2: one-shot up to this, two-shot above
  uint64_t l128SlotLines = 0;
  uint64_t l128Bytes = 0;
  int protoMask = 0;                // NCCL_PROTO at init: kProtoLL | kProtoLL128 | kProtoSimple
  bool ring = false;                // NCCL_ALGO=Ring at init
  bool multiGpu = false;            // the ranks span more than one physical GPU (PCI key)
  // Simple protocol (nbx_simple.h): staging [2][slots][n][grid][slice] and flag
  // words [4][n][grid] (uncached, IPC-mapped by every peer), counters [4][n][grid]
  char* stage = nullptr;
  uint64_t stageBytes = 0;
  uint64_t llBytes = 0, sflagsBytes = 0;   // used bytes of the LL buffer and the Simple flag words
  uint64_t stageHdrOff = 0;         // the Simple plan headers' offset in the staging (after the slices)
  int ipcRepairs = 0;               // connection buffers re-exported at init because a mapping was wrong (mpConnect)
  uint64_t* sflags = nullptr;
  uint64_t* scounters = nullptr;
  char** peerStageDev = nullptr;
  uint64_t** peerSFlagsDev = nullptr;
  uint64_t sliceBytes = 0;          // NBX_SIMPLE_SLICE_BYTES: staging bytes per (slot, source, workgroup)
  int slots = 2;                    // NBX_SIMPLE_SLOTS
  int simpleGrid = 0;               // workgroups of a full-size Simple call (NBX_SIMPLE_MAX_GRID, CU-capped)
  int simplePrefetch = 1;           // NBX_SIMPLE_PREFETCH: next round's pushes before this round's fold
  uint32_t llGridCap = 0, l128GridCap = 0;   // LL / LL128 workgroup caps: 4 / 1 per CU, split among ranks sharing a GPU
  // successive calls are ordered across streams, as NCCL serializes a
  // communicator's work: a call on another stream waits for the previous one
  hipStream_t lastStream = nullptr;
  bool streamOrder = true;          // NBX_MP_STREAM_ORDER=0: calls on different streams are not ordered (A/B only)
  // completion word of the communicator's kernels (MpDone, nbx_ll_args.h):
  // [0, 8) done (last completed eager call), [64, 64 + 9 * 64) arrival counters
  char* orderMem = nullptr;
  hipIpcMemHandle_t llHandle{}, l128Handle{}, stageHandle{}, sflagsHandle{};   // taken at allocation
  uint64_t callSeq = 0;             // eager calls numbered from 1
  uint64_t lastSeq = 0;             // number of the previous eager call that launched a kernel
  uint64_t curSeq = 0;              // number of the call being launched (0: captured)
  bool launched = false;            // the call being launched put a kernel on its stream
  std::vector<MpCall> group;        // calls queued inside ncclGroupStart/End (run at the outermost End)
  bool groupBatch = true;           // NBX_GROUP_BATCH=0: every grouped call its own kernel
  bool checkPlans = false;          // NBX_CHECK_PLANS (default NCCL_CHECK_POINTERS): plan words / headers
  std::vector<hipEvent_t> groupEvents;   // fan-in / fan-out of a group launch over several streams
  // clique ranks only: the previous call ran on the event-ordered fold path
  // (runCliqueColl / runCliqueBatch) on extStream; it is complete once every
  // rank's extDone event (the clique's evDone) is
  hipStream_t extStream = nullptr;
  std::vector<hipEvent_t> extDone;
};

// The LL-family transport of a communicator: its own (one process per rank)
// or, for a rank of an in-process clique, the one cliqueInitTransport built.
MpState* mpOf(const ncclComm* c) { return c->mp ? c->mp : c->lt; }

// Exchanged before anything is allocated: where every rank runs.
struct MpPreInfo {
  uint64_t pciKey;   // (domain, bus, device) of this rank's GPU: identifies it across processes
  int32_t device;
  int32_t cus;
};

struct MpInitInfo {
  int32_t pid;
  int32_t device;
  hipIpcMemHandle_t llHandle;
  hipIpcMemHandle_t l128Handle;
  hipIpcMemHandle_t stageHandle;
  hipIpcMemHandle_t sflagsHandle;
  uint64_t nonce;          // this communicator's mapping self-check pattern (mpConnect)
  // settings every rank must share: every rank must pick the same protocol,
  // grid and staging layout for the same call
  uint64_t llMaxBytes;
  uint64_t l128MaxBytes;
  uint64_t l128OneShotMax;
  uint64_t sliceBytes;
  int32_t protoMask;
  int32_t ring;            // NCCL_ALGO=Ring
  int32_t slots;
  int32_t simpleGrid;
  int32_t groupBatch;      // NBX_GROUP_BATCH: one launch per run of grouped calls, or one per call
  int32_t checkPlans;      // NBX_CHECK_PLANS: every launch stamps / checks its plan (or none does)
};

// NCCL_PROTO (tuning.cc:254-259, parseList): a comma-separated list of the
// enabled protocols among LL, LL128, Simple, or "^list" for all but those.
// Per message (per-rank block for ReduceScatter) the first enabled protocol
// whose buffer holds it is used: LL up to NBX_LL_MAX_BYTES (64 KiB), LL128 up
// to NBX_LL128_MAX_BYTES (1 MiB; n <= 8 ranks), else Simple (also the
// fallback when Simple is disabled and nothing else fits).
// Read when the communicator is created (as NCCL reads its tuning env at init).
enum { kProtoLL = 1, kProtoLL128 = 2, kProtoSimple = 4, kProtoAll = 7 };
int protoFromString(const char* v) {
  if (v == nullptr || *v == 0) return kProtoAll;
  bool exclude = v[0] == '^';
  std::string list(exclude ? v + 1 : v);
  int mask = 0;
  size_t pos = 0;
  while (pos <= list.size()) {
    size_t e = list.find(',', pos);
    if (e == std::string::npos) e = list.size();
    std::string tok = list.substr(pos, e - pos);
    if (strcasecmp(tok.c_str(), "ll") == 0) mask |= kProtoLL;
    else if (strcasecmp(tok.c_str(), "ll128") == 0) mask |= kProtoLL128;
    else if (strcasecmp(tok.c_str(), "simple") == 0) mask |= kProtoSimple;
    else if (!tok.empty()) warn("NCCL_PROTO: unknown protocol '%s' ignored", tok.c_str());
    pos = e + 1;
  }
  return exclude ? (kProtoAll & ~mask) : mask;
}
int protoFromEnv() { return protoFromString(std::getenv("NCCL_PROTO")); }

// LL128 across GPUs is enabled by default only where it was validated — the
// reference's rule (tuning.cc:250-297: protoEnable[LL128] = 2 "default", and
// parseList turns it into 1 only when NCCL_PROTO lists LL128; a "^list"
// leaves it at 2). LL128 trusts a 64-byte line written by one store to arrive
// whole; within one GPU that was stress-tested, over xGMI it has
// not been, so ranks on different GPUs drop LL128 from the default set until a
// node run validates it (DESIGN §6 states the flip rule). It stays on when
// NCCL_PROTO names it explicitly, or with NBX_LL128_ACROSS_GPUS=1.
// NBX_DEBUG_ASSUME_MULTI_GPU=1 (test hook) applies this gate to ranks that
// share a GPU, and nothing else of the multi-GPU settings.
long envLong(const char* name, long dflt);
bool protoLL128Explicit(const char* v) {
  if (v == nullptr || *v == 0 || v[0] == '^') return false;
  return (protoFromString(v) & kProtoLL128) != 0;
}
int protoGateAcrossGpus(int mask, bool multiGpu, const char* ncclProto) {
  const bool assume = envLong("NBX_DEBUG_ASSUME_MULTI_GPU", 0) != 0;
  if (!(multiGpu || assume) || protoLL128Explicit(ncclProto)) return mask;
  if (envLong("NBX_LL128_ACROSS_GPUS", 0) != 0) return mask;
  return mask & ~kProtoLL128;
}

// Per message: LL up to the LL max; LL128 up to the LL128 max: one-shot (every
// rank pushes the whole message to every target), for AllReduce / Reduce with
// more than 2 ranks only up to the one-shot max and the two-shot AllReduce /
// Reduce (reduce-scatter + gather hops, a rank's block in half an LL128 slot)
// above it; else Simple. ReduceScatter is one hop by nature: one-shot up to
// the LL128 max.
enum MpProto : int { kMpLL = 0, kMpLL128 = 1, kMpSimple = 2, kMpLL128x2 = 3 };
// Lines per (parity, source) slot: holds maxBytes one-shot, and each half (a
// two-shot sub-slot) holds maxBytes / 2.
uint64_t l128SlotLinesFor(uint64_t maxBytes) {
  const uint64_t half = (maxBytes + 1) / 2;
  return 2 * ((half + nbx::kL128DataBytesHost - 1) / nbx::kL128DataBytesHost);
}
MpProto chooseProtoFor(int mask, bool twoShotKind, uint64_t slotBytes, uint64_t blockBytes, int n, uint64_t llMax,
                       uint64_t l128Max, uint64_t oneShotMax) {
  if (slotBytes == 0 || n > 64) return kMpSimple;
  if ((mask & kProtoLL) && slotBytes <= llMax) return kMpLL;
  if ((mask & kProtoLL128) && l128Max != 0 && n <= nbx::kL128MaxRanksHost) {
    if (!twoShotKind || n <= 2 || slotBytes <= oneShotMax) {
      if (slotBytes <= l128Max) return kMpLL128;
    } else if (slotBytes <= l128Max && blockBytes <= (l128SlotLinesFor(l128Max) / 2) * nbx::kL128DataBytesHost) {
      return kMpLL128x2;
    }
  }
  return kMpSimple;
}

// NCCL_ALGO (tuning.cc:254-259): "Ring" selects the ring schedule for the
// Simple protocol; anything else (default) the direct schedule.
// Read when the communicator is created.
bool algoRingFromEnv() {
  const char* v = std::getenv("NCCL_ALGO");
  return v && strcasecmp(v, "ring") == 0;
}

long envLong(const char* name, long dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atol(v) : dflt;
}

// The reference's own tuning knobs on this path, read at communicator
// creation like NCCL reads them (init.cc:523-541 computeBuffSizes,
// connect.cc:314-315, tuning.cc:12), each mapped onto the setting that plays
// its role here; the NBX_* variable of that setting, when set, wins:
//   NCCL_BUFFSIZE       Simple connection buffer per (peer, channel): the
//                       Simple staging per (peer, workgroup, region) is
//                       slots x slice, so slice = NCCL_BUFFSIZE / slots
//                       (NBX_SIMPLE_SLICE_BYTES) — only below the 64 KiB
//                       default (mpTransportSettings);
//   NCCL_LL_BUFFSIZE    LL buffer: half of every 8-byte line is flag, so LL
//                       carries messages up to NCCL_LL_BUFFSIZE / 2 (NBX_LL_MAX_BYTES);
//   NCCL_LL128_BUFFSIZE LL128 buffer: 48 payload bytes per 64-byte line, so
//                       LL128 carries up to 3/4 of it (NBX_LL128_MAX_BYTES);
//   NCCL_MAX_NCHANNELS / NCCL_MIN_NCHANNELS  a channel is a workgroup here:
//                       the Simple grid (NBX_SIMPLE_MAX_GRID) and the LL /
//                       LL128 grids are capped at the max, and the Simple grid
//                       raised to the min (both within the co-residency cap).
// Unset, the measured defaults stay (64 KiB slices, 64 KiB LL, 4 MiB LL128,
// 128 Simple workgroups). NCCL_NTHREADS has no counterpart: every
// kernel is compiled for 256-thread workgroups (a warning says it is ignored).
long ncclEnvMapped(const char* nbxName, const char* ncclName, long dflt, long num, long den) {
  const char* v = std::getenv(nbxName);
  if (v && *v) return std::atol(v);
  const char* w = std::getenv(ncclName);
  if (w && *w && std::atol(w) > 0) return std::atol(w) / den * num;
  return dflt;
}

// Memory that other GPUs write and this GPU reads (LL lines, Simple staging
// and flag words). Uncached (MTYPE UC) by default: a peer's stores over xGMI
// land in HBM and no XCD L2 can hold a stale copy, which is what RCCL uses
// for its connection buffers too. NBX_SYNC_MEM=coarse selects plain hipMalloc
// (A/B measurement only).
// A connection buffer every peer maps: uncached device memory, its size
// rounded up to whole 2 MiB pages so the buffer is an allocation of its own,
// and its IPC handle taken at once.
// The runtime rule behind the retry (scripts/probe_ipc_export.py: N processes
// replaying communicator creation / destruction with the library's buffer
// sizes, raw HIP, no libnbxccl; profiles/r4/probe_ipc_export_r4*.jsonl):
// once exported allocations are freed, hipIpcGetMemHandle now and then refuses
// ('invalid argument') a new allocation — 25 of 62,400 exports, 20 of them at
// an address whose earlier allocation had been exported and freed; the same
// pointer was refused again on an immediate retry 23 times of 25, and a fresh
// allocation (the refused one still held, so at another address) was
// accepted 23 times of 23. With exported buffers never freed: 0 of 19,200. So
// a refused allocation is held aside while the next one is made (at most 4
// tries), then freed. The same runtime condition also makes a successful
// export name the wrong memory now and then (mpConnect, which verifies every
// mapping and re-exports what is wrong).
hipError_t allocSyncMem(void** p, size_t bytes, hipIpcMemHandle_t* handle /* nullptr: in-process only */) {
  static const bool coarse = [] {
    const char* v = std::getenv("NBX_SYNC_MEM");
    return v && strcasecmp(v, "coarse") == 0;
  }();
  const size_t page = (size_t)2 << 20;
  bytes = (bytes + page - 1) / page * page;
  std::vector<void*> refused;
  hipError_t e = hipSuccess;
  for (int attempt = 0; attempt < 4; attempt++) {
    *p = nullptr;
    e = coarse ? hipMalloc(p, bytes) : hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess || handle == nullptr) break;
    e = hipIpcGetMemHandle(handle, *p);
    if (e == hipSuccess) break;
    (void)hipGetLastError();
    info("hipIpcGetMemHandle refused a %zu-byte connection buffer at %p (%s): a reused exported address; "
         "allocating another", bytes, *p, hipGetErrorString(e));
    refused.push_back(*p);
    *p = nullptr;
  }
  for (void* q : refused) (void)hipFree(q);
  return e;
}

ncclResult_t mpLL128SelfTest(ncclComm* c);

// A device spin gave up (host error word set): name the wait, the peer, the
// value it waited for and the last one it saw (nbx_diag.h), once per record.
void mpReportDeviceError(ncclComm* c) {
  MpState* mp = mpOf(c);
  if (!mp || !mp->hostWords || mp->hostWords[1] == 0) return;
  const volatile uint64_t* d = (const volatile uint64_t*)((const volatile char*)mp->hostWords + nbx::kDiagByteOffset);
  static thread_local uint64_t lastReported[nbx::kDiagWords] = {};
  uint64_t rec[nbx::kDiagWords];
  for (int i = 0; i < nbx::kDiagWords; i++) rec[i] = d[i];
  if (std::memcmp(rec, lastReported, sizeof(rec)) == 0) return;
  std::memcpy(lastReported, rec, sizeof(rec));
  if (mp->hostWords[1] == 2) {
    warn("comm %p rank %d: a device wait was aborted (ncclCommAbort)", (void*)c, c->rank);
    return;
  }
  if (nbx::diagIsPlanCheck(rec[0])) {
    warn("comm %p rank %d: device check failed after %.3f s: %s: peer %lld, our plan %llx, its plan %llx "
         "(workgroup %llu)", (void*)c, c->rank, (double)rec[5] * 1e-8, nbx::diagSiteName(rec[0]),
         (long long)(int64_t)rec[1], (unsigned long long)rec[2], (unsigned long long)rec[3],
         (unsigned long long)rec[4]);
    return;
  }
  warn("comm %p rank %d: device wait timed out after %.3f s: %s of peer %lld, waited for %llu, last saw %llu "
       "(workgroup %llu)", (void*)c, c->rank, (double)rec[5] * 1e-8, nbx::diagSiteName(rec[0]),
       (long long)(int64_t)rec[1], (unsigned long long)rec[2], (unsigned long long)rec[3],
       (unsigned long long)rec[4]);
}

ncclResult_t mpOpenPeer(MpState* mp, const hipIpcMemHandle_t& h, void** p) {
  HIPCHECK(hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess));
  mp->peerMaps.push_back(*p);
  return ncclSuccess;
}

// The 16-byte mapping self-check word rank `from` leaves at slot `at`.
void checkWord(uint64_t nonce, int from, int at, uint64_t out[2]) {
  out[0] = nonce ^ (0x9e3779b97f4a7c15ull * (uint64_t)(from + 1));
  out[1] = ~nonce ^ (0xc2b2ae3d27d4eb4full * (uint64_t)(at + 1));
}

// Every connection buffer carries a check region after its used bytes:
// 16 bytes per writer rank plus the owner's own word (mpConnect).
uint64_t connCheckOff(uint64_t used) { return (used + 15) & ~(uint64_t)15; }
uint64_t connAllocBytes(uint64_t used, int n) { return connCheckOff(used) + 16ull * (uint64_t)(n + 1); }

// The connection buffers a multi-process rank exports (LL lines, LL128 lines,
// Simple staging, Simple flag words).
enum { kConnLL, kConnL128, kConnStage, kConnFlags, kNumConn };

// One rank's LL-family state on the current device: completion word,
// sequencing state, host abort / error words, and the LL and LL128 connection
// buffers (IPC handles taken when `ipc`; a clique's buffers stay in-process).
ncclResult_t mpAllocLL(MpState* mp, int n, bool ipc, const ncclComm* comm) {
  const char* t = std::getenv("NBX_TIMEOUT_SEC");
  if (t && std::atof(t) > 0) mp->timeoutSec = std::atof(t);
  mp->protoMask = protoFromEnv();
  mp->streamOrder = envLong("NBX_MP_STREAM_ORDER", 1) != 0;
  mp->groupBatch = envLong("NBX_GROUP_BATCH", 1) != 0;
  // Plan checks (nbx_ll.h plan words, nbx_simple.h slice headers): a launch
  // fails, naming the peer, when ranks issue mismatched calls or cut a group
  // differently — instead of a timeout or folded misplaced data. Off unless
  // asked for (NBX_CHECK_PLANS=1, or the reference's own argument-checking
  // knob NCCL_CHECK_POINTERS=1): they cost 0.7-1.9 us per small call on the
  // shared-GPU rig, and the reference does not check this either.
  mp->checkPlans = envLong("NBX_CHECK_PLANS", comm->checkPointers ? 1 : 0) != 0;
  HIPCHECK(hipMalloc((void**)&mp->orderMem, 1024));
  HIPCHECK(hipMemset(mp->orderMem, 0, 1024));
  HIPCHECK(hipMalloc((void**)&mp->llState, sizeof(nbx::LLState)));
  HIPCHECK(hipMemset(mp->llState, 0, sizeof(nbx::LLState)));
  if (comm->hostWords == nullptr) return ncclInternalError;
  mp->hostWords = comm->hostWords;
  mp->hostWordsDev = comm->hostWordsDev;
  // LL buffer: 2 parities x n sources x 2 lines per 8-byte pack
  {
    uint64_t mx = (uint64_t)ncclEnvMapped("NBX_LL_MAX_BYTES", "NCCL_LL_BUFFSIZE", 64 << 10, 1, 2);
    mx = (mx + 15) & ~(uint64_t)15;
    if (mx < 1024) mx = 1024;
    mp->llMaxBytes = mx;
    mp->llSlotLines = 2 * (mx / 8);
    mp->llDoneOff = 2 * (uint64_t)n * mp->llSlotLines;
    mp->llPlanOff = mp->llDoneOff + (uint64_t)n + 1;
    mp->llBytes = (mp->llPlanOff + 2 * (uint64_t)n) * sizeof(uint64_t);
    const uint64_t llAlloc = connAllocBytes(mp->llBytes, n);
    HIPCHECK(allocSyncMem((void**)&mp->ll, llAlloc, ipc ? &mp->llHandle : nullptr));
    HIPCHECK(hipMemset(mp->ll, 0, llAlloc));
  }
  // LL128 buffer: 2 parities x n sources x 64-byte lines of 48 payload bytes (n <= 8)
  if (n <= nbx::kL128MaxRanksHost) {
    // 1 MiB: where Simple overtakes LL128 (48 payload bytes per 64-byte line) on
    // the shared-GPU rig — 2 ranks: 1 MiB 15.4 vs 15.6 us, 2 MiB 25.8 vs 16.4,
    // 4 MiB 43.8 vs 18.7; 4 ranks: 2 MiB 34.5 vs 25.4 (profiles/r4/proto_sweep_r4z)
    uint64_t mx = (uint64_t)ncclEnvMapped("NBX_LL128_MAX_BYTES", "NCCL_LL128_BUFFSIZE", 1 << 20, 3, 4);
    mp->l128OneShotMax = (uint64_t)envLong("NBX_LL128_ONESHOT_MAX", 256 << 10);
    if (mx > (64u << 20)) mx = 64u << 20;   // keeps the buffer under the 4 GiB descriptor range
    if (mx != 0) {
      mx = (mx + 15) & ~(uint64_t)15;
      mp->l128MaxBytes = mx;
      mp->l128SlotLines = l128SlotLinesFor(mx);
      mp->l128Bytes = 2 * (uint64_t)n * mp->l128SlotLines * nbx::kL128LineBytesHost;
      const uint64_t l128Alloc = connAllocBytes(mp->l128Bytes, n);
      HIPCHECK(allocSyncMem((void**)&mp->l128, l128Alloc, ipc ? &mp->l128Handle : nullptr));
      HIPCHECK(hipMemset(mp->l128, 0, l128Alloc));
    }
  }
  return ncclSuccess;
}

// Grid caps and Simple settings of one rank's transport. Simple grid: one
// workgroup per CU, all co-resident (workgroup g of a rank waits on workgroup
// g of its peers); ranks sharing a GPU split its CUs, and so do the LL
// family's spinning grids (the env caps still apply on top).
void mpTransportSettings(MpState* mp, int minCus, int maxShare) {
  const long maxCh = envLong("NCCL_MAX_NCHANNELS", 0), minCh = envLong("NCCL_MIN_NCHANNELS", 0);
  long g = envLong("NBX_SIMPLE_MAX_GRID", 0);
  if (g <= 0) {
    g = 128;
    if (maxCh > 0) g = std::min(g, maxCh);
    if (minCh > 0) g = std::max(g, minCh);
  }
  g = std::min<long>(g, std::max(1, minCus / maxShare));
  mp->llGridCap = (uint32_t)std::max(1, 4 * minCus / maxShare);
  mp->l128GridCap = (uint32_t)std::max(1, minCus / maxShare);
  if (maxCh > 0) {   // a channel is a workgroup here
    mp->llGridCap = std::min<uint32_t>(mp->llGridCap, (uint32_t)maxCh);
    mp->l128GridCap = std::min<uint32_t>(mp->l128GridCap, (uint32_t)maxCh);
  }
  mp->simpleGrid = (int)std::max<long>(1, std::min<long>(g, nbx::kSimpleMaxGrid));
  mp->slots = (int)std::max<long>(2, std::min<long>(envLong("NBX_SIMPLE_SLOTS", 2), 8));
  // NCCL_BUFFSIZE is the reference's buffer per (peer, channel) and its own
  // default is 4 MiB, which job scripts often set explicitly; here it would
  // become a 1 MiB slice per (peer, workgroup, region, slot) — 4 GiB of staging
  // at 8 ranks. So it is honoured only where it LOWERS the slice
  // below the 64 KiB default (a memory cap, its use in the reference); an
  // explicit NBX_SIMPLE_SLICE_BYTES sets the slice (16 B .. 1 MiB) as asked.
  long sl = envLong("NBX_SIMPLE_SLICE_BYTES", 0);
  if (sl <= 0) {
    sl = 64 << 10;
    const long bs = envLong("NCCL_BUFFSIZE", 0);
    if (bs > 0 && bs / mp->slots < sl) sl = bs / mp->slots;
    else if (bs > 0)
      info("NCCL_BUFFSIZE=%ld ignored: the Simple slice stays %ld bytes (only smaller buffers are honoured)", bs, sl);
  }
  sl = std::max<long>(nbx::kSimpleMinSliceBytes, std::min<long>(sl, 1 << 20));
  mp->sliceBytes = (uint64_t)(sl + 15) & ~(uint64_t)15;
  if (const char* nt = std::getenv("NCCL_NTHREADS"); nt && *nt && std::atol(nt) != 256)
    info("NCCL_NTHREADS=%s ignored: every kernel of this library runs 256-thread workgroups", nt);
  mp->simplePrefetch = envLong("NBX_SIMPLE_PREFETCH", 1) != 0;
}

// The Simple protocol's staging and flag words (uncached, exported when
// `ipc`, with the check region mpConnect uses) and its counters.
ncclResult_t mpAllocSimple(MpState* mp, int n, bool ipc) {
  const uint64_t cells = (uint64_t)n * (uint64_t)mp->simpleGrid;
  // slices, then one 16-byte plan header per slice cell (nbx_simple.h simpleHdr)
  mp->stageHdrOff = 2ull * (uint64_t)mp->slots * cells * mp->sliceBytes;
  mp->stageBytes = mp->stageHdrOff + 2ull * (uint64_t)mp->slots * cells * 16u;
  HIPCHECK(allocSyncMem((void**)&mp->stage, connAllocBytes(mp->stageBytes, n), ipc ? &mp->stageHandle : nullptr));
  HIPCHECK(hipMemset(mp->stage, 0, connAllocBytes(mp->stageBytes, n)));
  mp->sflagsBytes = 4 * cells * sizeof(uint64_t);
  HIPCHECK(allocSyncMem((void**)&mp->sflags, connAllocBytes(mp->sflagsBytes, n), ipc ? &mp->sflagsHandle : nullptr));
  HIPCHECK(hipMemset(mp->sflags, 0, connAllocBytes(mp->sflagsBytes, n)));
  HIPCHECK(hipMalloc((void**)&mp->scounters, 4 * cells * sizeof(uint64_t)));
  HIPCHECK(hipMemset(mp->scounters, 0, 4 * cells * sizeof(uint64_t)));
  return ncclSuccess;
}

// Opens every peer's connection buffers and checks every mapping before first
// use, re-exporting any buffer whose mapping is wrong (the reference maps its
// peers' buffers once at connection time, transport/p2p.cc:290-330 p2pMap).
// Why the check is needed: scripts/probe_ipc_export.py (raw HIP, N processes
// on one GPU replaying communicator creation / destruction with this
// library's buffer sizes and memory kinds) found IPC mappings that do not
// show the exported allocation — an importer reads zeros or ANOTHER rank's
// buffer through it (89 canary reads), and its stores never reach the owner
// (164), out of 62,400 imports, in the library's own memory kind as in plain
// hipMalloc memory; the same wrong bytes are seen by every importer of that
// handle (so it is the export, not one importer's mapping, that is wrong),
// mostly at owner addresses that an earlier, freed allocation of the owner
// had been exported from; with exported buffers never freed, none. Round 2's
// wrong results (peers reading stale bytes through a mapping of a freshly
// allocated buffer, their stores lost) are the same failure.
// Check, per buffer and round (each with a fresh per-communicator nonce):
// every rank stores a 16-byte word through its mapping of every peer's buffer
// (slot = its rank) and its own word into its own buffer (slot n), all in the
// check region after the used bytes; after a bootstrap barrier every rank
// checks the words its peers stored into its buffers and reads every peer's
// own word through its mappings. A wrong (owner, buffer) seen by anyone —
// agreed by an allgather — is re-exported: its owner allocates a new buffer
// (the old one held until the end, so the new one lands elsewhere), every
// peer closes the wrong mapping and opens the new handle, and the round
// repeats (at most 4). Only then does ncclCommInitRank fail (ncclSystemError).
// NBX_IPC_VERIFY_FAIL=<rank>:<buffer> (test hook) makes round 0 report that
// rank's buffer (0 LL, 1 LL128, 2 staging, 3 flags) wrong.
ncclResult_t mpConnect(ncclComm* c, const std::vector<MpInitInfo>& all) {
  MpState* mp = c->mp;
  const int n = c->nRanks, me = c->rank;
  void** own[kNumConn] = {(void**)&mp->ll, (void**)&mp->l128, (void**)&mp->stage, (void**)&mp->sflags};
  hipIpcMemHandle_t* ownHandle[kNumConn] = {&mp->llHandle, &mp->l128Handle, &mp->stageHandle, &mp->sflagsHandle};
  const uint64_t used[kNumConn] = {mp->llBytes, mp->l128Bytes, mp->stageBytes, mp->sflagsBytes};
  const bool present[kNumConn] = {true, mp->l128 != nullptr, true, true};   // the same on every rank (n <= 8)
  auto handleOf = [](const MpInitInfo& i, int t) -> const hipIpcMemHandle_t& {
    return t == kConnLL ? i.llHandle : t == kConnL128 ? i.l128Handle : t == kConnStage ? i.stageHandle : i.sflagsHandle;
  };
  std::vector<std::array<char*, kNumConn>> peer(n);
  std::vector<hipIpcMemHandle_t> cur((size_t)n * kNumConn);   // the handle each mapping was opened from
  for (int j = 0; j < n; j++)
    for (int t = 0; t < kNumConn; t++) {
      peer[j][t] = nullptr;
      cur[(size_t)j * kNumConn + t] = handleOf(all[j], t);
    }
  auto open = [&](int j, int t) -> ncclResult_t {
    void* p = nullptr;
    NCCLCHECK(mpOpenPeer(mp, cur[(size_t)j * kNumConn + t], &p));
    peer[j][t] = (char*)p;
    return ncclSuccess;
  };
  for (int j = 0; j < n; j++)
    for (int t = 0; t < kNumConn; t++)
      if (j != me && present[t]) NCCLCHECK(open(j, t));
  int failRank = -1, failBuf = -1;
  if (const char* v = std::getenv("NBX_IPC_VERIFY_FAIL"); v && *v) std::sscanf(v, "%d:%d", &failRank, &failBuf);
  std::vector<void*> retired;
  ncclResult_t res = ncclSuccess;
  constexpr int kRounds = 4;
  for (int round = 0;; round++) {
    const uint64_t salt = 0x632be59bd9b4e019ull * (uint64_t)(round + 1);
    auto nonceOf = [&](int j, int t) { return all[j].nonce ^ salt ^ (0xd6e8feb86659fd93ull * (uint64_t)(t + 1)); };
    uint64_t w[2];
    for (int t = 0; t < kNumConn; t++) {
      if (!present[t]) continue;
      const uint64_t off = connCheckOff(used[t]);
      for (int j = 0; j < n; j++) {
        if (j == me) continue;
        checkWord(nonceOf(me, t), me, j, w);
        HIPCHECK(hipMemcpy(peer[j][t] + off + 16ull * (uint64_t)me, w, 16, hipMemcpyHostToDevice));
      }
      checkWord(nonceOf(me, t), me, n, w);
      HIPCHECK(hipMemcpy((char*)*own[t] + off + 16ull * (uint64_t)n, w, 16, hipMemcpyHostToDevice));
    }
    HIPCHECK(hipDeviceSynchronize());
    std::vector<uint8_t> bad((size_t)n * kNumConn, 0), allBad((size_t)n * n * kNumConn);
    int32_t dummy = 0;
    std::vector<int32_t> gathered(n);
    NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &dummy, sizeof(dummy), gathered.data()));   // every word stored
    std::vector<uint64_t> mine(2 * (size_t)(n + 1));
    for (int t = 0; t < kNumConn; t++) {
      if (!present[t]) continue;
      const uint64_t off = connCheckOff(used[t]);
      HIPCHECK(hipMemcpy(mine.data(), (char*)*own[t] + off, 16ull * (uint64_t)(n + 1), hipMemcpyDeviceToHost));
      for (int j = 0; j < n; j++) {
        if (j == me) continue;
        checkWord(nonceOf(j, t), j, me, w);
        if (mine[2 * j] != w[0] || mine[2 * j + 1] != w[1]) {
          info("comm %p rank %d: rank %d's store through its mapping of my buffer %d did not land (round %d)",
               (void*)c, me, j, t, round);
          bad[(size_t)me * kNumConn + t] = 1;
        }
        uint64_t got[2];
        HIPCHECK(hipMemcpy(got, peer[j][t] + off + 16ull * (uint64_t)n, 16, hipMemcpyDeviceToHost));
        checkWord(nonceOf(j, t), j, n, w);
        if (got[0] != w[0] || got[1] != w[1]) {
          info("comm %p rank %d: my mapping of rank %d's buffer %d shows other bytes (round %d)", (void*)c, me, j, t,
               round);
          bad[(size_t)j * kNumConn + t] = 1;
        }
      }
    }
    if (round == 0 && failRank == me && failBuf >= 0 && failBuf < kNumConn && present[failBuf])
      bad[(size_t)me * kNumConn + failBuf] = 1;
    NCCLCHECK(nbx::bootstrapAllGather(mp->bs, bad.data(), bad.size(), allBad.data()));
    for (int q = 0; q < n; q++)
      for (size_t i = 0; i < bad.size(); i++) bad[i] |= allBad[(size_t)q * bad.size() + i];
    int nBad = 0;
    for (uint8_t b : bad) nBad += b;
    if (nBad == 0) break;
    if (round + 1 == kRounds) {
      warn("ncclCommInitRank : %d peer mapping(s) still wrong after %d re-exports; giving up", nBad, kRounds - 1);
      res = ncclSystemError;
      break;
    }
    mp->ipcRepairs += nBad;
    // re-export: the owner of a wrong buffer allocates another (the old one held)
    struct Fresh {
      hipIpcMemHandle_t h[kNumConn];
    } fresh{};
    for (int t = 0; t < kNumConn; t++) {
      if (!bad[(size_t)me * kNumConn + t]) continue;
      retired.push_back(*own[t]);
      *own[t] = nullptr;
      const uint64_t bytes = connAllocBytes(used[t], n);
      HIPCHECK(allocSyncMem(own[t], bytes, ownHandle[t]));
      HIPCHECK(hipMemset(*own[t], 0, bytes));
      fresh.h[t] = *ownHandle[t];
      info("comm %p rank %d: buffer %d re-exported at %p (round %d)", (void*)c, me, t, *own[t], round);
    }
    HIPCHECK(hipDeviceSynchronize());
    std::vector<Fresh> allFresh(n);
    NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &fresh, sizeof(fresh), allFresh.data()));
    for (int j = 0; j < n; j++) {
      if (j == me) continue;
      for (int t = 0; t < kNumConn; t++) {
        if (!bad[(size_t)j * kNumConn + t]) continue;
        auto it = std::find(mp->peerMaps.begin(), mp->peerMaps.end(), (void*)peer[j][t]);
        if (it != mp->peerMaps.end()) mp->peerMaps.erase(it);
        HIPCHECK(hipIpcCloseMemHandle(peer[j][t]));
        cur[(size_t)j * kNumConn + t] = allFresh[j].h[t];
        NCCLCHECK(open(j, t));
      }
    }
  }
  for (void* q : retired) (void)hipFree(q);
  NCCLCHECK(res);
  // the device tables of peer buffers (own entry: own buffer)
  std::vector<uint64_t*> llTable(n), l128Table(n, nullptr), flagTable(n);
  std::vector<char*> stageTable(n);
  for (int j = 0; j < n; j++) {
    llTable[j] = j == me ? mp->ll : (uint64_t*)peer[j][kConnLL];
    l128Table[j] = j == me ? mp->l128 : (uint64_t*)peer[j][kConnL128];
    stageTable[j] = j == me ? mp->stage : peer[j][kConnStage];
    flagTable[j] = j == me ? mp->sflags : (uint64_t*)peer[j][kConnFlags];
  }
  auto upload = [](void** dev, const void* host, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(dev, bytes);
    return e != hipSuccess ? e : hipMemcpy(*dev, host, bytes, hipMemcpyHostToDevice);
  };
  HIPCHECK(upload((void**)&mp->peerLLDev, llTable.data(), n * sizeof(uint64_t*)));
  if (mp->l128) HIPCHECK(upload((void**)&mp->peerL128Dev, l128Table.data(), n * sizeof(uint64_t*)));
  HIPCHECK(upload((void**)&mp->peerStageDev, stageTable.data(), n * sizeof(char*)));
  HIPCHECK(upload((void**)&mp->peerSFlagsDev, flagTable.data(), n * sizeof(uint64_t*)));
  return ncclSuccess;
}

ncclResult_t mpInit(ncclComm* c, const ncclUniqueId& id) {
  MpState* mp = new MpState();
  c->mp = mp;
  const int n = c->nRanks, me = c->rank;
  mp->ring = algoRingFromEnv();
  NCCLCHECK(nbx::bootstrapConnect(id, me, n, &mp->bs));
  // where every rank runs: decides LL128's self-test and the Simple grid
  MpPreInfo pre{};
  {
    int dom = 0, bus = 0, dv = 0, cus = 0;
    (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->device);
    (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device);
    (void)hipDeviceGetAttribute(&dv, hipDeviceAttributePciDeviceId, c->device);
    HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
    pre.pciKey = ((uint64_t)(uint32_t)dom << 32) | ((uint64_t)(uint32_t)bus << 8) | (uint64_t)(uint32_t)dv;
    pre.device = c->device;
    pre.cus = cus;
  }
  std::vector<MpPreInfo> pres(n);
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &pre, sizeof(pre), pres.data()));
  int minCus = pre.cus, maxShare = 1;
  for (int j = 0; j < n; j++) {
    mp->multiGpu |= pres[j].pciKey != pre.pciKey;
    minCus = std::min(minCus, (int)pres[j].cus);
    int share = 0;
    for (int q = 0; q < n; q++) share += pres[q].pciKey == pres[j].pciKey;
    maxShare = std::max(maxShare, share);
  }
  mpTransportSettings(mp, minCus, maxShare);
  NCCLCHECK(mpAllocLL(mp, n, /*ipc=*/true, c));
  mp->protoMask = protoGateAcrossGpus(mp->protoMask, mp->multiGpu, std::getenv("NCCL_PROTO"));   // before the settings are compared
  NCCLCHECK(mpAllocSimple(mp, n, /*ipc=*/true));
  HIPCHECK(hipDeviceSynchronize());   // zeroed before any peer can map and write them

  MpInitInfo mine{};
  mine.pid = (int32_t)getpid();
  mine.device = c->device;
  mine.llMaxBytes = mp->llMaxBytes;
  mine.l128MaxBytes = mp->l128MaxBytes;
  mine.l128OneShotMax = mp->l128OneShotMax;
  mine.sliceBytes = mp->sliceBytes;
  mine.protoMask = mp->protoMask;
  mine.ring = mp->ring;
  mine.slots = mp->slots;
  mine.simpleGrid = mp->simpleGrid;
  mine.groupBatch = mp->groupBatch;
  mine.checkPlans = mp->checkPlans;
  mine.nonce = std::random_device{}() * 0x100000001ull ^ (uint64_t)std::random_device{}() ^
               ((uint64_t)getpid() << 20) ^ (uint64_t)(uintptr_t)mp;
  mine.llHandle = mp->llHandle;
  if (mp->l128) mine.l128Handle = mp->l128Handle;
  mine.stageHandle = mp->stageHandle;
  mine.sflagsHandle = mp->sflagsHandle;
  std::vector<MpInitInfo> all(n);
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &mine, sizeof(mine), all.data()));
  for (int j = 0; j < n; j++) {
    // every rank must pick the same protocol, grid and layout for the same call
    if (all[j].llMaxBytes != mp->llMaxBytes || all[j].l128MaxBytes != mp->l128MaxBytes ||
        all[j].l128OneShotMax != mp->l128OneShotMax || all[j].protoMask != mp->protoMask) {
      warn("ncclCommInitRank : NCCL_PROTO / NBX_LL_MAX_BYTES / NBX_LL128_MAX_BYTES / NBX_LL128_ONESHOT_MAX differ "
           "across ranks");
      return ncclInvalidUsage;
    }
    if (all[j].ring != mine.ring || all[j].sliceBytes != mine.sliceBytes || all[j].slots != mine.slots ||
        all[j].simpleGrid != mine.simpleGrid) {
      warn("ncclCommInitRank : NCCL_ALGO / NBX_SIMPLE_MAX_GRID / NBX_SIMPLE_SLICE_BYTES / NBX_SIMPLE_SLOTS differ "
           "across ranks");
      return ncclInvalidUsage;
    }
    // a group's calls become one launch or one per call, and every launch
    // advances the device-resident sequence by one: ranks must cut alike
    if (all[j].groupBatch != mine.groupBatch) {
      warn("ncclCommInitRank : NBX_GROUP_BATCH differs across ranks");
      return ncclInvalidUsage;
    }
    // a checking rank would wait for plan words a non-checking peer never stamps
    if (all[j].checkPlans != mine.checkPlans) {
      warn("ncclCommInitRank : NBX_CHECK_PLANS / NCCL_CHECK_POINTERS differ across ranks");
      return ncclInvalidUsage;
    }
    if (j == me || all[j].device == c->device) continue;
    int can = 0;
    HIPCHECK(hipDeviceCanAccessPeer(&can, c->device, all[j].device));
    if (!can) {
      // every data path here is a kernel store to peer memory; there is no
      // host-staged transport, so fail cleanly instead of faulting later
      warn("ncclCommInitRank : device %d cannot access peer device %d (no P2P)", c->device, all[j].device);
      return ncclSystemError;
    }
    hipError_t e = hipDeviceEnablePeerAccess(all[j].device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
    (void)hipGetLastError();
  }
  // every peer buffer mapped and checked before the first collective
  NCCLCHECK(mpConnect(c, all));
  NCCLCHECK(mpLL128SelfTest(c));
  info("comm %p rank %d nranks %d device %d: multi-process communicator ready (Simple grid %d, slice %llu B, "
       "staging %llu MiB)", (void*)c, me, n, c->device, mp->simpleGrid, (unsigned long long)mp->sliceBytes,
       (unsigned long long)(mp->stageBytes >> 20));
  return ncclSuccess;
}

void mpFreeState(MpState* mp, int device) {
  DevGuard g(device);
  (void)hipDeviceSynchronize();
  for (void* p : mp->peerMaps) (void)hipIpcCloseMemHandle(p);
  for (void* p : {(void*)mp->peerStageDev, (void*)mp->peerSFlagsDev, (void*)mp->scounters, (void*)mp->sflags,
                  (void*)mp->stage, (void*)mp->peerL128Dev, (void*)mp->l128, (void*)mp->peerLLDev, (void*)mp->ll,
                  (void*)mp->llState, (void*)mp->orderMem})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : mp->groupEvents) (void)hipEventDestroy(e);
  nbx::bootstrapClose(mp->bs);
  delete mp;
}

void mpFree(ncclComm* c) {
  if (c->mp) mpFreeState(c->mp, c->device);
  if (c->lt) mpFreeState(c->lt, c->device);
  c->mp = nullptr;
  c->lt = nullptr;
}

// The protocol of a call. It depends only on arguments every rank passes
// identically (and on the init-time settings checked equal), so every rank
// picks the same one.
MpProto mpProtoOf(const ncclComm* comm, const MpCall& c) {
  const MpState* mp = mpOf(comm);
  const int n = comm->nRanks;
  const int eb = typeSize(c.dt);
  const uint64_t slotBytes = (uint64_t)c.count * (uint64_t)eb;   // RS: recvcount per block
  size_t off0, per;
  blockRange(c.count, eb, n, 0, &off0, &per);   // the direct schedule's AllReduce block
  return chooseProtoFor(mp->protoMask, c.kind != kReduceScatter, slotBytes, (uint64_t)per * (uint64_t)eb, n,
                        mp->llMaxBytes, mp->l128MaxBytes, mp->l128OneShotMax);
}

// The completion word this launch publishes (runMpColl numbers the call).
nbx::MpDone mpOrderArgs(MpState* mp) {
  mp->launched = true;
  return nbx::MpDone{(uint64_t*)mp->orderMem, (uint32_t*)(mp->orderMem + 64), mp->curSeq};
}

// LL / LL128 protocols: small and medium collectives in one kernel (nbx_ll.h).
ncclResult_t mpLaunchLL(ncclComm* comm, const MpCall& c, MpProto proto, const MpCall* segs = nullptr,
                        int nSegs = 0) {
  MpState* mp = mpOf(comm);
  const int n = comm->nRanks, me = comm->rank;
  const int eb = typeSize(c.dt);
  const uint64_t slotBytes = (uint64_t)c.count * (uint64_t)eb;
  size_t off0, per;
  blockRange(c.count, eb, n, 0, &off0, &per);
  nbx::LLArgs la{};
  la.send = c.send;
  la.recv = c.recv;
  la.count = c.count;
  la.nPacks = (slotBytes + 7) / 8;
  la.peerLL = mp->peerLLDev;
  la.myLL = mp->ll;
  la.slotLines = mp->llSlotLines;
  la.doneOff = mp->llDoneOff;
  la.planOff = mp->llPlanOff;
  la.state = mp->llState;
  la.blockElts = per > 0 ? per : 1;
  la.abortWord = mp->hostWordsDev;
  la.errWord = mp->hostWordsDev + 1;
  la.timeoutTicks = (uint64_t)(mp->timeoutSec * 1.0e8);
  la.rank = me;
  la.nRanks = n;
  la.postOp = 1;
  la.mode = c.kind == kAllReduce       ? nbx::kLLAllReduce
            : c.kind == kReduceScatter ? nbx::kLLReduceScatter
                                       : nbx::kLLReduce;
  la.root = c.root;
  la.order = mpOrderArgs(mp);
  la.gridCap = proto == kMpLL ? mp->llGridCap : mp->l128GridCap;
  // a group's calls as one launch (runMpLLGroup): their slots concatenated, in
  // units of 8-byte packs (LL) or 48-byte lines (LL128 one-shot)
  const uint64_t unit = proto == kMpLL ? 8 : (uint64_t)nbx::kL128DataBytesHost;
  uint64_t units = 0;
  if (nSegs > 1) {
    for (int s = 0; s < nSegs; s++) {
      const MpCall& g = segs[s];
      size_t o, p;
      blockRange(g.count, eb, n, 0, &o, &p);
      la.seg[s] = nbx::LLSeg{g.send, g.recv, (uint64_t)g.count, units, p > 0 ? (uint64_t)p : 1};
      units += ((uint64_t)g.count * (uint64_t)eb + unit - 1) / unit;
    }
    la.nSegs = nSegs;
  }
  if (proto == kMpLL128 || proto == kMpLL128x2) {
    la.peerL128 = mp->peerL128Dev;
    la.myL128 = mp->l128;
    la.l128SlotLines = mp->l128SlotLines;
    la.l128Bytes = (uint32_t)mp->l128Bytes;
    if (proto == kMpLL128x2) {
      la.nSegs = 0;   // never grouped (runMpGroup)
      la.nLines = mp->l128SlotLines / 2;   // sub-slot lines: [parity][RS|AG][source]
      const uint64_t blockLines =
          ((uint64_t)per * (uint64_t)eb + nbx::kL128DataBytesHost - 1) / nbx::kL128DataBytesHost;
      la.planSig = mp->checkPlans ? nbx::llPlanSig(la, (int32_t)proto, (int32_t)c.dt, c.op.op) : 0;
      return nbx::launchLL128AllReduce2(c.dt, c.op, la, blockLines, c.stream);
    }
    la.nLines = nSegs > 1 ? units : (slotBytes + nbx::kL128DataBytesHost - 1) / nbx::kL128DataBytesHost;
    la.planSig = mp->checkPlans ? nbx::llPlanSig(la, (int32_t)proto, (int32_t)c.dt, c.op.op) : 0;
    return nbx::launchLL128Coll(c.dt, c.op, la, c.stream);
  }
  if (nSegs > 1) la.nPacks = units;
  la.planSig = mp->checkPlans ? nbx::llPlanSig(la, (int32_t)proto, (int32_t)c.dt, c.op.op) : 0;
  return nbx::launchLLColl(c.dt, c.op, la, c.stream);
}

// Simple protocol: one kernel (nbx_simple.h). Blocks: AllReduce / Reduce the
// direct schedule's 16-B aligned blocks (blockRange; the ring's chunks are the
// same blocks), ReduceScatter the API's recvcount blocks, ring Reduce the
// whole message as one block (a chain). A call of B-byte blocks runs on
// min(grid, B / 4 KiB) workgroups in rounds of one slice per workgroup and
// block, the slice at most the staging slice — every rank derives the same
// numbers from the same arguments. Several calls of one group (nc > 1, same
// kind / type / op / root) run as ONE launch: block b of the launch is block
// b of every message in turn (SimpleSeg), cut into the launch's slices.
ncclResult_t mpLaunchSimple(ncclComm* comm, const MpCall* calls, int nc, bool transport = false) {
  MpState* mp = mpOf(comm);
  const MpCall& c = calls[0];
  const int n = comm->nRanks, me = comm->rank;
  const uint64_t eb = (uint64_t)typeSize(c.dt);
  auto shape = [&](const MpCall& m, uint64_t* blockElts, uint64_t* total) {
    if (m.kind == kReduceScatter) {
      *blockElts = m.count;
      *total = (uint64_t)m.count * (uint64_t)n;
    } else if (m.kind == kReduce && mp->ring) {
      *blockElts = m.count;
      *total = m.count;
    } else {
      size_t o0, per;
      blockRange(m.count, (int)eb, n, 0, &o0, &per);
      *blockElts = per;
      *total = m.count;
    }
  };
  nbx::SimpleArgs sa{};
  sa.send = c.send;
  sa.recv = c.recv;
  shape(c, &sa.blockElts, &sa.total);
  uint64_t blockBytes = std::min<uint64_t>(sa.blockElts, sa.total) * eb;   // every message's block 0 together
  std::vector<uint64_t> segBlockBytes;
  if (nc > 1) {
    blockBytes = 0;
    for (int s = 0; s < nc; s++) {
      uint64_t be, tot;
      shape(calls[s], &be, &tot);
      sa.seg[s] = nbx::SimpleSeg{calls[s].send, calls[s].recv, tot, be, 0};
      segBlockBytes.push_back(std::min<uint64_t>(be, tot) * eb);
      blockBytes += segBlockBytes.back();
    }
    sa.nSegs = nc;
  }
  if (blockBytes == 0) return ncclSuccess;
  uint64_t grid = (blockBytes + nbx::kSimpleMinSliceBytes - 1) / nbx::kSimpleMinSliceBytes;
  grid = std::max<uint64_t>(1, std::min<uint64_t>(grid, (uint64_t)mp->simpleGrid));
  uint64_t slice = ((blockBytes + grid - 1) / grid + 15) & ~(uint64_t)15;
  slice = std::min<uint64_t>(slice, mp->sliceBytes);
  sa.sliceBytes = slice;
  if (nc > 1) {   // every message's slices of a block, back to back
    uint64_t off = 0;
    for (int s = 0; s < nc; s++) {
      sa.seg[s].sliceOff = off;
      off += (segBlockBytes[s] + slice - 1) / slice;
    }
    sa.nRounds = (off + grid - 1) / grid;
  } else {
    sa.nRounds = (blockBytes + grid * slice - 1) / (grid * slice);
  }
  sa.peerStage = mp->peerStageDev;
  sa.peerFlags = mp->peerSFlagsDev;
  sa.counters = mp->scounters;
  sa.stageSlice = mp->sliceBytes;
  sa.abortWord = mp->hostWordsDev;
  sa.errWord = mp->hostWordsDev + 1;
  sa.timeoutTicks = (uint64_t)(mp->timeoutSec * 1.0e8);
  sa.rank = me;
  sa.nRanks = n;
  sa.mode = transport                  ? nbx::kSimpleTransport
            : c.kind == kAllReduce     ? nbx::kSimpleAllReduce
            : c.kind == kReduceScatter ? nbx::kSimpleReduceScatter
                                       : nbx::kSimpleReduce;
  sa.root = c.root;
  sa.slots = mp->slots;
  sa.gridMax = mp->simpleGrid;
  sa.prefetch = mp->simplePrefetch;
  sa.hdrOff = mp->stageHdrOff;
  sa.planSig = mp->checkPlans ? nbx::simplePlanSig(sa, (uint32_t)grid, (int32_t)c.dt, c.op.op) : 0;
  sa.order = mpOrderArgs(mp);
  return nbx::launchSimple(c.dt, c.op, sa, (unsigned)grid, mp->ring && !transport, c.stream);
}

// One call of a multi-process communicator, ordered after the previous one:
// the kernels share the communicator's device-resident sequencing, and NCCL's
// calls on one communicator never overlap. Every eager call is numbered and
// its kernel's last block publishes the number in the communicator's done
// word (MpDone, nbx_order.h); a call on another stream than the previous
// one's is preceded on its stream by kMpWaitDone for the previous number. So
// the common one-stream path adds nothing to a call, where an event recorded
// behind every call cost ~5 us of device time per call
// (scripts/probe_order_cost.hip: 2.9 -> 7.9 us per back-to-back tiny
// kernel; nbx_perf 4 KiB LL AllReduce 9.7 vs 5.1 us,
// profiles/r3/nbx_perf_stream_order_r3f.txt), and nothing ever touches a
// stream other than the one the caller just passed (hipEventRecord on a
// destroyed stream's handle crashes the process: scripts/probe_stream_id.hip,
// r3g). Inside a stream capture the graph's own edges order the captured
// calls; they are numbered 0 and publish nothing.
// The cross-stream order around one launch on `stream` (see above).
template <class Launch>
ncclResult_t runMpOrdered(ncclComm* comm, hipStream_t stream, Launch&& launch) {
  MpState* mp = mpOf(comm);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(stream, &cap));
  const bool order = cap == hipStreamCaptureStatusNone && mp->streamOrder;
  if (order && mp->lastSeq != 0 && mp->lastStream != stream)
    NCCLCHECK(nbx::launchMpWaitDone((const uint64_t*)mp->orderMem, mp->lastSeq, mp->hostWordsDev, mp->hostWordsDev + 1,
                                    (uint64_t)(mp->timeoutSec * 1.0e8), stream));
  if (order && mp->extStream != nullptr && mp->extStream != stream)   // clique: after a fold-path call
    for (hipEvent_t e : mp->extDone) HIPCHECK(hipStreamWaitEvent(stream, e, 0));
  mp->curSeq = order ? mp->callSeq + 1 : 0;
  mp->launched = false;
  NCCLCHECK(launch());
  if (order && mp->launched) {
    mp->callSeq++;
    mp->lastSeq = mp->callSeq;
    mp->lastStream = stream;
    mp->extStream = nullptr;
  }
  return ncclSuccess;
}

ncclResult_t runMpColl(ncclComm* comm, const MpCall& c) {
  if (c.count == 0) return ncclSuccess;
  return runMpOrdered(comm, c.stream, [&]() -> ncclResult_t {
    const MpProto proto = mpProtoOf(comm, c);
    return proto == kMpSimple ? mpLaunchSimple(comm, &c, 1) : mpLaunchLL(comm, c, proto);
  });
}

// Several LL / LL128 one-shot / Simple calls of one group as ONE kernel (NCCL
// aggregates a group's collectives into one launch, enqueue.cc:67-91): their
// LL slots concatenated (LLSeg), or their Simple blocks (SimpleSeg). The
// launch goes on the first call's stream; if the calls use other
// streams too, the first waits for them before it and they wait for it after
// (NCCL's fan-in / fan-out, enqueue.cc:964-995, 1135-1148).
ncclResult_t runMpLLGroup(ncclComm* comm, const MpCall* calls, int nc, MpProto proto) {
  MpState* mp = mpOf(comm);
  hipStream_t s0 = calls[0].stream;
  std::vector<hipStream_t> others;
  for (int k = 1; k < nc; k++)
    if (calls[k].stream != s0 && std::find(others.begin(), others.end(), calls[k].stream) == others.end())
      others.push_back(calls[k].stream);
  while (mp->groupEvents.size() < others.size() + 1) {
    hipEvent_t e;
    HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    mp->groupEvents.push_back(e);
  }
  for (size_t k = 0; k < others.size(); k++) {
    HIPCHECK(hipEventRecord(mp->groupEvents[k + 1], others[k]));
    HIPCHECK(hipStreamWaitEvent(s0, mp->groupEvents[k + 1], 0));
  }
  NCCLCHECK(runMpOrdered(comm, s0, [&]() {
    return proto == kMpSimple ? mpLaunchSimple(comm, calls, nc) : mpLaunchLL(comm, calls[0], proto, calls, nc);
  }));
  if (!others.empty()) {
    HIPCHECK(hipEventRecord(mp->groupEvents[0], s0));
    for (hipStream_t s : others) HIPCHECK(hipStreamWaitEvent(s, mp->groupEvents[0], 0));
  }
  return ncclSuccess;
}

// LL128 correctness probe at communicator creation. LL128 relies on a 64-byte
// line written by one store instruction arriving whole (the flag in its last
// 8 bytes vouches for the 56 payload bytes, nbx_ll.h). That holds for every
// configuration measured here, but it is a property of the fabric between the
// GPUs of this communicator, so each communicator checks it before use:
// NBX_LL128_SELFTEST_ITERS (default 24; 0 = skip) AllReduces of integer data
// that changes every call, at one-shot and at two-shot sizes, each result
// compared exactly on the host. If any rank sees any wrong element, every rank
// drops LL128 from its protocol set (decided from an allgather, so the choice
// stays identical everywhere) and LL / Simple carry those sizes.
ncclResult_t mpLL128SelfTest(ncclComm* c) {
  MpState* mp = c->mp;
  if (!(mp->protoMask & kProtoLL128) || mp->l128MaxBytes == 0) return ncclSuccess;
  // only across GPUs (within one GPU the 64-byte line was stress-tested, DESIGN
  // §6), unless NBX_LL128_SELFTEST_ITERS asks for it explicitly; multiGpu is
  // the same on every rank (derived from every rank's PCI key)
  const char* v = std::getenv("NBX_LL128_SELFTEST_ITERS");
  const long iters = (v && *v) ? std::atol(v) : (mp->multiGpu ? 24 : 0);
  if (iters <= 0) return ncclSuccess;
  const int n = c->nRanks, me = c->rank;
  // one-shot (just above the LL limit) and two-shot (n > 2, above the one-shot limit) sizes
  std::vector<size_t> counts = {(size_t)(mp->llMaxBytes / 4 + 1024)};
  const uint64_t twoShot = std::min<uint64_t>(mp->l128OneShotMax * 2, mp->l128MaxBytes);
  if (n > 2 && twoShot > mp->l128OneShotMax) counts.push_back((size_t)(twoShot / 4 - 13));
  size_t maxCount = 0;
  for (size_t k : counts) maxCount = std::max(maxCount, k);
  DevGuard g(c->device);
  hipStream_t st = nullptr;
  int32_t* dSend = nullptr;
  int32_t* dRecv = nullptr;
  HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  HIPCHECK(hipMalloc((void**)&dSend, maxCount * sizeof(int32_t)));
  HIPCHECK(hipMalloc((void**)&dRecv, maxCount * sizeof(int32_t)));
  std::vector<int32_t> hIn(maxCount), hOut(maxCount);
  nbxDevRedOpFull sum{nbxDevSum, 0, 0};
  int32_t bad = 0;
  ncclResult_t r = ncclSuccess;
  for (size_t count : counts) {
    for (long it = 0; it < iters && r == ncclSuccess; it++) {
      for (size_t i = 0; i < count; i++) hIn[i] = (int32_t)((i * 7 + (size_t)me * 13 + (size_t)it * 101) % 1000);
      if (hipMemcpyAsync(dSend, hIn.data(), count * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
        r = ncclUnhandledCudaError;
        break;
      }
      const MpCall call{kAllReduce, dSend, dRecv, count, ncclInt32, sum, 0, st};
      r = runMpColl(c, call);
      if (r != ncclSuccess) break;
      if (hipMemcpyAsync(hOut.data(), dRecv, count * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        r = ncclUnhandledCudaError;
        break;
      }
      if (mp->hostWords[1] != 0) {   // a device wait gave up: an error, not a torn line
        mpReportDeviceError(c);
        warn("comm %p rank %d: LL128 self-test call %ld (%zu elements) did not complete", (void*)c, me, it, count);
        r = ncclRemoteError;
        break;
      }
      for (size_t i = 0; i < count && !bad; i++) {
        int64_t want = 0;
        for (int q = 0; q < n; q++) want += (int64_t)((i * 7 + (size_t)q * 13 + (size_t)it * 101) % 1000);
        if (hOut[i] != (int32_t)want) bad = 1;
      }
    }
  }
  const char* fail = std::getenv("NBX_LL128_SELFTEST_FAIL");   // test hook: simulate a torn line
  if (fail && std::strcmp(fail, "1") == 0) bad = 1;
  (void)hipStreamSynchronize(st);
  (void)hipFree(dSend);
  (void)hipFree(dRecv);
  (void)hipStreamDestroy(st);
  mp->lastSeq = 0;   // the probe's work is complete; its stream is gone
  if (r != ncclSuccess) return r;
  std::vector<int32_t> all(n);
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &bad, sizeof(bad), all.data()));
  bool anyBad = false;
  for (int32_t b : all) anyBad |= b != 0;
  if (anyBad) {
    warn("comm %p rank %d: LL128 self-test found torn lines on this fabric; LL128 disabled for this communicator",
         (void*)c, me);
    mp->protoMask &= ~kProtoLL128;
  }
  return ncclSuccess;
}


// ---------------------------------------------------------------------------
// Groups on a multi-process communicator (group.cc:82-103 semantics): calls
// inside ncclGroupStart/End are queued and launched, in order, at the
// outermost ncclGroupEnd, each as its own kernel on its stream. No host
// exchange keeps the ranks in step: every kernel's sequencing is per
// workgroup and device-resident, so the ranks only have to issue the same
// calls in the same order, as NCCL requires.
thread_local std::vector<ncclComm*> t_groupMpComms;

// Maximal runs of consecutive calls of the same protocol (LL, LL128
// one-shot, or Simple) with the same kind, datatype, op and root — LL / LL128
// runs whose slots fit one slot of that protocol together, at most
// kLLMaxSegs / kSimpleMaxSegs calls — run as one launch (runMpLLGroup): a
// decision made from arguments every rank passes identically, so every rank
// cuts the same runs. A run also ends before a call that reads or writes
// what an earlier call of the run writes (or writes what it reads): the
// segments of one launch run concurrently, so such a chain (AllReduce a->b,
// then b->c) must stay separate launches, in order. That cut looks at this
// rank's own buffers; the ranks of an SPMD program alias alike and cut alike.
// A Reduce never joins a run: its recv buffer is written on the root only (a
// non-root may even pass NULL), so a cut that looked at it would split the
// root's run where the non-roots batch theirs — every rank runs
// each grouped Reduce as its own launch instead, a rule every rank evaluates
// alike. A group whose AllReduce / ReduceScatter calls alias differently on
// different ranks is outside what the batching supports (LL / LL128 ranks then
// time out waiting for lines that never come; Simple ranks could fold
// misplaced slices; NBX_CHECK_PLANS=1 makes both fail loudly, naming the peer):
// NBX_GROUP_BATCH=0 runs every grouped call as its own kernel, in order.
void mpCallSpans(const MpCall& c, int n, std::vector<Span>* out) {
  const size_t eb = (size_t)typeSize(c.dt);
  const size_t sendBytes = (c.kind == kReduceScatter ? c.count * (size_t)n : c.count) * eb;
  out->push_back({(uintptr_t)c.send, (uintptr_t)c.send + sendBytes, false});
  if (c.recv != nullptr) out->push_back({(uintptr_t)c.recv, (uintptr_t)c.recv + c.count * eb, true});
}

ncclResult_t runMpGroup(ncclComm* comm) {
  DevGuard g(comm->device);
  MpState* mp = mpOf(comm);
  std::vector<MpCall> calls;
  calls.swap(mp->group);
  ncclResult_t r = ncclSuccess;
  // units of one call in its protocol's slot, and the slot's capacity
  auto unitsOf = [&](const MpCall& c, MpProto p) {
    const uint64_t unit = p == kMpLL ? 8 : (uint64_t)nbx::kL128DataBytesHost;
    return ((uint64_t)c.count * (uint64_t)typeSize(c.dt) + unit - 1) / unit;
  };
  auto capOf = [&](MpProto p) {
    return p == kMpLL ? mp->llSlotLines / 2 : p == kMpLL128 ? mp->l128SlotLines : ~(uint64_t)0;   // Simple: rounds
  };
  auto sameOp = [](const MpCall& a, const MpCall& b) {
    return a.kind == b.kind && a.dt == b.dt && a.op.op == b.op.op && a.op.scalarArg == b.op.scalarArg &&
           a.op.scalarArgIsPtr == b.op.scalarArgIsPtr && (a.kind != kReduce || a.root == b.root);
  };
  try {
    size_t i = 0;
    while (i < calls.size() && r == ncclSuccess) {
      size_t j = i + 1;
      const MpProto p = calls[i].count > 0 ? mpProtoOf(comm, calls[i]) : kMpSimple;
      const size_t maxSegs = p == kMpSimple ? (size_t)nbx::kSimpleMaxSegs : (size_t)nbx::kLLMaxSegs;
      if (mp->groupBatch && calls[i].kind != kReduce && (p == kMpLL || p == kMpLL128 || p == kMpSimple)) {
        uint64_t used = p == kMpSimple ? 0 : unitsOf(calls[i], p);
        std::vector<Span> spans, sj;
        mpCallSpans(calls[i], comm->nRanks, &spans);
        while (j < calls.size() && j - i < maxSegs && calls[j].count > 0 && sameOp(calls[i], calls[j]) &&
               mpProtoOf(comm, calls[j]) == p && (p == kMpSimple || used + unitsOf(calls[j], p) <= capOf(p))) {
          sj.clear();
          mpCallSpans(calls[j], comm->nRanks, &sj);
          if (spansConflict(spans, sj)) break;
          spans.insert(spans.end(), sj.begin(), sj.end());
          if (p != kMpSimple) used += unitsOf(calls[j], p);
          j++;
        }
      }
      r = j - i > 1 ? runMpLLGroup(comm, &calls[i], (int)(j - i), p) : runMpColl(comm, calls[i]);
      i = j;
    }
  } catch (const std::exception& e) {
    warn("internal exception: %s", e.what());
    r = ncclInternalError;
  }
  if (r != ncclSuccess) comm->asyncError.store(r);
  return r;
}

// Runs the queued calls of every multi-process communicator this thread used
// in the group that just ended; the first error is returned.
ncclResult_t flushMpGroups() {
  std::vector<ncclComm*> comms;
  comms.swap(t_groupMpComms);
  ncclResult_t first = ncclSuccess;
  for (ncclComm* c : comms) {
    if (c->magic != kCommMagic || c->mp == nullptr) continue;
    ncclResult_t r = runMpGroup(c);
    if (first == ncclSuccess) first = r;
  }
  return first;
}

// ---------------------------------------------------------------------------
// In-process clique over the LL family. Every rank of a clique whose devices
// are all distinct (NCCL's own rule for one communicator) gets the LL / LL128
// connection buffers a multi-process rank has, with its peers' buffers reached
// through plain device pointers — peer access is enabled by ncclCommInitAll,
// so nothing is IPC-mapped and nothing is exchanged. LL- and LL128-sized calls
// then run as ONE kernel per rank with the flow control inside it (nbx_ll.h),
// ordered across streams by the completion word (nbx_order.h), instead of the
// fold path's event exchange (2 markers and 2(n-1) waits per rank and call,
// ~5 us of device time per marker). Simple-sized calls keep the fold path
// (runCliqueColl): one kernel per rank that reads every rank's buffers in
// place, bandwidth-bound rather than latency-bound.
// NBX_CLIQUE_LL=1 forces the transport on for ranks sharing a GPU (each rank's
// kernel waits for its peers', so their streams must then be distinct and on
// distinct hardware queues, e.g. GPU_MAX_HW_QUEUES >= ranks + 2); 0 turns it
// off. A call whose ranks share a stream takes the fold path either way.
ncclResult_t cliqueInitTransport(Clique* cl) {
  const int n = cl->n;
  bool distinct = true;
  for (int r = 0; r < n; r++)
    for (int j = 0; j < r; j++) distinct &= cl->devs[r] != cl->devs[j];
  const char* v = std::getenv("NBX_CLIQUE_LL");
  if (!((v && *v) ? std::atoi(v) != 0 : distinct)) return ncclSuccess;
  // Simple sizes in-kernel too (the multi-process Simple kernels over the
  // clique's staging, reached by direct peer pointers) unless NBX_CLIQUE_SIMPLE=0
  // keeps them on the event-ordered fold
  const bool simple = envLong("NBX_CLIQUE_SIMPLE", 1) != 0;
  int minCus = 1 << 30, maxShare = 1;
  for (int r = 0; r < n; r++) {
    int cus = 0, share = 0;
    HIPCHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cl->devs[r]));
    minCus = std::min(minCus, cus);
    for (int j = 0; j < n; j++) share += cl->devs[j] == cl->devs[r];
    maxShare = std::max(maxShare, share);
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(cl->devs[r]);
    MpState* mp = new MpState();
    cl->comms[r]->lt = mp;
    NCCLCHECK(mpAllocLL(mp, n, /*ipc=*/false, cl->comms[r]));
    mp->multiGpu = distinct;
    mp->protoMask = protoGateAcrossGpus(mp->protoMask, mp->multiGpu, std::getenv("NCCL_PROTO"));
    mp->ring = algoRingFromEnv();
    mpTransportSettings(mp, minCus, maxShare);   // co-resident grids, as mpInit
    if (simple) NCCLCHECK(mpAllocSimple(mp, n, /*ipc=*/false));
    mp->extDone = cl->evDone;
  }
  std::vector<uint64_t*> llTable(n), l128Table(n), flagTable(n);
  std::vector<char*> stageTable(n);
  for (int r = 0; r < n; r++) {
    llTable[r] = cl->comms[r]->lt->ll;
    l128Table[r] = cl->comms[r]->lt->l128;
    stageTable[r] = cl->comms[r]->lt->stage;
    flagTable[r] = cl->comms[r]->lt->sflags;
  }
  for (int r = 0; r < n; r++) {
    DevGuard g(cl->devs[r]);
    MpState* mp = cl->comms[r]->lt;
    HIPCHECK(hipMalloc((void**)&mp->peerLLDev, n * sizeof(uint64_t*)));
    HIPCHECK(hipMemcpy(mp->peerLLDev, llTable.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice));
    if (mp->l128) {
      HIPCHECK(hipMalloc((void**)&mp->peerL128Dev, n * sizeof(uint64_t*)));
      HIPCHECK(hipMemcpy(mp->peerL128Dev, l128Table.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice));
    }
    if (simple) {
      HIPCHECK(hipMalloc((void**)&mp->peerStageDev, n * sizeof(char*)));
      HIPCHECK(hipMemcpy(mp->peerStageDev, stageTable.data(), n * sizeof(char*), hipMemcpyHostToDevice));
      HIPCHECK(hipMalloc((void**)&mp->peerSFlagsDev, n * sizeof(uint64_t*)));
      HIPCHECK(hipMemcpy(mp->peerSFlagsDev, flagTable.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice));
    }
    HIPCHECK(hipDeviceSynchronize());   // zeroed and uploaded before any peer's first kernel
  }
  cl->ll = true;
  cl->simple = simple;
  // above this the direct fold (peers' buffers read in place, no staging copy)
  // keeps large messages: on one GPU it wins from 64 MiB (the staging design
  // moves twice the HBM bytes there) and loses up to 16 MiB to the
  // event exchange; the xGMI crossover is for the first multi-GPU run to set
  cl->simpleMaxBytes = (uint64_t)envLong("NBX_CLIQUE_SIMPLE_MAX_BYTES", 32 << 20);
  info("clique of %d ranks: LL / LL128%s-sized calls run in-kernel (grid caps %u / %u)", n,
       simple ? " / Simple" : "", cl->comms[0]->lt->llGridCap, cl->comms[0]->lt->l128GridCap);
  return ncclSuccess;
}

// Whether a clique collective runs in-kernel on the in-process transport
// (one kernel per rank, its protocol chosen as on a multi-process
// communicator) or on the event-ordered fold path. Decided once for all ranks.
bool cliqueInKernel(Clique* c, const std::vector<PendingColl>& parts) {
  if (!c->ll || parts[0].count == 0 || !sameCollective(parts)) return false;
  for (int r = 0; r < c->n; r++) {
    if (c->comms[r] == nullptr || c->comms[r]->lt == nullptr) return false;
    for (int j = 0; j < r; j++)
      if (parts[j].stream == parts[r].stream) return false;   // one rank's kernel would queue behind another's
  }
  if (mpProtoOf(c->comms[0], parts[0]) != kMpSimple) return true;
  const PendingColl& p0 = parts[0];
  const uint64_t sendBytes =
      (uint64_t)p0.count * (uint64_t)typeSize(p0.dt) * (p0.kind == kReduceScatter ? (uint64_t)c->n : 1u);
  return c->simple && sendBytes <= c->simpleMaxBytes;
}

// Consecutive in-kernel collectives [lo, hi): every rank runs them as a group
// (runMpGroup cuts the same batched launches on every rank).
ncclResult_t cliqueRunLL(Clique* c, const std::vector<std::vector<PendingColl>>& rounds, size_t lo, size_t hi) {
  for (int r = 0; r < c->n; r++) {
    ncclComm* comm = c->comms[r];
    comm->lt->group.clear();
    for (size_t k = lo; k < hi; k++) comm->lt->group.push_back(rounds[k][r]);
    NCCLCHECK(runMpGroup(comm));
  }
  return ncclSuccess;
}

// Around a fold-path call on rank r's stream s: like runMpOrdered, it first
// waits for the communicator's previous call when that ran on another stream
// (the completion word after an in-kernel call, every rank's evDone after a
// fold-path call), and leaves the state the next call orders against.
ncclResult_t cliqueOrderBefore(Clique* c, int r, hipStream_t s) {
  MpState* mp = c->comms[r] ? c->comms[r]->lt : nullptr;
  if (mp == nullptr || !mp->streamOrder) return ncclSuccess;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return ncclSuccess;
  if (mp->lastSeq != 0 && mp->lastStream != s)
    NCCLCHECK(nbx::launchMpWaitDone((const uint64_t*)mp->orderMem, mp->lastSeq, mp->hostWordsDev, mp->hostWordsDev + 1,
                                    (uint64_t)(mp->timeoutSec * 1.0e8), s));
  if (mp->extStream != nullptr && mp->extStream != s)
    for (hipEvent_t e : mp->extDone) HIPCHECK(hipStreamWaitEvent(s, e, 0));
  return ncclSuccess;
}

ncclResult_t cliqueOrderAfter(Clique* c, int r, hipStream_t s) {
  MpState* mp = c->comms[r] ? c->comms[r]->lt : nullptr;
  if (mp == nullptr || !mp->streamOrder) return ncclSuccess;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(s, &cap));
  if (cap != hipStreamCaptureStatusNone) return ncclSuccess;
  mp->lastSeq = 0;   // complete once every evDone is: that is what a later call on another stream waits for
  mp->extStream = s;
  return ncclSuccess;
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
  if (comm->mp) {
    const MpCall call{kind, sendbuff, recvbuff, count, dt, opFull, root, stream};
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
    comm->clique->pending[comm->rank].push_back(PendingColl{kind, sendbuff, recvbuff, count, dt, opFull, root, stream});
  }
  if (t_groupDepth == 0) return flushPending();
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
  if (config && config->blocking != NCCL_CONFIG_UNDEF_INT) c->blocking = config->blocking;
  if (const char* be = std::getenv("NCCL_COMM_BLOCKING")) {   // init.cc:1444-1446: the env overrides the config
    char* end = nullptr;
    const long v = std::strtol(be, &end, 10);
    if (end != be && *end == '\0' && (v == 0 || v == 1)) c->blocking = (int)v;
  }
  *out = c;
  return ncclSuccess;
}

}  // namespace

// ===========================================================================
// Public C ABI

NBX_API(ncclResult_t, ncclGetVersion, int* version) {
  if (version == nullptr) return ncclInvalidArgument;
  *version = NCCL_VERSION_CODE;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclGetUniqueId, ncclUniqueId* out) {
  if (out == nullptr) return ncclInvalidArgument;
  return nbx::bootstrapCreateRoot(out);   // bootstrap.cc: the root listens for the ranks
}

NBX_API(ncclResult_t, ncclCommInitRankConfig, ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank,
        ncclConfig_t* config) {
  if (newcomm == nullptr) return ncclInvalidArgument;
  if (nranks < 1 || myrank < 0 || myrank >= nranks) {
    warn("Invalid rank requested : %d/%d", myrank, nranks);
    return ncclInvalidArgument;
  }
  if (config && (config->magic != 0xcafebeef || config->size != sizeof(ncclConfig_t))) {
    warn("ncclCommInitRankConfig : config is not initialized with NCCL_CONFIG_INITIALIZER");
    return ncclInvalidArgument;
  }
  if (std::memcmp(commId.internal, kIdMagic, sizeof(kIdMagic)) != 0) {
    warn("ncclCommInitRank : unique id was not produced by ncclGetUniqueId");
    return ncclInvalidArgument;
  }
  if (nranks > kMaxMpRanks) {   // one staging source region and one counter set per rank (kSimpleMaxRanks)
    warn("ncclCommInitRank : %d ranks requested, this build supports up to %d per communicator", nranks,
         kMaxMpRanks);
    return ncclInvalidArgument;
  }
  if (config && config->blocking != NCCL_CONFIG_UNDEF_INT && config->blocking != 0 && config->blocking != 1) {
    warn("Invalid config blocking attribute value %d", config->blocking);   // init.cc:1544-1547
    return ncclInvalidArgument;
  }
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  if (nranks == 1) {
    NCCLCHECK(newComm(newcomm, 1, 0, dev, config));
    return (*newcomm)->blocking ? ncclSuccess : ncclInProgress;   // nothing to wait for: already ready
  }
  if (!nbx::bootstrapIdHasRoot(commId)) {
    warn("ncclCommInitRank : unique id carries no bootstrap root");
    return ncclInvalidArgument;
  }
  ncclComm* c = nullptr;
  NCCLCHECK(newComm(&c, nranks, myrank, dev, config));
  auto init = [](ncclComm* cm, ncclUniqueId id) -> ncclResult_t {
    ncclResult_t r;
    try {
      r = mpInit(cm, id);
    } catch (const std::exception& e) {
      warn("internal exception: %s", e.what());
      r = ncclInternalError;
    }
    if (r != ncclSuccess) mpFree(cm);
    return r;
  };
  if (!c->blocking) {
    // non-blocking (init.cc:1757-1771, group.cc:390-415): the communicator is
    // handed out at once and initialised by a background thread;
    // ncclCommGetAsyncError reports ncclInProgress until it is done
    c->asyncError.store(ncclInProgress);
    *newcomm = c;
    try {
      c->initThread = std::thread([c, commId, dev, init] {
        (void)hipSetDevice(dev);
        nbx::bootstrapSetAbortFlag(&c->initAbort);
        c->asyncError.store(init(c, commId));
        nbx::bootstrapSetAbortFlag(nullptr);
      });
    } catch (const std::exception& e) {
      warn("ncclCommInitRankConfig : cannot start the initialisation thread: %s", e.what());
      c->asyncError.store(ncclSystemError);
      return ncclSystemError;
    }
    return ncclInProgress;
  }
  const ncclResult_t r = init(c, commId);
  if (r != ncclSuccess) {
    delete c;
    return r;
  }
  *newcomm = c;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommInitRank, ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank) {
  return ncclCommInitRankConfig(newcomm, nranks, commId, myrank, nullptr);
}

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
  if (config == nullptr) {
    cfg.blocking = comm->blocking;
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

NBX_API(ncclResult_t, ncclCommInitAll, ncclComm_t* comms, int ndev, const int* devlist) {
  // init.cc:1678-1734. Several ranks may share one device (emulation / testing).
  if (comms == nullptr || ndev < 1 || ndev > kMaxMpRanks) {
    warn("ncclCommInitAll : invalid arguments");
    return ncclInvalidArgument;
  }
  int nDevices = 0;
  HIPCHECK(hipGetDeviceCount(&nDevices));
  std::vector<int> devs(ndev);
  for (int i = 0; i < ndev; i++) {
    devs[i] = devlist ? devlist[i] : i;
    if (devs[i] < 0 || devs[i] >= nDevices) {
      warn("ncclCommInitAll : invalid device %d", devs[i]);
      return ncclInvalidArgument;
    }
  }
  if (ndev == 1) {
    DevGuard g(devs[0]);
    return newComm(&comms[0], 1, 0, devs[0], nullptr);
  }
  auto clique = std::make_shared<Clique>();
  clique->n = ndev;
  clique->devs = devs;
  clique->evEnter.resize(ndev);
  clique->evReduced.resize(ndev);
  clique->evDone.resize(ndev);
  clique->pending.resize(ndev);
  for (int r = 0; r < ndev; r++) {
    DevGuard g(devs[r]);
    for (int j = 0; j < ndev; j++) {
      if (devs[j] == devs[r]) continue;
      int can = 0;
      HIPCHECK(hipDeviceCanAccessPeer(&can, devs[r], devs[j]));
      if (!can) {
        warn("ncclCommInitAll : device %d cannot access peer %d", devs[r], devs[j]);
        return ncclUnhandledCudaError;
      }
      hipError_t e = hipDeviceEnablePeerAccess(devs[j], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
      (void)hipGetLastError();
    }
    HIPCHECK(hipEventCreateWithFlags(&clique->evEnter[r], hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&clique->evReduced[r], hipEventDisableTiming));
    HIPCHECK(hipEventCreateWithFlags(&clique->evDone[r], hipEventDisableTiming));
  }
  for (int r = 0; r < ndev; r++) {
    NCCLCHECK(newComm(&comms[r], ndev, r, devs[r], nullptr));
    comms[r]->clique = clique;
  }
  clique->comms.assign(comms, comms + ndev);
  if (cliqueInitTransport(clique.get()) != ncclSuccess) {   // every call keeps the fold path
    warn("ncclCommInitAll : in-process LL transport unavailable; every call uses the fold path");
    for (int r = 0; r < ndev; r++)
      if (comms[r]->lt) {
        mpFreeState(comms[r]->lt, devs[r]);
        comms[r]->lt = nullptr;
      }
    clique->ll = false;
  }
  {
    std::lock_guard<std::mutex> g(g_pendMu);
    g_cliques.push_back(clique);
  }
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommFinalize, ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclCommFinalize"));
  NCCLCHECK(commEnsureReady(comm));
  return flushPending();
}

static ncclResult_t commFree(ncclComm* comm) {
  std::shared_ptr<Clique> c = comm->clique;
  comm->magic = 0;
  // calls still queued in this thread's open group die with the communicator
  t_groupMpComms.erase(std::remove(t_groupMpComms.begin(), t_groupMpComms.end(), comm), t_groupMpComms.end());
  mpFree(comm);
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

NBX_EXPORT int nbxDebugProtoMask(const char* ncclProto) { return protoFromString(ncclProto); }

// The protocol set a communicator starts from (before its LL128 self-test):
// NCCL_PROTO = ncclProto, its ranks on more than one GPU or not (the LL128
// gate above; NBX_LL128_ACROSS_GPUS and NBX_DEBUG_ASSUME_MULTI_GPU apply).
NBX_EXPORT int nbxDebugGatedProtoMask(const char* ncclProto, int multiGpu) {
  return protoGateAcrossGpus(protoFromString(ncclProto), multiGpu != 0, ncclProto);
}

NBX_EXPORT int nbxDebugCommProtoMask(ncclComm_t comm) {
  if (comm == nullptr || comm->magic != kCommMagic || mpOf(comm) == nullptr) return -1;
  return mpOf(comm)->protoMask;   // a clique rank: its in-process transport's
}

// The transport settings a communicator runs with (its own, or a clique
// rank's in-process transport's): out[0] LL max bytes, [1] LL128 max bytes,
// [2] Simple slice bytes, [3] Simple slots, [4] Simple grid, [5] LL grid cap,
// [6] LL128 grid cap, [7] group batching, [8] connection buffers re-exported
// at creation because a peer's mapping of them was wrong (mpConnect), [9] plan
// checks on (NBX_CHECK_PLANS / NCCL_CHECK_POINTERS). Returns
// how many were written, -1
// for a bad handle or a communicator without that transport.
NBX_EXPORT int nbxDebugCommSettings(ncclComm_t comm, int64_t* out, int nOut) {
  if (comm == nullptr || comm->magic != kCommMagic || out == nullptr) return -1;
  if (comm->asyncError.load() != ncclSuccess) return -1;
  const MpState* mp = mpOf(comm);
  if (mp == nullptr) return -1;
  const int64_t v[10] = {(int64_t)mp->llMaxBytes, (int64_t)mp->l128MaxBytes, (int64_t)mp->sliceBytes, mp->slots,
                         mp->simpleGrid,          (int64_t)mp->llGridCap,    (int64_t)mp->l128GridCap, mp->groupBatch,
                         mp->ipcRepairs,          mp->checkPlans};
  int k = 0;
  for (; k < nOut && k < 10; k++) out[k] = v[k];
  return k;
}

// Config D's transport alone: an AllReduce-shaped call of the
// direct Simple schedule on a multi-process communicator that moves every
// byte the AllReduce moves between the ranks (pushes into the peers' staging,
// the finished blocks into theirs, the gather) with the fold reduced to a copy
// of the own input (kSimpleTransport). Collective: every rank calls it with
// the same count and datatype. recvbuff receives junk. Measurement only.
NBX_EXPORT ncclResult_t nbxDebugTransportAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                                                  ncclDataType_t datatype, ncclComm_t comm, ncclStream_t stream) {
  NCCLCHECK(commCheck(comm, "TransportAllReduce"));
  NCCLCHECK(commEnsureReady(comm));
  if (comm->mp == nullptr || typeSize(datatype) < 0 || count == 0 || sendbuff == nullptr || recvbuff == nullptr)
    return ncclInvalidArgument;
  DevGuard g(comm->device);
  const MpCall call{kAllReduce, sendbuff, recvbuff, count, datatype, nbxDevRedOpFull{nbxDevSum, 0, 0}, 0,
                    (hipStream_t)stream};
  try {
    return runMpOrdered(comm, call.stream, [&]() { return mpLaunchSimple(comm, &call, 1, /*transport=*/true); });
  } catch (const std::exception& e) {
    warn("internal exception: %s", e.what());
    return ncclInternalError;
  }
}

NBX_EXPORT int nbxDebugChooseProto(int protoMask, int twoShotKind, uint64_t slotBytes, uint64_t blockBytes, int nRanks,
                                   uint64_t llMaxBytes, uint64_t ll128MaxBytes, uint64_t ll128OneShotMax) {
  return (int)chooseProtoFor(protoMask, twoShotKind != 0, slotBytes, blockBytes, nRanks, llMaxBytes, ll128MaxBytes,
                             ll128OneShotMax);
}

NBX_EXPORT ncclResult_t nbxBootstrapSelfTest(const ncclUniqueId* id, int rank, int nranks, int rounds) {
  if (id == nullptr || nranks < 1 || rank < 0 || rank >= nranks || rounds < 0) return ncclInvalidArgument;
  nbx::Bootstrap* b = nullptr;
  NCCLCHECK(nbx::bootstrapConnect(*id, rank, nranks, &b));
  ncclResult_t res = ncclSuccess;
  for (int r = 0; r < rounds && res == ncclSuccess; r++) {
    const size_t len = 8 + (size_t)(r * 37) % 4096;
    std::vector<unsigned char> mine(len), all(len * (size_t)nranks);
    for (size_t i = 0; i < len; i++) mine[i] = (unsigned char)(rank * 31 + r * 7 + i);
    res = nbx::bootstrapAllGather(b, mine.data(), len, all.data());
    for (int j = 0; j < nranks && res == ncclSuccess; j++)
      for (size_t i = 0; i < len; i++)
        if (all[(size_t)j * len + i] != (unsigned char)(j * 31 + r * 7 + i)) {
          res = ncclInternalError;
          break;
        }
  }
  nbx::bootstrapClose(b);
  return res;
}
