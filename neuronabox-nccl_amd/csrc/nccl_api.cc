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
#include <vector>

#include "../../include/nbx_debug.h"
#include "../../include/nbx_reduce.h"
#include "nbx_bootstrap.h"
#include "nbx_shmx.h"
#include "nbx_sync.h"
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
  // 1. enter: every rank's stream reaches the collective
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
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
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    HIPCHECK(hipEventRecord(c->evReduced[r], parts[r].stream));
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
    if (batchable(rounds[i])) {
      collSpans(rounds[i], &spans);
      for (j = i + 1; j < rounds.size() && j - i < kMaxCliqueBatch; j++) {
        if (!batchable(rounds[j])) break;
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
// (bootstrap.cc, transport/p2p.cc:190-381) with: a TCP bootstrap for the
// allgathers, hipIpc handles of the caller's buffers exchanged per call
// (NCCL calls "may perform inter-CPU synchronization", nccl.h.in:253-261)
// and cached after the first map, and device flag barriers (nbx_sync.hip)
// ordering the phases on the caller's stream. The data path is the same
// one-shot direct exchange as the in-process clique.

enum { kSlotEnter = 0, kSlotReduced = 1, kSlotDone = 2, kSlotRing = 3, kNumSlots = 4 };
constexpr int kMaxMpRanks = 64;

// One reducing collective as enqueued on a multi-process communicator (the
// same record the in-process clique queues).
using MpCall = PendingColl;

struct MpState {
  nbx::Bootstrap* bs = nullptr;
  nbx::ShmExchange* shmx = nullptr;     // per-call exchange through /dev/shm (nullptr: TCP bootstrap)
  uint64_t* flags = nullptr;           // own phase flags (device memory, IPC-exported)
  uint64_t** peerFlagsDev = nullptr;   // device table: rank -> flags (self = flags)
  std::vector<void*> peerFlagMaps;     // IPC mappings to close
  int* hostWords = nullptr;            // pinned: [0] abort, [1] error
  int* hostWordsDev = nullptr;
  uint64_t seq = 0;
  double timeoutSec = 300.0;
  struct Mapping {
    void* base;
    uint64_t lastUse;   // seq of the last collective that used it; kPinned: used by a captured graph
  };
  static constexpr uint64_t kPinned = ~0ull;
  std::map<std::pair<int, std::string>, Mapping> maps;   // (peer, ipc handle) -> mapped base
  size_t mapsMax = 512;   // NBX_IPC_CACHE_MAX: beyond this, unused mappings are closed
  // LL protocol (nbx_ll.h): own buffer [2][n][slotLines] lines + [n] done words +
  // arrival counter; peers' buffers mapped
  uint64_t* ll = nullptr;
  uint64_t** peerLLDev = nullptr;
  std::vector<void*> peerLLMaps;
  uint64_t llMaxBytes = 0;
  uint64_t llSlotLines = 0;
  uint64_t llDoneOff = 0;
  nbx::LLState* llState = nullptr;  // device-resident LL-family sequencing (nbx_ll_args.h)
  uint64_t* epochs = nullptr;       // device-resident barrier epochs, one per flag slot
  // LL128 protocol (nbx_ll.h kLL128Coll): own buffer [2][n][l128SlotLines] 64-B lines;
  // shares the LL buffer's done words, arrival counter and parity credits
  uint64_t* l128 = nullptr;
  uint64_t** peerL128Dev = nullptr;
  std::vector<void*> peerL128Maps;
  uint64_t l128MaxBytes = 0;        // 0: LL128 unavailable (n > 8)
  uint64_t l128OneShotMax = 0;      // AllReduce, n > 2: one-shot up to this, two-shot above
  uint64_t l128SlotLines = 0;
  uint64_t l128Bytes = 0;
  int protoMask = 0;                // NCCL_PROTO at init: kProtoLL | kProtoLL128 | kProtoSimple
  bool ring = false;                // NCCL_ALGO=Ring at init
  bool multiGpu = false;            // the ranks span more than one physical GPU (PCI key)
  bool ringPipeline = true;         // ring as the pipelined kernel (nbx_ring.h); NBX_RING_PIPELINE=0: per-step kernels
  bool groupBatch = true;           // NBX_GROUP_BATCH at init: groups run as batched exchanges
  uint64_t* ringProg = nullptr;     // [kRingMaxGrid] progress words the left neighbour posts (uncached)
  uint64_t* rightRingProg = nullptr;// the right neighbour's words (peer mapping)
  nbx::RingState* ringState = nullptr;
  unsigned ringMaxGrid = nbx::kRingMaxGrid;   // NBX_RING_MAX_GRID
  // step FIFO of the ring ReduceScatter / chain Reduce (NCCL_ALGO=Ring only)
  void* fifo = nullptr;             // own FIFO (device memory, IPC-exported)
  uint64_t* fifoTail = nullptr;     // [kRingMaxGrid] entries the left neighbour produced (uncached)
  uint64_t* fifoHead = nullptr;     // [kRingMaxGrid] entries of `fifo` the right neighbour consumed (uncached)
  void* leftFifo = nullptr;         // peer mappings
  uint64_t* rightFifoTail = nullptr;
  uint64_t* leftFifoHead = nullptr;
  std::vector<MpCall> group;        // calls queued inside ncclGroupStart/End (run at the outermost End)
};

struct MpInitInfo {
  int32_t pid;
  int32_t device;
  hipIpcMemHandle_t flagsHandle;
  hipIpcMemHandle_t llHandle;
  hipIpcMemHandle_t l128Handle;
  hipIpcMemHandle_t ringHandle;
  hipIpcMemHandle_t fifoHandle, fifoTailHandle, fifoHeadHandle;   // NCCL_ALGO=Ring only
  uint64_t pciKey;   // (domain, bus, device) of this rank's GPU: identifies it across processes
  uint64_t llMaxBytes;
  uint64_t l128MaxBytes;
  uint64_t l128OneShotMax;
  int32_t protoMask;
  // schedule settings every rank must share: a workgroup of the pipelined ring
  // waits on its left neighbour's progress word of the same slice, so a
  // different grid (NBX_RING_MAX_GRID) or schedule would fold unfinished
  // partials or drift the barrier epochs apart
  int32_t ring;           // NCCL_ALGO=Ring
  int32_t ringPipeline;   // NBX_RING_PIPELINE
  int32_t ringMaxGrid;    // NBX_RING_MAX_GRID
  int32_t groupBatch;     // NBX_GROUP_BATCH
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

// Per message: LL up to the LL max; LL128 one-shot (every rank pushes the
// whole message to every target) up to the LL128 max — for AllReduce / Reduce
// with more than 2 ranks only up to the one-shot max; above that the LL128
// two-shot AllReduce / Reduce (reduce-scatter + gather hops) while a rank's
// block fits half an LL128 slot; else Simple. ReduceScatter is one hop by
// nature: one-shot up to the LL128 max.
enum MpProto { kMpLL = 0, kMpLL128 = 1, kMpSimple = 2, kMpLL128x2 = 3 };
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
    } else if (blockBytes <= (l128SlotLinesFor(l128Max) / 2) * nbx::kL128DataBytesHost) {
      return kMpLL128x2;
    }
  }
  return kMpSimple;
}

struct MpCallInfo {
  uint64_t seq;
  int32_t kind, dt, op, root;
  uint64_t count;
  int32_t flags;   // kMpContig
  int32_t hasSend, hasRecv;
  hipIpcMemHandle_t sendH, recvH;
  uint64_t sendOff, recvOff;
};

// The Simple path's per-call allgather: shared memory when every rank could
// attach the segment at init, the TCP bootstrap otherwise.
ncclResult_t mpExchange(MpState* mp, uint64_t seq, const void* mine, size_t len, void* all) {
  if (mp->shmx) return nbx::shmxAllGather(mp->shmx, seq, mine, len, all, mp->timeoutSec, mp->hostWords);
  return nbx::bootstrapAllGather(mp->bs, mine, len, all);
}

// Name of the communicator's exchange segment, derived from its unique id.
std::string shmxName(const ncclUniqueId& id) {
  uint64_t h = 1469598103934665603ull;   // FNV-1a over the id bytes
  for (int i = 0; i < NCCL_UNIQUE_ID_BYTES; i++) h = (h ^ (uint8_t)id.internal[i]) * 1099511628211ull;
  char buf[64];
  std::snprintf(buf, sizeof(buf), "/nbx-shmx-%016llx", (unsigned long long)h);
  return buf;
}

// Collective: rank 0 creates the segment, the others attach; used only if
// every rank succeeded (NBX_HOST_EXCHANGE=tcp on any rank keeps TCP).
ncclResult_t mpSetupShmx(ncclComm* c, const ncclUniqueId& id) {
  MpState* mp = c->mp;
  const char* env = std::getenv("NBX_HOST_EXCHANGE");
  const bool want = !(env && strcasecmp(env, "tcp") == 0);
  const std::string name = shmxName(id);
  std::vector<int32_t> ok(c->nRanks);
  int32_t mine = 0;
  if (c->rank == 0 && want) {
    nbx::shmxUnlink(name.c_str());   // a stale segment of a crashed run with the same id (practically never)
    mp->shmx = nbx::shmxOpen(name.c_str(), 0, c->nRanks, sizeof(MpCallInfo), true);
    mine = mp->shmx != nullptr;
  }
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &mine, sizeof(mine), ok.data()));   // created?
  const bool created = ok[0] != 0;
  if (c->rank != 0) {
    if (created && want) mp->shmx = nbx::shmxOpen(name.c_str(), c->rank, c->nRanks, sizeof(MpCallInfo), false);
    mine = mp->shmx != nullptr;
  }
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &mine, sizeof(mine), ok.data()));   // everyone attached?
  if (c->rank == 0 && created) nbx::shmxUnlink(name.c_str());
  bool all = true;
  for (int32_t v : ok) all &= v != 0;
  if (!all && mp->shmx) {
    nbx::shmxClose(mp->shmx);
    mp->shmx = nullptr;
  }
  info("comm %p rank %d: per-call exchange over %s", (void*)c, c->rank, mp->shmx ? "shared memory" : "TCP");
  return ncclSuccess;
}

// Closing a peer-buffer mapping frees its virtual range, and the next import
// in this process can land at the same address. A call through such a
// reused address read zeros / garbage from the peer's buffer and its stores
// to it vanished (bench N = 2 rehearsals: 8 of 22 runs, always the first call
// through a new mapping whose address an earlier, closed mapping had used —
// a stale translation for the old mapping). Retired mappings are
// therefore kept open, up to NBX_IPC_RETIRED_MAX (4096) process-wide, oldest
// closed first, so addresses are not reused while their translations may be live.
void retirePeerMapping(void* base) {
  static std::mutex mu;
  static std::deque<void*> retired;
  static const size_t maxRetired = [] {
    const char* v = std::getenv("NBX_IPC_RETIRED_MAX");
    return (v && *v) ? (size_t)std::strtoull(v, nullptr, 10) : (size_t)4096;
  }();
  std::lock_guard<std::mutex> g(mu);
  retired.push_back(base);
  while (retired.size() > maxRetired) {
    (void)hipIpcCloseMemHandle(retired.front());
    retired.pop_front();
  }
}

ncclResult_t ipcHandleOf(const void* p, hipIpcMemHandle_t* h, uint64_t* off) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIPCHECK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p));
  HIPCHECK(hipIpcGetMemHandle(h, (void*)base));
  *off = (uint64_t)((const char*)p - (const char*)base);
  return ncclSuccess;
}

// `pin`: the call is being captured into a graph, whose replays keep using the
// mapping — it is never evicted.
ncclResult_t mapPeer(MpState* mp, int peer, const hipIpcMemHandle_t& h, void** base, bool pin) {
  auto key = std::make_pair(peer, std::string((const char*)&h, sizeof(h)));
  const uint64_t use = pin ? MpState::kPinned : mp->seq;
  auto it = mp->maps.find(key);
  if (it != mp->maps.end()) {
    if (it->second.lastUse != MpState::kPinned) it->second.lastUse = use;
    *base = it->second.base;
    return ncclSuccess;
  }
  void* p = nullptr;
  HIPCHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  mp->maps[key] = MpState::Mapping{p, use};
  *base = p;
  return ncclSuccess;
}

// Advance this rank's epoch of `slot`, post it, wait for the ranks in `mask`
// to reach it (epochs live on the device: graph replays stay in step).
ncclResult_t mpSignalWait(ncclComm* comm, int slot, uint64_t mask, hipStream_t stream) {
  MpState* mp = comm->mp;
  HIPCHECK(nbx::launchPeerBarrier(mp->flags, mp->peerFlagsDev, comm->nRanks, slot, mask, mp->epochs,
                                  mp->hostWordsDev, mp->hostWordsDev + 1, mp->timeoutSec, stream));
  return ncclSuccess;
}

ncclResult_t mpBarrier(ncclComm* comm, int slot, hipStream_t stream) {
  const int n = comm->nRanks;
  const uint64_t all = n >= 64 ? ~0ull : ((1ull << n) - 1ull);
  return mpSignalWait(comm, slot, all, stream);
}


// NCCL_ALGO (tuning.cc:254-259): "Ring" selects the ring schedule for
// AllReduce; anything else (default) the one-shot direct exchange.
// Read when the communicator is created.
bool algoRingFromEnv() {
  const char* v = std::getenv("NCCL_ALGO");
  return v && strcasecmp(v, "ring") == 0;
}

// Memory that other GPUs write and this GPU polls (barrier flags, LL lines).
// Uncached (fine-grained, MTYPE UC) by default: a peer's system-scope store
// over xGMI lands in HBM and no XCD L2 can hold a stale copy, which is what
// RCCL uses for its flags too. NBX_SYNC_MEM=coarse selects plain hipMalloc
// (A/B measurement only).
hipError_t allocSyncMem(void** p, size_t bytes) {
  static const bool coarse = [] {
    const char* v = std::getenv("NBX_SYNC_MEM");
    return v && strcasecmp(v, "coarse") == 0;
  }();
  if (coarse) return hipMalloc(p, bytes);
  return hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
}

ncclResult_t mpLL128SelfTest(ncclComm* c);
bool groupBatchEnabled();

// A device spin gave up (host error word set): name the wait, the peer, the
// value it waited for and the last one it saw (nbx_diag.h), once per record.
void mpReportDeviceError(ncclComm* c) {
  MpState* mp = c->mp;
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
  warn("comm %p rank %d: device wait timed out after %.3f s: %s of peer %lld, waited for %llu, last saw %llu "
       "(workgroup %llu)", (void*)c, c->rank, (double)rec[5] * 1e-8, nbx::diagSiteName(rec[0]),
       (long long)(int64_t)rec[1], (unsigned long long)rec[2], (unsigned long long)rec[3],
       (unsigned long long)rec[4]);
}

ncclResult_t mpInit(ncclComm* c, const ncclUniqueId& id) {
  MpState* mp = new MpState();
  c->mp = mp;
  const char* t = std::getenv("NBX_TIMEOUT_SEC");
  if (t && std::atof(t) > 0) mp->timeoutSec = std::atof(t);
  const char* cm = std::getenv("NBX_IPC_CACHE_MAX");
  if (cm && std::atol(cm) > 0) mp->mapsMax = (size_t)std::atol(cm);
  mp->protoMask = protoFromEnv();
  mp->ring = algoRingFromEnv();
  {
    const char* v = std::getenv("NBX_RING_PIPELINE");
    mp->ringPipeline = !(v && std::strcmp(v, "0") == 0);
    const char* gcap = std::getenv("NBX_RING_MAX_GRID");
    const long gv = (gcap && *gcap) ? std::atol(gcap) : nbx::kRingMaxGrid;
    mp->ringMaxGrid = (unsigned)(gv < 1 ? 1 : gv > nbx::kRingMaxGrid ? nbx::kRingMaxGrid : gv);
  }
  NCCLCHECK(nbx::bootstrapConnect(id, c->rank, c->nRanks, &mp->bs));
  HIPCHECK(allocSyncMem((void**)&mp->flags, kNumSlots * sizeof(uint64_t)));
  HIPCHECK(hipMemset(mp->flags, 0, kNumSlots * sizeof(uint64_t)));
  HIPCHECK(hipMalloc((void**)&mp->epochs, kNumSlots * sizeof(uint64_t)));
  HIPCHECK(hipMemset(mp->epochs, 0, kNumSlots * sizeof(uint64_t)));
  HIPCHECK(hipMalloc((void**)&mp->llState, sizeof(nbx::LLState)));
  HIPCHECK(hipMemset(mp->llState, 0, sizeof(nbx::LLState)));
  HIPCHECK(allocSyncMem((void**)&mp->ringProg, nbx::kRingMaxGrid * sizeof(uint64_t)));
  HIPCHECK(hipMemset(mp->ringProg, 0, nbx::kRingMaxGrid * sizeof(uint64_t)));
  HIPCHECK(hipMalloc((void**)&mp->ringState, sizeof(nbx::RingState)));
  HIPCHECK(hipMemset(mp->ringState, 0, sizeof(nbx::RingState)));
  if (mp->ring) {
    HIPCHECK(hipMalloc(&mp->fifo, nbx::kRingFifoBytes));
    HIPCHECK(allocSyncMem((void**)&mp->fifoTail, nbx::kRingMaxGrid * sizeof(uint64_t)));
    HIPCHECK(hipMemset(mp->fifoTail, 0, nbx::kRingMaxGrid * sizeof(uint64_t)));
    HIPCHECK(allocSyncMem((void**)&mp->fifoHead, nbx::kRingMaxGrid * sizeof(uint64_t)));
    HIPCHECK(hipMemset(mp->fifoHead, 0, nbx::kRingMaxGrid * sizeof(uint64_t)));
  }
  HIPCHECK(hipHostMalloc((void**)&mp->hostWords, 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(mp->hostWords, 0, 64);
  HIPCHECK(hipHostGetDevicePointer((void**)&mp->hostWordsDev, mp->hostWords, 0));
  // LL buffer: 2 parities x n sources x 2 lines per 8-byte pack
  {
    const char* v = std::getenv("NBX_LL_MAX_BYTES");
    uint64_t mx = (v && *v) ? std::strtoull(v, nullptr, 10) : (64u << 10);
    mx = (mx + 15) & ~(uint64_t)15;
    if (mx < 1024) mx = 1024;
    mp->llMaxBytes = mx;
    mp->llSlotLines = 2 * (mx / 8);
    mp->llDoneOff = 2 * (uint64_t)c->nRanks * mp->llSlotLines;
    const size_t llBytes = (mp->llDoneOff + (uint64_t)c->nRanks + 1) * sizeof(uint64_t);
    HIPCHECK(allocSyncMem((void**)&mp->ll, llBytes));
    HIPCHECK(hipMemset(mp->ll, 0, llBytes));
  }
  // LL128 buffer: 2 parities x n sources x 64-byte lines of 56 payload bytes (n <= 8)
  if (c->nRanks <= nbx::kL128MaxRanksHost) {
    const char* v = std::getenv("NBX_LL128_MAX_BYTES");
    uint64_t mx = (v && *v) ? std::strtoull(v, nullptr, 10) : (4u << 20);
    const char* o = std::getenv("NBX_LL128_ONESHOT_MAX");
    mp->l128OneShotMax = (o && *o) ? std::strtoull(o, nullptr, 10) : (256u << 10);
    if (mx > (64u << 20)) mx = 64u << 20;   // keeps the buffer under the 4 GiB descriptor range
    if (mx != 0) {
      mx = (mx + 15) & ~(uint64_t)15;
      mp->l128MaxBytes = mx;
      mp->l128SlotLines = l128SlotLinesFor(mx);
      mp->l128Bytes = 2 * (uint64_t)c->nRanks * mp->l128SlotLines * nbx::kL128LineBytesHost;
      HIPCHECK(allocSyncMem((void**)&mp->l128, mp->l128Bytes));
      HIPCHECK(hipMemset(mp->l128, 0, mp->l128Bytes));
    }
  }
  MpInitInfo mine{};
  mine.pid = (int32_t)getpid();
  mine.device = c->device;
  mine.llMaxBytes = mp->llMaxBytes;
  mine.l128MaxBytes = mp->l128MaxBytes;
  mine.l128OneShotMax = mp->l128OneShotMax;
  mine.protoMask = mp->protoMask;
  mp->groupBatch = groupBatchEnabled();
  mine.ring = mp->ring;
  mine.ringPipeline = mp->ringPipeline;
  mine.ringMaxGrid = (int32_t)mp->ringMaxGrid;
  mine.groupBatch = mp->groupBatch;
  HIPCHECK(hipIpcGetMemHandle(&mine.flagsHandle, mp->flags));
  HIPCHECK(hipIpcGetMemHandle(&mine.llHandle, mp->ll));
  if (mp->l128) HIPCHECK(hipIpcGetMemHandle(&mine.l128Handle, mp->l128));
  HIPCHECK(hipIpcGetMemHandle(&mine.ringHandle, mp->ringProg));
  if (mp->ring) {
    HIPCHECK(hipIpcGetMemHandle(&mine.fifoHandle, mp->fifo));
    HIPCHECK(hipIpcGetMemHandle(&mine.fifoTailHandle, mp->fifoTail));
    HIPCHECK(hipIpcGetMemHandle(&mine.fifoHeadHandle, mp->fifoHead));
  }
  {
    int dom = 0, bus = 0, dv = 0;
    (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->device);
    (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device);
    (void)hipDeviceGetAttribute(&dv, hipDeviceAttributePciDeviceId, c->device);
    mine.pciKey = ((uint64_t)(uint32_t)dom << 32) | ((uint64_t)(uint32_t)bus << 8) | (uint64_t)(uint32_t)dv;
  }
  std::vector<MpInitInfo> all(c->nRanks);
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &mine, sizeof(mine), all.data()));
  for (int j = 0; j < c->nRanks; j++) mp->multiGpu |= all[j].pciKey != mine.pciKey;
  std::vector<uint64_t*> table(c->nRanks), llTable(c->nRanks), l128Table(c->nRanks, nullptr);
  for (int j = 0; j < c->nRanks; j++) {
    // every rank must pick the same protocol for the same call
    if (all[j].llMaxBytes != mp->llMaxBytes || all[j].l128MaxBytes != mp->l128MaxBytes ||
        all[j].l128OneShotMax != mp->l128OneShotMax || all[j].protoMask != mp->protoMask) {
      warn("ncclCommInitRank : NCCL_PROTO / NBX_LL_MAX_BYTES / NBX_LL128_MAX_BYTES / NBX_LL128_ONESHOT_MAX differ "
           "across ranks");
      return ncclInvalidUsage;
    }
    if (all[j].ring != mine.ring || all[j].ringPipeline != mine.ringPipeline ||
        all[j].ringMaxGrid != mine.ringMaxGrid || all[j].groupBatch != mine.groupBatch) {
      warn("ncclCommInitRank : NCCL_ALGO / NBX_RING_PIPELINE / NBX_RING_MAX_GRID / NBX_GROUP_BATCH differ across ranks");
      return ncclInvalidUsage;
    }
    if (j == c->rank) {
      table[j] = mp->flags;
      llTable[j] = mp->ll;
      l128Table[j] = mp->l128;
      continue;
    }
    if (all[j].device != c->device) {
      int can = 0;
      HIPCHECK(hipDeviceCanAccessPeer(&can, c->device, all[j].device));
      if (!can) {
        // every data path here is a kernel load/store of peer memory; there is
        // no host-staged transport, so fail cleanly instead of faulting later
        warn("ncclCommInitRank : device %d cannot access peer device %d (no P2P)", c->device, all[j].device);
        return ncclSystemError;
      }
      hipError_t e = hipDeviceEnablePeerAccess(all[j].device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
      (void)hipGetLastError();
    }
    void* p = nullptr;
    HIPCHECK(hipIpcOpenMemHandle(&p, all[j].flagsHandle, hipIpcMemLazyEnablePeerAccess));
    mp->peerFlagMaps.push_back(p);
    table[j] = (uint64_t*)p;
    void* q = nullptr;
    HIPCHECK(hipIpcOpenMemHandle(&q, all[j].llHandle, hipIpcMemLazyEnablePeerAccess));
    mp->peerLLMaps.push_back(q);
    llTable[j] = (uint64_t*)q;
    if (mp->l128) {
      void* w = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&w, all[j].l128Handle, hipIpcMemLazyEnablePeerAccess));
      mp->peerL128Maps.push_back(w);
      l128Table[j] = (uint64_t*)w;
    }
    if (j == (c->rank + 1) % c->nRanks) {   // the ring's right neighbour: this rank posts its progress there
      void* w = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&w, all[j].ringHandle, hipIpcMemLazyEnablePeerAccess));
      mp->rightRingProg = (uint64_t*)w;
      if (mp->ring) {   // ... and its FIFO tail words
        HIPCHECK(hipIpcOpenMemHandle(&w, all[j].fifoTailHandle, hipIpcMemLazyEnablePeerAccess));
        mp->rightFifoTail = (uint64_t*)w;
      }
    }
    if (mp->ring && j == (c->rank + c->nRanks - 1) % c->nRanks) {   // the left neighbour: its FIFO and head words
      void* w = nullptr;
      HIPCHECK(hipIpcOpenMemHandle(&w, all[j].fifoHandle, hipIpcMemLazyEnablePeerAccess));
      mp->leftFifo = w;
      HIPCHECK(hipIpcOpenMemHandle(&w, all[j].fifoHeadHandle, hipIpcMemLazyEnablePeerAccess));
      mp->leftFifoHead = (uint64_t*)w;
    }
  }
  HIPCHECK(hipMalloc((void**)&mp->peerFlagsDev, c->nRanks * sizeof(uint64_t*)));
  HIPCHECK(hipMemcpy(mp->peerFlagsDev, table.data(), c->nRanks * sizeof(uint64_t*), hipMemcpyHostToDevice));
  HIPCHECK(hipMalloc((void**)&mp->peerLLDev, c->nRanks * sizeof(uint64_t*)));
  HIPCHECK(hipMemcpy(mp->peerLLDev, llTable.data(), c->nRanks * sizeof(uint64_t*), hipMemcpyHostToDevice));
  if (mp->l128) {
    HIPCHECK(hipMalloc((void**)&mp->peerL128Dev, c->nRanks * sizeof(uint64_t*)));
    HIPCHECK(hipMemcpy(mp->peerL128Dev, l128Table.data(), c->nRanks * sizeof(uint64_t*), hipMemcpyHostToDevice));
  }
  // everyone has mapped everyone before the first collective
  int dummy = 0;
  std::vector<int> sink(c->nRanks);
  NCCLCHECK(nbx::bootstrapAllGather(mp->bs, &dummy, sizeof(dummy), sink.data()));
  NCCLCHECK(mpSetupShmx(c, id));
  NCCLCHECK(mpLL128SelfTest(c));
  info("comm %p rank %d nranks %d device %d: multi-process communicator ready", (void*)c, c->rank, c->nRanks,
       c->device);
  return ncclSuccess;
}

void mpFree(ncclComm* c) {
  MpState* mp = c->mp;
  if (!mp) return;
  DevGuard g(c->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : mp->maps) retirePeerMapping(kv.second.base);
  for (void* p : mp->peerFlagMaps) (void)hipIpcCloseMemHandle(p);
  for (void* p : mp->peerLLMaps) (void)hipIpcCloseMemHandle(p);
  for (void* p : mp->peerL128Maps) (void)hipIpcCloseMemHandle(p);
  if (mp->rightRingProg) (void)hipIpcCloseMemHandle(mp->rightRingProg);
  if (mp->rightFifoTail) (void)hipIpcCloseMemHandle(mp->rightFifoTail);
  if (mp->leftFifo) (void)hipIpcCloseMemHandle(mp->leftFifo);
  if (mp->leftFifoHead) (void)hipIpcCloseMemHandle(mp->leftFifoHead);
  if (mp->fifo) (void)hipFree(mp->fifo);
  if (mp->fifoTail) (void)hipFree(mp->fifoTail);
  if (mp->fifoHead) (void)hipFree(mp->fifoHead);
  if (mp->ringProg) (void)hipFree(mp->ringProg);
  if (mp->ringState) (void)hipFree(mp->ringState);
  if (mp->peerL128Dev) (void)hipFree(mp->peerL128Dev);
  if (mp->l128) (void)hipFree(mp->l128);
  if (mp->peerFlagsDev) (void)hipFree(mp->peerFlagsDev);
  if (mp->peerLLDev) (void)hipFree(mp->peerLLDev);
  if (mp->ll) (void)hipFree(mp->ll);
  if (mp->epochs) (void)hipFree(mp->epochs);
  if (mp->llState) (void)hipFree(mp->llState);
  if (mp->flags) (void)hipFree(mp->flags);
  if (mp->hostWords) (void)hipHostFree(mp->hostWords);
  nbx::shmxClose(mp->shmx);
  nbx::bootstrapClose(mp->bs);
  delete mp;
  c->mp = nullptr;
}

// The protocol of a call. It depends only on arguments every rank passes
// identically (and on the init-time settings checked equal), so every rank
// picks the same one.
MpProto mpProtoOf(const ncclComm* comm, const MpCall& c) {
  const MpState* mp = comm->mp;
  const int n = comm->nRanks;
  const int eb = typeSize(c.dt);
  const uint64_t slotBytes = (uint64_t)c.count * (uint64_t)eb;   // RS: recvcount per block
  size_t off0, per;
  blockRange(c.count, eb, n, 0, &off0, &per);   // the direct schedule's AllReduce block
  return chooseProtoFor(mp->protoMask, c.kind != kReduceScatter, slotBytes, (uint64_t)per * (uint64_t)eb, n,
                        mp->llMaxBytes, mp->l128MaxBytes, mp->l128OneShotMax);
}

// LL / LL128 protocols: small and medium collectives in one kernel, no host
// exchange (nbx_ll.h).
ncclResult_t mpLaunchLL(ncclComm* comm, const MpCall& c, MpProto proto) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks, me = comm->rank;
  const int eb = typeSize(c.dt);
  const uint64_t slotBytes = (uint64_t)c.count * (uint64_t)eb;
  size_t off0, per;
  blockRange(c.count, eb, n, 0, &off0, &per);
  if (c.send == nullptr || (c.recv == nullptr && (c.kind != kReduce || me == c.root))) {
    warn("rank %d passed a NULL buffer", me);
    return ncclInvalidArgument;
  }
  ++mp->seq;
  nbx::LLArgs la{};
  la.send = c.send;
  la.recv = c.recv;
  la.count = c.count;
  la.nPacks = (slotBytes + 7) / 8;
  la.peerLL = mp->peerLLDev;
  la.myLL = mp->ll;
  la.slotLines = mp->llSlotLines;
  la.doneOff = mp->llDoneOff;
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
  if (proto == kMpLL128 || proto == kMpLL128x2) {
    la.peerL128 = mp->peerL128Dev;
    la.myL128 = mp->l128;
    la.l128SlotLines = mp->l128SlotLines;
    la.l128Bytes = (uint32_t)mp->l128Bytes;
    if (proto == kMpLL128x2) {
      la.nLines = mp->l128SlotLines / 2;   // sub-slot lines: [parity][RS|AG][source]
      const uint64_t blockLines =
          ((uint64_t)per * (uint64_t)eb + nbx::kL128DataBytesHost - 1) / nbx::kL128DataBytesHost;
      return nbx::launchLL128AllReduce2(c.dt, c.op, la, blockLines, c.stream);
    }
    la.nLines = (slotBytes + nbx::kL128DataBytesHost - 1) / nbx::kL128DataBytesHost;
    return nbx::launchLL128Coll(c.dt, c.op, la, c.stream);
  }
  return nbx::launchLLColl(c.dt, c.op, la, c.stream);
}

// Simple path, step 0: allgather the call (kind, type, op, count) and the IPC
// handles of every rank's buffers, and check that the ranks agree.
// `flags` is this rank's kMpContig bit, exchanged so that group batching
// decisions are identical on every rank.
constexpr int32_t kMpContig = 1;   // same stream as the previous call of the group
ncclResult_t mpExchangeCall(ncclComm* comm, const MpCall& c, int32_t flags, std::vector<MpCallInfo>* all) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks, me = comm->rank;
  const uint64_t seq = ++mp->seq;
  MpCallInfo mine{};
  mine.seq = seq;
  mine.kind = (int32_t)c.kind;
  mine.dt = (int32_t)c.dt;
  mine.op = c.op.op;
  mine.root = c.root;
  mine.count = c.count;
  mine.flags = flags;
  mine.hasSend = c.count > 0 && c.send != nullptr;
  mine.hasRecv = c.count > 0 && c.recv != nullptr;
  if (mine.hasSend) NCCLCHECK(ipcHandleOf(c.send, &mine.sendH, &mine.sendOff));
  if (mine.hasRecv) NCCLCHECK(ipcHandleOf(c.recv, &mine.recvH, &mine.recvOff));
  all->assign(n, MpCallInfo{});
  NCCLCHECK(mpExchange(mp, seq, &mine, sizeof(mine), all->data()));
  for (int j = 0; j < n; j++) {
    const MpCallInfo& a = (*all)[j];
    if (a.seq != seq || a.kind != mine.kind || a.dt != mine.dt || a.op != mine.op || a.root != c.root ||
        a.count != c.count) {
      warn("collective mismatch across ranks (rank %d vs %d)", j, me);
      return ncclInvalidUsage;
    }
  }
  return ncclSuccess;
}

// Bound the mapping cache: a peer's freed-and-reallocated buffers come back
// with new handles, and every open mapping pins the peer's old allocation.
// Past the bound, wait for this device's work (no kernel in flight uses a
// mapping), then close every mapping not used since the call before `seq`.
ncclResult_t mpEvictMappings(MpState* mp, uint64_t seq, bool capturing) {
  if (mp->maps.size() <= mp->mapsMax || capturing) return ncclSuccess;
  HIPCHECK(hipDeviceSynchronize());
  for (auto it = mp->maps.begin(); it != mp->maps.end();) {
    if (it->second.lastUse != MpState::kPinned && it->second.lastUse + 1 < seq) {
      retirePeerMapping(it->second.base);
      it = mp->maps.erase(it);
    } else {
      ++it;
    }
  }
  return ncclSuccess;
}

// Every rank's send / recv base for one call (own buffers as passed, peers'
// through the IPC mapping cache).
ncclResult_t mpMapCall(ncclComm* comm, const MpCall& c, const std::vector<MpCallInfo>& all, bool capturing,
                       std::vector<const char*>* sendP, std::vector<char*>* recvP) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks, me = comm->rank;
  sendP->assign(n, nullptr);
  recvP->assign(n, nullptr);
  for (int j = 0; j < n; j++) {
    if (j == me) {
      (*sendP)[j] = (const char*)c.send;
      (*recvP)[j] = (char*)c.recv;
      continue;
    }
    void* b = nullptr;
    if (all[j].hasSend) {
      NCCLCHECK(mapPeer(mp, j, all[j].sendH, &b, capturing));
      (*sendP)[j] = (const char*)b + all[j].sendOff;
    }
    if (all[j].hasRecv) {
      NCCLCHECK(mapPeer(mp, j, all[j].recvH, &b, capturing));
      (*recvP)[j] = (char*)b + all[j].recvOff;
    }
  }
  for (int j = 0; j < n; j++)
    if (!(*sendP)[j] || ((c.kind != kReduce || j == c.root) && !(*recvP)[j])) {
      warn("rank %d passed a NULL buffer", j);
      return ncclInvalidArgument;
    }
  return ncclSuccess;
}

// This rank's block of the direct schedule: block `me` of every rank's send
// buffer in fold order, and where the folded block goes. AllReduce /
// ReduceScatter fold in ring order me+1, ..., me; Reduce in chain order
// root+1, ..., root for every block (reduce.h:44-67). AllReduce with
// n <= NBX_MAX_DSTS pushes the block into every rank's output (push-gather,
// all_reduce.h:343-360), so there is no separate gather phase.
RankBlock mpDirectBlock(const MpCall& c, int n, int me, const std::vector<const char*>& sendP,
                        const std::vector<char*>& recvP) {
  const int eb = typeSize(c.dt);
  const size_t total = c.kind == kReduceScatter ? c.count * (size_t)n : c.count;
  RankBlock b;
  size_t off;
  if (c.kind == kReduceScatter) {
    off = (size_t)me * c.count;
    b.len = c.count;
  } else {
    blockRange(total, eb, n, me, &off, &b.len);
  }
  if (b.len == 0) return b;
  const int first = (c.kind == kReduce ? c.root : me) + 1;
  for (int k = 0; k < n; k++) b.srcs.push_back(sendP[(first + k) % n] + off * (size_t)eb);
  if (c.kind == kReduceScatter) b.dsts.push_back(recvP[me]);
  else if (c.kind == kReduce) b.dsts.push_back(recvP[c.root] + off * (size_t)eb);
  else if (n > NBX_MAX_DSTS) b.dsts.push_back(recvP[me] + off * (size_t)eb);
  else
    for (int k = 0; k < n; k++) b.dsts.push_back(recvP[(me + k) % n] + off * (size_t)eb);
  return b;
}

// NCCL_ALGO=Ring ReduceScatter / Reduce through the step FIFO (kRingFifo):
// every rank's buffers 16-B aligned (decided from the exchanged offsets, so
// every rank decides alike) and, for ReduceScatter, blocks of whole 16-B packs
// (block c starts at c * recvcount elements). Otherwise the direct schedule.
bool mpRingFifoEligible(const MpCall& c, int n, const std::vector<MpCallInfo>& all) {
  if (c.kind != kReduceScatter && c.kind != kReduce) return false;
  const int eb = typeSize(c.dt);
  if (c.kind == kReduceScatter && ((uint64_t)c.count * (uint64_t)eb) % 16 != 0) return false;
  for (int j = 0; j < n; j++) {
    const MpCallInfo& ai = all[j];
    if ((ai.sendOff & 15u) != 0) return false;
    if (ai.hasRecv && (ai.recvOff & 15u) != 0) return false;
  }
  return true;
}

// Simple path, after the exchange: map, barriers, reduce (direct or ring), gather.
ncclResult_t mpRunSimple(ncclComm* comm, const MpCall& c, const std::vector<MpCallInfo>& all) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks, me = comm->rank;
  const int eb = typeSize(c.dt);
  hipStream_t stream = c.stream;
  if (c.count == 0) return ncclSuccess;
  hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(stream, &capture));
  const bool capturing = capture != hipStreamCaptureStatusNone;
  NCCLCHECK(mpEvictMappings(mp, all[me].seq, capturing));
  std::vector<const char*> sendP;
  std::vector<char*> recvP;
  const size_t mapsBefore = mp->maps.size();
  NCCLCHECK(mpMapCall(comm, c, all, capturing, &sendP, &recvP));
  if (traceOn()) {   // NBX_TRACE=1: every rank's send / recv as this rank sees them
    auto hsh = [](const hipIpcMemHandle_t& h) {
      uint64_t x = 1469598103934665603ull;
      for (size_t i = 0; i < sizeof(h); i++) x = (x ^ (unsigned char)((const char*)&h)[i]) * 1099511628211ull;
      return x;
    };
    for (int j = 0; j < n; j++)
      NBX_TRACE("mp simple seq=%llu rank %d count=%zu: rank %d send %p (h %016llx off %llu) recv %p (h %016llx off %llu)%s",
                (unsigned long long)all[me].seq, me, c.count, j, (const void*)sendP[j],
                (unsigned long long)hsh(all[j].sendH), (unsigned long long)all[j].sendOff, (void*)recvP[j],
                (unsigned long long)hsh(all[j].recvH), (unsigned long long)all[j].recvOff,
                mp->maps.size() != mapsBefore ? " [new mapping]" : "");
  }
  // 1. every rank's stream has reached the collective (its inputs are written,
  //    its output may be written by peers)
  NCCLCHECK(mpBarrier(comm, kSlotEnter, stream));
  const size_t total = c.kind == kReduceScatter ? c.count * (size_t)n : c.count;
  const bool push = c.kind == kAllReduce && n <= NBX_MAX_DSTS;
  if (c.kind == kAllReduce && n > 2 && mp->ring) {
    // 2'. ring reduce-scatter (all_reduce.h:60-79): chunk c starts at rank c+1 and
    // visits c+2, ..., c; at step s this rank folds chunk c = me-2-s as
    // Fn(pre(local), received) — NCCL's operand order (recvReduceSend: srcs[0] is
    // the local input, srcs[1] the received partial) — into its own recv buffer,
    // where the right neighbour reads it at step s+1. Step 0 reads the left
    // neighbour's raw input (its `send`, PreOp applies to both sources); the last
    // step (c == me) applies postOp and, with push, stores into every output.
    // Every rank works on a different chunk at each step, so all ring links
    // carry 1/n of the data concurrently.
    const int left = (me + n - 1) % n;
    // pipelined: one kernel, slices flow through the ring on device progress
    // words (nbx_ring.h). It needs 16-B aligned buffers, and every rank must
    // choose it or none: decided from the exchanged offsets of all ranks
    // (allocation bases are >= 256-B aligned, so an offset's alignment is the
    // pointer's).
    const int nOuts = push ? n : 1;
    bool aligned = true;
    for (const MpCallInfo& ai : all) aligned &= ((ai.sendOff | ai.recvOff) & 15u) == 0;
    if (mp->ringPipeline && aligned) {
      size_t o0, per;
      blockRange(total, eb, n, 0, &o0, &per);
      const uint64_t epp = (uint64_t)(16 / eb);
      const uint64_t maxPacks = per / epp;
      uint64_t grid = (maxPacks + 1023) / 1024;   // slices of >= 16 KiB
      if (grid < 1) grid = 1;
      if (grid > mp->ringMaxGrid) grid = mp->ringMaxGrid;
      nbx::RingArgs ra{};
      ra.sendMe = sendP[me];
      ra.sendLeft = sendP[left];
      ra.recvMe = recvP[me];
      ra.recvLeft = recvP[left];
      for (int k = 0; k < nOuts; k++) ra.outs[k] = recvP[(me + k) % n];
      ra.myProgress = mp->ringProg;
      ra.rightProgress = mp->rightRingProg;
      ra.state = mp->ringState;
      ra.total = total;
      ra.blockElts = per;
      ra.slicePacks = (maxPacks + grid - 1) / grid;
      ra.abortWord = mp->hostWordsDev;
      ra.errWord = mp->hostWordsDev + 1;
      ra.timeoutTicks = (uint64_t)(mp->timeoutSec * 1.0e8);
      ra.rank = me;
      ra.nRanks = n;
      ra.nOuts = nOuts;
      NCCLCHECK(nbx::launchRingAllReduce(c.dt, c.op, ra, (unsigned)grid, stream));
    } else {
    std::vector<void*> pushDsts;
    for (int st = 0; st < n - 1; st++) {
      const int ch = ((me - 2 - st) % n + n) % n;
      size_t off, len;
      blockRange(total, eb, n, ch, &off, &len);
      if (len > 0) {
        const void* srcs[2] = {sendP[me] + off * (size_t)eb,
                               st == 0 ? (const void*)(sendP[left] + off * (size_t)eb)
                                       : (const void*)(recvP[left] + off * (size_t)eb)};
        void* dsts[1] = {recvP[me] + off * (size_t)eb};
        const bool last = st == n - 2;
        pushDsts.clear();
        for (int k = 0; k < n; k++) pushDsts.push_back(recvP[(me + k) % n] + off * (size_t)eb);
        NCCLCHECK(nbx::reduceMultiEx(last && push ? pushDsts.data() : dsts, last && push ? n : 1, srcs, 2, len,
                                     c.dt, c.op, st == 0 ? 2 : 1, last ? 1 : 0, (ncclStream_t)stream,
                                     nbx::kReduceAcquireSystem));
      }
      if (st < n - 2) NCCLCHECK(mpSignalWait(comm, kSlotRing, 1ull << left, stream));
    }
    }
  } else if (mp->ring && mp->ringPipeline && n > 1 && mpRingFifoEligible(c, n, all)) {
    // 2''. ring ReduceScatter / chain Reduce through the step FIFO (nbx_ring.h
    // kRingFifo; reduce_scatter.h:13-66, reduce.h:12-68)
    const int left = (me + n - 1) % n;
    const uint64_t epp = (uint64_t)(16 / eb);
    const uint64_t blockPacks = ((uint64_t)c.count + epp - 1) / epp;   // RS: recvcount, Reduce: count
    uint64_t grid = (blockPacks + 1023) / 1024;   // slices of >= 16 KiB
    if (grid < 1) grid = 1;
    if (grid > mp->ringMaxGrid) grid = mp->ringMaxGrid;
    nbx::RingFifoArgs fa{};
    fa.sendMe = sendP[me];
    fa.sendLeft = sendP[left];
    fa.recv = recvP[me];
    fa.fifoMe = mp->fifo;
    fa.fifoLeft = mp->leftFifo;
    fa.myTail = mp->fifoTail;
    fa.rightTail = mp->rightFifoTail;
    fa.myHead = mp->fifoHead;
    fa.leftHead = mp->leftFifoHead;
    fa.state = mp->ringState;
    fa.blockElts = c.count;
    fa.slicePacks = (blockPacks + grid - 1) / grid;
    fa.abortWord = mp->hostWordsDev;
    fa.errWord = mp->hostWordsDev + 1;
    fa.timeoutTicks = (uint64_t)(mp->timeoutSec * 1.0e8);
    fa.rank = me;
    fa.nRanks = n;
    fa.root = c.root;
    fa.mode = c.kind == kReduceScatter ? nbx::kRingFifoReduceScatter : nbx::kRingFifoReduce;
    NCCLCHECK(nbx::launchRingFifo(c.dt, c.op, fa, (unsigned)grid, stream));
  } else {
    // 2. direct reduce of this rank's block
    const RankBlock b = mpDirectBlock(c, n, me, sendP, recvP);
    if (b.len > 0)
      NCCLCHECK(nbx::reduceMultiEx(b.dsts.data(), (int)b.dsts.size(), b.srcs.data(), n, b.len, c.dt, c.op, n, 1,
                                   (ncclStream_t)stream, nbx::kReduceAcquireSystem));
  }
  // 3. AllReduce with n > NBX_MAX_DSTS: gather the peers' reduced blocks
  if (c.kind == kAllReduce && !push) {
    NCCLCHECK(mpBarrier(comm, kSlotReduced, stream));
    nbxDevRedOpFull copyOp{nbxDevSum, 0, 0};
    for (int k = 1; k < n; k++) {
      const int j = (me + k) % n;
      size_t o, l;
      blockRange(total, eb, n, j, &o, &l);
      if (l == 0) continue;
      void* d[1] = {recvP[me] + o * (size_t)eb};
      const void* s1[1] = {recvP[j] + o * (size_t)eb};
      NCCLCHECK(nbx::reduceMultiEx(d, 1, s1, 1, l * (size_t)eb, ncclUint8, copyOp, 0, 0, (ncclStream_t)stream,
                                   nbx::kReduceAcquireSystem));
    }
  }
  // 4. nobody reuses its buffers while a peer may still read them
  NCCLCHECK(mpBarrier(comm, kSlotDone, stream));
  return ncclSuccess;
}

ncclResult_t runMpColl(ncclComm* comm, const MpCall& c) {
  const MpProto proto = mpProtoOf(comm, c);
  if (proto != kMpSimple) return mpLaunchLL(comm, c, proto);
  std::vector<MpCallInfo> all;
  NCCLCHECK(mpExchangeCall(comm, c, 0, &all));
  return mpRunSimple(comm, c, all);
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
// Groups on a multi-process communicator. Inside ncclGroupStart/End the calls
// are queued and run at the outermost ncclGroupEnd, in order: every
// Simple-protocol call is exchanged first (one allgather each, flags
// included), then maximal runs of direct-schedule calls that every rank issued
// on one stream and that touch no buffer an earlier member of the run writes
// (or write one it reads) run as ONE exchange — one enter barrier, one
// nbxReduceMultiBatch per (datatype, op), one done barrier — the way NCCL packs
// a group's collectives into one kernel's work list (enqueue.cc:67-91
// appendWorkElemColl). Every decision uses only exchanged data, so all ranks
// make the same one. LL / LL128 calls and the ring / gather schedules run
// one by one, in order. NBX_GROUP_BATCH=0 runs every call at enqueue instead.
thread_local std::vector<ncclComm*> t_groupMpComms;
constexpr size_t kMaxMpBatch = 64;

bool groupBatchEnabled() {
  static const bool on = [] {
    const char* v = std::getenv("NBX_GROUP_BATCH");
    return !(v && std::strcmp(v, "0") == 0);
  }();
  return on;
}

// Bytes of every rank's buffers a call reads (send) and writes (recv),
// identified by (IPC handle of the allocation, offset range).
struct HSpan {
  hipIpcMemHandle_t h;
  uint64_t lo, hi;
  bool write;
};

void callSpans(const MpCall& c, int n, const std::vector<MpCallInfo>& all, std::vector<HSpan>* out) {
  const uint64_t eb = (uint64_t)typeSize(c.dt);
  const uint64_t sendBytes = (c.kind == kReduceScatter ? (uint64_t)c.count * (uint64_t)n : c.count) * eb;
  const uint64_t recvBytes = (uint64_t)c.count * eb;
  for (const MpCallInfo& a : all) {
    if (a.hasSend) out->push_back({a.sendH, a.sendOff, a.sendOff + sendBytes, false});
    if (a.hasRecv) out->push_back({a.recvH, a.recvOff, a.recvOff + recvBytes, true});
  }
}

bool hspansConflict(const std::vector<HSpan>& a, const std::vector<HSpan>& b) {
  for (const HSpan& x : a)
    for (const HSpan& y : b)
      if ((x.write || y.write) && x.lo < y.hi && y.lo < x.hi && std::memcmp(&x.h, &y.h, sizeof(x.h)) == 0)
        return true;
  return false;
}

// One batched exchange over calls[lo, hi) (all Simple, direct schedule, one stream).
ncclResult_t mpRunBatch(ncclComm* comm, const std::vector<MpCall>& calls,
                        const std::vector<std::vector<MpCallInfo>>& alls, size_t lo, size_t hi) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks, me = comm->rank;
  hipStream_t stream = calls[lo].stream;
  hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
  HIPCHECK(hipStreamIsCapturing(stream, &capture));
  const bool capturing = capture != hipStreamCaptureStatusNone;
  NCCLCHECK(mpEvictMappings(mp, alls[lo][me].seq, capturing));
  std::vector<RankBlock> blocks;
  std::vector<const PendingColl*> colls;
  for (size_t k = lo; k < hi; k++) {
    std::vector<const char*> sendP;
    std::vector<char*> recvP;
    NCCLCHECK(mpMapCall(comm, calls[k], alls[k], capturing, &sendP, &recvP));
    blocks.push_back(mpDirectBlock(calls[k], n, me, sendP, recvP));
    colls.push_back(&calls[k]);
  }
  NBX_TRACE("mp group batch of %zu collectives", hi - lo);
  NCCLCHECK(mpBarrier(comm, kSlotEnter, stream));
  NCCLCHECK(foldBlocksBatched(colls, blocks, n, stream));
  NCCLCHECK(mpBarrier(comm, kSlotDone, stream));
  return ncclSuccess;
}

ncclResult_t runMpGroupImpl(ncclComm* comm) {
  MpState* mp = comm->mp;
  const int n = comm->nRanks;
  std::vector<MpCall> calls;
  calls.swap(mp->group);
  const size_t m = calls.size();
  std::vector<MpProto> protos(m);
  std::vector<std::vector<MpCallInfo>> alls(m);
  for (size_t k = 0; k < m; k++) {
    protos[k] = mpProtoOf(comm, calls[k]);
    if (protos[k] != kMpSimple) continue;
    const int32_t flags = (k > 0 && protos[k - 1] == kMpSimple && calls[k].stream == calls[k - 1].stream) ? kMpContig : 0;
    NCCLCHECK(mpExchangeCall(comm, calls[k], flags, &alls[k]));
  }
  auto directSimple = [&](size_t k) {
    const MpCall& c = calls[k];
    return protos[k] == kMpSimple && c.count > 0 && !(c.kind == kAllReduce && n > NBX_MAX_DSTS) &&
           !(c.kind == kAllReduce && n > 2 && mp->ring) &&
           !(mp->ring && mp->ringPipeline && mpRingFifoEligible(c, n, alls[k]));   // ring RS / Reduce: alone
  };
  auto contigEverywhere = [&](size_t k) {
    for (const MpCallInfo& a : alls[k])
      if (!(a.flags & kMpContig)) return false;
    return true;
  };
  size_t k = 0;
  while (k < m) {
    if (protos[k] != kMpSimple) {
      NCCLCHECK(mpLaunchLL(comm, calls[k], protos[k]));
      k++;
      continue;
    }
    size_t j = k + 1;
    if (directSimple(k)) {
      std::vector<HSpan> spans;
      callSpans(calls[k], n, alls[k], &spans);
      for (; j < m && j - k < kMaxMpBatch; j++) {
        if (!directSimple(j) || !contigEverywhere(j)) break;
        std::vector<HSpan> sj;
        callSpans(calls[j], n, alls[j], &sj);
        if (hspansConflict(spans, sj)) break;
        spans.insert(spans.end(), sj.begin(), sj.end());
      }
    }
    if (j == k + 1) NCCLCHECK(mpRunSimple(comm, calls[k], alls[k]));
    else NCCLCHECK(mpRunBatch(comm, calls, alls, k, j));
    k = j;
  }
  return ncclSuccess;
}

ncclResult_t runMpGroup(ncclComm* comm) {
  DevGuard g(comm->device);
  ncclResult_t r;
  try {
    r = runMpGroupImpl(comm);
  } catch (const std::exception& e) {
    warn("internal exception: %s", e.what());
    r = ncclInternalError;
  }
  comm->mp->group.clear();
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

// ncclEnqueueCheck + taskAppend for the reducing collectives.
ncclResult_t enqueueColl(CollKind kind, const char* opName, const void* sendbuff, void* recvbuff, size_t count,
                         ncclDataType_t dt, ncclRedOp_t op, int root, ncclComm* comm, hipStream_t stream) {
  NCCLCHECK(commCheck(comm, opName));
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
    if (t_groupDepth > 0 && comm->mp->groupBatch) {   // run at the outermost ncclGroupEnd
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
  if (config && config->blocking != NCCL_CONFIG_UNDEF_INT) c->blocking = config->blocking;
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
  if (nranks > kMaxMpRanks) {   // 64-bit rank masks in the barrier kernel, one source per rank
    warn("ncclCommInitRank : %d ranks requested, this build supports up to %d per communicator", nranks,
         kMaxMpRanks);
    return ncclInvalidArgument;
  }
  int dev = 0;
  HIPCHECK(hipGetDevice(&dev));
  if (nranks == 1) return newComm(newcomm, 1, 0, dev, config);
  if (!nbx::bootstrapIdHasRoot(commId)) {
    warn("ncclCommInitRank : unique id carries no bootstrap root");
    return ncclInvalidArgument;
  }
  ncclComm* c = nullptr;
  NCCLCHECK(newComm(&c, nranks, myrank, dev, config));
  ncclResult_t r;
  try {
    r = mpInit(c, commId);
  } catch (const std::exception& e) {
    warn("internal exception: %s", e.what());
    r = ncclInternalError;
  }
  if (r != ncclSuccess) {
    mpFree(c);
    delete c;
    return r;
  }
  *newcomm = c;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommInitRank, ncclComm_t* newcomm, int nranks, ncclUniqueId commId, int myrank) {
  return ncclCommInitRankConfig(newcomm, nranks, commId, myrank, nullptr);
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
  {
    std::lock_guard<std::mutex> g(g_pendMu);
    g_cliques.push_back(clique);
  }
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommFinalize, ncclComm_t comm) {
  NCCLCHECK(commCheck(comm, "ncclCommFinalize"));
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
  return commFree(comm);
}

NBX_API(ncclResult_t, ncclCommAbort, ncclComm_t comm) {
  if (comm == nullptr) return ncclSuccess;
  NCCLCHECK(commCheck(comm, "ncclCommAbort"));
  if (comm->mp && comm->mp->hostWords) comm->mp->hostWords[0] = 1;   // ends every spinning barrier
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
  if (*asyncError == ncclSuccess && comm->mp && comm->mp->hostWords && comm->mp->hostWords[1] != 0) {
    *asyncError = ncclRemoteError;   // a peer barrier timed out or was aborted
    mpReportDeviceError(comm);
  }
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommCount, const ncclComm_t comm, int* count) {
  NCCLCHECK(commCheck(comm, "CommCount"));
  if (count == nullptr) return ncclInvalidArgument;
  *count = comm->nRanks;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommCuDevice, const ncclComm_t comm, int* devid) {
  NCCLCHECK(commCheck(comm, "CommCuDevice"));
  if (devid == nullptr) return ncclInvalidArgument;
  *devid = comm->device;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclCommUserRank, const ncclComm_t comm, int* rank) {
  NCCLCHECK(commCheck(comm, "CommUserRank"));
  if (rank == nullptr) return ncclInvalidArgument;
  *rank = comm->rank;
  return ncclSuccess;
}

NBX_API(ncclResult_t, ncclRedOpCreatePreMulSum, ncclRedOp_t* op, void* scalar, ncclDataType_t datatype,
        ncclScalarResidence_t residence, ncclComm_t comm) {
  // enqueue.cc:1648-1685
  NCCLCHECK(commCheck(comm, "ncclRedOpCreatePreMulSum"));
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

NBX_EXPORT int nbxDebugCommProtoMask(ncclComm_t comm) {
  if (comm == nullptr || comm->magic != kCommMagic || comm->mp == nullptr) return -1;
  return comm->mp->protoMask;
}

NBX_EXPORT int nbxDebugChooseProto(int protoMask, int twoShotKind, uint64_t slotBytes, uint64_t blockBytes, int nRanks,
                                   uint64_t llMaxBytes, uint64_t ll128MaxBytes, uint64_t ll128OneShotMax) {
  return (int)chooseProtoFor(protoMask, twoShotKind != 0, slotBytes, blockBytes, nRanks, llMaxBytes, ll128MaxBytes,
                             ll128OneShotMax);
}

NBX_EXPORT ncclResult_t nbxShmxSelfTest(const char* name, int rank, int nranks, int rounds, int jitterUs) {
  if (name == nullptr || nranks < 1 || rank < 0 || rank >= nranks || rounds < 0) return ncclInvalidArgument;
  constexpr size_t kMax = 256;
  nbx::ShmExchange* x = nullptr;
  if (rank == 0) {
    x = nbx::shmxOpen(name, 0, nranks, kMax, true);
  } else {
    for (int i = 0; i < 20000 && x == nullptr; i++) {   // wait for rank 0's segment (<= ~20 s)
      x = nbx::shmxOpen(name, rank, nranks, kMax, false);
      if (!x) usleep(1000);
    }
  }
  if (!x) return ncclSystemError;
  std::mt19937 rng(1234u + (unsigned)rank);
  std::vector<unsigned char> mine(kMax), all(kMax * (size_t)nranks);
  ncclResult_t r = ncclSuccess;
  for (int k = 1; k <= rounds && r == ncclSuccess; k++) {
    const size_t len = 1 + (size_t)(k * 37) % kMax;
    for (size_t i = 0; i < len; i++) mine[i] = (unsigned char)(rank * 31 + k * 7 + (int)i);
    if (jitterUs > 0) usleep(rng() % (unsigned)jitterUs);
    r = nbx::shmxAllGather(x, (uint64_t)(3 * k + (k % 2)), mine.data(), len, all.data(), 60.0, nullptr);
    for (int j = 0; r == ncclSuccess && j < nranks; j++)
      for (size_t i = 0; i < len; i++)
        if (all[(size_t)j * len + i] != (unsigned char)(j * 31 + k * 7 + (int)i)) r = ncclInternalError;
  }
  nbx::shmxClose(x);
  return r;
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
