// nbx_comm.h — the communicator layer behind the NCCL C ABI (include/nccl.h),
// shared by its units (library-internal; every symbol here has hidden
// visibility, -fvisibility=hidden):
//   nccl_api.cc        argument checks, hostToDevRedOp, the one-rank path,
//                      enqueue, the collective / group / redop / error entry points
//   comm_mp_init.cc    multi-process communicator (ncclCommInitRank, nranks > 1):
//                      settings, connection buffers, IPC mapping check, LL128 probe
//   comm_mp_launch.cc  multi-process launches: protocol choice, LL / LL128 /
//                      Simple kernels, cross-stream order, group batching
//   comm_clique.cc     in-process clique (ncclCommInitAll): event-ordered fold,
//                      batched folds, the in-kernel transport
//   comm_lifecycle.cc  split, register, finalize / destroy / abort, async error, queries
// Reference host path: src/collectives.cc:29-124, src/enqueue.cc:1436-1717,
// src/misc/argcheck.cc:28-75, src/init.cc (lifecycle), src/group.cc:82-103.
#pragma once
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nbx_debug.h"
#include "../../include/nbx_reduce.h"
#include "nbx_bootstrap.h"
#include "nbx_diag.h"
#include "nbx_internal.h"
#include "nbx_ll_args.h"

#define NBX_EXPORT extern "C" __attribute__((visibility("default")))
// NCCL_API (src/include/core.h:17-32): every entry point plus a p-prefixed alias.
#define NBX_API(ret, func, ...)                                                     \
  NBX_EXPORT ret func(__VA_ARGS__);                                                 \
  NBX_EXPORT __attribute__((alias(#func))) ret p##func(__VA_ARGS__);                \
  NBX_EXPORT ret func(__VA_ARGS__)

#define NBX_TRACE(...)                                   \
  do {                                                   \
    if (nbxcomm::traceOn()) {                            \
      std::fprintf(stderr, "[nbx] " __VA_ARGS__);        \
      std::fprintf(stderr, "\n");                        \
      std::fflush(stderr);                               \
    }                                                    \
  } while (0)

#define HIPCHECK(cmd)                                                         \
  do {                                                                        \
    hipError_t e_ = (cmd);                                                    \
    if (e_ != hipSuccess) {                                                   \
      nbxcomm::warn("HIP failure '%s' at %s:%d", hipGetErrorString(e_), __FILE__, __LINE__); \
      return ncclUnhandledCudaError;                                          \
    }                                                                         \
  } while (0)
#define NCCLCHECK(cmd)                          \
  do {                                          \
    ncclResult_t r_ = (cmd);                    \
    if (r_ != ncclSuccess) return r_;           \
  } while (0)

namespace nbxcomm {

// ---- logging (NCCL_DEBUG=WARN|INFO, debug.cc:26-147) and the last-error string
extern char g_lastError[1024];
void warn(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void info(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
bool traceOn();

int typeSize(ncclDataType_t t);

constexpr uint64_t kCommMagic = 0x4e42584343434f4dull;  // "NBXCCCOM"
constexpr char kIdMagic[8] = {'N', 'B', 'X', 'U', 'I', 'D', '0', '1'};

struct UserRedOp {   // comm.h ncclUserRedOp
  int freeNext;      // -1 = allocated
  ncclDataType_t datatype;
  nbxDevRedOpFull opFull;
};

struct Clique;
struct MpState;

}  // namespace nbxcomm

struct ncclComm {
  uint64_t magic = nbxcomm::kCommMagic;
  int nRanks = 1;
  int rank = 0;
  int device = 0;
  int blocking = 1;
  // ncclConfig_t minCTAs / maxCTAs after NCCL_MIN_CTAS / NCCL_MAX_CTAS
  // (init.cc:1455-1494); NCCL_CONFIG_UNDEF_INT: not set. A CTA (channel) is a
  // workgroup here: they bound the transports' grids (mpTransportSettings).
  int minCTAs = NCCL_CONFIG_UNDEF_INT;
  int maxCTAs = NCCL_CONFIG_UNDEF_INT;
  int cgaClusterSize = NCCL_CONFIG_UNDEF_INT;   // accepted and kept (no clusters on CDNA)
  int splitShare = NCCL_CONFIG_UNDEF_INT;       // accepted and kept (children share nothing here)
  bool checkPointers = false;
  std::atomic<int> asyncError{ncclSuccess};
  std::mutex opsMu;
  std::vector<nbxcomm::UserRedOp> userOps;
  int freeHead = 0;
  std::shared_ptr<nbxcomm::Clique> clique;  // nRanks > 1 (single process)
  nbxcomm::MpState* mp = nullptr;           // nRanks > 1 (one process per rank)
  nbxcomm::MpState* lt = nullptr;           // clique rank: in-process LL / LL128 transport (cliqueInitTransport)
  std::thread initThread;         // non-blocking ncclCommInitRankConfig: mpInit in the background
  int initAbort = 0;               // set by ncclCommAbort: the init thread's bootstrap waits end
  // pinned, device-mapped words every device wait of this rank polls: [0]
  // abort, [1] error, diag record at byte 16 (nbx_diag.h). Owned here, not by
  // the transport state, so ncclCommAbort can end a wait of a background
  // initialisation (the LL128 self-test's kernels) before it joins that thread.
  int* hostWords = nullptr;
  int* hostWordsDev = nullptr;
  // user PreMulSum across ranks (localPreScratch): this rank's input
  // pre-multiplied by its own scalar; superseded buffers are kept until the
  // communicator is freed (an earlier call may still read them)
  void* preScratch = nullptr;
  size_t preScratchBytes = 0;
  std::vector<void*> preScratchOld;
  // recorded (on the call's stream) behind the last call that read preScratch:
  // after the clique's leave step, every peer's fold of it is complete. The
  // next pre-pass waits for it, whatever stream either call ran on (ADVICE r5:
  // a clique without the in-kernel transport has no other cross-stream order)
  hipEvent_t preScratchFree = nullptr;
  bool preScratchPending = false;
  ~ncclComm() {
    if (hostWords) (void)hipHostFree(hostWords);
  }
};

namespace nbxcomm {

// ---- collectives as enqueued (both multi-rank communicator kinds)
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
  // a user PreMulSum (ncclRedOpCreatePreMulSum) across ranks: the scalar
  // multiplies THIS rank's input only — the reference applies the pre-op to
  // the local Input source alone (prims_simple.h:269-270) and exchanges the
  // peers' own scalars for the direct paths (:617-628), so the result is
  // sum_r s_r * x_r. Run as a pre-pass into scratch, then a Sum (localPreOp).
  bool localPre = false;
};

// One reducing collective as enqueued on a multi-process communicator (the
// same record the in-process clique queues).
using MpCall = PendingColl;

// In-process clique (ncclCommInitAll): per-rank streams are the caller's; the
// clique owns the events used to order the exchange across devices.
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
// g_pendMu together with every clique's pending queues (comm_clique.cc).
extern std::mutex g_pendMu;
extern std::vector<std::weak_ptr<Clique>> g_cliques;

// Group depth (group.cc:82-103: thread-local); the multi-process
// communicators this thread queued calls on inside the open group.
extern thread_local int t_groupDepth;
extern thread_local std::vector<ncclComm*> t_groupMpComms;

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

// Byte ranges one collective reads and writes.
struct Span {
  uintptr_t lo, hi;
  bool write;
};
bool spansConflict(const std::vector<Span>& a, const std::vector<Span>& b);

// ---- nccl_api.cc: checks, op encoding, enqueue
ncclResult_t commCheck(ncclComm* comm, const char* opName);
ncclResult_t commEnsureReady(ncclComm* comm);
ncclRedOp_t userRedOpMangle(ncclComm* comm, ncclRedOp_t op);
ncclResult_t hostToDevRedOp(nbxDevRedOpFull* opFull, ncclRedOp_t op, ncclDataType_t dt, ncclComm* comm);
// Element range of block b when `count` is split over n ranks, aligned so
// every block starts on a 16-byte boundary relative to the buffer.
void blockRange(size_t count, int eb, int n, int b, size_t* off, size_t* len);
ncclResult_t newComm(ncclComm** out, int nRanks, int rank, int dev, const ncclConfig_t* config);
// parseCommConfig (init.cc:1526-1594): the caller's config copied up to its
// own size (older versions get the defaults of the fields they predate), then
// checked; ncclInvalidArgument, with the reference's WARN, for a bad one.
ncclResult_t parseConfig(const ncclConfig_t* config, ncclConfig_t* out);

// ---- comm_clique.cc
ncclResult_t flushPending();   // launch every complete collective queued for every clique

// ---- multi-process transport state (comm_mp_init.cc)
constexpr int kMaxMpRanks = nbx::kSimpleMaxRanks;   // one staging source region per rank

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
  uint32_t* probeSink = nullptr;    // nbxDebugLinkProbe's never-written pull sink (allocated on first use)
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
  bool checkSlices = false;         // NBX_CHECK_SLICES: Simple slices carry a checksum the consumer verifies
  int sliceFaultRank = -1;          // NBX_DEBUG_SLICE_FAULT (test hook): this rank's workgroup 0 stamps wrong sums
  std::vector<hipEvent_t> groupEvents;   // fan-in / fan-out of a group launch over several streams
  // clique ranks only: the previous call ran on the event-ordered fold path
  // (runCliqueColl / runCliqueBatch) on extStream; it is complete once every
  // rank's extDone event (the clique's evDone) is
  hipStream_t extStream = nullptr;
  std::vector<hipEvent_t> extDone;
};

// The LL-family transport of a communicator: its own (one process per rank)
// or, for a rank of an in-process clique, the one cliqueInitTransport built.
inline MpState* mpOf(const ncclComm* c) { return c->mp ? c->mp : c->lt; }

// NCCL_PROTO bits (tuning.cc:254-259) and the per-message protocols.
enum { kProtoLL = 1, kProtoLL128 = 2, kProtoSimple = 4, kProtoAll = 7 };
enum MpProto : int { kMpLL = 0, kMpLL128 = 1, kMpSimple = 2, kMpLL128x2 = 3 };

int protoFromString(const char* v);
int protoGateAcrossGpus(int mask, bool multiGpu, const char* ncclProto);
MpProto chooseProtoFor(int mask, bool twoShotKind, uint64_t slotBytes, uint64_t blockBytes, int n, uint64_t llMax,
                       uint64_t l128Max, uint64_t oneShotMax);
bool algoRingFromEnv();
long envLong(const char* name, long dflt);
ncclResult_t mpAllocLL(MpState* mp, int n, bool ipc, const ncclComm* comm);
void mpTransportSettings(MpState* mp, int minCus, int maxShare, const ncclComm* comm);
ncclResult_t mpAllocSimple(MpState* mp, int n, bool ipc);
ncclResult_t mpInit(ncclComm* c, const ncclUniqueId& id);
ncclResult_t mpLL128SelfTest(ncclComm* c);
void mpReportDeviceError(ncclComm* c);
void mpFreeState(MpState* mp, int device);
void mpFree(ncclComm* c);

// ---- comm_mp_launch.cc
MpProto mpProtoOf(const ncclComm* comm, const MpCall& c);
ncclResult_t mpLaunchLL(ncclComm* comm, const MpCall& c, MpProto proto, const MpCall* segs = nullptr,
                        int nSegs = 0);
ncclResult_t mpLaunchSimple(ncclComm* comm, const MpCall* calls, int nc, bool transport = false);
ncclResult_t runMpColl(ncclComm* comm, const MpCall& c);
// localPre calls: scratch = this rank's input x its own scalar (one pre-op
// reduce on c.stream), then *c sums the scratch (op Sum, localPre cleared)
ncclResult_t localPreOp(ncclComm* comm, int device, PendingColl* c, int nRanks);
ncclResult_t preScratchDone(ncclComm* comm, int device, hipStream_t stream);
ncclResult_t runMpGroup(ncclComm* comm);
ncclResult_t flushMpGroups();

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

}  // namespace nbxcomm
