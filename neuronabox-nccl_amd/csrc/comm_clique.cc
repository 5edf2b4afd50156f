// comm_clique.cc — the in-process clique (ncclCommInitAll, init.cc:1678-1734):
// every rank of one process, one thread driving them. Collectives are queued
// per rank and run once every rank has enqueued its part (flushPending): the
// event-ordered direct fold (rank r folds block r of every send buffer, in
// NCCL's ring order r+1, ..., r, and pushes it into every output), batched
// folds for a group's independent collectives, and — ranks on distinct GPUs
// — the multi-process kernels in-kernel over in-process connection buffers.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <exception>
#include "nbx_comm.h"

namespace nbxcomm {

std::mutex g_pendMu;
std::vector<std::weak_ptr<Clique>> g_cliques;

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


bool cliqueInKernel(Clique* c, const std::vector<PendingColl>& parts);
ncclResult_t cliqueRunLL(Clique* c, const std::vector<std::vector<PendingColl>>& rounds, size_t lo, size_t hi);
ncclResult_t cliqueOrderBefore(Clique* c, int r, hipStream_t s);
ncclResult_t cliqueOrderAfter(Clique* c, int r, hipStream_t s);

// Run one collective across every rank of an in-process clique.
ncclResult_t runCliqueColl(Clique* c, const std::vector<PendingColl>& parts0) {
  const int n = c->n;
  if (!sameCollective(parts0)) {
    warn("collective mismatch across ranks of the clique");
    return ncclInvalidUsage;
  }
  std::vector<PendingColl> parts = parts0;   // localPre: each rank's pre-multiplied scratch, summed
  const PendingColl& p0 = parts[0];
  const int eb = typeSize(p0.dt);
  NBX_TRACE("clique coll kind=%d n=%d count=%zu dt=%d op=%d", (int)p0.kind, n, p0.count, (int)p0.dt, p0.op.op);
  // 1. enter: every rank's stream reaches the collective (after the previous
  //    call of the rank when that ran on another stream)
  for (int r = 0; r < n; r++) {
    DevGuard g(c->devs[r]);
    NCCLCHECK(cliqueOrderBefore(c, r, parts[r].stream));
    if (parts[r].localPre) NCCLCHECK(localPreOp(c->comms[r], c->devs[r], &parts[r], n));
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
    if (parts0[r].localPre) NCCLCHECK(preScratchDone(c->comms[r], c->devs[r], parts[r].stream));
  }
  return ncclSuccess;
}

// Byte ranges one clique collective reads and writes (every rank's buffers).
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
    return sameCollective(parts) && !(parts[0].kind == kAllReduce && n > NBX_MAX_DSTS) && !parts[0].localPre;
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
    mpTransportSettings(mp, minCus, maxShare, cl->comms[r]);   // co-resident grids, as mpInit
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

}  // namespace nbxcomm

using namespace nbxcomm;

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
