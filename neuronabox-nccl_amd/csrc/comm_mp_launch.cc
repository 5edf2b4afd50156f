// comm_mp_launch.cc — launches on a multi-process communicator (and on a
// clique rank's in-process transport): the per-message protocol choice, the
// LL / LL128 and Simple kernels' arguments, the cross-stream order
// (runMpOrdered, nbx_comm.h), and group batching (group.cc:82-103 semantics,
// enqueue.cc:67-91 work aggregation).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <string>
#include <exception>
#include "nbx_comm.h"

namespace nbxcomm {

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
ncclResult_t mpLaunchLL(ncclComm* comm, const MpCall& c, MpProto proto, const MpCall* segs,
                        int nSegs) {
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
ncclResult_t mpLaunchSimple(ncclComm* comm, const MpCall* calls, int nc, bool transport) {
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
  sa.checkSlices = mp->checkSlices ? (mp->sliceFaultRank == me ? 2 : 1) : 0;   // 2: test hook, a wrong stamp
  sa.order = mpOrderArgs(mp);
  return nbx::launchSimple(c.dt, c.op, sa, (unsigned)grid, mp->ring && !transport, c.stream);
}

ncclResult_t runMpColl(ncclComm* comm, const MpCall& c0) {
  if (c0.count == 0) return ncclSuccess;
  return runMpOrdered(comm, c0.stream, [&]() -> ncclResult_t {
    MpCall c = c0;   // after the cross-stream wait: the pre-pass reuses scratch an earlier call read
    if (c.localPre) NCCLCHECK(localPreOp(comm, comm->device, &c, comm->nRanks));
    const MpProto proto = mpProtoOf(comm, c);
    NCCLCHECK(proto == kMpSimple ? mpLaunchSimple(comm, &c, 1) : mpLaunchLL(comm, c, proto));
    // only this rank's kernel reads its scratch (peers see staging / lines)
    return c0.localPre ? preScratchDone(comm, comm->device, c.stream) : ncclSuccess;
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
// alike. A user PreMulSum (localPre) runs alone too: its pre-pass fills the
// communicator's one scratch buffer. A group whose AllReduce / ReduceScatter calls alias differently on
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
      if (mp->groupBatch && calls[i].kind != kReduce && !calls[i].localPre &&
          (p == kMpLL || p == kMpLL128 || p == kMpSimple)) {
        uint64_t used = p == kMpSimple ? 0 : unitsOf(calls[i], p);
        std::vector<Span> spans, sj;
        mpCallSpans(calls[i], comm->nRanks, &spans);
        while (j < calls.size() && j - i < maxSegs && calls[j].count > 0 && !calls[j].localPre &&
               sameOp(calls[i], calls[j]) &&
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

}  // namespace nbxcomm

using namespace nbxcomm;

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

// Per-link fabric rate (the roofline config D's entries are priced against):
// every rank moves `bytesPerPeer` to (pull = 0: the transport's system-scope
// stores) or from (pull = 1: its system-scope loads) each peer's Simple
// staging at once, in its own part of the peer's data area (the slices, never
// the flag words or plan headers), with workgroupsPerPeer workgroups per peer
// (0: 32). One kernel on `stream`; *bytesMovedPerPeer receives what one launch
// moves per peer (bytesPerPeer rounded to whole passes over the part). NOT
// ordered against collectives: the caller keeps every rank's communicator
// quiet around it (no Simple call in flight on any rank) — it overwrites the
// peers' staging slices. Measurement only.
NBX_EXPORT ncclResult_t nbxDebugLinkProbe(ncclComm_t comm, size_t bytesPerPeer, int pull, int workgroupsPerPeer,
                                         ncclStream_t stream, size_t* bytesMovedPerPeer) {
  NCCLCHECK(commCheck(comm, "LinkProbe"));
  NCCLCHECK(commEnsureReady(comm));
  MpState* mp = comm->mp;
  const int n = comm->nRanks;
  if (mp == nullptr || n < 2 || bytesPerPeer == 0 || bytesMovedPerPeer == nullptr || workgroupsPerPeer < 0)
    return ncclInvalidArgument;
  const int wg = workgroupsPerPeer > 0 ? workgroupsPerPeer : 32;
  // this rank's part of a peer's slices (16-B packs, < 2 GiB for the buffer
  // resource), cut into one whole chunk per workgroup
  const uint64_t part = std::min<uint64_t>(mp->stageHdrOff / (uint64_t)n, 1ull << 30) & ~15ull;
  const uint64_t chunkPacks = part / 16 / (uint64_t)wg;
  if (chunkPacks == 0) return ncclInvalidArgument;
  const uint64_t perPass = chunkPacks * 16 * (uint64_t)wg;
  const uint64_t passes = std::max<uint64_t>(1, (bytesPerPeer + perPass - 1) / perPass);
  if (passes > (1u << 20)) return ncclInvalidArgument;
  DevGuard g(comm->device);
  if (mp->probeSink == nullptr) HIPCHECK(hipMalloc((void**)&mp->probeSink, nbx::kLinkProbeSinkWords * sizeof(uint32_t)));
  *bytesMovedPerPeer = (size_t)(passes * perPass);
  return nbx::launchLinkProbe(mp->peerStageDev, comm->rank, n, part, chunkPacks, wg, (int)passes, pull != 0,
                              mp->probeSink, (hipStream_t)stream);
}
