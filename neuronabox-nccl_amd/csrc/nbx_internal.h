// nbx_internal.h — library-internal entry points shared between host units.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <mutex>
#include <utility>

#include "../../include/nbx_reduce.h"

namespace nbx {
struct KArgs;
// Dynamic tiles (nbx_tiles.h forEachTile): begin() gives the launch its
// stream's counter and base (a.dynCtr / a.dynBase) and holds the counter lock
// until done(), which advances the base by the launch's tile count if the
// launch went out. begin() returns false (static grid stride) while the
// stream is being captured, for hipStreamPerThread, or with
// NBX_DYNAMIC_TILES=0 (nbx_reduce.cc).
class DynLaunch {
 public:
  bool begin(int dev, hipStream_t st, uint64_t nTiles, KArgs& a);
  void done(bool launched);

 private:
  std::unique_lock<std::mutex> lk_;
  std::pair<uint32_t*, uint32_t>* slot_ = nullptr;
  uint64_t tiles_ = 0;
};
struct LLArgs;
struct SimpleArgs;
// nbxReduceMulti with internal flags: kReduceAcquireSystem makes every
// workgroup issue a system-scope acquire before its first load (sources in
// peer GPU memory, written before the launch and ordered by a flag barrier).
constexpr int kReduceAcquireSystem = 1;
ncclResult_t reduceMultiEx(void* const* dsts, int nDsts, const void* const* srcs, int nSrcs, size_t count,
                           ncclDataType_t datatype, nbxDevRedOpFull op, int nPreOpSrcs, int postOp,
                           ncclStream_t stream, int flags);
// nbxReduceMultiBatch with the same internal flags.
ncclResult_t reduceMultiBatchEx(const nbxReduceTask* tasks, int nTasks, ncclDataType_t datatype, nbxDevRedOpFull op,
                                int nPreOpSrcs, int postOp, ncclStream_t stream, int flags);
// Launch the LL collective kernel of (datatype, op) (nbx_ll.h); sequencing is
// device-resident (args.state).
ncclResult_t launchLLColl(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, hipStream_t stream);
// The same for the LL128 kernel (args.nLines 64-byte lines).
ncclResult_t launchLL128Coll(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, hipStream_t stream);
// Simple protocol collective (nbx_simple.h): the direct schedule, or the ring
// schedule when `ring`; `grid` workgroups (<= args.gridMax).
ncclResult_t launchSimple(ncclDataType_t dt, const nbxDevRedOpFull& op, SimpleArgs& args, unsigned grid, bool ring,
                          hipStream_t stream);
// kMpWaitDone on `stream` (nbx_order.hip): the stream waits until *done >= target.
ncclResult_t launchMpWaitDone(const uint64_t* done, uint64_t target, const volatile int* abortWord,
                              volatile int* errWord, uint64_t timeoutTicks, hipStream_t stream);
// Every rank of the one-process Simple rig in one dispatch (fp32 sum; PMC
// measurement only, nbx_simple_bench.cc): n x grid workgroups, argsDev[n].
ncclResult_t launchSimpleFusedF32Sum(const SimpleArgs* argsDev, int n, unsigned grid, bool ring, hipStream_t stream);
int simpleFusedMaxResident(bool ring);   // workgroups of kSimpleFused resident at once (-1: HIP error)
// nbxDebugLinkProbe's kernel (nbx_ll_debug.hip): (n - 1) x wgPerPeer workgroups,
// each moving chunkPacks 16-B packs of this rank's part of one peer's staging,
// `passes` times; sink[kLinkProbeSinkWords] is written only by a pull, and only in theory.
constexpr int kLinkProbeSinkWords = 256;   // = kBlock (nbx_kargs.h)
ncclResult_t launchLinkProbe(char* const* peerStageDev, int me, int n, uint64_t part, uint64_t chunkPacks,
                             int wgPerPeer, int passes, bool pull, uint32_t* sink, hipStream_t stream);
// LL128 two-shot AllReduce (args.nLines = sub-slot lines; blockLines sizes the grid).
ncclResult_t launchLL128AllReduce2(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& args, uint64_t blockLines,
                                   hipStream_t stream);
}  // namespace nbx
