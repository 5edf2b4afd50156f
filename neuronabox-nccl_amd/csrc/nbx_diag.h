// nbx_diag.h — what a bounded device spin saw when it gave up.
//
// The multi-process communicator's host words (pinned, device-mapped, 64 B):
//   int32 [0] abort word (ncclCommAbort), [1] error word (1 timeout, 2 abort),
//   uint64 at byte 16: the diagnostic record of a timed-out wait —
//     [0] site (kDiag*), [1] the peer rank waited on, [2] the value waited for,
//     [3] the value last observed, [4] the workgroup, [5] wall-clock ticks spent
// so a timeout names the wait, the peer and how far it got (NCCL prints the
// equivalent from its proxy / abort path, init.cc:2016, prims_simple.h:103-113).
// Several waves may time out together; the record is the last writer's (the
// site word is written last, after the fields), except that a failed plan
// check is never replaced by a timeout.
#pragma once
#include <stdint.h>

namespace nbx {

enum DiagSite : uint64_t {
  kDiagNone = 0,
  kDiagCredit = 1,       // LL family: a target's done word (slot credit)
  kDiagLLLine = 2,       // LL: a {data, flag} line of a peer
  kDiagLL128Line = 3,    // LL128 one-shot: a peer's line
  kDiagLL128RS = 4,      // LL128 two-shot: a reduce-scatter sub-slot line
  kDiagLL128AG = 5,      // LL128 two-shot: an all-gather sub-slot line
  kDiagRing = 6,         // pipelined ring: the left neighbour's progress word
  kDiagBarrier = 7,      // phase barrier: a peer's flag
  kDiagSimpleRs = 8,     // Simple: a peer's RS-region slice (rsReady)
  kDiagSimpleRsCredit = 9,   // Simple: a peer's credit for this rank's RS slot (rsCredit)
  kDiagSimpleAg = 10,    // Simple: a peer's AG-region slice (agReady)
  kDiagSimpleAgCredit = 11,  // Simple: a peer's credit for this rank's AG slot (agCredit)
  kDiagOrder = 12,       // a call on another stream: the previous call's done word (kMpWaitDone)
  kDiagSimplePlan = 13,  // Simple: a peer's slice was cut by another plan (mismatched calls or group runs)
  kDiagLLPlan = 14,      // LL family: a peer at the same call runs another plan
  kDiagLLPlanWord = 15,  // LL family: a peer's plan word for this call (its lines had arrived)
  kDiagSimpleSlice = 16, // Simple (NBX_CHECK_SLICES): a slice read differs from what its producer wrote
};
constexpr int kDiagWords = 6;
constexpr int kDiagByteOffset = 16;   // from the start of the host words

// a site that records a failed consistency check, not a wait that gave up
constexpr bool diagIsPlanCheck(uint64_t s) { return s == kDiagSimplePlan || s == kDiagLLPlan || s == kDiagSimpleSlice; }

inline const char* diagSiteName(uint64_t s) {
  switch (s) {
    case kDiagCredit: return "slot credit (peer done word)";
    case kDiagLLLine: return "LL line flag";
    case kDiagLL128Line: return "LL128 line flag";
    case kDiagLL128RS: return "LL128 two-shot reduce-scatter line flag";
    case kDiagLL128AG: return "LL128 two-shot all-gather line flag";
    case kDiagRing: return "ring progress word";
    case kDiagBarrier: return "phase barrier flag";
    case kDiagSimpleRs: return "Simple reduce-scatter slice (peer's ready word)";
    case kDiagSimpleRsCredit: return "Simple reduce-scatter slot credit";
    case kDiagSimpleAg: return "Simple all-gather slice (peer's ready word)";
    case kDiagSimpleAgCredit: return "Simple all-gather slot credit";
    case kDiagOrder: return "previous call's completion (stream switch)";
    case kDiagSimplePlan: return "Simple slice from a peer running a different plan (mismatched call or group cut)";
    case kDiagLLPlan: return "LL / LL128 lines from a peer running a different plan (mismatched call or group cut)";
    case kDiagLLPlanWord: return "LL / LL128 plan word of a peer";
    case kDiagSimpleSlice: return "Simple slice checksum (the bytes read differ from the bytes the peer wrote)";
    default: return "unknown";
  }
}

#if defined(__HIPCC__)
// Called by the lane that timed out; errWord points at host word [1].
__device__ __forceinline__ void diagTimeout(volatile int* errWord, uint64_t site, int peer, uint64_t target,
                                            uint64_t observed, uint64_t ticks) {
  volatile uint64_t* d = (volatile uint64_t*)((volatile char*)errWord - 4 + kDiagByteOffset);
  // a failed plan check names the cause; a later call's wait that then times
  // out (the peers have diverged) does not replace it
  if (!diagIsPlanCheck(site) && diagIsPlanCheck(d[0])) return;
  d[1] = (uint64_t)(int64_t)peer;
  d[2] = target;
  d[3] = observed;
  d[4] = blockIdx.x;
  d[5] = ticks;
  d[0] = site;
}
#endif

}  // namespace nbx
