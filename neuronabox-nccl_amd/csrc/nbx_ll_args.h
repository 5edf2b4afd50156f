// nbx_ll_args.h — kernel arguments of the LL-protocol collectives (nbx_ll.h);
// device-free so host units can fill them.
#pragma once
#include <stdint.h>

namespace nbx {

enum LLMode : int32_t { kLLAllReduce = 0, kLLReduceScatter = 1, kLLReduce = 2 };
constexpr int kL128MaxRanksHost = 8;   // LL128 kernel keeps one line per rank in registers
constexpr int kL128LineBytesHost = 64;  // LL128 line: 4 x {12 payload bytes + 4-byte flag} (nbx_ll.h)
constexpr int kL128DataBytesHost = 48;
constexpr int kL128LanesHost = 4;       // lanes (16 bytes each) per LL128 line

// Device-resident sequencing of the LL-family calls of one communicator
// (plain device memory of this rank, zero at init). Kept on the device, not
// passed by the host, so a captured graph replays with fresh sequence numbers:
// every block of a launch reads seq at its start; the launch's last block
// (found by the MpDone arrival counters, nbx_order.h) publishes the done
// words, then advances seq / lastSeq for the next launch.
struct LLState {
  uint64_t seq;         // last completed LL-family call (the pending one is seq + 1)
  uint64_t lastSeq[2];  // last call that used each parity's slots (credit target)
  uint64_t recvAllSeq;  // last call in which this rank took lines from every peer
};

// Cross-stream order of one communicator's calls (comm_mp_launch.cc runMpColl):
// every eager call carries its sequence number; the launch's last block, once
// every block's memory operations have completed, publishes it in `done`
// (device memory). A call on another stream than the previous one is preceded
// by kMpWaitDone on its stream, spinning until `done` reaches the previous
// call's number — no event behind every call (an event marker cost ~5 us of
// device time per call, scripts/probe_order_cost.hip). seq = 0 (captured
// calls): nothing is published. `arrive`: 8 per-XCD arrival counters and one
// top counter, each on its own 64-byte line, zero between launches.
constexpr int kMpArriveStride = 16;   // u32 words between arrival counters (64 B)
struct MpDone {
  uint64_t* done;
  uint32_t* arrive;   // [9 * kMpArriveStride]
  uint64_t seq;
};

// A group of small collectives as ONE LL launch (comm_mp_launch.cc runMpGroup; NCCL
// packs a group's collectives into one kernel's work, enqueue.cc:67-91): the
// messages' slots are concatenated, 8-byte packs [packOff, packOff + packs of
// this message) of the launch belong to segment s. Every segment has the
// launch's kind, datatype, op (and root). nSegs = 0: the single message of
// send / recv / count / blockElts.
constexpr int kLLMaxSegs = 16;
struct LLSeg {
  const void* send;
  void* recv;
  uint64_t count;       // elements per slot (ReduceScatter: recvcount)
  uint64_t packOff;     // first pack of this message in the launch's slot
  uint64_t blockElts;   // AllReduce: the message's direct-schedule block (fold order)
};

struct LLArgs {
  const void* send;
  void* recv;
  uint64_t count;          // elements per slot: AllReduce/Reduce = count, ReduceScatter = recvcount
  uint64_t nPacks;         // 8-byte packs covering `count` elements
  uint64_t* const* peerLL; // device table: rank -> LL buffer base
  uint64_t* myLL;
  uint64_t slotLines;      // lines per (parity, source) slot = 2 * max packs
  uint64_t doneOff;        // line index of the done words (one per writer rank) in every LL buffer
  uint64_t planOff;        // line index of the plan words [parity 2][source n] in every LL buffer
  LLState* state;          // this rank's sequencing state (device memory)
  uint64_t blockElts;      // AllReduce: direct-schedule block size (elements) -> fold order
  uint64_t arg;            // functor scalar (by value)
  const void* argPtr;      // device scalar or nullptr
  const volatile int* abortWord;
  volatile int* errWord;
  uint64_t timeoutTicks;
  // LL128 (kLL128Coll only): 64-byte lines, 4 x {12 payload bytes + 4-byte flag}
  uint64_t* const* peerL128;  // device table: rank -> LL128 buffer base
  uint64_t* myL128;
  uint64_t l128SlotLines;     // lines per (parity, source) slot
  uint64_t nLines;            // lines covering this call's slot bytes
  uint32_t l128Bytes;         // size of myL128 (buffer-descriptor range, < 4 GiB)
  int32_t rank;
  int32_t nRanks;
  int32_t postOp;
  int32_t mode;            // LLMode
  int32_t root;            // kLLReduce
  MpDone order;
  int32_t nSegs;           // kLLColl group launch: segments in seg[] (0: one message)
  uint32_t gridCap;        // the communicator's workgroup cap (ranks sharing a GPU split it), 0: none
  uint32_t planSig;        // llPlanSig: the same on every rank iff the ranks cut the call alike; 0: no plan checks
  uint32_t pad;
  LLSeg seg[kLLMaxSegs];
};

// An LL-family launch's plan: what decides which line of a slot carries which
// bytes and how a receiver folds them (protocol, kind, type, op, root, ranks,
// message sizes and blocks, a group's cut; never a pointer, the rank or the
// grid), hashed (FNV-1a, folded to 32 bits). Every source stamps it with the
// call's flag into its plan word in each target's buffer (nbx_ll.h llPlanStamp).
inline uint32_t llPlanSig(const LLArgs& a, int32_t proto, int32_t dtype, int32_t op) {
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&h](uint64_t v) {
    for (int b = 0; b < 8; b++) {
      h ^= (v >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ull;
    }
  };
  mix((uint64_t)(uint32_t)proto);
  mix((uint64_t)(uint32_t)a.mode);
  mix((uint64_t)(uint32_t)a.root);
  mix((uint64_t)(uint32_t)a.nRanks);
  mix((uint64_t)(uint32_t)dtype);
  mix((uint64_t)(uint32_t)op);
  mix(a.count);
  mix(a.nPacks);
  mix(a.nLines);
  mix(a.blockElts);
  mix((uint64_t)(uint32_t)a.nSegs);
  for (int s = 0; s < a.nSegs; s++) {
    mix(a.seg[s].count);
    mix(a.seg[s].packOff);
    mix(a.seg[s].blockElts);
  }
  return (uint32_t)(h ^ (h >> 32)) | 1u;   // never 0 (0: checks off)
}

// ---------------------------------------------------------------------------
// Simple protocol over init-mapped staging (nbx_simple.h). Peers never touch
// the caller's buffers: each rank owns an uncached staging area and a set of
// uncached flag words, allocated and IPC-mapped by every peer ONCE, at
// ncclCommInitRank (the p2pMap / p2pSendConnect step of the reference,
// transport/p2p.cc:290-330,450-520). A rank's kernels move data between its
// own user buffers and staging; peer traffic is stores into the peer's
// staging plus flag words (waitPeer / postPeer of prims_simple.h:129-185).
//   staging  [region 2: RS | AG][slot][source rank n][workgroup gridMax][stageSlice bytes]
//            then, at hdrOff, one 16-byte plan header per slice cell in the same order
//            ({plan signature, round}: written with the slice, checked by the consumer)
//   flags    [kind 4][peer n][workgroup gridMax] u64      (written by the peer)
//   counters [kind 4][peer n][workgroup gridMax] u64      (this rank's, device-resident)
// Counter / flag kinds per (ordered pair, workgroup), monotonic over the
// communicator's life, so producer and consumer agree without the host:
//   rsSent  / flag rsReady  : RS-region slices this rank pushed to the peer / the peer pushed here
//   rsRecv  / flag rsCredit : RS-region slices this rank consumed from the peer / the peer consumed from here
//   agSent  / flag agReady  : the same for the AG region
//   agRecv  / flag agCredit
// kSimpleTransport (measurement only, nbxDebugTransportAllReduce): the direct
// AllReduce schedule moving every byte it moves across the peers (pushes,
// gather) with the fold reduced to a copy of the own input — the staging
// slots are waited for and credited, not read — so its time is the xGMI
// transport alone; its output is not the sum.
enum SimpleMode : int32_t { kSimpleAllReduce = 0, kSimpleReduceScatter = 1, kSimpleReduce = 2, kSimpleTransport = 3 };
enum SimpleAlgo : int32_t { kSimpleAlgoDirect = 0, kSimpleAlgoRing = 1 };
// flag words (written by the peer named by their index)
enum SimpleFlag : int32_t { kFlRsReady = 0, kFlRsCredit = 1, kFlAgReady = 2, kFlAgCredit = 3 };
// this rank's counters (per peer, per workgroup)
enum SimpleCounter : int32_t { kCtRsSent = 0, kCtRsRecv = 1, kCtAgSent = 2, kCtAgRecv = 3 };
constexpr int kSimpleMaxGrid = 256;
constexpr int kSimpleMaxRanks = 64;
constexpr int kSimpleMinSliceBytes = 4096;   // a call uses at most ceil(block / 4 KiB) workgroups

// A group of Simple-sized collectives as ONE launch (comm_mp_launch.cc runMpGroup;
// NCCL packs a group's collectives into one kernel's work, enqueue.cc:67-91):
// every block b of the launch is the concatenation of block b of each
// message, cut into the launch's slices; segment s owns the virtual slices
// [sliceOff, next sliceOff) of every block. Every segment has the launch's
// kind, datatype, op (and root). nSegs = 0: the single message of send / recv
// / total / blockElts.
constexpr int kSimpleMaxSegs = 16;
struct SimpleSeg {
  const void* send;
  void* recv;
  uint64_t total;       // elements of the message (ReduceScatter: recvcount * n)
  uint64_t blockElts;   // its block (as SimpleArgs::blockElts)
  uint64_t sliceOff;    // its first virtual slice of every block
};

struct SimpleArgs {
  const void* send;
  void* recv;                  // nullptr on Reduce non-roots
  char* const* peerStage;      // device table [n]: rank -> staging base (own entry: own staging)
  uint64_t* const* peerFlags;  // device table [n]: rank -> flag words (own entry: own flags)
  uint64_t* counters;          // this rank's [4][n][gridMax]
  uint64_t total;              // elements of the message (ReduceScatter: recvcount * n)
  uint64_t blockElts;          // elements per block: AllReduce/Reduce direct = blockRange, RS = recvcount, ring Reduce = count
  uint64_t sliceBytes;         // bytes per (workgroup, block, round) of this call (multiple of 16)
  uint64_t nRounds;
  uint64_t stageSlice;         // staging bytes per (region, slot, source, workgroup)
  uint64_t arg;
  const void* argPtr;
  const volatile int* abortWord;
  volatile int* errWord;
  uint64_t timeoutTicks;
  uint64_t planSig;            // simplePlanSig: the same on every rank iff the ranks cut the call alike; 0: no checks
  uint64_t hdrOff;             // byte offset of the plan headers in every rank's staging
  int32_t rank;
  int32_t nRanks;
  int32_t mode;                // SimpleMode
  int32_t root;
  int32_t slots;               // staging slots per (region, source, workgroup), >= 2
  int32_t gridMax;
  int32_t prefetch;            // direct: push round k+1 before folding round k (a rank-local choice)
  int32_t nSegs;               // group launch: segments in seg[] (0: one message)
  int32_t checkSlices;         // NBX_CHECK_SLICES: producers stamp, consumers verify every slice's checksum
  int32_t pad0;
  MpDone order;
  SimpleSeg seg[kSimpleMaxSegs];
};

// A launch's plan: everything that decides which elements go into which
// staging slice in which round (never a pointer, never the rank), hashed
// (FNV-1a). Ranks whose calls or group cuts differ get different signatures;
// a consumer that finds a slice stamped with another signature fails the
// launch (kDiagSimplePlan) instead of folding misplaced data.
inline uint64_t simplePlanSig(const SimpleArgs& a, uint32_t grid, int32_t dtype, int32_t op) {
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&h](uint64_t v) {
    for (int b = 0; b < 8; b++) {
      h ^= (v >> (8 * b)) & 0xffu;
      h *= 0x100000001b3ull;
    }
  };
  mix((uint64_t)a.mode);
  mix((uint64_t)(uint32_t)a.root);
  mix((uint64_t)a.nRanks);
  mix((uint64_t)(uint32_t)dtype);
  mix((uint64_t)(uint32_t)op);
  mix(grid);
  mix(a.sliceBytes);
  mix(a.nRounds);
  mix((uint64_t)a.nSegs);
  if (a.nSegs == 0) {
    mix(a.total);
    mix(a.blockElts);
  }
  for (int s = 0; s < a.nSegs; s++) {
    mix(a.seg[s].total);
    mix(a.seg[s].blockElts);
    mix(a.seg[s].sliceOff);
  }
  return h | 1u;   // never 0: zeroed staging never matches
}

}  // namespace nbx
