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
// (the one whose arrival completes `arrive`) publishes the done words, then
// advances seq / lastSeq and resets `arrive` for the next launch.
struct LLState {
  uint64_t seq;         // last completed LL-family call (the pending one is seq + 1)
  uint64_t lastSeq[2];  // last call that used each parity's slots (credit target)
  uint64_t arrive;      // blocks of the running launch that have finished
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
};

constexpr int kRingMaxGrid = 256;   // slices per chunk = workgroups; one progress word each

// Pipelined ring AllReduce (nbx_ring.h kRingAllReduce): device-resident
// sequencing, as LLState. The step-FIFO kernels (kRingFifo) keep, per
// workgroup, how many FIFO entries this rank has produced and consumed over
// all calls — every rank counts the same calls, so producer and consumer
// agree without the host passing values (graph replays included).
struct RingState {
  uint64_t seq;      // completed ring calls
  uint64_t arrive;   // workgroups of the running launch that have finished
  uint64_t produced[kRingMaxGrid];   // kRingFifo: entries written into this rank's FIFO, per workgroup
  uint64_t consumed[kRingMaxGrid];   // kRingFifo: entries of the left neighbour's FIFO read, per workgroup
};

// Step-FIFO ring ReduceScatter / chain Reduce (nbx_ring.h kRingFifo): NCCL's
// Simple-protocol FIFO (prims_simple.h:129-185: the receiver waits on the
// sender's tail, the sender on the receiver's head credit) with the FIFO in
// the producer's HBM, read in place by the right neighbour over xGMI.
enum RingFifoMode : int32_t { kRingFifoReduceScatter = 0, kRingFifoReduce = 1 };
constexpr int kRingFifoSlots = 4;          // entries in flight per workgroup (NCCL_STEPS analogue)
constexpr int kRingFifoEntryPacks = 2048;  // 16-B packs per entry: 32 KiB per workgroup per step
constexpr uint64_t kRingFifoBytes = (uint64_t)kRingMaxGrid * kRingFifoSlots * kRingFifoEntryPacks * 16;

struct RingFifoArgs {
  const void* sendMe;     // this rank's input
  const void* sendLeft;   // the left neighbour's input (peer mapping): the chain's first hop reads it raw
  void* recv;             // RS: this rank's block; Reduce: the root's output (root only)
  void* fifoMe;           // this rank's FIFO [kRingMaxGrid][kRingFifoSlots][kRingFifoEntryPacks] packs
  const void* fifoLeft;   // the left neighbour's FIFO (peer mapping)
  uint64_t* myTail;       // [kRingMaxGrid] entries the left neighbour has produced (it posts here; uncached)
  uint64_t* rightTail;    // the right neighbour's tail words (peer mapping): this rank posts there
  uint64_t* myHead;       // [kRingMaxGrid] entries of this rank's FIFO the right neighbour has consumed
  uint64_t* leftHead;     // the left neighbour's head words (peer mapping): this rank posts there
  RingState* state;
  uint64_t blockElts;     // RS: recvcount (a whole number of 16-B packs); Reduce: count
  uint64_t slicePacks;    // 16-B packs per workgroup slice of a block (Reduce: of the message)
  uint64_t arg;
  const void* argPtr;
  const volatile int* abortWord;
  volatile int* errWord;
  uint64_t timeoutTicks;
  int32_t rank;
  int32_t nRanks;
  int32_t root;           // Reduce
  int32_t mode;           // RingFifoMode
};

struct RingArgs {
  const void* sendMe;     // this rank's input
  const void* sendLeft;   // the left neighbour's input (peer mapping): step 0 reads it raw
  void* recvMe;           // this rank's output: partials of steps 0..n-3 live here
  const void* recvLeft;   // the left neighbour's output (peer mapping): its partials
  void* outs[8];          // last step: rank (me + k) % n's output for k < nOuts (push-gather)
  uint64_t* myProgress;   // [kRingMaxGrid] words the LEFT neighbour posts (uncached, this rank's memory)
  uint64_t* rightProgress;// the right neighbour's words (peer mapping): this rank posts there
  RingState* state;
  uint64_t total;         // elements of the message
  uint64_t blockElts;     // direct-schedule block (multiple of 16 B / element)
  uint64_t slicePacks;    // 16-B packs per slice (one slice per workgroup per chunk)
  uint64_t arg;
  const void* argPtr;
  const volatile int* abortWord;
  volatile int* errWord;
  uint64_t timeoutTicks;
  int32_t rank;
  int32_t nRanks;
  int32_t nOuts;          // 1: own output only (gather follows), n: push to every rank
  int32_t pad;
};

}  // namespace nbx
