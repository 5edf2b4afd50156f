// nbx_ll.h — LL ("low latency") protocol for small messages on the
// multi-process communicator: one kernel per collective, no host exchange.
//
// Wire format (the idea of NCCL's LL protocol, prims_ll.h:226-294 /
// device.h ncclLLFifoLine): every 8-byte line is {u32 data, u32 flag} written
// by ONE 64-bit system-scope store, so a reader that sees flag == seq also
// sees that line's data (single-copy atomicity; no separate flag, no fence).
// Each rank owns an IPC-registered, uncached LL buffer laid out
//   [parity 2][source rank n][lines 2 * maxPacks]   data lines (8 bytes)
//   [done n]                                        done words, one per writer
// plus a private LLState (seq, per-parity last seq, block-arrival counter) in
// plain device memory; the sequence lives on the device so a graph-captured
// call replays with fresh numbers. The kernel of rank r
//   -. reads seq = state.seq + 1 (parity seq & 1, credit target
//      state.lastSeq[parity]);
//   0. waits until every peer it pushes to has finished reading the last LL
//      call that used this parity (that peer's done word >= needDone) — the
//      credit that makes a slot reusable even when a rank never waits for
//      data (Reduce non-roots); implied, and skipped, when the previous call
//      took lines from every peer (llBegin);
//   1. pushes its message, 8 bytes per thread, as two lines into slot
//      [seq & 1][r] of each target's buffer (remote stores over xGMI):
//        AllReduce      — the whole message to every peer
//        ReduceScatter  — send block j (recvcount elements) to peer j
//        Reduce         — the whole message to the root only;
//   2. polls its own slots [seq & 1][j] until the flags equal seq (bounded
//      spin: timeout + abort word), takes its own contribution from `send`,
//      and folds all n sources per element in the direct schedule's order so
//      the result is bitwise the direct path's:
//        AllReduce      — element in block c: ranks c+1, ..., c
//        ReduceScatter  — ranks r+1, ..., r       (reduce_scatter.h:50-64)
//        Reduce (root)  — ranks root+1, ..., root (reduce.h:44-67);
//   3. stores the result; the last block to finish publishes this rank's
//      done word (= seq) into every peer's buffer and advances the state.
// Plan words (when the communicator checks plans, NBX_CHECK_PLANS: the
// kernels' CHECK instantiation, LLArgs.planSig != 0; the default instantiation
// carries none of this code): [parity 2][source n] after the done words. Every source
// stamps {plan signature, flag} into each target's buffer, performed before
// its lines go out (llPlanStamp), so a receiver can tell a peer that runs the
// same call with another plan (mismatched counts / types / ops, a group cut
// differently) and fail the launch naming it (kDiagLLPlan) — instead of timing
// out on lines the peer never writes (every stuck line wait reads the plan
// word in its slow path), or folding lines it cut differently (block 0's
// threads j compare peer j's word after the fold, llPlanCheck).
#pragma once
#include "nbx_diag.h"
#include "nbx_order.h"
#include "nbx_functors.h"
#include "nbx_ll_args.h"

namespace nbx {

template <class Fn>
__device__ __forceinline__ uint64_t llLoadArg(const LLArgs& a) {
  if (a.argPtr != nullptr) return (uint64_t) * (const typename Fn::Elt*)a.argPtr;
  return a.arg;
}

// 8 bytes of `p` starting at byte `off`, zero past `limit` (any alignment)
__device__ __forceinline__ uint64_t llLoadBytes(const unsigned char* p, uint64_t off, uint64_t limit) {
  if (off + 8 <= limit && (((uintptr_t)(p + off)) & 7u) == 0) return *(const uint64_t*)(p + off);
  uint64_t v = 0;
  for (int b = 0; b < 8; b++)
    if (off + b < limit) v |= (uint64_t)p[off + b] << (8 * b);
  return v;
}

__device__ __forceinline__ void llStoreBytes(unsigned char* p, uint64_t off, uint64_t limit, uint64_t v) {
  if (off + 8 <= limit && (((uintptr_t)(p + off)) & 7u) == 0) {
    *(uint64_t*)(p + off) = v;
    return;
  }
  for (int b = 0; b < 8; b++)
    if (off + b < limit) p[off + b] = (unsigned char)(v >> (8 * b));
}

// A bounded spin gives up: error word (1 timeout, 2 abort) + what it waited for.
__device__ __forceinline__ void llGiveUp(const LLArgs& a, uint64_t site, int peer, uint64_t target, uint64_t seen,
                                         uint64_t t0, bool record = true) {
  const bool aborted = *a.abortWord != 0;
  if (!aborted && record) diagTimeout(a.errWord, site, peer, target, seen, wall_clock64() - t0);
  *a.errWord = aborted ? 2 : 1;
}

__device__ __forceinline__ bool llExpired(const LLArgs& a, uint64_t t0) {
  return *a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks;
}

// Bounded spin until *w >= target (peer `peer`'s word); false on timeout/abort.
__device__ __forceinline__ bool llWait(const uint64_t* w, uint64_t target, const LLArgs& a, uint64_t t0, int peer) {
  uint32_t spins = 0;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v >= target) return true;
    if ((++spins & 1023u) == 0u && llExpired(a, t0)) {
      llGiveUp(a, kDiagCredit, peer, target, v, t0);
      return false;
    }
  }
}

__device__ __forceinline__ bool llIsTarget(const LLArgs& a, int j) {
  if (j == a.rank) return false;
  return a.mode != kLLReduce || j == a.root;
}

// This launch's sequence number, parity and credit target (see LLState).
struct LLCall {
  uint64_t seq;
  uint64_t needDone;
  int parity;
  uint32_t flag;
};

// The state words are loaded together (one round trip, not two: the previous
// launch on this stream wrote all of them before it completed).
// Implied credits: if the previous call took lines from every peer, each peer
// had started ITS previous call, so (a communicator's calls run in order on
// every rank) each peer had finished the call before that — the last one that
// used this call's parity — and with it every read of the slots this call
// overwrites. The explicit wait on the done words (needDone != 0) is then
// skipped: one uncached round trip less per call in a run of AllReduce /
// ReduceScatter calls. A Reduce non-root (it takes no lines) keeps the wait.
__device__ __forceinline__ LLCall llBegin(const LLArgs& a) {
  LLCall c;
  const uint64_t s = __hip_atomic_load(&a.state->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t l0 = __hip_atomic_load(&a.state->lastSeq[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t l1 = __hip_atomic_load(&a.state->lastSeq[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t ra = __hip_atomic_load(&a.state->recvAllSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c.seq = s + 1;
  c.parity = (int)(c.seq & 1u);
  c.needDone = (s != 0 && ra == s) ? 0 : (c.parity ? l1 : l0);
  c.flag = (uint32_t)c.seq;
  return c;
}

// Plan word of source `src` for `parity` in the LL buffer at `base`.
__device__ __forceinline__ uint64_t* llPlanWord(uint64_t* const base, const LLArgs& a, int parity, int src) {
  return base + a.planOff + (uint64_t)(parity * a.nRanks + src);
}

// Block 0, thread j: this call's plan into target j's buffer. Stamped BEFORE
// j's credit wait and drained after it: the word is performed at
// j's memory before this thread's unit goes out, at no added latency (the
// credit poll's round trip covers the write). So it can reach j while j still
// runs the call two back on this parity; j's checks take a newer flag as
// "moved on" (llPlanAge), never as a mismatch.
__device__ __forceinline__ void llPlanStamp(const LLArgs& a, const LLCall& c, int j) {
  __hip_atomic_store(llPlanWord(a.peerLL[j], a, c.parity, a.rank), ((uint64_t)c.flag << 32) | a.planSig,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// plan word flag vs this call's: < 0 older (not stamped yet), 0 this call, > 0 newer
__device__ __forceinline__ int32_t llPlanAge(uint64_t h, uint32_t flag) { return (int32_t)((uint32_t)(h >> 32) - flag); }

// Slow path of a wait on peer j's lines: true (and the launch's error recorded)
// if j is at this call with another plan. `w`: j's plan word; nullptr: none.
__device__ __forceinline__ bool llPlanMismatch(const LLArgs& a, const uint64_t* w, uint32_t flag, int j, uint64_t t0,
                                               bool record = true) {
  if (w == nullptr) return false;
  const uint64_t h = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if ((uint32_t)(h >> 32) != flag || (uint32_t)h == a.planSig) return false;
  if (record) diagTimeout(a.errWord, kDiagLLPlan, j, a.planSig, (uint32_t)h, wall_clock64() - t0);
  *a.errWord = 1;
  return true;
}

// Block 0, thread j (a source of this rank), after the fold: peer j's plan
// word for this call (bounded wait; already there in the common case, since j
// performed it before pushing) must carry this rank's signature.
__device__ __forceinline__ bool llPlanCheck(const LLArgs& a, const LLCall& c, int j, uint64_t t0) {
  const uint64_t* w = llPlanWord(a.myLL, a, c.parity, j);
  uint32_t spins = 0;
  for (;;) {
    const uint64_t h = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int32_t age = llPlanAge(h, c.flag);
    if (age > 0) return true;
    if (age == 0) return !llPlanMismatch(a, w, c.flag, j, t0);
    if ((++spins & 1023u) == 0u && llExpired(a, t0)) {
      llGiveUp(a, kDiagLLPlanWord, j, c.flag, (uint32_t)(h >> 32), t0);
      return false;
    }
  }
}

// Every thread of every block, as the launch's last statement: the block's
// memory operations complete, thread 0 arrives (nbx_order.h, per-XCD
// counters), and the launch's last block publishes this rank's done word
// (= seq) in every peer's buffer, advances the state for the next launch and
// publishes the call's completion number (MpDone).
// `receivedAll`: this launch took lines from every peer (llBegin's implied credits).
__device__ __forceinline__ void llEnd(const LLArgs& a, const LLCall& c, bool receivedAll) {
  mpDrain();
  if (threadIdx.x != 0 || !mpLastBlock(a.order.arrive)) return;
  for (int j = 0; j < a.nRanks; j++) {
    if (j == a.rank) continue;
    __hip_atomic_store(a.peerLL[j] + a.doneOff + a.rank, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (receivedAll)   // (after a failed call the communicator is broken until aborted, as in the reference)
    __hip_atomic_store(&a.state->recvAllSeq, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&a.state->lastSeq[c.parity], c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&a.state->seq, c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // write-through (nbx_order.h)
  mpPublish(a.order);
}

// The message that unit k of the launch belongs to (a group launch's segment,
// or the launch's single message) and k's index inside it. The unit is the
// 8-byte pack in kLLColl and the 48-byte line in kLL128Coll (LLSeg.packOff
// counts the launch's units).
struct LLMsg {
  const unsigned char* send;
  unsigned char* recv;
  uint64_t bytes;       // bytes per slot of this message
  uint64_t k;           // pack index inside the message
  uint64_t blockElts;
};

template <class E>
__device__ __forceinline__ LLMsg llMsg(const LLArgs& a, uint64_t k) {
  if (a.nSegs == 0)
    return LLMsg{(const unsigned char*)a.send, (unsigned char*)a.recv, a.count * sizeof(E), k, a.blockElts};
  int s = 0;
  for (int q = 1; q < a.nSegs; q++)
    if (k >= a.seg[q].packOff) s = q;
  const LLSeg& g = a.seg[s];
  return LLMsg{(const unsigned char*)g.send, (unsigned char*)g.recv, g.count * sizeof(E), k - g.packOff, g.blockElts};
}

template <class Fn, bool CHECK>
__global__ __launch_bounds__(256) void kLLColl(LLArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPK = 8 / (int)sizeof(E);   // elements per 8-byte pack
  const Fn fn(llLoadArg<Fn>(a));
  const int n = a.nRanks, me = a.rank;
  const LLCall call = llBegin(a);
  const uint64_t flagHi = (uint64_t)call.flag << 32;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = wall_clock64();
  // this thread's first pack of the caller's input, loaded while the credits
  // are checked (AllReduce / Reduce: one pack for every target)
  const uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool pre = a.mode != kLLReduceScatter && k0 < a.nPacks;
  uint64_t first = 0;
  if (pre) {
    const LLMsg m0 = llMsg<E>(a, k0);
    first = llLoadBytes(m0.send, m0.k * 8, m0.bytes);
  }
  __shared__ int sFailed;
  if (threadIdx.x == 0) sFailed = 0;
  __syncthreads();

  // 0. plan words (checks on: block 0's thread j for target j, performed before
  // the lines go out), credits: each target has finished reading this parity's previous use
  const bool stamps = CHECK && blockIdx.x == 0 && (int)threadIdx.x < n && llIsTarget(a, threadIdx.x);
  if (stamps) llPlanStamp(a, call, threadIdx.x);
  if (call.needDone != 0 && (int)threadIdx.x < n && llIsTarget(a, threadIdx.x)) {
    if (!llWait(a.myLL + a.doneOff + threadIdx.x, call.needDone, a, t0, (int)threadIdx.x)) sFailed = 1;
  }
  if (stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool failed = sFailed != 0;

  // 1. push two {data, flag} lines per pack into each target's slot [parity][me]
  if (!failed) {
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.nPacks; k += stride) {
      const LLMsg m = llMsg<E>(a, k);
      uint64_t whole = 0;
      if (a.mode != kLLReduceScatter) whole = (pre && k == k0) ? first : llLoadBytes(m.send, m.k * 8, m.bytes);
      for (int j = 0; j < n; j++) {
        if (!llIsTarget(a, j)) continue;
        const uint64_t v = a.mode == kLLReduceScatter ? llLoadBytes(m.send + (uint64_t)j * m.bytes, m.k * 8, m.bytes)
                                                      : whole;
        const uint64_t l0 = (v & 0xffffffffull) | flagHi, l1 = (v >> 32) | flagHi;
        uint64_t* line = a.peerLL[j] + ((uint64_t)(call.parity * n + me) * a.slotLines + 2 * k);
        __hip_atomic_store(line, l0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(line + 1, l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }

  // 2.+3. poll own slots, fold in the direct order, store the result
  const bool receives = a.mode != kLLReduce || me == a.root;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; receives && k < a.nPacks; k += stride) {
    union Pk {
      uint64_t u;
      E e[EPK];
    };
    const LLMsg m = llMsg<E>(a, k);
    const unsigned char* own = m.send + (a.mode == kLLReduceScatter ? (uint64_t)me * m.bytes : 0);
    int first;
    if (a.mode == kLLAllReduce) {
      const int c = (int)((m.k * EPK) / m.blockElts);   // packs never straddle 16-B-aligned blocks
      first = (c + 1) % n;
    } else {
      first = ((a.mode == kLLReduce ? a.root : me) + 1) % n;
    }
    Pk acc;
    acc.u = 0;
    for (int q = 0; q < n; q++) {
      const int j = (first + q) % n;
      Pk x;
      if (j == me) {
        x.u = llLoadBytes(own, m.k * 8, m.bytes);
      } else {
        const uint64_t* line = a.myLL + ((uint64_t)(call.parity * n + j) * a.slotLines + 2 * k);
        const uint64_t* pw = CHECK ? llPlanWord(a.myLL, a, call.parity, j) : nullptr;
        uint64_t l0 = 0, l1 = 0;
        uint32_t spins = 0;
        while (!failed) {
          l0 = __hip_atomic_load(line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          l1 = __hip_atomic_load(line + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((uint32_t)(l0 >> 32) == call.flag && (uint32_t)(l1 >> 32) == call.flag) break;
          if ((++spins & 1023u) == 0u) {
            if (llPlanMismatch(a, pw, call.flag, j, t0)) {
              failed = true;
            } else if (llExpired(a, t0)) {
              llGiveUp(a, kDiagLLLine, j, call.flag, (uint32_t)(l0 >> 32), t0);
              failed = true;
            }
          }
        }
        x.u = (l0 & 0xffffffffull) | (l1 << 32);
      }
#pragma unroll
      for (int e = 0; e < EPK; e++) {
        E v = x.e[e];
        if constexpr (Fn::kHasPre) v = fn.pre(v);   // PreMulSum: every contribution pre-multiplied once
        acc.e[e] = q == 0 ? v : fn.red(acc.e[e], v);
      }
    }
    if constexpr (Fn::kHasPost) {
      if (a.postOp) {
#pragma unroll
        for (int e = 0; e < EPK; e++) acc.e[e] = fn.post(acc.e[e]);
      }
    }
    llStoreBytes(m.recv, m.k * 8, m.bytes, acc.u);
  }
  if (CHECK && receives && !failed && blockIdx.x == 0 && (int)threadIdx.x < n && (int)threadIdx.x != me)
    (void)llPlanCheck(a, call, threadIdx.x, t0);

  // done word: after every block of this launch has consumed its lines
  llEnd(a, call, receives);
}


// ---------------------------------------------------------------------------
// LL128 protocol for medium messages (NCCL's LL128 idea, prims_ll128.h:185-291:
// lines of several 16-byte lane chunks moved by ONE wave store instruction and
// polled by ONE wave load instruction, most of each line payload).
// NCCL's 128-byte line carries ONE flag and relies on NVLink delivering a
// 128-byte store whole. gfx950 does not: a 128-byte line tore at its 64-byte
// halves (scripts/ll128_stress.py, profiles/r1/ll128_stress_128B.jsonl), and
// nothing guarantees that a 64-byte line crossing xGMI arrives whole either.
// So here EVERY 16-byte lane chunk carries its own 32-bit flag (= seq) in
// dword 3 — the LL idea ({data, flag} per store, prims_ll.h:226-294) at
// 16-byte granularity: a reader accepts a line only when all four chunks show
// the flag, so a line torn at any 16-byte boundary is waited on, never folded
// (tests/test_multiprocess_gpu.py::test_ll128_torn_line_is_waited_on). The
// remaining assumption is that one 16-byte aligned buffer_store_dwordx4 lands
// whole.
// Line: 64 bytes = 4 lanes x {12 payload bytes, flag}; 48 payload bytes as two
// pairs of lanes, each pair 24 bytes = 8-byte words W0, W1, W2:
//   lane A (even) {W0.lo, W0.hi, W1.lo, flag}   lane B (odd) {W2.lo, W2.hi, W1.hi, flag}
// so every 8-byte word is folded whole by one lane (A: W0 and W1, taking
// W1.hi from B by a lane shuffle; B: W2) in its own direct-schedule order.
// Writer: buffer_store_dwordx4 sc0 sc1 (system scope); reader:
// buffer_load_dwordx4 sc0 sc1 (volatile) and a wave ballot per 4-lane line.
// Payload efficiency 75 % (LL: 50 %). Buffers, parities, done words and
// credits are the LL protocol's (above). Restricted to n <= 8 ranks (one
// node): a lane keeps the chunk of every source in registers.
constexpr int kL128Lanes = 4;                 // lanes per line
constexpr int kL128LineBytes = 64;
constexpr int kL128DataBytes = 48;
constexpr int kL128PairBytes = 24;            // payload of a lane pair: words W0, W1, W2
constexpr int kL128MaxRanks = kL128MaxRanksHost;
constexpr int kL128LoadAux = 1 | 16 | (int)(1u << 31);   // sc0 sc1 (system scope), volatile
static_assert(kL128LineBytes == kL128LineBytesHost && kL128DataBytes == kL128DataBytesHost &&
                  kL128Lanes == kL128LanesHost, "host/device layout");

// One 16-byte chunk of a line into a peer's LL128 buffer (`base`, uniform;
// `word`: 8-byte word index of the chunk) by ONE buffer_store_dwordx4 sc0 sc1
// (system scope, write-through). A buffer store rather than inline asm: the
// compiler's hazard recognizer cannot see an asm dwordx4 store, so a VALU write
// to its data registers right behind it could change what is stored.
typedef unsigned int l128V4U __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void l128StoreLine16(uint64_t* base, uint32_t bytes, uint64_t word, u32x4 v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(l128V4U, v), rs, (int)(word * 8u), 0, 1 | 16);
}

// byte offset (in the message) of lane t's pair in line i, and of its first whole word
__device__ __forceinline__ uint64_t l128PairOff(uint64_t i, int t) {
  return i * kL128DataBytes + (uint64_t)(t >> 1) * kL128PairBytes;
}
__device__ __forceinline__ uint64_t l128WordOff(uint64_t i, int t) { return l128PairOff(i, t) + ((t & 1) ? 16u : 0u); }

// lane t's chunk of line i of `src` (bytes long) from its words, flag in dword 3
__device__ __forceinline__ u32x4 l128Chunk(const unsigned char* src, uint64_t bytes, uint64_t i, int t,
                                           uint32_t flag) {
  const uint64_t w = llLoadBytes(src, l128WordOff(i, t), bytes);
  const uint64_t w1 = llLoadBytes(src, l128PairOff(i, t) + 8, bytes);
  return (u32x4){(uint32_t)w, (uint32_t)(w >> 32), (t & 1) ? (uint32_t)(w1 >> 32) : (uint32_t)w1, flag};
}

// every lane of this lane's 4-lane line group sees `ok` (lanes of a group are
// always active together, so their ballot bits are current)
__device__ __forceinline__ bool l128LineReady(bool ok) {
  const uint64_t b = __ballot((int)ok);
  const uint64_t gm = 0xFull << ((threadIdx.x & 63u) & ~3u);
  return (b & gm) == gm;
}

// the other lane of the pair's dword (every lane of the group participates)
__device__ __forceinline__ uint32_t l128Partner(uint32_t x) { return (uint32_t)__shfl_xor((int)x, 1, kL128Lanes); }

// word k of source j's chunk for a runtime j < 8 (select chain, no scratch):
// k = 0 the lane's whole word (x, y); k = 1 (lane A only) W1 = (z, pz = B's z)
__device__ __forceinline__ uint64_t l128Pick(const u32x4 (&v)[kL128MaxRanks], const uint32_t (&pz)[kL128MaxRanks],
                                             int j, int k) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int q = 0; q < kL128MaxRanks; q++) {
    const bool m = q == j;
    lo = m ? (k ? v[q].z : v[q].x) : lo;
    hi = m ? (k ? pz[q] : v[q].y) : hi;
  }
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t l128FlagOf(const u32x4 (&v)[kL128MaxRanks], int j) {
  uint32_t f = 0;
#pragma unroll
  for (int q = 0; q < kL128MaxRanks; q++) f = q == j ? v[q].w : f;
  return f;
}

// Poll the chunks of the sources in `need` (slot byte offset slotOff(q)) until
// every chunk of the line shows `flag`; false if the wait gave up, or if the
// source's plan word (`plan` + q, or `plan` itself for a fixed `planPeer` >= 0;
// nullptr: none) shows this call with another plan.
template <class SlotOff>
__device__ __forceinline__ bool l128Poll(const LLArgs& a, __amdgpu_buffer_rsrc_t rs, u32x4 (&v)[kL128MaxRanks],
                                         uint32_t need, uint32_t flag, uint64_t site, uint64_t t0, int t,
                                         SlotOff slotOff, const uint64_t* plan, int planPeer) {
  uint32_t spins = 0;
  while (need != 0) {
#pragma unroll
    for (int q = 0; q < kL128MaxRanks; q++)
      if ((need >> q) & 1u)
        v[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, slotOff(q) + (uint32_t)t * 16u, 0,
                                                                               kL128LoadAux));
#pragma unroll
    for (int q = 0; q < kL128MaxRanks; q++)
      if (((need >> q) & 1u) && l128LineReady(v[q].w == flag)) need &= ~(1u << q);
    if (need != 0 && (++spins & 1023u) == 0u) {
      const int q = __builtin_ctz(need);
      const int peer = planPeer >= 0 ? planPeer : q;
      if (plan != nullptr && llPlanMismatch(a, planPeer >= 0 ? plan : plan + q, flag, peer, t0, t == 0)) return false;
      if (llExpired(a, t0)) {
        llGiveUp(a, site, peer, flag, l128FlagOf(v, q), t0, t == 0);
        return false;
      }
    }
  }
  return true;
}

// Fold lane t's words of line i over the n sources in v (own contribution
// included) in the direct schedule's order, apply postOp, and hand each word
// to `sink(k, byteOffset, word)`: lane A words k = 0 (W0), 1 (W1); lane B k = 0 (W2).
template <class Fn, class Sink>
__device__ __forceinline__ void l128FoldLine(const Fn& fn, const LLArgs& a, const u32x4 (&v)[kL128MaxRanks], uint64_t i,
                                             int t, int fixedFirst, uint64_t blockElts, Sink sink) {
  using E = typename Fn::Elt;
  constexpr int EPK = 8 / (int)sizeof(E);
  const int n = a.nRanks;
  uint32_t pz[kL128MaxRanks];
#pragma unroll
  for (int q = 0; q < kL128MaxRanks; q++) pz[q] = l128Partner(v[q].z);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (k == 1 && (t & 1)) break;   // lane B owns one word
    const uint64_t off = k ? l128PairOff(i, t) + 8 : l128WordOff(i, t);
    int first = fixedFirst;
    if (first < 0) {   // AllReduce: the word's block c folds c+1, ..., c (8-byte words never straddle blocks)
      const int c = (int)((off / sizeof(E)) / blockElts);
      first = (c + 1) % n;
    }
    union Pk {
      uint64_t u;
      E e[EPK];
    };
    Pk acc;
    acc.u = 0;
    for (int q = 0; q < n; q++) {
      const int j = first + q < n ? first + q : first + q - n;
      Pk x;
      x.u = l128Pick(v, pz, j, k);
#pragma unroll
      for (int e = 0; e < EPK; e++) {
        E y = x.e[e];
        if constexpr (Fn::kHasPre) y = fn.pre(y);   // PreMulSum: every contribution pre-multiplied once
        acc.e[e] = q == 0 ? y : fn.red(acc.e[e], y);
      }
    }
    if constexpr (Fn::kHasPost) {
      if (a.postOp) {
#pragma unroll
        for (int e = 0; e < EPK; e++) acc.e[e] = fn.post(acc.e[e]);
      }
    }
    sink(k, off, acc.u);
  }
}

template <class Fn, bool CHECK>
__global__ __launch_bounds__(256) void kLL128Coll(LLArgs a) {
  using E = typename Fn::Elt;
  const Fn fn(llLoadArg<Fn>(a));
  const int n = a.nRanks, me = a.rank;
  const int t = (int)(threadIdx.x % kL128Lanes);   // lane within the line's group
  const uint64_t groups = ((uint64_t)gridDim.x * blockDim.x) / kL128Lanes;
  const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kL128Lanes;
  const uint64_t t0 = wall_clock64();
  const LLCall call = llBegin(a);
  // this lane's chunk of its first line, loaded while the credits are checked
  const bool pre = a.mode != kLLReduceScatter && g0 < a.nLines;
  u32x4 first = {0, 0, 0, 0};
  if (pre) {
    const LLMsg m0 = llMsg<E>(a, g0);
    first = l128Chunk(m0.send, m0.bytes, m0.k, t, call.flag);
  }
  __shared__ int sFailed;
  if (threadIdx.x == 0) sFailed = 0;
  __syncthreads();

  // 0. plan words, credits (as kLLColl)
  const bool stamps = CHECK && blockIdx.x == 0 && (int)threadIdx.x < n && llIsTarget(a, threadIdx.x);
  if (stamps) llPlanStamp(a, call, threadIdx.x);
  if (call.needDone != 0 && (int)threadIdx.x < n && llIsTarget(a, threadIdx.x)) {
    if (!llWait(a.myLL + a.doneOff + threadIdx.x, call.needDone, a, t0, (int)threadIdx.x)) sFailed = 1;
  }
  if (stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool failed = sFailed != 0;

  // 1. push: line i of the launch (line m.k of its message) into slot [parity][me] of every target
  if (!failed) {
    for (uint64_t i = g0; i < a.nLines; i += groups) {
      const LLMsg m = llMsg<E>(a, i);
      u32x4 whole = {0, 0, 0, 0};
      if (a.mode != kLLReduceScatter) whole = (pre && i == g0) ? first : l128Chunk(m.send, m.bytes, m.k, t, call.flag);
      for (int j = 0; j < n; j++) {
        if (!llIsTarget(a, j)) continue;
        const u32x4 v = a.mode == kLLReduceScatter ? l128Chunk(m.send + (uint64_t)j * m.bytes, m.bytes, m.k, t, call.flag)
                                                   : whole;
        l128StoreLine16(a.peerL128[j], a.l128Bytes,
                        ((uint64_t)(call.parity * n + me) * a.l128SlotLines + i) * (kL128LineBytes / 8) + 2 * t, v);
      }
    }
  }

  // 2.+3. poll own slots (every source's chunk of line i in registers), fold, store
  const bool receives = a.mode != kLLReduce || me == a.root;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.myL128, (short)0, (int)a.l128Bytes,
                                                                      0x00020000);
  const int fixedFirst = a.mode == kLLAllReduce ? -1 : ((a.mode == kLLReduce ? a.root : me) + 1) % n;
  const uint64_t* const plan = CHECK ? llPlanWord(a.myLL, a, call.parity, 0) : nullptr;
  for (uint64_t i = g0; receives && !failed && i < a.nLines; i += groups) {
    const LLMsg m = llMsg<E>(a, i);
    const unsigned char* own = m.send + (a.mode == kLLReduceScatter ? (uint64_t)me * m.bytes : 0);
    u32x4 v[kL128MaxRanks];
    uint32_t need = 0;
#pragma unroll
    for (int q = 0; q < kL128MaxRanks; q++) {
      v[q] = (u32x4){0, 0, 0, 0};
      if (q < n) {
        if (q == me) v[q] = l128Chunk(own, m.bytes, m.k, t, 0);
        else need |= 1u << q;
      }
    }
    failed = !l128Poll(
        a, rs, v, need, call.flag, kDiagLL128Line, t0, t,
        [&](int q) { return (uint32_t)((((uint64_t)(call.parity * n + q)) * a.l128SlotLines + i) * kL128LineBytes); },
        plan, -1);
    l128FoldLine(fn, a, v, m.k, t, fixedFirst, m.blockElts, [&](int, uint64_t off, uint64_t w) {
      llStoreBytes(m.recv, off, m.bytes, w);
    });
  }
  if (CHECK && receives && !failed && blockIdx.x == 0 && (int)threadIdx.x < n && (int)threadIdx.x != me)
    (void)llPlanCheck(a, call, threadIdx.x, t0);

  // done word (as kLLColl)
  llEnd(a, call, receives);
}


// ---------------------------------------------------------------------------
// LL128 two-shot AllReduce / Reduce (medium messages, n <= 8 ranks): the
// one-shot kernel above sends the whole message to every target ((n-1) x M per
// rank for AllReduce, (n-1) x M into the root for Reduce); this one moves
// 2 (n-1)/n x M per rank (AllReduce; Reduce: (n-1)/n x M into the root), in one
// kernel and two hops:
//   A. push block j of `send` (the direct schedule's 16-byte-aligned blocks)
//      into peer j's reduce-scatter sub-slot [parity][RS][me];
//   B. for this rank's block: poll the n-1 RS sub-slots, fold with the own
//      contribution in the direct order (AllReduce me+1, ..., me; Reduce
//      root+1, ..., root — bitwise the direct path's result), then AllReduce:
//      store it to `recv` and push the folded lines into every peer's
//      all-gather sub-slot [parity][AG][me]; Reduce: the root stores it, the
//      others push it into the root's sub-slot only;
//   C. (AllReduce: every rank; Reduce: the root) for every other block j:
//      poll AG sub-slot [parity][AG][j], copy the payload into `recv`.
// The LL128 buffer's per-parity region (n slots of l128SlotLines lines) is
// split into 2n sub-slots of subSlotLines lines ([RS][source], [AG][source]).
// Credits, sequencing and done words are the LL family's (llBegin / llEnd).
__device__ __forceinline__ void l128BlockRange(const LLArgs& a, int j, int eb, uint64_t* offBytes,
                                               uint64_t* lenBytes) {
  uint64_t lo = a.blockElts * (uint64_t)j, hi = lo + a.blockElts;
  if (lo > a.count) lo = a.count;
  if (hi > a.count) hi = a.count;
  *offBytes = lo * (uint64_t)eb;
  *lenBytes = (hi - lo) * (uint64_t)eb;
}

template <class Fn, bool CHECK>
__global__ __launch_bounds__(256) void kLL128AllReduce2(LLArgs a) {
  using E = typename Fn::Elt;
  constexpr int eb = (int)sizeof(E);
  const Fn fn(llLoadArg<Fn>(a));
  const int n = a.nRanks, me = a.rank;
  const int t = (int)(threadIdx.x % kL128Lanes);
  const uint64_t groups = ((uint64_t)gridDim.x * blockDim.x) / kL128Lanes;
  const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / kL128Lanes;
  const uint64_t t0 = wall_clock64();
  const LLCall call = llBegin(a);
  const uint64_t S = a.nLines;   // sub-slot lines (nLines carries subSlotLines here)
  auto subSlot = [&](int region, int src) { return (uint64_t)((call.parity * 2 + region) * n + src) * S; };
  __shared__ int sFailed;
  if (threadIdx.x == 0) sFailed = 0;
  __syncthreads();
  // plan words, credits (as kLLColl)
  const bool stamps = CHECK && blockIdx.x == 0 && (int)threadIdx.x < n && (int)threadIdx.x != me;
  if (stamps) llPlanStamp(a, call, threadIdx.x);
  if (call.needDone != 0 && (int)threadIdx.x < n && (int)threadIdx.x != me) {
    if (!llWait(a.myLL + a.doneOff + threadIdx.x, call.needDone, a, t0, (int)threadIdx.x)) sFailed = 1;
  }
  if (stamps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bool failed = sFailed != 0;
  const uint64_t* const plan = CHECK ? llPlanWord(a.myLL, a, call.parity, 0) : nullptr;
  const unsigned char* send = (const unsigned char*)a.send;
  unsigned char* recv = (unsigned char*)a.recv;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.myL128, (short)0, (int)a.l128Bytes,
                                                                      0x00020000);
  // A. reduce-scatter pushes
  for (int j = 0; j < n && !failed; j++) {
    if (j == me) continue;
    uint64_t off, len;
    l128BlockRange(a, j, eb, &off, &len);
    const uint64_t lines = (len + kL128DataBytes - 1) / kL128DataBytes;
    for (uint64_t i = g0; i < lines; i += groups) {
      const u32x4 v = l128Chunk(send + off, len, i, t, call.flag);
      l128StoreLine16(a.peerL128[j], a.l128Bytes, (subSlot(0, me) + i) * (kL128LineBytes / 8) + 2 * t, v);
    }
  }
  // B. own block: fold, store, all-gather pushes
  {
    uint64_t off, len;
    l128BlockRange(a, me, eb, &off, &len);
    const uint64_t lines = (len + kL128DataBytes - 1) / kL128DataBytes;
    const bool reduce = a.mode == kLLReduce;
    const int first = ((reduce ? a.root : me) + 1) % n;
    for (uint64_t i = g0; i < lines && !failed; i += groups) {
      u32x4 v[kL128MaxRanks];
      uint32_t need = 0;
#pragma unroll
      for (int q = 0; q < kL128MaxRanks; q++) {
        v[q] = (u32x4){0, 0, 0, 0};
        if (q < n) {
          if (q == me) v[q] = l128Chunk(send + off, len, i, t, 0);
          else need |= 1u << q;
        }
      }
      failed = !l128Poll(a, rs, v, need, call.flag, kDiagLL128RS, t0, t,
                         [&](int q) { return (uint32_t)((subSlot(0, q) + i) * kL128LineBytes); }, plan, -1);
      uint64_t w[2] = {0, 0};
      l128FoldLine(fn, a, v, i, t, first, a.blockElts, [&](int k, uint64_t o, uint64_t r) {
        w[k] = r;
        if (!reduce || me == a.root) llStoreBytes(recv + off, o, len, r);
      });
      // the folded line in the chunk layout: lane B takes W1.hi from lane A
      const uint32_t w1hi = l128Partner((uint32_t)(w[1] >> 32));
      const u32x4 line = {(uint32_t)w[0], (uint32_t)(w[0] >> 32), (t & 1) ? w1hi : (uint32_t)w[1], call.flag};
      for (int j = 0; j < n; j++) {
        if (j == me || failed || (reduce && j != a.root)) continue;
        l128StoreLine16(a.peerL128[j], a.l128Bytes, (subSlot(1, me) + i) * (kL128LineBytes / 8) + 2 * t, line);
      }
    }
  }
  // C. the other blocks arrive folded: copy them into recv
  for (int j = 0; j < n && !failed && (a.mode != kLLReduce || me == a.root); j++) {
    if (j == me) continue;
    uint64_t off, len;
    l128BlockRange(a, j, eb, &off, &len);
    const uint64_t lines = (len + kL128DataBytes - 1) / kL128DataBytes;
    for (uint64_t i = g0; i < lines && !failed; i += groups) {
      u32x4 v[kL128MaxRanks];
#pragma unroll
      for (int q = 0; q < kL128MaxRanks; q++) v[q] = (u32x4){0, 0, 0, 0};
      failed = !l128Poll(a, rs, v, 1u, call.flag, kDiagLL128AG, t0, t,
                         [&](int) { return (uint32_t)((subSlot(1, j) + i) * kL128LineBytes); }, plan ? plan + j : nullptr, j);
      const uint32_t pz = l128Partner(v[0].z);
      llStoreBytes(recv + off, l128WordOff(i, t), len, ((uint64_t)v[0].y << 32) | v[0].x);
      if (!(t & 1)) llStoreBytes(recv + off, l128PairOff(i, t) + 8, len, ((uint64_t)pz << 32) | v[0].z);
    }
  }
  // every peer pushed its reduce-scatter lines here (both modes)
  if (CHECK && !failed && blockIdx.x == 0 && (int)threadIdx.x < n && (int)threadIdx.x != me)
    (void)llPlanCheck(a, call, threadIdx.x, t0);
  uint64_t myOff, myLen;   // every peer pushes lines of a non-empty own block here
  l128BlockRange(a, me, eb, &myOff, &myLen);
  llEnd(a, call, myLen > 0);
}

}  // namespace nbx
