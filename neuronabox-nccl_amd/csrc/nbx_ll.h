// nbx_ll.h — LL ("low latency") protocol AllReduce for small messages on the
// multi-process communicator: one kernel, no host exchange per call.
//
// Wire format (the idea of NCCL's LL protocol, prims_ll.h:226-294 /
// device.h ncclLLFifoLine): every 8-byte line is {u32 data, u32 flag} written
// by ONE 64-bit system-scope store, so a reader that sees flag == seq also
// sees that line's data (single-copy atomicity; no separate flag, no fence).
// Each rank owns an IPC-registered LL buffer laid out
//   [parity 2][source rank n][lines 2 * maxPacks]   (8-byte lines)
// and the kernel of rank r
//   1. pushes its message, 8 bytes per thread, as two lines into slot
//      [seq & 1][r] of every peer's buffer (remote stores over xGMI);
//   2. polls its own buffer's slots [seq & 1][j] for every peer j until the
//      flags equal seq (bounded spin: timeout + abort word), reads its own
//      contribution from `send`, and folds all n sources per element in the
//      direct schedule's order (element in block c: ranks c+1, ..., c), so the
//      result is bitwise the direct path's;
//   3. stores the full result to `recv` — every rank computes the whole
//      message, so there is no gather phase.
// Parity buffers + stream order make reuse safe: a rank writes parity p again
// only at seq+2, after it has seen every peer's seq+1 lines (LL) or passed the
// seq+1 done-barrier (direct), i.e. after every peer finished reading seq.
#pragma once
#include "nbx_functors.h"
#include "nbx_ll_args.h"

namespace nbx {



template <class Fn>
__device__ __forceinline__ uint64_t llLoadArg(const LLArgs& a) {
  if (a.argPtr != nullptr) return (uint64_t) * (const typename Fn::Elt*)a.argPtr;
  return a.arg;
}

// 8 bytes of `p` starting at byte `off`, zero past `limit`
__device__ __forceinline__ uint64_t llLoadBytes(const unsigned char* p, uint64_t off, uint64_t limit) {
  if (off + 8 <= limit) return *(const uint64_t*)(p + off);
  uint64_t v = 0;
  for (int b = 0; b < 8; b++)
    if (off + b < limit) v |= (uint64_t)p[off + b] << (8 * b);
  return v;
}

template <class Fn>
__global__ __launch_bounds__(256) void kLLAllReduce(LLArgs a) {
  using E = typename Fn::Elt;
  constexpr int EPK = 8 / (int)sizeof(E);   // elements per 8-byte pack
  const Fn fn(llLoadArg<Fn>(a));
  const int n = a.nRanks, me = a.rank;
  const uint64_t bytes = a.count * sizeof(E);
  const uint64_t flagHi = (uint64_t)a.flag << 32;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = wall_clock64();
  bool failed = false;

  // 1. push: two {data, flag} lines per pack into every peer's slot [parity][me]
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.nPacks; k += stride) {
    const uint64_t v = llLoadBytes((const unsigned char*)a.send, k * 8, bytes);
    const uint64_t l0 = (v & 0xffffffffull) | flagHi, l1 = (v >> 32) | flagHi;
    for (int j = 0; j < n; j++) {
      if (j == me) continue;
      uint64_t* line = a.peerLL[j] + ((uint64_t)(a.parity * n + me) * a.slotLines + 2 * k);
      __hip_atomic_store(line, l0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(line + 1, l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }

  // 2.+3. poll own slots, fold in the direct order, store the result
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < a.nPacks; k += stride) {
    union Pk {
      uint64_t u;
      E e[EPK];
    };
    const uint64_t firstElt = k * EPK;
    const int c = (int)(firstElt / a.blockElts);       // packs never straddle 16-B-aligned blocks
    const int first = (c + 1) % n;
    Pk acc;
    acc.u = 0;
    for (int q = 0; q < n; q++) {
      const int j = (first + q) % n;
      Pk x;
      if (j == me) {
        x.u = llLoadBytes((const unsigned char*)a.send, k * 8, bytes);
      } else {
        const uint64_t* line = a.myLL + ((uint64_t)(a.parity * n + j) * a.slotLines + 2 * k);
        uint64_t l0, l1;
        uint32_t spins = 0;
        for (;;) {
          l0 = __hip_atomic_load(line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          l1 = __hip_atomic_load(line + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if ((uint32_t)(l0 >> 32) == a.flag && (uint32_t)(l1 >> 32) == a.flag) break;
          if (failed) break;
          if ((++spins & 1023u) == 0u) {
            if (*a.abortWord != 0 || wall_clock64() - t0 > a.timeoutTicks) {
              *a.errWord = *a.abortWord != 0 ? 2 : 1;
              failed = true;
              break;
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
    unsigned char* out = (unsigned char*)a.recv;
    if (k * 8 + 8 <= bytes) {
      *(uint64_t*)(out + k * 8) = acc.u;
    } else {
      for (int b = 0; b < 8; b++)
        if (k * 8 + b < bytes) out[k * 8 + b] = (unsigned char)(acc.u >> (8 * b));
    }
  }
}

}  // namespace nbx
