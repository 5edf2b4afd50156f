// sweep_shift.hip — experiment for the realigning kernel (kReduceShifted),
// not part of the product: sources whose alignment mod 16 differs from the
// destination's. fp32 sum, NSRC x 64 MiB -> 64 MiB, destination one element
// past a 16-B boundary (so every source is read 12 B off its packs).
//
// Variants:
//   temporal Ux  : lane loads packs q and q+1 of each source (plain loads;
//                  q+1 is the next lane's q, served by L2) — the production
//                  shape at U = 1, here also unrolled to U packs per lane;
//   dpp Ux       : lane loads pack q only (nontemporal) and takes q+1 from
//                  the next lane with a DPP wave shift (VALU, no LDS); lane 63
//                  and the lane holding the last pack load q+1 themselves.
// Outputs are checked bit-exact against the first variant.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/sweep_shift.hip -o scripts/sweep_shift
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Args {
  const u32x4* base[8];   // 16-B aligned-down source bases
  uint32_t sh[8];         // byte offset of each source inside its first pack
  u32x4* dst;
  uint64_t nPacks;
};

__device__ __forceinline__ u32x4 funnel16(const u32x4& lo, const u32x4& hi, uint32_t m) {
  const uint32_t b = m & 3u;
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 r;
  switch (m >> 2) {
    case 0:
      r = u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], b), __builtin_amdgcn_alignbyte(w[2], w[1], b),
                __builtin_amdgcn_alignbyte(w[3], w[2], b), __builtin_amdgcn_alignbyte(w[4], w[3], b)};
      break;
    case 1:
      r = u32x4{__builtin_amdgcn_alignbyte(w[2], w[1], b), __builtin_amdgcn_alignbyte(w[3], w[2], b),
                __builtin_amdgcn_alignbyte(w[4], w[3], b), __builtin_amdgcn_alignbyte(w[5], w[4], b)};
      break;
    case 2:
      r = u32x4{__builtin_amdgcn_alignbyte(w[3], w[2], b), __builtin_amdgcn_alignbyte(w[4], w[3], b),
                __builtin_amdgcn_alignbyte(w[5], w[4], b), __builtin_amdgcn_alignbyte(w[6], w[5], b)};
      break;
    default:
      r = u32x4{__builtin_amdgcn_alignbyte(w[4], w[3], b), __builtin_amdgcn_alignbyte(w[5], w[4], b),
                __builtin_amdgcn_alignbyte(w[6], w[5], b), __builtin_amdgcn_alignbyte(w[7], w[6], b)};
      break;
  }
  return r;
}

__device__ __forceinline__ u32x4 add4(u32x4 a, u32x4 b) {
  f32x4 x = __builtin_bit_cast(f32x4, a), y = __builtin_bit_cast(f32x4, b);
  return __builtin_bit_cast(u32x4, x + y);
}

// wave_shl:1 (DPP control 0x130): lane i receives lane i+1's value
__device__ __forceinline__ u32x4 fromNextLane(const u32x4& v) {
  return u32x4{(uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x130, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x130, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x130, 0xf, 0xf, false),
               (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x130, 0xf, 0xf, false)};
}

template <int NSRC, int U, bool DPP>
__global__ __launch_bounds__(256) void kshift(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t p0 = blockIdx.x * tile + threadIdx.x; p0 - threadIdx.x < n; p0 += stride) {
    u32x4 lo[NSRC][U], hi[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t q = p0 + (uint64_t)u * 256;
        if (q >= n) q = n - 1;   // clamp: every lane stays active for the shift
        if constexpr (DPP) {
          lo[s][u] = __builtin_nontemporal_load(a.base[s] + q);
        } else {
          lo[s][u] = a.base[s][q];
          hi[s][u] = a.base[s][q + 1];
        }
      }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DPP) {
#pragma unroll
      for (int s = 0; s < NSRC; s++)
#pragma unroll
        for (int u = 0; u < U; u++) hi[s][u] = fromNextLane(lo[s][u]);
#pragma unroll
      for (int s = 0; s < NSRC; s++)
#pragma unroll
        for (int u = 0; u < U; u++) {
          uint64_t q = p0 + (uint64_t)u * 256;
          if (q >= n) q = n - 1;
          if (lane == 63u || q + 1 >= n) hi[s][u] = a.base[s][q + 1];
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = p0 + (uint64_t)u * 256;
      u32x4 acc = funnel16(lo[0][u], hi[0][u], a.sh[0]);
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = add4(acc, funnel16(lo[s][u], hi[s][u], a.sh[s]));
      if (q < n) a.dst[q] = acc;
    }
  }
}

// two loads per lane, q nontemporal and q+1 temporal (the next lane's q is
// then read nontemporally by that lane while this lane's copy hits L2)
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kshiftMix(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p0 = blockIdx.x * tile + threadIdx.x; p0 - threadIdx.x < n; p0 += stride) {
    u32x4 lo[NSRC][U], hi[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t q = p0 + (uint64_t)u * 256;
        if (q >= n) q = n - 1;
        lo[s][u] = __builtin_nontemporal_load(a.base[s] + q);
        hi[s][u] = a.base[s][q + 1];
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = p0 + (uint64_t)u * 256;
      u32x4 acc = funnel16(lo[0][u], hi[0][u], a.sh[0]);
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = add4(acc, funnel16(lo[s][u], hi[s][u], a.sh[s]));
      if (q < n) a.dst[q] = acc;
    }
  }
}

// dpp, with the own loads of lane 63 / the last pack issued in the load
// phase (no extra memory round trip after the shift)
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kshiftPre(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t p0 = blockIdx.x * tile + threadIdx.x; p0 - threadIdx.x < n; p0 += stride) {
    u32x4 lo[NSRC][U], own[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t q = p0 + (uint64_t)u * 256;
        if (q >= n) q = n - 1;
        lo[s][u] = __builtin_nontemporal_load(a.base[s] + q);
        if (lane == 63u || q + 1 >= n) own[s][u] = a.base[s][q + 1];
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t q = p0 + (uint64_t)u * 256;
      const bool mine = lane == 63u || (q >= n ? n - 1 : q) + 1 >= n;
      u32x4 h = fromNextLane(lo[0][u]);
      u32x4 acc = funnel16(lo[0][u], mine ? own[0][u] : h, a.sh[0]);
#pragma unroll
      for (int s = 1; s < NSRC; s++) {
        h = fromNextLane(lo[s][u]);
        acc = add4(acc, funnel16(lo[s][u], mine ? own[s][u] : h, a.sh[s]));
      }
      if (q < n) a.dst[q] = acc;
    }
  }
}

// dpp-pre with the source count a run-time value and arrays sized for 8
// sources (the library's kReduceShiftedDpp shape)
template <int U>
__global__ __launch_bounds__(256) void kshiftPreRt(Args a, int nSrcs) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t p0 = blockIdx.x * tile + threadIdx.x; p0 - threadIdx.x < n; p0 += stride) {
    u32x4 lo[8][U], own[8][U];
#pragma unroll
    for (int s = 0; s < 8; s++)
      if (s < nSrcs) {
#pragma unroll
        for (int u = 0; u < U; u++) {
          uint64_t q = p0 + (uint64_t)u * 256;
          if (q >= n) q = n - 1;
          lo[s][u] = __builtin_nontemporal_load(a.base[s] + q);
          if (lane == 63u || q + 1 >= n) own[s][u] = a.base[s][q + 1];
        }
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t q = p0 + (uint64_t)u * 256;
      const bool mine = lane == 63u || (q >= n ? n - 1 : q) + 1 >= n;
      u32x4 h = fromNextLane(lo[0][u]);
      u32x4 acc = funnel16(lo[0][u], mine ? own[0][u] : h, a.sh[0]);
#pragma unroll
      for (int s = 1; s < 8; s++)
        if (s < nSrcs) {
          h = fromNextLane(lo[s][u]);
          acc = add4(acc, funnel16(lo[s][u], mine ? own[s][u] : h, a.sh[s]));
        }
      if (q < n) a.dst[q] = acc;
    }
  }
}

// 63 output packs per wave: lane 63 only loads (the pack lane 62 needs), so
// every lane's q+1 comes from the next lane by DPP and nothing is loaded
// twice inside a wave; loads clamp at the last pack the source range touches
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kshift63(Args a) {
  const uint64_t n = a.nPacks, span = (uint64_t)U * 63;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t waves = (uint64_t)gridDim.x * 4, wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint64_t lim[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; s++) lim[s] = a.sh[s] ? n : n - 1;
  for (uint64_t w0 = wave * span; w0 < n; w0 += waves * span) {
    u32x4 lo[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = w0 + (uint64_t)u * 63 + lane;
        lo[s][u] = __builtin_nontemporal_load(a.base[s] + (q < lim[s] ? q : lim[s]));
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = w0 + (uint64_t)u * 63 + lane;
      u32x4 acc = funnel16(lo[0][u], fromNextLane(lo[0][u]), a.sh[0]);
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = add4(acc, funnel16(lo[s][u], fromNextLane(lo[s][u]), a.sh[s]));
      if (lane < 63u && q < n) a.dst[q] = acc;
    }
  }
}

// reference point: the same fold with every source aligned to the
// destination (pack q of each source, no shift) — the aligned kernel's rate
// at this size, same process, same buffers
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kaligned(Args a) {
  const uint64_t n = a.nPacks, tile = (uint64_t)U * 256, stride = (uint64_t)gridDim.x * tile;
  for (uint64_t p0 = blockIdx.x * tile + threadIdx.x; p0 < n; p0 += stride) {
    u32x4 v[NSRC][U];
#pragma unroll
    for (int s = 0; s < NSRC; s++)
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t q = p0 + (uint64_t)u * 256;
        v[s][u] = __builtin_nontemporal_load(a.base[s] + (q < n ? q : n - 1));
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = p0 + (uint64_t)u * 256;
      u32x4 acc = v[0][u];
#pragma unroll
      for (int s = 1; s < NSRC; s++) acc = add4(acc, v[s][u]);
      if (q < n) a.dst[q] = acc;
    }
  }
}

// LDS-staged: a workgroup's tile of U*256 output packs needs source packs
// [p0, p0 + U*256] of every source; they are loaded aligned (nontemporal, the
// workgroup's extra last pack by thread 0) and written to LDS, and each lane
// reads its 16 output bytes back at byte offset 16 (q - p0) + sh as five
// dwords + one byte funnel shift. Every pack is loaded once and no lane
// exchange is needed; the cost is LDS traffic and two barriers per tile.
template <int NSRC, int U>
__global__ __launch_bounds__(256) void kshiftLds(Args a) {
  constexpr int T = U * 256;
  __shared__ u32x4 sm[NSRC][T + 1];
  const uint64_t n = a.nPacks, stride = (uint64_t)gridDim.x * T;
  const int tid = (int)threadIdx.x;
  for (uint64_t b0 = (uint64_t)blockIdx.x * T; b0 < n; b0 += stride) {
    u32x4 v[NSRC][U], ex[NSRC];
#pragma unroll
    for (int s = 0; s < NSRC; s++) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = b0 + (uint64_t)u * 256 + tid;
        v[s][u] = __builtin_nontemporal_load(a.base[s] + (q < n ? q : n));   // pack n holds the range's last bytes
      }
      if (tid == 0) ex[s] = a.base[s][b0 + T < n ? b0 + T : n];
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();   // the previous tile's LDS reads are done
#pragma unroll
    for (int s = 0; s < NSRC; s++) {
#pragma unroll
      for (int u = 0; u < U; u++) sm[s][u * 256 + tid] = v[s][u];
      if (tid == 0) sm[s][T] = ex[s];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = b0 + (uint64_t)u * 256 + tid;
      u32x4 acc;
#pragma unroll
      for (int s = 0; s < NSRC; s++) {
        const uint32_t o = (uint32_t)(u * 256 + tid) * 16u + a.sh[s];
        const uint32_t* w = (const uint32_t*)&sm[s][0] + (o >> 2);
        const uint32_t b = o & 3u;
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = b ? w[4] : 0u;
        const u32x4 x = {__builtin_amdgcn_alignbyte(w1, w0, b), __builtin_amdgcn_alignbyte(w2, w1, b),
                         __builtin_amdgcn_alignbyte(w3, w2, b), __builtin_amdgcn_alignbyte(w4, w3, b)};
        acc = s == 0 ? x : add4(acc, x);
      }
      if (q < n) a.dst[q] = acc;
    }
  }
}

// LDS-DMA realign: a wave's tile is U x 64 output packs; it needs source
// packs [p0, p0 + U*64] — U full DMA instructions (global_load_lds_dwordx4,
// nt, 64 lanes x 16 B straight into LDS) plus one single-lane DMA for the
// extra pack — per source, into a stage buffer private to the wave. S stages:
// the wave issues tile j+S-1's DMA, waits (vmcnt) for tile j, reads each
// output's 16 bytes back from LDS at byte offset 16 (q - p0) + sh (five
// dwords + one byte funnel shift), folds and stores. Nothing goes through
// VGPRs on the load side, so several tiles can be in flight per wave.
typedef __attribute__((address_space(3))) void* lds_ptr;
#define WAIT_VM(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
template <int N>
__device__ __forceinline__ void waitVm() {
  if constexpr (N == 9) WAIT_VM(9);
  else if constexpr (N == 18) WAIT_VM(18);
  else if constexpr (N == 24) WAIT_VM(24);
  else if constexpr (N == 27) WAIT_VM(27);
  else if constexpr (N == 36) WAIT_VM(36);
  else if constexpr (N == 40) WAIT_VM(40);
  else if constexpr (N == 32) WAIT_VM(32);
  else if constexpr (N == 48) WAIT_VM(48);
  else if constexpr (N == 80) WAIT_VM(63);
  else if constexpr (N == 10) WAIT_VM(10);
  else if constexpr (N == 12) WAIT_VM(12);
  else if constexpr (N == 15) WAIT_VM(15);
  else if constexpr (N == 6) WAIT_VM(6);
  else if constexpr (N == 20) WAIT_VM(20);
  else if constexpr (N == 30) WAIT_VM(30);
  else if constexpr (N == 5) WAIT_VM(5);
  else if constexpr (N == 3) WAIT_VM(3);
  else if constexpr (N == 4) WAIT_VM(4);
  else if constexpr (N == 8) WAIT_VM(8);
  else if constexpr (N == 16) WAIT_VM(16);
  else WAIT_VM(0);
}

template <int NSRC, int U, int S, int W>
__global__ __launch_bounds__(W * 64) void kshiftDma(Args a) {
  constexpr int P = U * 64 + 1;   // packs per source per stage
  __shared__ u32x4 sm[W][S][NSRC][P];
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  constexpr uint64_t kTile = (uint64_t)U * 64;
  const uint64_t n = a.nPacks;
  const uint64_t nTiles = (n + kTile - 1) / kTile;
  const uint64_t nWaves = (uint64_t)gridDim.x * W, gw = (uint64_t)blockIdx.x * W + wave;
  auto issue = [&](uint64_t t, int st) {
    const uint64_t p0 = t * kTile;
#pragma unroll
    for (int s = 0; s < NSRC; s++) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t q = p0 + u * 64 + lane;
        q = q < n ? q : n;   // pack n holds the range's last bytes
        __builtin_amdgcn_global_load_lds((const void*)(a.base[s] + q), (lds_ptr)&sm[wave][st][s][u * 64], 16, 0, 2);
      }
      if (lane == 0) {
        const uint64_t q = p0 + kTile < n ? p0 + kTile : n;
        __builtin_amdgcn_global_load_lds((const void*)(a.base[s] + q), (lds_ptr)&sm[wave][st][s][kTile], 16, 0, 2);
      }
    }
  };
#pragma unroll
  for (int k = 0; k < S - 1; k++) {
    const uint64_t t = gw + (uint64_t)k * nWaves;
    if (t < nTiles) issue(t, k);
  }
  int st = 0;
  for (uint64_t t = gw; t < nTiles; t += nWaves) {
    const uint64_t ahead = t + (uint64_t)(S - 1) * nWaves;
    if (ahead < nTiles) {
      issue(ahead, (st + S - 1) % S);
      waitVm<(S - 1) * NSRC * (U + 1)>();   // lane 0 issued U+1 per source: the other lanes' counts are smaller, so stricter
    } else {
      waitVm<0>();
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t q = t * kTile + u * 64 + lane;
      u32x4 acc;
#pragma unroll
      for (int s = 0; s < NSRC; s++) {
        const uint32_t o = (uint32_t)(u * 64 + lane) * 16u + a.sh[s];
        const uint32_t* w = (const uint32_t*)&sm[wave][st][s][0] + (o >> 2);
        const uint32_t b = o & 3u;
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = b ? w[4] : 0u;
        const u32x4 x = {__builtin_amdgcn_alignbyte(w1, w0, b), __builtin_amdgcn_alignbyte(w2, w1, b),
                         __builtin_amdgcn_alignbyte(w3, w2, b), __builtin_amdgcn_alignbyte(w4, w3, b)};
        acc = s == 0 ? x : add4(acc, x);
      }
      if (q < n) a.dst[q] = acc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    st = st + 1 == S ? 0 : st + 1;
  }
}

struct Variant {
  std::string name;
  const void* fn;
  int unroll, blocksPerCU;
};

template <int NSRC>
int run(int cus, int rounds, int iters, int mib) {
  const size_t count = ((size_t)mib << 20) / 4;   // fp32 elements per input
  std::vector<void*> src(NSRC);
  std::vector<float> h(count + 64);
  for (int s = 0; s < NSRC; s++) {
    CK(hipMalloc(&src[s], (count + 64) * 4));
    for (size_t i = 0; i < h.size(); i++) h[i] = (float)((i * 2654435761u + s * 97u) % 100003u) / 1000.0f;
    CK(hipMemcpy(src[s], h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  // destination one element past a 16-B boundary: 3 head elements, then
  // packs; source element k of the body sits 12 B into pack (k*4+12)/16
  float *dstRaw, *refRaw;
  CK(hipMalloc(&dstRaw, (count + 128) * 4));
  CK(hipMalloc(&refRaw, (count + 128) * 4));
  const size_t head = 3;
  const uint64_t nPacks = (count - head) / 4;
  Args a;
  for (int s = 0; s < NSRC; s++) {
    uintptr_t qa = (uintptr_t)src[s] + head * 4;
    a.sh[s] = (uint32_t)(qa & 15u);
    a.base[s] = (const u32x4*)(qa - a.sh[s]);
  }
  a.nPacks = nPacks;
  std::vector<Variant> vs = {
      {"temporal u2 bpc4 (library, 1-3 src)", (const void*)&kshift<NSRC, 2, false>, 2, 4},
      {"dpp-pre u2 bpc2 (library, 4-8 src)", (const void*)&kshiftPre<NSRC, 2>, 2, 2},
      {"temporal u1 bpc8", (const void*)&kshift<NSRC, 1, false>, 1, 8},
      {"temporal u2 bpc2", (const void*)&kshift<NSRC, 2, false>, 2, 2},
      {"lo-nt/hi-temporal u2 bpc4", (const void*)&kshiftMix<NSRC, 2>, 2, 4},
      {"lo-nt/hi-temporal u2 bpc2", (const void*)&kshiftMix<NSRC, 2>, 2, 2},
      {"lo-nt/hi-temporal u1 bpc8", (const void*)&kshiftMix<NSRC, 1>, 1, 8},
      {"dpp-pre u2 bpc4", (const void*)&kshiftPre<NSRC, 2>, 2, 4},
      {"dpp-pre u1 bpc8", (const void*)&kshiftPre<NSRC, 1>, 1, 8},
      {"63-lane u4 bpc2", (const void*)&kshift63<NSRC, 4>, -4, 2},
      {"dpp-pre u4 bpc1", (const void*)&kshiftPre<NSRC, 4>, 4, 1},
      {"dpp-pre u1 bpc4", (const void*)&kshiftPre<NSRC, 1>, 1, 4},
      {"lds u1 bpc4", (const void*)&kshiftLds<NSRC, 1>, 1, 4},
      {"lds u2 bpc2", (const void*)&kshiftLds<NSRC, 2>, 2, 2},
      {"lds u2 bpc3", (const void*)&kshiftLds<NSRC, 2>, 2, 3},
      {"lds u4 bpc1", (const void*)&kshiftLds<NSRC, 4>, 4, 1},
      {"dma W4 U2 S2 bpc1", (const void*)&kshiftDma<NSRC, 2, 2, 4>, -4002, 1},
      {"dma W4 U1 S3 bpc1", (const void*)&kshiftDma<NSRC, 1, 3, 4>, -4001, 1},
      {"dma W2 U4 S2 bpc1", (const void*)&kshiftDma<NSRC, 4, 2, 2>, -2004, 1},
      {"dma W2 U2 S2 bpc2", (const void*)&kshiftDma<NSRC, 2, 2, 2>, -2002, 2},
      {"dma W4 U1 S2 bpc2", (const void*)&kshiftDma<NSRC, 1, 2, 4>, -4001, 2},
      {"dma W2 U2 S3 bpc1", (const void*)&kshiftDma<NSRC, 2, 3, 2>, -2002, 1},
      {"dma W1 U4 S3 bpc1", (const void*)&kshiftDma<NSRC, 4, 3, 1>, -1004, 1},
      {"dma W1 U4 S2 bpc2", (const void*)&kshiftDma<NSRC, 4, 2, 1>, -1004, 2},
      {"dma W2 U4 S1 bpc2", (const void*)&kshiftDma<NSRC, 4, 1, 2>, -2004, 2},
  };
  // the aligned fold (reference rate, not a realigning kernel): its output
  // differs, so it is timed but not compared
  const Variant aligned = NSRC >= 4 ? Variant{"ALIGNED u4 bpc1 (reference)", (const void*)&kaligned<NSRC, 4>, 4, 1}
                                    : Variant{"ALIGNED u1 bpc4 (reference)", (const void*)&kaligned<NSRC, 1>, 1, 4};

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // destination body: DSTOFF bytes into its (256-B aligned) allocation; 16 =
  // the library's layout for a destination one element off (body on the
  // next 16-B boundary), 128 / 256 = a body on a cache-line boundary
  const char* dv = getenv("DSTOFF");
  const size_t dstOff = dv ? (size_t)atoi(dv) : 16;
  printf("destination body at byte %zu of its allocation\n", dstOff);
  auto launch = [&](const Variant& v, float* outRaw) {
    Args b = a;
    b.dst = (u32x4*)((char*)outRaw + dstOff);
    // unroll < 0: 63-lane variant, a workgroup covers 4 x 63 x |unroll| packs;
    // <= -1000: LDS-DMA variant, -(1000 x waves + U): waves x U x 64 packs
    int threads = 256;
    uint64_t tile;
    if (v.unroll > 0) tile = (uint64_t)v.unroll * 256;
    else if (v.unroll > -1000) tile = (uint64_t)(-v.unroll) * 252;
    else {
      const int w = (-v.unroll) / 1000, u = (-v.unroll) % 1000;
      threads = 64 * w;
      tile = (uint64_t)w * u * 64;
    }
    uint64_t grid = std::min<uint64_t>((nPacks + tile - 1) / tile, (uint64_t)cus * v.blocksPerCU);
    int ns = NSRC;
    void* args[] = {&b, &ns};
    CK(hipLaunchKernel(v.fn, dim3((unsigned)grid), dim3(threads), args, 0, 0));
  };
  CK(hipMemset(refRaw, 0, (count + 64) * 4));
  launch(vs[0], refRaw);
  CK(hipDeviceSynchronize());
  // host check of the reference variant: ordered left fold of the sources
  std::vector<float> r(count + 64), o(count + 64);
  CK(hipMemcpy(r.data(), refRaw, r.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  {
    std::vector<std::vector<float>> hs(NSRC, std::vector<float>(count + 64));
    for (int s = 0; s < NSRC; s++) CK(hipMemcpy(hs[s].data(), src[s], hs[s].size() * 4, hipMemcpyDeviceToHost));
    for (uint64_t k = 0; k < nPacks * 4; k++) {
      float acc = hs[0][head + k];
      for (int s = 1; s < NSRC; s++) acc = acc + hs[s][head + k];
      if (memcmp(&acc, &r[dstOff / 4 + k], 4) != 0) {
        if (bad < 4) printf("host mismatch at %llu\n", (unsigned long long)k);
        bad++;
      }
    }
  }
  for (auto& v : vs) {
    CK(hipMemset(dstRaw, 0, (count + 64) * 4));
    launch(v, dstRaw);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), dstRaw, o.size() * 4, hipMemcpyDeviceToHost));
    if (memcmp(o.data(), r.data(), o.size() * 4) != 0) {
      printf("MISMATCH in %s\n", v.name.c_str());
      bad++;
    }
  }
  vs.push_back(aligned);
  std::vector<std::vector<float>> t(vs.size());
  for (int rd = 0; rd < rounds; rd++)
    for (size_t i = 0; i < vs.size(); i++) {
      launch(vs[i], dstRaw);
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < iters; it++) launch(vs[i], dstRaw);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[i].push_back(ms / iters);
    }
  printf("%d x %d MiB fp32 -> %d MiB, sources 12 B off their packs\n", NSRC, mib, mib);
  printf("%-40s %10s %10s %9s\n", "variant", "med_ms", "min_ms", "GB/s(med)");
  for (size_t i = 0; i < vs.size(); i++) {
    auto x = t[i];
    std::sort(x.begin(), x.end());
    double med = x[x.size() / 2];
    printf("%-40s %10.4f %10.4f %9.1f\n", vs[i].name.c_str(), med, x[0],
           (double)(NSRC + 1) * nPacks * 16 / (med * 1e-3) / 1e9);
  }
  printf("mismatches: %d\n", bad);
  for (auto p : src) CK(hipFree(p));
  CK(hipFree(dstRaw));
  CK(hipFree(refRaw));
  return bad;
}

int main(int argc, char** argv) {
  int rounds = argc > 1 ? atoi(argv[1]) : 7, iters = argc > 2 ? atoi(argv[2]) : 10;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int mib = argc > 3 ? atoi(argv[3]) : 64;
  int bad = run<8>(cus, rounds, iters, mib);
  bad += run<4>(cus, rounds, iters, mib);
  bad += run<2>(cus, rounds, iters, mib);
  printf("total mismatches: %d\n", bad);
  return bad ? 1 : 0;
}
