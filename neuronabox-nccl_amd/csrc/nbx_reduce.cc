// nbx_reduce.cc — host side of the reduction core: argument checks, pointer
// alignment analysis, multi-pass folding for > 8 sources, grid sizing and the
// kernel launch. Exposes the C ABI of include/nbx_reduce.h.
//
// Reference behaviour mirrored:
//   * alignment fallback — reduceCopy checks every pointer for 16-B alignment
//     and otherwise runs sizeof(T) packs (common_kernel.h:209-238). Here the
//     fast kernel also accepts pointers that share ONE misalignment modulo 16
//     (peeling < 16 B of head elements), so only genuinely mixed alignments
//     take the element kernel.
//   * opArg: by value, or a device pointer dereferenced by the kernel
//     (ncclScalarDevice; common.h:100-119, onerank.cu:32-42).
//   * PreOp on sources s < nPreOpSrcs, postOp after the fold
//     (common_kernel.h:79-137).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/nbx_reduce.h"
#include "nbx_registry.h"
#include "nbx_internal.h"
#include "nbx_ll_args.h"

using namespace nbx;

namespace {

KernelTable g_table;
std::once_flag g_tableOnce;

void buildTable() {
  std::memset(&g_table, 0, sizeof(g_table));
  fillInt8(g_table);
  fillInt32(g_table);
  fillInt64(g_table);
  fillF16(g_table);
  fillBF16(g_table);
  fillF32(g_table);
  fillF64(g_table);
  fillFp8(g_table);
}

const KernelTable& table() {
  std::call_once(g_tableOnce, buildTable);
  return g_table;
}

// Launch configuration (NCCL_NTHREADS / NCCL_MAX_NCHANNELS analogues).
std::atomic<int> g_maxBlocksPerCU{0};   // 0 = default per variant
std::atomic<int> g_variant{0};          // 0 = auto, 1 = force small tile, 2 = force big tile

int envInt(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

constexpr int kMaxDevices = 64;
std::atomic<int> g_cuCount[kMaxDevices];

int cuCount(int dev) {
  if (dev < 0 || dev >= kMaxDevices) return 256;
  int c = g_cuCount[dev].load(std::memory_order_relaxed);
  if (c > 0) return c;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
  g_cuCount[dev].store(c, std::memory_order_relaxed);
  return c;
}

// Workgroups per CU: big tiles keep ~32 dwordx4 loads in flight per lane
// slot — one 256-thread workgroup per CU (4 waves, ~128 KiB in flight per CU)
// when nSrcs x U >= 32, proportionally more when the unroll is capped. Small
// tiles (one pack per lane per source): 5 / 4 / 3 workgroups per CU for 1 / 2
// / 3 sources, 4 above — measured on MI355X (profiles/r1/tiles_sweep_r1n.jsonl:
// 2 sources at 256 MiB 6.80 TB/s with 4 per CU vs 6.12 with 8 and 5.91 with
// one big-tile workgroup; 3 sources 6.58 vs 6.38 big-tile). classic = true
// keeps 8 small workgroups per CU: the element kernel, and passes that read
// peer GPUs' memory (the collectives' direct and ring schedules) — xGMI
// latency wants more bytes in flight, and the local-HBM measurement does not
// carry over (no multi-GPU box to measure it on).
int maxBlocksPerCU(bool big, int loadsPerLane, bool classic = false) {
  int v = g_maxBlocksPerCU.load(std::memory_order_relaxed);
  if (v > 0) return v;
  static const int envBig = envInt("NBX_BLOCKS_PER_CU", 0);
  if (envBig > 0) return envBig;
  if (!big) {
    if (classic) return 8;
    return loadsPerLane <= 1 ? 5 : loadsPerLane == 2 ? 4 : loadsPerLane == 3 ? 3 : 4;
  }
  int b = (32 + loadsPerLane - 1) / loadsPerLane;
  return b < 1 ? 1 : (b > 8 ? 8 : b);
}

// Realigning kernels: 8 workgroups per CU for the run-time-count kernel
// (profiles/r1/sweep_shift.txt); per source count, the LDS-DMA kernel's
// shiftLdsBlocksPerCU (profiles/r2/sweep_shift_256MiB_r2f.txt).
int shiftedBlocksPerCU(bool perCount, int nSrcs) {
  int v = g_maxBlocksPerCU.load(std::memory_order_relaxed);
  if (v > 0) return v;
  static const int env = envInt("NBX_BLOCKS_PER_CU", 0);
  if (env > 0) return env;
  if (!perCount) return 8;
  return shiftLdsBlocksPerCU(nSrcs);
}

// The device a launch on `st` runs on (the per-device arenas and tile
// counters must live there): the stream's own device, the current one for
// the null / per-thread stream.
int launchDevice(hipStream_t st) {
  if (st != nullptr && st != hipStreamPerThread) {
    hipDevice_t d = 0;
    if (hipStreamGetDevice(st, &d) == hipSuccess) return (int)d;
  }
  int dev = 0;
  (void)hipGetDevice(&dev);
  return dev;
}

// Makes `dev` current for an allocation, restoring the caller's device.
struct CurDev {
  int prev = -1;
  explicit CurDev(int dev) {
    if (hipGetDevice(&prev) != hipSuccess || prev == dev || hipSetDevice(dev) != hipSuccess) prev = -1;
  }
  ~CurDev() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

bool isFloatType(int dt) {
  return dt == ncclFloat16 || dt == ncclFloat32 || dt == ncclFloat64 || dt == ncclBfloat16 ||
         dt == ncclFloat8e4m3 || dt == ncclFloat8e5m2;
}

int typeSize(int dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return -1;
  }
}

// Elements folded one by one before the 16-B pack body, so that the body of
// dsts[0] starts on a 128-B cache-line boundary (NBX_PEEL_BYTES: 16 keeps
// the smallest peel). Streams that start mid-line cost every wave
// instruction a partial line at each end: all pointers one element off ran
// 9 % slower at 256 MiB per input than aligned ones with a 16-B peel, and a
// destination body on a line boundary gains 2-5 % for the realigning kernels
// (profiles/r2/realign_probe_r2d.jsonl, sweep_shift_256MiB_r2d.txt).
size_t peelElts(uintptr_t dst, int eb) {
  static const unsigned line = [] {
    const int v = envInt("NBX_PEEL_BYTES", 128);
    return (unsigned)(v == 16 || v == 32 || v == 64 || v == 128 || v == 256 ? v : 128);
  }();
  const unsigned mis = (unsigned)(dst & (line - 1));
  return mis ? (size_t)((line - mis) / (unsigned)eb) : 0;
}

bool overlaps(const void* a, const void* b, size_t bytes) {
  uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
  return x < y + bytes && y < x + bytes;
}

// Dynamic tiles (kernels' forEachTile): one 32-bit counter per (device,
// stream) in device memory. Every launch on a stream advances its counter by
// exactly its tile count, so the host knows each launch's base without the
// kernel resetting anything; launches on one stream run in order, so no two
// launches ever share a counter concurrently. The lock is held from reading
// the base to the launch, so calls racing on one stream from several threads
// still enqueue in base order. Not used while the stream is being captured
// (a replay would reuse a stale base), for hipStreamPerThread (one handle,
// many streams), or with NBX_DYNAMIC_TILES=0.
// Keyed by the stream handle. HIP hands a destroyed stream's handle to the
// next stream created (63 of 64 create / destroy cycles), but hipStreamDestroy
// returns only once the stream's work has completed (20 ms of pending kernels:
// destroy took 21.4 ms on the ROCm 7.2 runtime, 39 ms on torch's 7.0 runtime,
// nothing left running after it; scripts/probe_stream_id.hip,
// scripts/probe_stream_destroy.py, profiles/r3/probe_stream_*_r3f.log). So a
// new stream that inherits a handle inherits an idle counter whose value is
// the base the host tracks, and streams created per iteration keep reusing
// the same few counters (tests/test_reduce_gpu.py::
// test_dynamic_counters_with_stream_churn).
constexpr int kDynCounters = 4096;

struct DynTiles {
  std::mutex mu;
  uint32_t* pool = nullptr;
  int used = 0;
  bool failed = false;
  std::unordered_map<hipStream_t, std::pair<uint32_t*, uint32_t>> next;   // stream -> (counter, base)
};
DynTiles g_dyn[kMaxDevices];

// Tiles per workgroup from which a big-tile launch is dynamic (launchPass);
// env NBX_DYN_MIN_TILES_PER_WG, nbxDebugSetDynMinTiles.
std::atomic<int> g_dynMinTiles{0};
int dynMinTilesPerWG() {
  int v = g_dynMinTiles.load(std::memory_order_relaxed);
  if (v < 1) {
    const int e = envInt("NBX_DYN_MIN_TILES_PER_WG", 16);
    int expect = v;
    g_dynMinTiles.compare_exchange_strong(expect, e < 1 ? 1 : e);
    v = g_dynMinTiles.load();
  }
  return v;
}

// Class counters of the realigning kernel's dynamic schedule: kShiftDynClasses
// counters kShiftDynStride words apart per (device, stream). The kernel resets
// each class counter on its last fetch, so a launch always starts from zero
// and the host tracks no base; launches on one stream run in order, so no two
// share a block at once. nullptr (static schedule) while the stream is being
// captured (a captured launch may be replayed on any stream), for
// hipStreamPerThread, with NBX_DYNAMIC_TILES=0 or once the pool is used up.
constexpr int kShiftDynBlocks = 64;
constexpr size_t kShiftDynBlockWords = (size_t)kShiftDynClasses * kShiftDynStride;
struct ShiftDyn {
  std::mutex mu;
  uint32_t* pool = nullptr;
  int used = 0;
  bool failed = false;
  std::unordered_map<hipStream_t, uint32_t*> block;
};
ShiftDyn g_shiftDyn[kMaxDevices];

uint32_t* shiftDynCounters(int dev, hipStream_t st) {
  static const int on = envInt("NBX_DYNAMIC_TILES", 1);
  if (!on || dev < 0 || dev >= kMaxDevices || st == hipStreamPerThread) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  ShiftDyn& D = g_shiftDyn[dev];
  std::lock_guard<std::mutex> lk(D.mu);
  if (D.pool == nullptr) {
    if (D.failed) return nullptr;
    CurDev cur(dev);
    void* p = nullptr;
    const size_t bytes = (size_t)kShiftDynBlocks * kShiftDynBlockWords * sizeof(uint32_t);
    if (hipMalloc(&p, bytes) != hipSuccess) {
      D.failed = true;
      return nullptr;
    }
    D.pool = (uint32_t*)p;
  }
  auto it = D.block.find(st);
  if (it != D.block.end()) return it->second;
  if (D.used >= kShiftDynBlocks) return nullptr;
  uint32_t* b = D.pool + (size_t)D.used * kShiftDynBlockWords;
  // zeroed in the stream's own order, ahead of its first launch
  if (hipMemsetAsync(b, 0, kShiftDynBlockWords * sizeof(uint32_t), st) != hipSuccess) return nullptr;
  D.used++;
  D.block.emplace(st, b);
  return b;
}

// One kernel pass over <= kMaxKSrcs sources.
ncclResult_t launchPass(const KernelSet& ks, void* const* dsts, int nDsts, const void* const* srcs,
                        int nSrcs, size_t count, const nbxDevRedOpFull& op, uint32_t preMask,
                        int postOp, int acquireSystem, hipStream_t stream) {
  KArgs a;
  std::memset(&a, 0, sizeof(a));
  a.acquireSystem = acquireSystem;
  for (int s = 0; s < nSrcs; s++) a.src[s] = srcs[s];
  for (int d = 0; d < kMaxKDsts; d++) a.dst[d] = dsts[d < nDsts ? d : 0];
  a.nElts = count;
  a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
  a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
  a.preMask = preMask;
  a.nSrcs = nSrcs;
  a.nDsts = nDsts;
  a.postOp = postOp;

  const int eb = ks.eltBytes;
  const int epp = 16 / eb;
  // shared misalignment modulo 16?
  const unsigned mis = (unsigned)((uintptr_t)srcs[0] & 15u);
  bool shared = true;
  for (int s = 1; s < nSrcs; s++) shared &= (((uintptr_t)srcs[s] & 15u) == mis);
  for (int d = 0; d < nDsts; d++) shared &= (((uintptr_t)dsts[d] & 15u) == mis);

  const int dev = launchDevice(stream);
  const int cus = cuCount(dev);
  void* args[] = {&a};
  hipError_t err;
  if (shared) {
    size_t head = peelElts((uintptr_t)dsts[0], eb);
    if (head > count) head = count;
    const size_t nPacks = (count - head) / (size_t)epp;
    a.headElts = (int)head;
    a.nPacks = nPacks;
    // big tiles once every CU gets at least one, for 4+ sources; small tiles
    // below that, and always for 1-3 sources (more workgroups per CU beat
    // deeper unrolling when a quarter or more of the traffic is stores:
    // profiles/r1/tiles_sweep_r1n.jsonl)
    const size_t bigTile = (size_t)ks.unroll[nSrcs - 1] * kBlock;
    const size_t bigTiles = (nPacks + bigTile - 1) / bigTile;
    const int force = g_variant.load(std::memory_order_relaxed);
    const bool big = force == 2 || (force == 0 && (nSrcs > 3 || acquireSystem) && bigTiles >= (size_t)cus);
    const size_t tile = big ? bigTile : (size_t)kBlock;
    const size_t tiles = (nPacks + tile - 1) / tile;
    int perCU = maxBlocksPerCU(big, nSrcs * (big ? ks.unroll[nSrcs - 1] : 1), acquireSystem != 0);
    static const bool envPerCU = envInt("NBX_BLOCKS_PER_CU", 0) > 0;
    if (big && !envPerCU && g_maxBlocksPerCU.load(std::memory_order_relaxed) == 0 && perCU < ks.bigBlocksPerCU)
      perCU = ks.bigBlocksPerCU;   // VALU-heavy functors: a second wave per SIMD
    // Few big tiles per CU (config C's mid-size buckets): one tile per
    // workgroup, up to NBX_MID_BLOCKS_PER_CU workgroups per CU, so every tile's
    // loads are in flight at once instead of a workgroup's second tile waiting
    // for its first tile's fold (scripts/steps/r4-o.txt, r4-p.txt)
    static const int midPerCU = envInt("NBX_MID_BLOCKS_PER_CU", 4);
    if (big && !envPerCU && g_maxBlocksPerCU.load(std::memory_order_relaxed) == 0 && midPerCU > 1) {
      const size_t need = (tiles + (size_t)cus - 1) / (size_t)cus;
      if (need > (size_t)perCU && need <= (size_t)midPerCU) perCU = (int)need;
    }
    const size_t maxBlocks = (size_t)cus * (size_t)perCU;
    size_t grid = tiles < maxBlocks ? tiles : maxBlocks;
    if (grid == 0) grid = 1;
    a.variant = big ? 1 : 0;
    // dynamic tiles for big tiles only: small tiles (1-3 sources, 3-5
    // workgroups per CU, 16x the atomics) collapse to 0.7-1.4 TB/s on the
    // counter's contention (profiles/r2/probe_dyn_r2x.jsonl), and fetching
    // chunks of 4-16 consecutive small tiles per atomic still lost 15-60 % to
    // the static grid stride (profiles/r2/probe_dyn_small_chunk_r3k.jsonl).
    // And only for launches of >= 16 tiles per workgroup: every workgroup's
    // fetch goes to one address, and device-scope atomics on one address
    // serialize (~11 ns each), so the launch's first and last round of
    // fetches — one per workgroup, all at once — add ~3 us, which only long
    // launches win back (8 x fp32 sources: 4 MiB per input 7.50 vs 4.71 us
    // static, 16 MiB 27.4 vs 24.4 us, 64 MiB 97.4 vs 98.1, 256 MiB 376 vs 395;
    // scripts/sweep_dyn_xcd.hip, profiles/r2/sweep_dyn_xcd_r4e.txt,
    // profiles/r2/probe_mid_sizes_r4d.jsonl)
    DynLaunch dyn;
    if (big && tiles >= (size_t)dynMinTilesPerWG() * grid) dyn.begin(dev, stream, tiles, a);
    err = hipLaunchKernel((const void*)ks.packs[big ? 1 : 0][nSrcs - 1], dim3((unsigned)grid), dim3(kBlock), args,
                          0, stream);
    dyn.done(err == hipSuccess);
  } else {
    const unsigned dmis = (unsigned)((uintptr_t)dsts[0] & 15u);
    bool dstShared = true;
    for (int d = 1; d < nDsts; d++) dstShared &= (((uintptr_t)dsts[d] & 15u) == dmis);
    if (dstShared && ks.shifted != nullptr) {
      // destinations share one alignment: 16-B packs on their side, the
      // sources realigned in registers (kReduceShifted)
      size_t head = peelElts((uintptr_t)dsts[0], eb);
      if (head > count) head = count;
      const size_t nPacks = (count - head) / (size_t)epp;
      a.headElts = (int)head;
      a.nPacks = nPacks;
      // one kernel per source count staging the sources through LDS by
      // LDS-DMA (profiles/r2/sweep_shift_256MiB_r2f.txt);
      // NBX_SHIFT_N=0 or launch variant 1 (small tiles) selects the
      // run-time-count register kernel (1 pack per lane, 8 workgroups/CU)
      static const int useN = envInt("NBX_SHIFT_N", 1);
      const bool small = g_variant.load(std::memory_order_relaxed) == 1;
      const void* fn = (useN && !small) ? ks.shiftedN[nSrcs - 1] : nullptr;
      const size_t tile = fn ? (size_t)shiftLdsUnroll(nSrcs) * 64 * kShiftLdsWaves : (size_t)kBlock;
      size_t blocks = (nPacks + tile - 1) / tile;
      if (blocks == 0) blocks = 1;
      const size_t maxBlocks = (size_t)cus * (size_t)shiftedBlocksPerCU(fn != nullptr, nSrcs);
      const size_t grid = blocks < maxBlocks ? blocks : maxBlocks;
      const unsigned threads = fn ? (unsigned)(kShiftLdsWaves * 64) : (unsigned)kBlock;
      // dynamic schedule for long eager launches from 3 sources, over
      // kShiftDynClasses class counters (kReduceShiftedLds): one counter for
      // all workgroup tiles ran 1.1-4.9 TB/s here — 4-8x the big kernel's
      // atomics on one address (profiles/r2/realign_dyn_r3a.jsonl). At 256 MiB
      // per input the classes give 8 sources +4.7 %, 4 sources +1.1 % over
      // the static stride; 2 sources (1-pack wave tiles, 2 workgroups per CU:
      // 8x the fetches per byte) lost 28 % to the counters' contention, so
      // they stay static (profiles/r2/realign_probe_r4q.jsonl)
      if (fn && nSrcs >= 3 && blocks >= (size_t)dynMinTilesPerWG() * grid) a.dynCtr = shiftDynCounters(dev, stream);
      if (!fn) fn = ks.shifted;
      err = hipLaunchKernel(fn, dim3((unsigned)grid), dim3(threads), args, 0, stream);
    } else {
      size_t blocks = (count + kBlock - 1) / kBlock;
      size_t maxBlocks = (size_t)cus * (size_t)maxBlocksPerCU(false, nSrcs, /*classic=*/true);
      size_t grid = blocks < maxBlocks ? blocks : maxBlocks;
      err = hipLaunchKernel((const void*)ks.elts, dim3((unsigned)grid), dim3(kBlock), args, 0, stream);
    }
  }
  if (err != hipSuccess) {
    std::fprintf(stderr, "nbx: kernel launch failed: %s\n", hipGetErrorString(err));
    return ncclUnhandledCudaError;
  }
  return ncclSuccess;
}

}  // namespace

namespace nbx {
bool DynLaunch::begin(int dev, hipStream_t st, uint64_t nTiles, KArgs& a) {
  static const int on = envInt("NBX_DYNAMIC_TILES", 1);
  if (!on || dev < 0 || dev >= kMaxDevices || st == hipStreamPerThread || nTiles == 0 || nTiles > 0xffffffffull)
    return false;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  DynTiles& D = g_dyn[dev];
  lk_ = std::unique_lock<std::mutex>(D.mu);
  if (D.pool == nullptr) {
    CurDev cur(dev);
    void* p = nullptr;
    if (D.failed || hipMalloc(&p, kDynCounters * sizeof(uint32_t)) != hipSuccess) {
      D.failed = true;
      lk_.unlock();
      return false;
    }
    D.pool = (uint32_t*)p;
  }
  auto it = D.next.find(st);
  if (it == D.next.end()) {
    // a stream's counter is zeroed in that stream's own order, ahead of its
    // first launch (a memset on the null stream would not order a
    // non-blocking stream's kernel after it)
    if (D.used >= kDynCounters || hipMemsetAsync(D.pool + D.used, 0, sizeof(uint32_t), st) != hipSuccess) {
      lk_.unlock();
      return false;
    }
    it = D.next.emplace(st, std::make_pair(D.pool + D.used++, 0u)).first;
  }
  slot_ = &it->second;
  tiles_ = nTiles;
  a.dynCtr = slot_->first;
  a.dynBase = slot_->second;
  return true;
}

void DynLaunch::done(bool launched) {
  if (slot_ && launched) slot_->second += (uint32_t)tiles_;   // mod 2^32, as the kernel's arithmetic
  slot_ = nullptr;
  if (lk_.owns_lock()) lk_.unlock();
}
}  // namespace nbx

namespace nbx {
// Workgroup cap of the LL-family kernels from an env knob, clamped to [1, 1024].
size_t gridCapFromEnv(const char* name, long dflt) {
  const char* v = std::getenv(name);
  long g = (v && *v) ? std::atol(v) : dflt;
  return (size_t)(g < 1 ? 1 : g > 1024 ? 1024 : g);
}

ncclResult_t launchLLColl(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& a, hipStream_t stream) {
  if ((int)dt < 0 || (int)dt >= kNumTypes || op.op < 0 || op.op >= kNumDevOps) return ncclInvalidArgument;
  const KernelSet& ks = table()[(int)dt][op.op];
  if (!ks.valid || ks.ll == nullptr || ks.llChk == nullptr) return ncclInvalidArgument;
  a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
  a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
  // one 8-byte pack per thread; NBX_LL_MAX_GRID caps the workgroups (default
  // 1024), e.g. when several ranks share one GPU and every rank's grid must
  // stay co-resident for the ranks' spinning blocks to make progress
  static const size_t maxGrid = gridCapFromEnv("NBX_LL_MAX_GRID", 1024);
  size_t grid = (a.nPacks + 255) / 256;
  if (grid < 1) grid = 1;
  if (grid > maxGrid) grid = maxGrid;
  if (a.gridCap != 0 && grid > a.gridCap) grid = a.gridCap;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(a.planSig != 0 ? ks.llChk : ks.ll, dim3((unsigned)grid), dim3(256), args, 0, stream);
  if (e != hipSuccess) return ncclUnhandledCudaError;
  return ncclSuccess;
}

ncclResult_t launchLL128Coll(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& a, hipStream_t stream) {
  if ((int)dt < 0 || (int)dt >= kNumTypes || op.op < 0 || op.op >= kNumDevOps) return ncclInvalidArgument;
  const KernelSet& ks = table()[(int)dt][op.op];
  if (!ks.valid || ks.ll128 == nullptr || ks.ll128Chk == nullptr) return ncclInvalidArgument;
  a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
  a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
  // 64 lines (4 lanes each) per 256-thread workgroup, at most one workgroup per
  // CU by default (every block of the grid co-resident on its GPU, so a block
  // waiting for its peers' lines never holds back a block they wait for).
  // NBX_LL128_MAX_GRID lowers the cap, e.g. when several ranks share one GPU.
  static const size_t maxGrid = gridCapFromEnv("NBX_LL128_MAX_GRID", 256);
  const size_t linesPerBlock = 256 / kL128LanesHost;
  size_t grid = (a.nLines + linesPerBlock - 1) / linesPerBlock;
  if (grid < 1) grid = 1;
  if (grid > maxGrid) grid = maxGrid;
  if (a.gridCap != 0 && grid > a.gridCap) grid = a.gridCap;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(a.planSig != 0 ? ks.ll128Chk : ks.ll128, dim3((unsigned)grid), dim3(256), args, 0, stream);
  if (e != hipSuccess) return ncclUnhandledCudaError;
  return ncclSuccess;
}

ncclResult_t launchSimple(ncclDataType_t dt, const nbxDevRedOpFull& op, SimpleArgs& a, unsigned grid, bool ring,
                          hipStream_t stream) {
  if ((int)dt < 0 || (int)dt >= kNumTypes || op.op < 0 || op.op >= kNumDevOps) return ncclInvalidArgument;
  const KernelSet& ks = table()[(int)dt][op.op];
  const void* k = a.checkSlices ? (ring ? ks.simpleRingChk : ks.simpleChk) : (ring ? ks.simpleRing : ks.simple);
  if (!ks.valid || k == nullptr || grid < 1 || grid > (unsigned)a.gridMax || a.gridMax > kSimpleMaxGrid ||
      a.nRanks < 2 || a.nRanks > kSimpleMaxRanks)
    return ncclInvalidArgument;
  a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
  a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(k, dim3(grid), dim3(kBlock), args, 0, stream);
  if (e != hipSuccess) return ncclUnhandledCudaError;
  return ncclSuccess;
}

ncclResult_t launchLL128AllReduce2(ncclDataType_t dt, const nbxDevRedOpFull& op, LLArgs& a, uint64_t blockLines,
                                   hipStream_t stream) {
  if ((int)dt < 0 || (int)dt >= kNumTypes || op.op < 0 || op.op >= kNumDevOps) return ncclInvalidArgument;
  const KernelSet& ks = table()[(int)dt][op.op];
  if (!ks.valid || ks.ll128x2 == nullptr || ks.ll128x2Chk == nullptr) return ncclInvalidArgument;
  a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
  a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
  static const size_t maxGrid = gridCapFromEnv("NBX_LL128_MAX_GRID", 256);
  const size_t linesPerBlock = 256 / kL128LanesHost;
  size_t grid = (blockLines + linesPerBlock - 1) / linesPerBlock;
  if (grid < 1) grid = 1;
  if (grid > maxGrid) grid = maxGrid;
  if (a.gridCap != 0 && grid > a.gridCap) grid = a.gridCap;
  void* args[] = {&a};
  hipError_t e = hipLaunchKernel(a.planSig != 0 ? ks.ll128x2Chk : ks.ll128x2, dim3((unsigned)grid), dim3(256), args, 0, stream);
  if (e != hipSuccess) return ncclUnhandledCudaError;
  return ncclSuccess;
}
}  // namespace nbx

extern "C" {

__attribute__((visibility("default"))) ncclResult_t nbxHostToDevRedOp(nbxDevRedOpFull* out, ncclRedOp_t op,
                                                                       ncclDataType_t datatype, int nRanks) {
  // enqueue.cc:1436-1512 for the built-in ops.
  if (out == nullptr) return ncclInvalidArgument;
  const int sz = typeSize((int)datatype);
  if (sz < 0) return ncclInvalidArgument;
  const int nbits = 8 * sz;
  const uint64_t allBits = ~0ull >> (64 - nbits);
  const uint64_t signBit = allBits ^ (allBits >> 1);
  out->scalarArgIsPtr = 0;
  out->scalarArg = 0;
  switch ((int)op) {
    case ncclSum: out->op = nbxDevSum; return ncclSuccess;
    case ncclProd: out->op = nbxDevProd; return ncclSuccess;
    case ncclMin:
    case ncclMax:
      out->op = nbxDevMinMax;
      if (datatype == ncclInt8 || datatype == ncclInt32 || datatype == ncclInt64) out->scalarArg ^= signBit;
      out->scalarArg ^= ((int)op == ncclMax) ? allBits : 0;
      return ncclSuccess;
    case ncclAvg: {
      if (nRanks < 1) return ncclInvalidArgument;
      if (!isFloatType((int)datatype)) {
        out->op = nbxDevSumPostDiv;
        out->scalarArg = (uint64_t)nRanks;
        return ncclSuccess;
      }
      out->op = nbxDevPreMulSum;
      const float f = (float)(1.0 / nRanks);
      uint32_t fb;
      std::memcpy(&fb, &f, 4);
      switch ((int)datatype) {
        case ncclFloat16: {  // __float2half(float(1.0/n)) — enqueue.cc:1483
          _Float16 h = (_Float16)f;
          uint16_t hb;
          std::memcpy(&hb, &h, 2);
          out->scalarArg = hb;
          break;
        }
        case ncclBfloat16: {  // __float2bfloat16(float(1.0/n)) — enqueue.cc:1488, RNE
          uint32_t u = fb + 0x7fffu + ((fb >> 16) & 1u);
          out->scalarArg = (uint16_t)(u >> 16);
          break;
        }
        case ncclFloat32: out->scalarArg = fb; break;
        case ncclFloat64: {
          double d = 1.0 / nRanks;
          std::memcpy(&out->scalarArg, &d, 8);
          break;
        }
        case ncclFloat8e4m3:
        case ncclFloat8e5m2: {
          // this build's extension: the element type's RNE encoding of float(1/n)
          // (e4m3fn: E=4,M=3,bias=7; e5m2: E=5,M=2,bias=15). 1/n <= 1, never overflows.
          const bool e4 = datatype == ncclFloat8e4m3;
          const int E = e4 ? 4 : 5, M = e4 ? 3 : 2;
          const int bias = (1 << (E - 1)) - 1, emin = 1 - bias;
          const int e = (int)((fb >> 23) & 0xff) - 127;
          const int et = e < emin ? emin : e;
          int shift = (23 - M) + (et - e);
          if (shift > 31) shift = 31;
          const uint32_t mant = (fb & 0x7fffffu) | 0x800000u;
          uint32_t q = mant >> shift;
          const uint32_t rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1);
          if (rem > half || (rem == half && (q & 1u))) q++;
          out->scalarArg = (uint64_t)((uint32_t)((et + bias - 1) << M) + q);
          break;
        }
      }
      return ncclSuccess;
    }
    default: return ncclInvalidArgument;
  }
}

namespace {
// Datatype / op checks shared by the single and batched entry points; on
// success *ks is the functor's kernel set.
ncclResult_t checkOp(ncclDataType_t datatype, const nbxDevRedOpFull& op, const KernelSet** ks) {
  const int dt = (int)datatype;
  if (dt < 0 || dt >= kNumTypes) return ncclInvalidArgument;
  if (op.op < 0 || op.op >= kNumDevOps) return ncclInvalidArgument;
  const KernelSet& k = table()[dt][op.op];
  if (!k.valid) return ncclInvalidArgument;   // e.g. SumPostDiv on floats
  if (op.op == nbxDevSumPostDiv && !op.scalarArgIsPtr && (int)op.scalarArg == 0) return ncclInvalidArgument;
  if (op.scalarArgIsPtr && op.scalarArg == 0) return ncclInvalidArgument;
  *ks = &k;
  return ncclSuccess;
}

// Per-bucket checks: counts of sources and destinations, non-null pointers
// aligned to the element size (count == 0 accepts anything but NULL arrays).
ncclResult_t checkBucket(const KernelSet& ks, void* const* dsts, int nDsts, const void* const* srcs, int nSrcs,
                         size_t count) {
  if (nSrcs < 1 || nSrcs > NBX_MAX_SRCS || nDsts < 1 || nDsts > NBX_MAX_DSTS) return ncclInvalidArgument;
  if (srcs == nullptr || dsts == nullptr) return ncclInvalidArgument;
  if (count == 0) return ncclSuccess;
  const int eb = ks.eltBytes;
  for (int s = 0; s < nSrcs; s++)
    if (srcs[s] == nullptr || ((uintptr_t)srcs[s] % (uintptr_t)eb) != 0) return ncclInvalidArgument;
  for (int d = 0; d < nDsts; d++)
    if (dsts[d] == nullptr || ((uintptr_t)dsts[d] % (uintptr_t)eb) != 0) return ncclInvalidArgument;
  return ncclSuccess;
}

ncclResult_t reduceMultiImpl(void* const* dsts, int nDsts, const void* const* srcs, int nSrcs, size_t count,
                             ncclDataType_t datatype, nbxDevRedOpFull op, int nPreOpSrcs, int postOp,
                             ncclStream_t stream, int flags) {
  const int acq = (flags & nbx::kReduceAcquireSystem) ? 1 : 0;
  const KernelSet* ksp = nullptr;
  if (nSrcs < 1 || nSrcs > NBX_MAX_SRCS || nDsts < 1 || nDsts > NBX_MAX_DSTS) return ncclInvalidArgument;
  if (srcs == nullptr || dsts == nullptr) return ncclInvalidArgument;
  ncclResult_t cr = checkOp(datatype, op, &ksp);
  if (cr != ncclSuccess) return cr;
  const KernelSet& ks = *ksp;
  if (count == 0) return ncclSuccess;
  cr = checkBucket(ks, dsts, nDsts, srcs, nSrcs, count);
  if (cr != ncclSuccess) return cr;
  const int eb = ks.eltBytes;
  if (nPreOpSrcs < 0) nPreOpSrcs = 0;
  hipStream_t st = (hipStream_t)stream;
  const bool pre = op.op == nbxDevPreMulSum;
  const int post = (op.op == nbxDevSumPostDiv && postOp) ? 1 : 0;

  if (nSrcs <= kMaxKSrcs) {
    uint32_t mask = 0;
    if (pre)
      for (int s = 0; s < nSrcs; s++)
        if (s < nPreOpSrcs) mask |= 1u << s;
    return launchPass(ks, dsts, nDsts, srcs, nSrcs, count, op, mask, post, acq, st);
  }

  // > 8 sources: ordered multi-pass left fold through a partial buffer:
  //   pass 0: part = fold(srcs[0..8)); pass k: part = fold(part, next <= 7 srcs);
  //   the last pass writes every destination.
  // The partial lives in dsts[0] unless dsts[0] overlaps a source read by a
  // later pass — in-place collectives past 8 ranks put the rank's own send
  // block (= its output) last in fold order — then in stream-ordered scratch
  // memory, so the fold order (and the result) is unchanged.
  const size_t bytes = count * (size_t)eb;
  bool alias = false;
  for (int s = kMaxKSrcs; s < nSrcs; s++) alias |= overlaps(dsts[0], srcs[s], bytes);
  void* part = dsts[0];
  if (alias) {
    // graph-capturable (a stream-ordered allocation node); freed after the last pass
    if (hipMallocAsync(&part, bytes, st) != hipSuccess) return ncclUnhandledCudaError;
  }
  void* partDst[1] = {part};
  uint32_t mask = 0;
  if (pre)
    for (int s = 0; s < kMaxKSrcs; s++)
      if (s < nPreOpSrcs) mask |= 1u << s;
  ncclResult_t r = launchPass(ks, partDst, 1, srcs, kMaxKSrcs, count, op, mask, 0, acq, st);
  int next = kMaxKSrcs;
  while (r == ncclSuccess && next < nSrcs) {
    const void* ps[kMaxKSrcs];
    ps[0] = part;
    int n = 1;
    uint32_t m = 0;
    while (n < kMaxKSrcs && next < nSrcs) {
      if (pre && next < nPreOpSrcs) m |= 1u << n;
      ps[n++] = srcs[next++];
    }
    const bool last = next >= nSrcs;
    r = launchPass(ks, last ? dsts : partDst, last ? nDsts : 1, ps, n, count, op, m, last ? post : 0, acq, st);
  }
  if (alias && hipFreeAsync(part, st) != hipSuccess && r == ncclSuccess) r = ncclUnhandledCudaError;
  return r;
}

// Shared misalignment modulo 16 of every pointer of a bucket (-1: mixed).
int sharedMisalignment(void* const* dsts, int nDsts, const void* const* srcs, int nSrcs) {
  const unsigned mis = (unsigned)((uintptr_t)srcs[0] & 15u);
  for (int s = 1; s < nSrcs; s++)
    if (((uintptr_t)srcs[s] & 15u) != mis) return -1;
  for (int d = 0; d < nDsts; d++)
    if (((uintptr_t)dsts[d] & 15u) != mis) return -1;
  return (int)mis;
}

// Packs bucket records (nbx_kargs.h BatchArgs) for kReduceBatch launches of
// one source count; a launch goes out when the table is full, or on flush().
struct BatchPacker {
  const KernelSet& ks;
  int nSrcs;
  const nbxDevRedOpFull& op;
  uint32_t preMask;
  int postOp, acquireSystem;
  hipStream_t stream;
  BatchArgs a;
  int used = 0;

  BatchPacker(const KernelSet& k, int ns, const nbxDevRedOpFull& o, uint32_t pm, int post, int acq, hipStream_t st)
      : ks(k), nSrcs(ns), op(o), preMask(pm), postOp(post), acquireSystem(acq), stream(st) {
    static_assert(sizeof(BatchArgs) <= 4096, "batch table must fit the kernel-argument segment");
    reset();
  }
  void reset() {
    std::memset(&a, 0, offsetof(BatchArgs, w));
    used = 0;
  }
  // appends one bucket (count > 0, one shared misalignment)
  ncclResult_t add(const nbxReduceTask& t) {
    const int len = 2 + nSrcs + t.nDsts;
    if (used + len > kBatchWords) {
      ncclResult_t r = flush();
      if (r != ncclSuccess) return r;
    }
    const int eb = ks.eltBytes;
    const uint64_t epp = (uint64_t)(16 / eb);
    const unsigned mis = (unsigned)((uintptr_t)t.srcs[0] & 15u);
    uint64_t head = mis ? (uint64_t)((16u - mis) / (unsigned)eb) : 0;
    if (head > t.count) head = t.count;
    const uint64_t nPacks = (t.count - head) / epp;
    const uint64_t tiles = (nPacks + kBatchTilePacks - 1) / kBatchTilePacks;
    a.totalTiles += tiles ? tiles : 1;   // a bucket below one pack still owns a tile (its elements)
    uint64_t* w = a.w + used;
    w[0] = a.totalTiles;
    w[1] = (uint64_t)t.count | head << 56 | (uint64_t)t.nDsts << 60;
    for (int s = 0; s < nSrcs; s++) w[2 + s] = (uint64_t)(uintptr_t)t.srcs[s];
    for (int d = 0; d < t.nDsts; d++) w[2 + nSrcs + d] = (uint64_t)(uintptr_t)t.dsts[d];
    used += len;
    a.nTasks++;
    return ncclSuccess;
  }
  ncclResult_t flush() {
    if (a.nTasks == 0) return ncclSuccess;
    a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
    a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
    a.preMask = preMask;
    a.postOp = postOp;
    a.acquireSystem = acquireSystem;
    const uint64_t maxBlocks =
        (uint64_t)cuCount(launchDevice(stream)) * (uint64_t)maxBlocksPerCU(false, nSrcs, acquireSystem != 0);
    const uint64_t grid = a.totalTiles < maxBlocks ? a.totalTiles : maxBlocks;
    void* args[] = {&a};
    hipError_t err = hipLaunchKernel(ks.batch[nSrcs - 1], dim3((unsigned)grid), dim3(kBlock), args, 0, stream);
    reset();
    if (err != hipSuccess) {
      std::fprintf(stderr, "nbx: batch kernel launch failed: %s\n", hipGetErrorString(err));
      return ncclUnhandledCudaError;
    }
    return ncclSuccess;
  }
};

// Work-list tables (kReduceBatchList): one arena of kListSlots fixed-size
// slots per device, allocated on first use outside stream capture. Where the
// device's memory is CPU-visible (large BAR) the arena is uncached device
// memory the host writes directly — a workgroup's dependent record read then
// costs ~110 ns instead of ~1.2 us from pinned host memory
// (scripts/probe_table_mem.hip, profiles/r2/probe_table_mem_r2.txt); uncached,
// so no GPU cache can keep an earlier table of a reused slot. Otherwise the
// arena is pinned, coherent host memory the kernel reads in place.
// A slot written for an eager launch is reusable once the event recorded after
// that launch has completed; every eager call sweeps a few slots' events so
// completed slots return to the free pool (a capture cannot query events). A
// slot written while the stream is being captured belongs to the graph (every
// replay reads it); a user object retained by the graph hands it back when
// the graph is destroyed. Nothing ever waits for a slot: with none free the
// caller falls back to kernel-argument batches.
constexpr int kListSlots = 128;
constexpr int kListSweep = 8;   // eager calls query at most this many in-flight slots

struct ListArena {
  std::mutex mu;
  char* base = nullptr;
  bool onDevice = false;
  hipEvent_t ev[kListSlots] = {};
  std::atomic<int> state[kListSlots];   // 0 free, 1 eager (event pending), 2 owned by a graph
  std::atomic<long> fallbacks{0};       // launches that found no free slot
  int cursor = 0, sweep = 0;
  ListArena() {
    for (auto& s : state) s.store(0);
  }
};
ListArena g_lists[kMaxDevices];

void releaseGraphSlot(void* p) { static_cast<std::atomic<int>*>(p)->store(0); }

bool allocArena(ListArena& A, int dev) {
  CurDev cur(dev);
  const size_t bytes = (size_t)kListSlots * kBatchListSlotBytes;
  int largeBar = 0;
  static const int want = envInt("NBX_BATCH_TABLE_DEVICE", 1);
  void* p = nullptr;
  if (want && hipDeviceGetAttribute(&largeBar, hipDeviceAttributeIsLargeBar, dev) == hipSuccess && largeBar &&
      hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) {
    A.onDevice = true;
  } else {
    p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocCoherent) != hipSuccess) return false;
    A.onDevice = false;
  }
  for (int i = 0; i < kListSlots; i++) {
    if (hipEventCreateWithFlags(&A.ev[i], hipEventDisableTiming) != hipSuccess) {
      for (int j = 0; j < i; j++) (void)hipEventDestroy(A.ev[j]);
      if (A.onDevice) (void)hipFree(p);
      else (void)hipHostFree(p);
      return false;
    }
  }
  A.base = (char*)p;
  return true;
}

// A free slot of this device's arena (index, *ptr = its memory), or -1.
int acquireListSlot(int dev, bool capturing, char** ptr) {
  if (dev < 0 || dev >= kMaxDevices) return -1;
  ListArena& A = g_lists[dev];
  std::lock_guard<std::mutex> lk(A.mu);
  if (A.base == nullptr) {
    if (capturing) return -1;   // no allocation inside a capture
    if (!allocArena(A, dev)) return -1;
  }
  if (!capturing) {   // return a few completed slots to the free pool
    for (int j = 0; j < kListSweep; j++) {
      const int i = A.sweep;
      A.sweep = (A.sweep + 1) % kListSlots;
      if (A.state[i].load() == 1 && hipEventQuery(A.ev[i]) == hipSuccess) A.state[i].store(0);
    }
  }
  int pick = -1;
  for (int j = 0; j < kListSlots && pick < 0; j++) {
    const int i = (A.cursor + j) % kListSlots;
    if (A.state[i].load() == 0) pick = i;
  }
  if (pick < 0 && !capturing) {   // the oldest in-flight slot, if it has completed
    for (int j = 0; j < kListSlots && pick < 0; j++) {
      const int i = (A.cursor + j) % kListSlots;
      if (A.state[i].load() == 1) {
        if (hipEventQuery(A.ev[i]) == hipSuccess) pick = i;
        break;
      }
    }
  }
  if (pick < 0) {
    A.fallbacks++;
    return -1;
  }
  A.state[pick].store(2);   // reserved until released by the launch
  A.cursor = (pick + 1) % kListSlots;
  *ptr = A.base + (size_t)pick * kBatchListSlotBytes;
  return pick;
}

// Make the host's writes into a device-memory slot land before the launch
// (posted PCIe writes, write-combined mapping): fence, then read one back.
void publishListSlot(int dev, const volatile uint32_t* last) {
  if (!g_lists[dev].onDevice) return;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  (void)*last;
}

// After the launch that reads slot i: eager -> its event; captured -> the
// graph owns it until destroyed; launch failed -> free again.
void releaseListSlot(int dev, int i, hipStream_t st, hipGraph_t graph, bool launched) {
  ListArena& A = g_lists[dev];
  if (!launched) {
    A.state[i].store(0);
    return;
  }
  if (graph != nullptr) {
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, &A.state[i], releaseGraphSlot, 1, hipUserObjectNoDestructorSync) == hipSuccess &&
        hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) == hipSuccess)
      return;   // state stays 2 until the graph lets go of it
    return;     // could not attach: the slot stays the graph's for good (never reused)
  }
  if (hipEventRecord(A.ev[i], st) != hipSuccess) {
    (void)hipStreamSynchronize(st);
    A.state[i].store(0);
    return;
  }
  A.state[i].store(1);
}

// NBX_BATCH_LIST: 1 (default) = work-list launches (sets of <= 16 buckets
// that fit one kernel-argument table excepted), 2 = work lists for every set,
// 0 = kernel-argument batches only (also settable through nbxDebugSetBatchMode).
std::atomic<int> g_batchMode{-1};
int batchMode() {
  int m = g_batchMode.load(std::memory_order_relaxed);
  if (m < 0) {
    const int e = envInt("NBX_BATCH_LIST", 1);
    m = e == 0 ? 0 : (e == 2 ? 2 : 1);
    int expect = -1;
    g_batchMode.compare_exchange_strong(expect, m);
    m = g_batchMode.load();
  }
  return m;
}
bool batchListEnabled() { return batchMode() != 0; }

// Slots of the device's work-list arena by state (free / eager / graph-owned).
int listSlotCount(int dev, int state) {
  if (dev < 0 || dev >= kMaxDevices) return -1;
  ListArena& A = g_lists[dev];
  std::lock_guard<std::mutex> lk(A.mu);
  if (state == 3) return (int)A.fallbacks.load();
  if (A.base == nullptr) return state == 0 ? kListSlots : 0;
  int n = 0;
  for (auto& s : A.state) n += s.load() == state;
  return n;
}

// Launches the buckets of one source count as work-list kernels (as many
// launches as slots they need). Returns the number of buckets launched from
// the front of `ts` (fewer than ts.size() when no slot was free).
ncclResult_t launchBatchList(const KernelSet& ks, int nSrcs, const std::vector<const nbxReduceTask*>& ts,
                             const nbxDevRedOpFull& op, uint32_t preMask, int postOp, int acq, hipStream_t st,
                             size_t* done) {
  *done = 0;
  const int dev = launchDevice(st);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipGraph_t graph = nullptr;
  if (hipStreamGetCaptureInfo_v2(st, &cs, nullptr, &graph, nullptr, nullptr) != hipSuccess) {
    cs = hipStreamCaptureStatusNone;
    graph = nullptr;
  }
  const bool capturing = cs != hipStreamCaptureStatusNone;
  if (capturing && (cs != hipStreamCaptureStatusActive || graph == nullptr)) return ncclSuccess;
  const uint64_t maxG = (uint64_t)cuCount(dev) * (uint64_t)maxBlocksPerCU(false, nSrcs, acq != 0);
  // 4 consecutive tiles per workgroup turn: the best of 1 / 4 / 16 on every
  // config-C bucket set (profiles/r2/batch_list_chunk_r2p.jsonl)
  static const uint64_t chunkEnv = (uint64_t)envInt("NBX_BATCH_CHUNK", 4);
  const uint64_t chunk = chunkEnv < 1 ? 1 : chunkEnv;
  const int eb = ks.eltBytes;
  const uint64_t epp = (uint64_t)(16 / eb);
  static_assert(sizeof(BatchListArgs) <= 4096, "work-list arguments must fit the kernel-argument segment");
  BatchListArgs a;
  size_t i = 0;
  while (i < ts.size()) {
    // this launch's buckets: up to kListMaxRecs, running tile totals < 2^32
    size_t nRec = 0;
    uint64_t tiles = 0;
    int maxD = 1;
    while (nRec < (size_t)kListMaxRecs && i + nRec < ts.size()) {
      const nbxReduceTask& t = *ts[i + nRec];
      if (t.nDsts > maxD) maxD = t.nDsts;
      const unsigned mis = (unsigned)((uintptr_t)t.srcs[0] & 15u);
      uint64_t head = mis ? (uint64_t)((16u - mis) / (unsigned)eb) : 0;
      if (head > t.count) head = t.count;
      const uint64_t bt = ((t.count - head) / epp + kBatchTilePacks - 1) / kBatchTilePacks;
      const uint64_t next = tiles + (bt ? bt : 1);   // a bucket below one pack still owns a tile
      if (next > 0xffffffffull) break;
      tiles = next;
      a.tileEnd[nRec++] = (uint32_t)tiles;
    }
    if (nRec == 0) return ncclSuccess;   // a bucket of >= 2^32 tiles: the caller's fallback
    char* mem = nullptr;
    const int slot = acquireListSlot(dev, capturing, &mem);
    if (slot < 0) return ncclSuccess;
    uint64_t* recs = (uint64_t*)mem;   // write-only: the slot may be device memory behind the BAR
    const int recWords = 3 + nSrcs + maxD;   // <= kBatchRecWords
    for (size_t r = 0; r < nRec; r++) {
      const nbxReduceTask& t = *ts[i + r];
      const unsigned mis = (unsigned)((uintptr_t)t.srcs[0] & 15u);
      uint64_t head = mis ? (uint64_t)((16u - mis) / (unsigned)eb) : 0;
      if (head > t.count) head = t.count;
      uint64_t* w = recs + r * (size_t)recWords;
      w[0] = r ? a.tileEnd[r - 1] : 0;
      w[1] = a.tileEnd[r];
      w[2] = (uint64_t)t.count | head << 56 | (uint64_t)t.nDsts << 60;
      for (int s = 0; s < nSrcs; s++) w[3 + s] = (uint64_t)(uintptr_t)t.srcs[s];
      for (int d = 0; d < maxD; d++) w[3 + nSrcs + d] = d < t.nDsts ? (uint64_t)(uintptr_t)t.dsts[d] : 0;
    }
    const uint64_t chunks = (tiles + chunk - 1) / chunk;
    const uint64_t G = chunks < maxG ? chunks : maxG;
    a.recs = recs;
    a.nRecs = (int)nRec;
    a.chunk = (uint32_t)chunk;
    a.recWords = (uint32_t)recWords;
    a.totalTiles = tiles;
    a.arg = op.scalarArgIsPtr ? 0 : op.scalarArg;
    a.argPtr = op.scalarArgIsPtr ? (const void*)(uintptr_t)op.scalarArg : nullptr;
    a.preMask = preMask;
    a.postOp = postOp;
    a.acquireSystem = acq;
    publishListSlot(dev, (const volatile uint32_t*)(recs + nRec * (size_t)recWords - 1));
    void* args[] = {&a};
    const hipError_t err =
        hipLaunchKernel(ks.batchList[nSrcs - 1], dim3((unsigned)G), dim3(kBlock), args, 0, st);
    releaseListSlot(dev, slot, st, capturing ? graph : nullptr, err == hipSuccess);
    if (err != hipSuccess) {
      std::fprintf(stderr, "nbx: batch-list kernel launch failed: %s\n", hipGetErrorString(err));
      return ncclUnhandledCudaError;
    }
    i += nRec;
    *done = i;
  }
  return ncclSuccess;
}

ncclResult_t reduceMultiBatchImpl(const nbxReduceTask* tasks, int nTasks, ncclDataType_t datatype,
                                  nbxDevRedOpFull op, int nPreOpSrcs, int postOp, ncclStream_t stream, int flags) {
  if (nTasks < 0 || (nTasks > 0 && tasks == nullptr)) return ncclInvalidArgument;
  const KernelSet* ksp = nullptr;
  ncclResult_t r = checkOp(datatype, op, &ksp);
  if (r != ncclSuccess) return r;
  const KernelSet& ks = *ksp;
  // every bucket is checked before anything is enqueued
  for (int i = 0; i < nTasks; i++) {
    r = checkBucket(ks, tasks[i].dsts, tasks[i].nDsts, tasks[i].srcs, tasks[i].nSrcs, tasks[i].count);
    if (r != ncclSuccess) return r;
  }
  if (nPreOpSrcs < 0) nPreOpSrcs = 0;
  const bool pre = op.op == nbxDevPreMulSum;
  const int post = (op.op == nbxDevSumPostDiv && postOp) ? 1 : 0;
  const int acq = (flags & nbx::kReduceAcquireSystem) ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  // buckets with <= 8 sources and one shared alignment go into batches per
  // source count, in order; the rest (mixed alignment, > 8 sources) take the
  // single-bucket path, and so do buckets of 4+ sources big enough to give
  // every CU a big tile on their own (they fill the GPU alone, at the big
  // tile's higher rate; 1-3 sources use the batch kernel's tile shape anyway). Launch variant 1 (force small tiles) batches those too; variant 2
  // (force big tiles) batches nothing.
  const int force = g_variant.load(std::memory_order_relaxed);
  const uint64_t cus = (uint64_t)cuCount(launchDevice(st));
  std::unique_ptr<BatchPacker> packers[kMaxKSrcs];
  std::vector<const nbxReduceTask*> lists[kMaxKSrcs];
  const bool useList = batchListEnabled();
  for (int i = 0; i < nTasks; i++) {
    const nbxReduceTask& t = tasks[i];
    if (t.count == 0) continue;
    bool single = force == 2 || t.nSrcs > kMaxKSrcs || t.count > kBatchCountMask ||
                  sharedMisalignment(t.dsts, t.nDsts, t.srcs, t.nSrcs) < 0;
    if (!single && force == 0 && (t.nSrcs > 3 || acq)) {
      const uint64_t bigTile = (uint64_t)ks.unroll[t.nSrcs - 1] * kBlock;
      single = t.count / (uint64_t)(16 / ks.eltBytes) >= bigTile * cus;
    }
    if (single) {
      r = reduceMultiImpl(t.dsts, t.nDsts, t.srcs, t.nSrcs, t.count, datatype, op, nPreOpSrcs, postOp, stream,
                          flags);
      if (r != ncclSuccess) return r;
      continue;
    }
    lists[t.nSrcs - 1].push_back(&t);
  }
  for (int q = 0; q < kMaxKSrcs; q++) {
    if (lists[q].empty()) continue;
    const int ns = q + 1;
    uint32_t mask = 0;
    if (pre)
      for (int s = 0; s < ns; s++)
        if (s < nPreOpSrcs) mask |= 1u << s;
    size_t done = 0;
    // a handful of buckets that fit one kernel-argument table run faster from
    // it (records in the scalar cache, a short cursor walk); longer lists,
    // whose cursor walk dominates, take the work list
    bool fitsKernarg = batchMode() != 2 && lists[q].size() <= (size_t)kBatchKernargMaxBuckets;
    if (fitsKernarg) {
      size_t words = 0;
      for (const nbxReduceTask* t : lists[q]) words += (size_t)(2 + ns + t->nDsts);
      fitsKernarg = words <= (size_t)kBatchWords;
    }
    if (useList && !fitsKernarg) {
      r = launchBatchList(ks, ns, lists[q], op, mask, post, acq, st, &done);
      if (r != ncclSuccess) return r;
    }
    if (done == lists[q].size()) continue;
    // the rest as kernel-argument batches (work lists off, or no table slot free)
    packers[q].reset(new BatchPacker(ks, ns, op, mask, post, acq, st));
    for (size_t j = done; j < lists[q].size(); j++) {
      r = packers[q]->add(*lists[q][j]);
      if (r != ncclSuccess) return r;
    }
    r = packers[q]->flush();
    if (r != ncclSuccess) return r;
  }
  return ncclSuccess;
}
}  // namespace

}  // extern "C"

namespace nbx {
ncclResult_t reduceMultiEx(void* const* dsts, int nDsts, const void* const* srcs, int nSrcs, size_t count,
                           ncclDataType_t datatype, nbxDevRedOpFull op, int nPreOpSrcs, int postOp,
                           ncclStream_t stream, int flags) {
  return reduceMultiImpl(dsts, nDsts, srcs, nSrcs, count, datatype, op, nPreOpSrcs, postOp, stream, flags);
}
ncclResult_t reduceMultiBatchEx(const nbxReduceTask* tasks, int nTasks, ncclDataType_t datatype, nbxDevRedOpFull op,
                                int nPreOpSrcs, int postOp, ncclStream_t stream, int flags) {
  return reduceMultiBatchImpl(tasks, nTasks, datatype, op, nPreOpSrcs, postOp, stream, flags);
}
}  // namespace nbx

extern "C" {

__attribute__((visibility("default"))) ncclResult_t nbxReduceMulti(void* const* dsts, int nDsts,
                                                                    const void* const* srcs, int nSrcs, size_t count,
                                                                    ncclDataType_t datatype, nbxDevRedOpFull op,
                                                                    int nPreOpSrcs, int postOp, ncclStream_t stream) {
  return reduceMultiImpl(dsts, nDsts, srcs, nSrcs, count, datatype, op, nPreOpSrcs, postOp, stream, 0);
}

__attribute__((visibility("default"))) ncclResult_t nbxReduceMultiBatch(const nbxReduceTask* tasks, int nTasks,
                                                                         ncclDataType_t datatype, nbxDevRedOpFull op,
                                                                         int nPreOpSrcs, int postOp,
                                                                         ncclStream_t stream) {
  return reduceMultiBatchImpl(tasks, nTasks, datatype, op, nPreOpSrcs, postOp, stream, 0);
}

__attribute__((visibility("default"))) ncclResult_t nbxSetLaunchConfig(int blocksPerCU, int variant) {
  if (blocksPerCU < 0 || blocksPerCU > 64 || variant < 0 || variant > 2) return ncclInvalidArgument;
  g_maxBlocksPerCU.store(blocksPerCU);
  g_variant.store(variant);
  return ncclSuccess;
}

__attribute__((visibility("default"))) ncclResult_t nbxGetLaunchConfig(int* blocksPerCU, int* variant) {
  if (blocksPerCU) *blocksPerCU = g_maxBlocksPerCU.load();
  if (variant) *variant = g_variant.load();
  return ncclSuccess;
}

__attribute__((visibility("default"))) int nbxKernelCount(void) {
  int n = 0;
  const KernelTable& t = table();
  for (int ty = 0; ty < kNumTypes; ty++)
    for (int o = 0; o < kNumDevOps; o++)
      if (t[ty][o].valid) n++;
  return n;
}

__attribute__((visibility("default"))) int nbxAbiVersion(void) { return 1; }

__attribute__((visibility("default"))) int nbxDebugSetBatchMode(int mode) {
  const int prev = batchMode();
  if (mode >= 0 && mode <= 2) g_batchMode.store(mode);
  return prev;
}

__attribute__((visibility("default"))) int nbxDebugBatchListSlots(int device, int state) {
  return listSlotCount(device, state);
}

__attribute__((visibility("default"))) int nbxDebugDynStreamSlots(int device, int which) {
  if (device < 0 || device >= kMaxDevices) return -1;
  if (which == 0) {
    std::lock_guard<std::mutex> lk(g_dyn[device].mu);
    return g_dyn[device].used;
  }
  std::lock_guard<std::mutex> lk(g_shiftDyn[device].mu);
  return g_shiftDyn[device].used;
}

__attribute__((visibility("default"))) int nbxDebugSetDynMinTiles(int tilesPerWorkgroup) {
  const int prev = dynMinTilesPerWG();
  if (tilesPerWorkgroup >= 1) g_dynMinTiles.store(tilesPerWorkgroup);
  return prev;
}

}  // extern "C"
