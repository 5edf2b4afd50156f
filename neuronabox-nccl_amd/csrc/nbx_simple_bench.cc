// nbx_simple_bench.cc — the Simple protocol's kernels (nbx_simple.h) driven
// for n ranks from ONE process on one GPU, for tuning and tests: the staging,
// flag words and counters of every "rank" are allocated here exactly as
// ncclCommInitRank lays them out (uncached memory), every rank's kernel is
// launched on its own stream, and the n launches of a call run concurrently —
// the multi-process communicator's data path without its processes, IPC or
// bootstrap. Diagnostics only (include/nbx_debug.h); nothing in the
// collectives calls it.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <vector>

#include "../../include/nbx_debug.h"
#include "nbx_internal.h"
#include "nbx_ll_args.h"

namespace {

struct Rig {
  int n = 0;
  std::vector<char*> stage;
  std::vector<uint64_t*> flags, counters;
  char** stageTab = nullptr;
  uint64_t** flagTab = nullptr;
  std::vector<hipStream_t> streams;
  int* hostWords = nullptr;
  int* hostWordsDev = nullptr;

  ~Rig() {
    (void)hipDeviceSynchronize();
    for (auto* p : stage) (void)hipFree(p);
    for (auto* p : flags) (void)hipFree(p);
    for (auto* p : counters) (void)hipFree(p);
    if (stageTab) (void)hipFree(stageTab);
    if (flagTab) (void)hipFree(flagTab);
    for (auto s : streams) (void)hipStreamDestroy(s);
    if (hostWords) (void)hipHostFree(hostWords);
  }
};

int typeBytes(int dt) {
  switch (dt) {
    case 0: case 1: case 10: case 11: return 1;
    case 6: case 9: return 2;
    case 2: case 3: case 7: return 4;
    case 4: case 5: case 8: return 8;
    default: return -1;
  }
}

}  // namespace

extern "C" __attribute__((visibility("default"))) int nbxDebugSimpleRun(
    int n, int kind, int ring, size_t count, int datatype, int op, const void* const* sends, void* const* recvs,
    int root, int gridMax, size_t sliceBytes, int slots, int prefetch, int iters, float* msPerCall) {
  const int eb = typeBytes(datatype);
  if (n < 2 || n > nbx::kSimpleMaxRanks || kind < 0 || kind > 2 || eb < 0 || gridMax < 1 ||
      gridMax > nbx::kSimpleMaxGrid || slots < 2 || sliceBytes < 16 || (sliceBytes & 15u) || iters < 1 ||
      sends == nullptr || recvs == nullptr || root < 0 || root >= n)
    return ncclInvalidArgument;
  nbxDevRedOpFull opFull;
  if (nbxHostToDevRedOp(&opFull, (ncclRedOp_t)op, (ncclDataType_t)datatype, n) != ncclSuccess) return ncclInvalidArgument;
  Rig rig;
  rig.n = n;
  const uint64_t cells = (uint64_t)n * (uint64_t)gridMax;
  const uint64_t hdrOff = 2ull * (uint64_t)slots * cells * sliceBytes;   // then the plan headers (nbx_simple.h)
  const uint64_t stageBytes = hdrOff + 2ull * (uint64_t)slots * cells * 16u;
  for (int r = 0; r < n; r++) {
    void *s = nullptr, *f = nullptr, *c = nullptr;
    if (hipExtMallocWithFlags(&s, stageBytes, hipDeviceMallocUncached) != hipSuccess ||
        hipExtMallocWithFlags(&f, 4 * cells * 8, hipDeviceMallocUncached) != hipSuccess ||
        hipMalloc(&c, 4 * cells * 8) != hipSuccess)
      return ncclUnhandledCudaError;
    rig.stage.push_back((char*)s);
    rig.flags.push_back((uint64_t*)f);
    rig.counters.push_back((uint64_t*)c);
    if (hipMemset(f, 0, 4 * cells * 8) != hipSuccess || hipMemset(c, 0, 4 * cells * 8) != hipSuccess)
      return ncclUnhandledCudaError;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return ncclUnhandledCudaError;
    rig.streams.push_back(st);
  }
  if (hipMalloc((void**)&rig.stageTab, n * sizeof(char*)) != hipSuccess ||
      hipMalloc((void**)&rig.flagTab, n * sizeof(uint64_t*)) != hipSuccess ||
      hipMemcpy(rig.stageTab, rig.stage.data(), n * sizeof(char*), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(rig.flagTab, rig.flags.data(), n * sizeof(uint64_t*), hipMemcpyHostToDevice) != hipSuccess ||
      hipHostMalloc((void**)&rig.hostWords, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void**)&rig.hostWordsDev, rig.hostWords, 0) != hipSuccess)
    return ncclUnhandledCudaError;
  for (int i = 0; i < 16; i++) rig.hostWords[i] = 0;
  if (hipDeviceSynchronize() != hipSuccess) return ncclUnhandledCudaError;

  // the call's shape, as mpLaunchSimple derives it
  uint64_t blockElts, total;
  if (kind == 1) {
    blockElts = count;
    total = (uint64_t)count * (uint64_t)n;
  } else if (kind == 2 && ring) {
    blockElts = count;
    total = count;
  } else {
    const uint64_t epp = (uint64_t)(16 / eb);
    uint64_t per = ((uint64_t)count + n - 1) / n;
    blockElts = (per + epp - 1) / epp * epp;
    total = count;
  }
  const uint64_t blockBytes = (blockElts < total ? blockElts : total) * (uint64_t)eb;
  if (blockBytes == 0) return ncclSuccess;
  uint64_t grid = (blockBytes + nbx::kSimpleMinSliceBytes - 1) / nbx::kSimpleMinSliceBytes;
  if (grid > (uint64_t)gridMax) grid = gridMax;
  if (grid < 1) grid = 1;
  uint64_t slice = ((blockBytes + grid - 1) / grid + 15) & ~(uint64_t)15;
  if (slice > sliceBytes) slice = sliceBytes;
  std::vector<nbx::SimpleArgs> args(n);
  for (int r = 0; r < n; r++) {
    nbx::SimpleArgs& sa = args[r];
    sa = nbx::SimpleArgs{};
    sa.send = sends[r];
    sa.recv = recvs[r];
    sa.peerStage = rig.stageTab;
    sa.peerFlags = rig.flagTab;
    sa.counters = rig.counters[r];
    sa.total = total;
    sa.blockElts = blockElts;
    sa.sliceBytes = slice;
    sa.nRounds = (blockBytes + grid * slice - 1) / (grid * slice);
    sa.stageSlice = sliceBytes;
    sa.abortWord = rig.hostWordsDev;
    sa.errWord = rig.hostWordsDev + 1;
    sa.timeoutTicks = 30ull * 100000000ull;
    sa.rank = r;
    sa.nRanks = n;
    sa.mode = kind;
    sa.root = root;
    sa.slots = slots;
    sa.gridMax = gridMax;
    sa.prefetch = prefetch;
    sa.hdrOff = hdrOff;
    const char* cp = std::getenv("NBX_CHECK_PLANS");   // as the communicator's default: off
    sa.planSig = (cp && std::atoi(cp) != 0) ? nbx::simplePlanSig(sa, (uint32_t)grid, datatype, opFull.op) : 0;
  }
  // NBX_DEBUG_SIMPLE_FUSED=1: every rank's workgroups in ONE dispatch (fp32
  // sum), so a rocprofv3 PMC pass (which serializes dispatches) can count the
  // call's HBM bytes; the per-rank launches wait on each other and cannot be
  // serialized
  const char* fv = std::getenv("NBX_DEBUG_SIMPLE_FUSED");
  const bool fused = fv && *fv == '1';
  nbx::SimpleArgs* argsDev = nullptr;
  if (fused) {
    if (datatype != 7 || opFull.op != nbxDevSum || (uint64_t)n * grid > 2048) return ncclInvalidArgument;
    // every workgroup of the one dispatch must be resident at once (they wait on each other)
    const int resident = nbx::simpleFusedMaxResident(ring != 0);
    if (resident < 0 || (uint64_t)n * grid > (uint64_t)resident) return ncclInvalidArgument;
    for (auto& sa : args) {
      sa.arg = 0;
      sa.argPtr = nullptr;
    }
    if (hipMalloc((void**)&argsDev, n * sizeof(nbx::SimpleArgs)) != hipSuccess ||
        hipMemcpy(argsDev, args.data(), n * sizeof(nbx::SimpleArgs), hipMemcpyHostToDevice) != hipSuccess)
      return ncclUnhandledCudaError;
  }
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return ncclUnhandledCudaError;
  float ms = 0.f;
  // one untimed call, then `iters` timed ones; the n launches of a call run together
  for (int it = 0; it <= iters; it++) {
    if (it == 1 && hipEventRecord(e0, rig.streams[0]) != hipSuccess) return ncclUnhandledCudaError;
    if (fused) {
      if (nbx::launchSimpleFusedF32Sum(argsDev, n, (unsigned)grid, ring != 0, rig.streams[0]) != ncclSuccess)
        return ncclUnhandledCudaError;
      continue;
    }
    for (int r = 0; r < n; r++) {
      if (it == 1 && r > 0 && hipStreamWaitEvent(rig.streams[r], e0, 0) != hipSuccess) return ncclUnhandledCudaError;
      if (nbx::launchSimple((ncclDataType_t)datatype, opFull, args[r], (unsigned)grid, ring != 0, rig.streams[r]) !=
          ncclSuccess)
        return ncclUnhandledCudaError;
    }
  }
  for (int r = 1; r < n; r++) {
    hipEvent_t er;
    if (hipEventCreateWithFlags(&er, hipEventDisableTiming) != hipSuccess || hipEventRecord(er, rig.streams[r]) != hipSuccess ||
        hipStreamWaitEvent(rig.streams[0], er, 0) != hipSuccess)
      return ncclUnhandledCudaError;
    (void)hipEventDestroy(er);
  }
  if (hipEventRecord(e1, rig.streams[0]) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
      hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
    return ncclUnhandledCudaError;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (hipDeviceSynchronize() != hipSuccess) return ncclUnhandledCudaError;
  if (argsDev) (void)hipFree(argsDev);
  if (msPerCall) *msPerCall = ms / (float)iters;
  return rig.hostWords[1] != 0 ? ncclRemoteError : ncclSuccess;
}
