// nbx_host.cc — host-staged reduction: nbxReduceMultiHost.
//
// The reference's NET/SHM paths stage data in host memory — the proxy's
// host-pinned FIFOs (net.cc:735/883, 1018-1141) and /dev/shm buffers
// (shm.cc:86-114) — which is where the NeuronaBox emulator's proxy/net
// buffers live. This entry point reduces sources that live in host memory
// into host destinations, through a device staging ring:
//
//   in-stream   : H2D of chunk k's sources into slot k%2
//   comp-stream : nbxReduceMulti(slot inputs -> slot output)
//   out-stream  : D2H of slot output into every host destination
//
// so the H2D of chunk k+1, the reduce of chunk k and the D2H of chunk k-1 run
// concurrently (PCIe is full duplex; the reduce runs at HBM speed). Events
// guard slot reuse (inputs: reduce k-2 done; output: D2H k-2 done). The call
// is blocking: it returns when the host destinations hold the result.
// Pinned, device-mapped buffers skip the ring: the reduce kernel reads and
// writes them in place over PCIe (NBX_HOST_MODE selects).
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nbx_reduce.h"

namespace {

#define HCHECK(cmd)                                  \
  do {                                               \
    if ((cmd) != hipSuccess) return ncclUnhandledCudaError; \
  } while (0)

int typeSizeH(ncclDataType_t t) {
  switch ((int)t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return -1;
  }
}

constexpr int kSlots = 2;

// Per-device staging state (streams, events, a growable arena). One call at a
// time per device (the mutex is held for the whole blocking call).
struct HostStage {
  std::mutex mu;
  bool init = false;
  hipStream_t sIn = nullptr, sComp = nullptr, sOut = nullptr;
  hipEvent_t evIn[kSlots], evRed[kSlots], evOut[kSlots], evStart, evDone;
  char* arena = nullptr;
  size_t arenaBytes = 0;
};

constexpr int kMaxDev = 64;
HostStage g_stage[kMaxDev];

size_t chunkBytesPerSource() {
  const char* v = std::getenv("NBX_HOST_CHUNK_BYTES");
  size_t b = (v && *v) ? (size_t)std::strtoull(v, nullptr, 10) : (size_t)(16u << 20);
  if (b < (64u << 10)) b = 64u << 10;
  return b & ~(size_t)255;
}

ncclResult_t stageInit(HostStage& st) {
  if (st.init) return ncclSuccess;
  HCHECK(hipStreamCreateWithFlags(&st.sIn, hipStreamNonBlocking));
  HCHECK(hipStreamCreateWithFlags(&st.sComp, hipStreamNonBlocking));
  HCHECK(hipStreamCreateWithFlags(&st.sOut, hipStreamNonBlocking));
  for (int i = 0; i < kSlots; i++) {
    HCHECK(hipEventCreateWithFlags(&st.evIn[i], hipEventDisableTiming));
    HCHECK(hipEventCreateWithFlags(&st.evRed[i], hipEventDisableTiming));
    HCHECK(hipEventCreateWithFlags(&st.evOut[i], hipEventDisableTiming));
  }
  HCHECK(hipEventCreateWithFlags(&st.evStart, hipEventDisableTiming));
  HCHECK(hipEventCreateWithFlags(&st.evDone, hipEventDisableTiming));
  st.init = true;
  return ncclSuccess;
}

// NBX_HOST_MODE: "staged" (always the device staging ring), "zerocopy"
// (the kernel reads and writes pinned host memory directly over PCIe when
// every buffer is pinned and device-mapped), "auto" (default: zero-copy for
// pinned buffers, staged otherwise).
enum HostMode { kHostAuto, kHostStaged, kHostZeroCopy };
HostMode hostMode() {   // read per call (a blocking, PCIe-bound call: getenv is noise)
  const char* v = std::getenv("NBX_HOST_MODE");
  if (v && std::strcmp(v, "staged") == 0) return kHostStaged;
  if (v && std::strcmp(v, "zerocopy") == 0) return kHostZeroCopy;
  return kHostAuto;
}

// Device address of pinned, device-mapped host memory (nullptr if `p` is
// pageable or not mapped for this device).
void* mappedAlias(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || a.devicePointer == nullptr || a.hostPointer == nullptr) return nullptr;
  return (char*)a.devicePointer + ((const char*)p - (const char*)a.hostPointer);
}

}  // namespace

extern "C" __attribute__((visibility("default"))) ncclResult_t nbxReduceMultiHost(
    void* const* hostDsts, int nDsts, const void* const* hostSrcs, int nSrcs, size_t count, ncclDataType_t datatype,
    nbxDevRedOpFull op, int nPreOpSrcs, int postOp, ncclStream_t stream) {
  const int eb = typeSizeH(datatype);
  if (eb < 0 || nSrcs < 1 || nSrcs > NBX_MAX_SRCS || nDsts < 1 || nDsts > NBX_MAX_DSTS) return ncclInvalidArgument;
  if (hostSrcs == nullptr || hostDsts == nullptr) return ncclInvalidArgument;
  if (op.op < 0 || op.op >= nbxNumDevRedOps) return ncclInvalidArgument;
  if (count == 0) return ncclSuccess;
  for (int s = 0; s < nSrcs; s++)
    if (hostSrcs[s] == nullptr) return ncclInvalidArgument;
  for (int d = 0; d < nDsts; d++)
    if (hostDsts[d] == nullptr) return ncclInvalidArgument;
  // zero-copy: every buffer pinned and mapped — one kernel reads the sources
  // over PCIe and writes the destinations back over PCIe (full duplex), no
  // staging copies
  if (hostMode() != kHostStaged) {
    const void* zs[NBX_MAX_SRCS];
    void* zd[NBX_MAX_DSTS];
    bool all = true;
    for (int s = 0; s < nSrcs && all; s++) all = (zs[s] = mappedAlias(hostSrcs[s])) != nullptr;
    for (int d = 0; d < nDsts && all; d++) all = (zd[d] = mappedAlias(hostDsts[d])) != nullptr;
    if (all) {
      ncclResult_t r = nbxReduceMulti(zd, nDsts, zs, nSrcs, count, datatype, op, nPreOpSrcs, postOp, stream);
      if (r != ncclSuccess) return r;
      HCHECK(hipStreamSynchronize((hipStream_t)stream));
      return ncclSuccess;
    }
    if (hostMode() == kHostZeroCopy) return ncclInvalidArgument;   // zero-copy forced on unpinned memory
  }
  int dev = 0;
  HCHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDev) return ncclInternalError;
  HostStage& st = g_stage[dev];
  std::lock_guard<std::mutex> lock(st.mu);
  ncclResult_t r = stageInit(st);
  if (r != ncclSuccess) return r;

  // chunk: a multiple of 16 B so every slot buffer stays 16-B aligned
  size_t chunkElts = chunkBytesPerSource() / (size_t)eb;
  chunkElts -= chunkElts % (size_t)(16 / eb);
  if (chunkElts > count) chunkElts = count;
  const size_t chunkB = ((chunkElts * (size_t)eb) + 255) & ~(size_t)255;
  const size_t slotB = chunkB * (size_t)(nSrcs + 1);
  if (st.arenaBytes < slotB * kSlots) {
    if (st.arena) HCHECK(hipFree(st.arena));
    st.arena = nullptr;
    st.arenaBytes = 0;
    HCHECK(hipMalloc((void**)&st.arena, slotB * kSlots));
    st.arenaBytes = slotB * kSlots;
  }
  const size_t nChunks = (count + chunkElts - 1) / chunkElts;
  if (nChunks == 1) {
    // one chunk: nothing to overlap — run the three steps on the caller's stream
    // (the three-stream hand-off costs more than it hides at this size)
    hipStream_t cs = (hipStream_t)stream;
    const size_t bytes = count * (size_t)eb;
    const void* dsrc[NBX_MAX_SRCS];
    for (int s = 0; s < nSrcs; s++) {
      char* d = st.arena + (size_t)s * chunkB;
      HCHECK(hipMemcpyAsync(d, hostSrcs[s], bytes, hipMemcpyHostToDevice, cs));
      dsrc[s] = d;
    }
    void* dout[1] = {st.arena + (size_t)nSrcs * chunkB};
    r = nbxReduceMulti(dout, 1, dsrc, nSrcs, count, datatype, op, nPreOpSrcs, postOp, stream);
    if (r != ncclSuccess) return r;
    for (int d = 0; d < nDsts; d++) HCHECK(hipMemcpyAsync(hostDsts[d], dout[0], bytes, hipMemcpyDeviceToHost, cs));
    HCHECK(hipStreamSynchronize(cs));
    return ncclSuccess;
  }
  // order after prior work of the caller's stream
  HCHECK(hipEventRecord(st.evStart, (hipStream_t)stream));
  HCHECK(hipStreamWaitEvent(st.sIn, st.evStart, 0));
  HCHECK(hipStreamWaitEvent(st.sComp, st.evStart, 0));
  HCHECK(hipStreamWaitEvent(st.sOut, st.evStart, 0));

  for (size_t k = 0; k < nChunks; k++) {
    const int slot = (int)(k % kSlots);
    const size_t off = k * chunkElts;
    const size_t n = count - off < chunkElts ? count - off : chunkElts;
    const size_t bytes = n * (size_t)eb;
    char* base = st.arena + (size_t)slot * slotB;
    // inputs: the reduce of chunk k-2 must be done with this slot
    if (k >= kSlots) HCHECK(hipStreamWaitEvent(st.sIn, st.evRed[slot], 0));
    const void* dsrc[NBX_MAX_SRCS];
    for (int s = 0; s < nSrcs; s++) {
      char* d = base + (size_t)s * chunkB;
      HCHECK(hipMemcpyAsync(d, (const char*)hostSrcs[s] + off * (size_t)eb, bytes, hipMemcpyHostToDevice, st.sIn));
      dsrc[s] = d;
    }
    HCHECK(hipEventRecord(st.evIn[slot], st.sIn));
    // reduce: inputs landed; output slot free (D2H of chunk k-2 done)
    HCHECK(hipStreamWaitEvent(st.sComp, st.evIn[slot], 0));
    if (k >= kSlots) HCHECK(hipStreamWaitEvent(st.sComp, st.evOut[slot], 0));
    void* dout[1] = {base + (size_t)nSrcs * chunkB};
    r = nbxReduceMulti(dout, 1, dsrc, nSrcs, n, datatype, op, nPreOpSrcs, postOp, (ncclStream_t)st.sComp);
    if (r != ncclSuccess) return r;
    HCHECK(hipEventRecord(st.evRed[slot], st.sComp));
    // outputs
    HCHECK(hipStreamWaitEvent(st.sOut, st.evRed[slot], 0));
    for (int d = 0; d < nDsts; d++)
      HCHECK(hipMemcpyAsync((char*)hostDsts[d] + off * (size_t)eb, dout[0], bytes, hipMemcpyDeviceToHost, st.sOut));
    HCHECK(hipEventRecord(st.evOut[slot], st.sOut));
  }
  HCHECK(hipEventRecord(st.evDone, st.sOut));
  HCHECK(hipStreamWaitEvent((hipStream_t)stream, st.evDone, 0));
  HCHECK(hipStreamSynchronize(st.sIn));
  HCHECK(hipStreamSynchronize(st.sComp));
  HCHECK(hipStreamSynchronize(st.sOut));
  return ncclSuccess;
}
