// probe_table_mem.hip — where should the batch work list live? (not product
// code). Measures, on the GPU box:
//   1. whether the CPU can write device memory from hipMalloc /
//      hipExtMallocWithFlags(fine-grained) / (uncached) directly (large BAR),
//      and the host write rate into each;
//   2. the latency of a chain of dependent loads a kernel issues into pinned
//      host memory vs device memory (what a workgroup pays per record it reads).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe_table_mem.hip -o scripts/probe_table_mem
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <csetjmp>
#include <csignal>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 2; } } while (0)

static sigjmp_buf g_jmp;
static void onSegv(int) { siglongjmp(g_jmp, 1); }

// one lane walks a pointer chain of `hops` dependent loads; the time per hop
__global__ void kchase(const uint64_t* p, int hops, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint64_t idx = 0;
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < hops; i++) idx = ((const volatile uint64_t*)p)[idx];   // L1 bypassed, L2 as the record reads
  const uint64_t t1 = wall_clock64();
  out[0] = t1 - t0;
  out[1] = idx;
}

static int hostWriteTest(const char* name, void* p, size_t bytes) {
  struct sigaction sa = {}, old = {};
  sa.sa_handler = onSegv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  if (sigsetjmp(g_jmp, 1) == 0) {
    auto t0 = std::chrono::steady_clock::now();
    std::memset(p, 0x5a, bytes);
    auto t1 = std::chrono::steady_clock::now();
    volatile unsigned char v = ((volatile unsigned char*)p)[bytes - 1];
    (void)v;
    const double us = std::chrono::duration<double, std::micro>(t1 - t0).count();
    printf("%-28s CPU write OK: %zu B in %.1f us (%.2f GB/s)\n", name, bytes, us, bytes / us * 1e-3);
    sigaction(SIGSEGV, &old, nullptr);
    return 1;
  }
  printf("%-28s CPU write FAULTED (not host-accessible)\n", name);
  sigaction(SIGSEGV, &old, nullptr);
  return 0;
}

static int chase(const char* name, uint64_t* table, bool hostPtr, uint64_t* dout) {
  const int n = 4096, hops = 200;
  uint64_t h[n];
  for (int i = 0; i < n; i++) h[i] = (uint64_t)((i * 977 + 131) % n);   // 16-B+ strided chain
  if (hostPtr) std::memcpy(table, h, sizeof(h));
  else CK(hipMemcpy(table, h, sizeof(h), hipMemcpyHostToDevice));
  uint64_t r[2];
  for (int rep = 0; rep < 3; rep++) {
    kchase<<<1, 64>>>(table, hops, dout);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r, dout, sizeof(r), hipMemcpyDeviceToHost));
  }
  printf("%-28s dependent load: %.0f ns per hop (100 MHz wall clock)\n", name, r[0] * 10.0 / hops);
  return 0;
}

int main() {
  const size_t bytes = 64 << 10;
  uint64_t* dout;
  CK(hipMalloc(&dout, 64));
  void* pin = nullptr;
  CK(hipHostMalloc(&pin, bytes, hipHostMallocCoherent));
  void* dm = nullptr;
  CK(hipMalloc(&dm, bytes));
  void* fg = nullptr;
  CK(hipExtMallocWithFlags(&fg, bytes, hipDeviceMallocFinegrained));
  void* uc = nullptr;
  CK(hipExtMallocWithFlags(&uc, bytes, hipDeviceMallocUncached));
  hostWriteTest("pinned host (coherent)", pin, bytes);
  const int okDm = hostWriteTest("hipMalloc", dm, bytes);
  const int okFg = hostWriteTest("device fine-grained", fg, bytes);
  const int okUc = hostWriteTest("device uncached", uc, bytes);
  const char* names[4] = {"pinned host (coherent)", "hipMalloc", "device fine-grained", "device uncached"};
  void* ptrs[4] = {pin, dm, fg, uc};
  for (int i = 0; i < 4; i++) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, ptrs[i]) == hipSuccess)
      printf("%-28s attributes: type %d hostPointer %p devicePointer %p (ptr %p)\n", names[i], (int)at.type,
             at.hostPointer, at.devicePointer, ptrs[i]);
  }
  // host cost of the calls a batch launch makes
  hipStream_t st;
  CK(hipStreamCreate(&st));
  {
    hipStreamCaptureStatus cs;
    hipGraph_t g;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) (void)hipStreamGetCaptureInfo_v2(st, &cs, nullptr, &g, nullptr, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    printf("hipStreamGetCaptureInfo_v2: %.2f us per call\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) (void)hipStreamIsCapturing(st, &cs);
    t1 = std::chrono::steady_clock::now();
    printf("hipStreamIsCapturing: %.2f us per call\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) (void)hipEventRecord(ev, st);
    t1 = std::chrono::steady_clock::now();
    printf("hipEventRecord: %.2f us per call\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    CK(hipStreamSynchronize(st));
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) (void)hipEventQuery(ev);
    t1 = std::chrono::steady_clock::now();
    printf("hipEventQuery: %.2f us per call\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) (void)hipStreamWriteValue64(st, pin, (uint64_t)i, 0);
    t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(st));
    printf("hipStreamWriteValue64: %.2f us per call (host), last value %llu\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000, (unsigned long long)*(volatile uint64_t*)pin);
    // CPU write of a 20 KiB table into uncached device memory + read-back of its last word
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100; i++) {
      std::memset(uc, i, 20 << 10);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      (void)((volatile uint64_t*)uc)[(20 << 10) / 8 - 1];
    }
    t1 = std::chrono::steady_clock::now();
    printf("20 KiB table into uncached device memory + read-back: %.2f us\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 100);
  }
  chase("pinned host (coherent)", (uint64_t*)pin, true, dout);
  chase("hipMalloc", (uint64_t*)dm, okDm != 0, dout);
  chase("device fine-grained", (uint64_t*)fg, okFg != 0, dout);
  chase("device uncached", (uint64_t*)uc, okUc != 0, dout);
  return 0;
}
