// probe_host_cost.hip — host-side cost per call of the library's entry points
// against the HIP calls they make (not part of the product): mean host time
// per call of N back-to-back calls (no synchronization inside the timed loop),
// the GPU drained between measurements. Small buckets, so the host enqueue is
// what is measured, not the kernel.
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 -I include scripts/probe_host_cost.hip
//        -L neuronabox-nccl_amd/lib -lnbxccl -Wl,-rpath,$PWD/neuronabox-nccl_amd/lib -o scripts/probe_host_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nbx_reduce.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(2); } } while (0)

__global__ void kEmpty(int) {}

template <class F>
double usPerCall(F f, int n, hipStream_t st) {
  for (int i = 0; i < 50; i++) f();
  CK(hipStreamSynchronize(st));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) f();
  const auto t1 = std::chrono::steady_clock::now();
  CK(hipStreamSynchronize(st));
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t count = 1 << 16;   // 256 KiB fp32 per source
  std::vector<void*> src(8);
  for (auto& p : src) CK(hipMalloc(&p, count * 4));
  void* dst;
  CK(hipMalloc(&dst, count * 4));
  nbxDevRedOpFull op{};
  op.op = 0;
  const int n = 2000;
  printf("{\"what\": \"host us per call, %d back-to-back calls\"", n);
  printf(", \"hipLaunchKernel_empty\": %.3f", usPerCall([&] { hipLaunchKernelGGL(kEmpty, dim3(1), dim3(64), 0, st, 0); }, n, st));
  printf(", \"hipStreamGetDevice\": %.3f", usPerCall([&] { hipDevice_t d; (void)hipStreamGetDevice(st, &d); }, n, st));
  printf(", \"hipGetDevice\": %.3f", usPerCall([&] { int d; (void)hipGetDevice(&d); }, n, st));
  printf(", \"hipStreamIsCapturing\": %.3f", usPerCall([&] { hipStreamCaptureStatus c; (void)hipStreamIsCapturing(st, &c); }, n, st));
  for (int ns : {2, 8}) {
    printf(", \"nbxReduceMulti_%dsrc_256KiB\": %.3f", ns,
           usPerCall([&] { (void)nbxReduceMulti(&dst, 1, (const void* const*)src.data(), ns, count, ncclFloat32, op, 0, 0, st); },
                     n, st));
  }
  // a config-B-sized launch takes the dynamic schedule (>= 16 tiles per workgroup)
  const size_t big = 64ull << 20;
  std::vector<void*> bsrc(8);
  for (auto& p : bsrc) CK(hipMalloc(&p, big * 4));
  void* bdst;
  CK(hipMalloc(&bdst, big * 4));
  printf(", \"nbxReduceMulti_8src_256MiB_dynamic\": %.3f",
         usPerCall([&] { (void)nbxReduceMulti(&bdst, 1, (const void* const*)bsrc.data(), 8, big, ncclFloat32, op, 0, 0, st); },
                   50, st));
  std::vector<nbxReduceTask> tasks(128);
  std::vector<void*> dsts(128);
  for (int i = 0; i < 128; i++) {
    CK(hipMalloc(&dsts[i], 16384 * 4));
    tasks[i].dsts = &dsts[i];
    tasks[i].nDsts = 1;
    tasks[i].srcs = (const void* const*)src.data();
    tasks[i].nSrcs = 2;
    tasks[i].count = 16384;
  }
  printf(", \"nbxReduceMultiBatch_128x64KiB_2src\": %.3f",
         usPerCall([&] { (void)nbxReduceMultiBatch(tasks.data(), 128, ncclFloat32, op, 0, 0, st); }, 500, st));
  printf("}\n");
  return 0;
}
