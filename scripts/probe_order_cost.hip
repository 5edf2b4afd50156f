// probe_order_cost.hip — what it costs per call to leave a marker behind a
// collective so that a later call on ANOTHER stream can wait for it (the
// multi-process communicator orders its calls across streams): a tiny kernel
// launched back to back alone, and followed each time by hipEventRecord with
// several event flags, or by hipStreamWriteValue64 (signal memory). Wall time
// per call (host throughput) and device time per call (events around the
// batch). Also: what hipEventRecord does on a destroyed stream's handle is
// NOT probed here (it crashed this probe's predecessor: never do it).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void kTiny(unsigned* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

int main() {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
  unsigned* d = nullptr;
  (void)hipMalloc(&d, 64);
  void* sig = nullptr;
  const bool haveSig = hipExtMallocWithFlags(&sig, 64, hipMallocSignalMemory) == hipSuccess;
  hipEvent_t t0, t1;
  (void)hipEventCreate(&t0);
  (void)hipEventCreate(&t1);
  struct V {
    const char* name;
    unsigned flags;   // event flags; ~0u = no marker; 1u = write value
  } vs[] = {{"kernel_only", ~0u},
            {"event_disable_timing", hipEventDisableTiming},
            {"event_disable_timing_no_system_fence", hipEventDisableTiming | hipEventDisableSystemFence},
            {"event_disable_timing_release_to_device", hipEventDisableTiming | hipEventReleaseToDevice},
            {"write_value64_signal_mem", 1u}};
  const int iters = 2000;
  for (const V& v : vs) {
    if (v.flags == 1u && !haveSig) continue;
    hipEvent_t ev = nullptr;
    if (v.flags != ~0u && v.flags != 1u) (void)hipEventCreateWithFlags(&ev, v.flags);
    for (int rep = 0; rep < 2; rep++) {
      (void)hipStreamSynchronize(s);
      (void)hipEventRecord(t0, s);
      const auto a = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; i++) {
        kTiny<<<1, 64, 0, s>>>(d);
        if (ev) (void)hipEventRecord(ev, s);
        if (v.flags == 1u) (void)hipStreamWriteValue64(s, sig, (uint64_t)i + 1, 0);
      }
      const auto b = std::chrono::steady_clock::now();
      (void)hipEventRecord(t1, s);
      (void)hipEventSynchronize(t1);
      const auto c = std::chrono::steady_clock::now();
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, t0, t1);
      if (rep == 1)
        std::printf("{\"variant\": \"%s\", \"enqueue_us_per_call\": %.3f, \"wall_us_per_call\": %.3f, "
                    "\"device_us_per_call\": %.3f}\n",
                    v.name, std::chrono::duration<double, std::micro>(b - a).count() / iters,
                    std::chrono::duration<double, std::micro>(c - a).count() / iters, ms * 1e3 / iters);
    }
    if (ev) (void)hipEventDestroy(ev);
  }
  std::fflush(stdout);
  return 0;
}
