// probe_stream_id.hip — does a destroyed stream's handle or id come back for a
// new stream? (the dynamic-tile counters are keyed per stream.)
// Creates and destroys streams, with and without pending work, and prints the
// handle and hipStreamGetId of each; reports reuse of either.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <set>

__global__ void kSpin(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int main() {
  std::set<void*> handles;
  std::set<unsigned long long> ids;
  int handleReuse = 0, idReuse = 0;
  for (int i = 0; i < 64; i++) {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, (i & 1) ? hipStreamNonBlocking : hipStreamDefault) != hipSuccess) return 2;
    unsigned long long id = 0;
    const hipError_t e = hipStreamGetId(s, &id);
    if (e != hipSuccess) {
      std::printf("hipStreamGetId: %s\n", hipGetErrorString(e));
      return 3;
    }
    if (!handles.insert((void*)s).second) handleReuse++;
    if (!ids.insert(id).second) idReuse++;
    if (i % 4 == 0) kSpin<<<1, 64, 0, s>>>(100000ull);   // 1 ms pending at destroy
    if (i < 8) std::printf("stream %d handle %p id %llu\n", i, (void*)s, id);
    (void)hipStreamDestroy(s);
  }
  // does hipStreamDestroy wait for pending work? a 20 ms kernel, then destroy
  double destroyMs = -1.0, kernelLeftMs = -1.0;
  {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
    hipEvent_t done;
    (void)hipEventCreate(&done);
    kSpin<<<1, 64, 0, s>>>(2000000ull);   // 20 ms at 100 MHz
    (void)hipEventRecord(done, s);
    const auto t0 = std::chrono::steady_clock::now();
    (void)hipStreamDestroy(s);
    const auto t1 = std::chrono::steady_clock::now();
    destroyMs = std::chrono::duration<double, std::milli>(t1 - t0).count();
    const bool pending = hipEventQuery(done) == hipErrorNotReady;
    (void)hipEventSynchronize(done);
    kernelLeftMs = pending ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count() : 0.0;
    (void)hipEventDestroy(done);
  }
  std::printf("{\"destroy_with_20ms_pending_ms\": %.3f, \"kernel_still_running_after_destroy_ms\": %.3f}\n", destroyMs,
              kernelLeftMs);
  // (an hipEventRecord on a destroyed stream's handle segfaulted this probe on
  // ROCm 7.2, gpurun_out r3g: the library must never touch a stream it did not
  // just receive from the caller)
  unsigned long long nullId = 0;
  const hipError_t en = hipStreamGetId(nullptr, &nullId);
  (void)hipDeviceSynchronize();
  std::printf("{\"streams\": 64, \"handle_reuse\": %d, \"id_reuse\": %d, \"null_stream_id_rc\": %d, \"null_stream_id\": %llu}\n",
              handleReuse, idReuse, (int)en, nullId);
  return 0;
}
