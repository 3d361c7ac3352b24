// Host cost of the HIP calls on the protocol engine's round path (a 1 MiB
// round spends ~60 us outside its kernel). Each call is timed in a loop of N on one thread,
// (a) alone and (b) while a second thread polls hipEventQuery on a pending event the way the
// plane's completion thread does (contention on the runtime's locks).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/api_cost_probe tools/api_cost_probe.hip -lpthread
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e = (x);                                                                         \
    if (e != hipSuccess) {                                                                      \
      std::fprintf(stderr, "HIP error %s at %s:%d: %s\n", #x, __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(2);                                                                             \
    }                                                                                           \
  } while (0)

__global__ void empty_k() {}
__global__ void spin_k(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

static double us_per(int n, const std::function<void()>& f) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t s, s2;
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
  hipEvent_t ev, ev2;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
  hipMemPool_t mp = nullptr;
  CK(hipDeviceGetDefaultMemPool(&mp, 0));
  uint64_t keep = UINT64_MAX;
  CK(hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep));
  void* warm = nullptr;
  CK(hipMallocAsync(&warm, 8 << 20, s));
  CK(hipFreeAsync(warm, s));
  CK(hipDeviceSynchronize());
  const int N = 2000;
  struct Case {
    const char* name;
    std::function<void()> f;
  };
  std::vector<Case> cases = {
      {"hipMallocAsync+hipFreeAsync 1 MiB (plane stream)",
       [&] {
         void* p = nullptr;
         (void)hipMallocAsync(&p, 1 << 20, s);
         (void)hipFreeAsync(p, s);
       }},
      {"hipFreeAsync on the null stream (after a malloc on the plane stream)",
       [&] {
         void* p = nullptr;
         (void)hipMallocAsync(&p, 1 << 20, s);
         (void)hipFreeAsync(p, nullptr);
       }},
      {"hipLaunchKernel (empty)", [&] { hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s); }},
      {"hipEventRecord", [&] { (void)hipEventRecord(ev, s); }},
      {"hipStreamWaitEvent", [&] { (void)hipStreamWaitEvent(s, ev, 0); }},
      {"hipStreamQuery", [&] { (void)hipStreamQuery(s); }},
      {"hipEventQuery", [&] { (void)hipEventQuery(ev); }},
      {"hipSetDevice", [&] { (void)hipSetDevice(0); }},
      {"hipGetLastError", [&] { (void)hipGetLastError(); }},
      {"hipStreamIsCapturing", [&] {
         hipStreamCaptureStatus st;
         (void)hipStreamIsCapturing(s, &st);
       }},
      {"hipEventCreate+Record+Destroy", [&] {
         hipEvent_t e;
         (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
         (void)hipEventRecord(e, s);
         (void)hipEventDestroy(e);
       }},
  };
  std::printf("{\"rows\": [\n");
  bool first = true;
  for (int contended = 0; contended < 2; ++contended) {
    std::atomic<bool> stop{false};
    std::thread poller;
    if (contended) {
      // a long kernel on the second stream keeps ev2 pending; the poller spins on it
      hipLaunchKernelGGL(spin_k, dim3(1), dim3(64), 0, s2, 100000000ull);  // 1 s
      CK(hipEventRecord(ev2, s2));
      poller = std::thread([&] {
        while (!stop.load()) {
          (void)hipEventQuery(ev2);
          std::this_thread::yield();
        }
      });
    }
    for (auto& c : cases) {
      for (int i = 0; i < 50; ++i) c.f();
      CK(hipStreamSynchronize(s));
      const double us = us_per(N, c.f);
      CK(hipStreamSynchronize(s));
      std::printf("%s {\"call\": \"%s\", \"contended\": %d, \"us\": %.3f}\n", first ? " " : ",", c.name, contended,
                  us);
      first = false;
    }
    if (contended) {
      stop = true;
      poller.join();
    }
    CK(hipDeviceSynchronize());
  }
  std::printf("]}\n");
  return 0;
}
