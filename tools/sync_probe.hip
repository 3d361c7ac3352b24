// Which HIP runtime calls wait for a kernel that is still running on ANOTHER stream?
//
// The round engine's peers spin in persistent kernels until this process does its part.
// A runtime call that implicitly synchronises the device, made while a peer spins, waits for
// that peer, and the peer waits for us: a deadlock until the kernel's deadline. This probe
// launches a spinning kernel on stream A that waits for a pinned host flag and gives up
// after 2 s, so every wave exits. It then times each call. A call that takes about 2 s waited
// for the kernel.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/sync_probe tools/sync_probe.hip && build/sync_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                 \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

__global__ void spin(const uint32_t* flag, uint64_t ticks) {
  const uint64_t until = __builtin_amdgcn_s_memrealtime() + ticks;  // 100 MHz
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u &&
         __builtin_amdgcn_s_memrealtime() < until)
    __builtin_amdgcn_s_sleep(8);
}

int main() {
  CHECK(hipSetDevice(0));
  hipStream_t a = nullptr, b = nullptr;
  CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  uint32_t* flag = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* dflag = nullptr;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0));
  void* keep = nullptr;
  CHECK(hipMalloc(&keep, 64 << 20));
  void* keep2 = nullptr;
  CHECK(hipMalloc(&keep2, 64 << 20));
  void* pooled = nullptr;
  std::vector<std::pair<std::string, std::function<hipError_t()>>> probes = {
      {"hipMalloc 1 MiB", [&] { void* p; return hipMalloc(&p, 1 << 20); }},
      {"hipMalloc 1 GiB", [&] { void* p; return hipMalloc(&p, size_t(1) << 30); }},
      {"hipFree", [&] { hipError_t e = hipFree(keep); keep = nullptr; return e; }},
      {"hipExtMallocWithFlags fine 64 MiB", [&] { void* p; return hipExtMallocWithFlags(&p, 64 << 20, hipDeviceMallocFinegrained); }},
      {"hipMallocAsync 256 MiB (pool growth)", [&] { return hipMallocAsync(&pooled, size_t(256) << 20, b); }},
      {"hipFreeAsync", [&] { return hipFreeAsync(pooled, b); }},
      {"hipMemset (sync API)", [&] { return hipMemset(keep2, 0, 4096); }},
      {"hipMemsetAsync other stream", [&] { return hipMemsetAsync(keep2, 0, 4096, b); }},
      {"hipHostMalloc 1 MiB", [&] { void* p; return hipHostMalloc(&p, 1 << 20, hipHostMallocMapped); }},
      {"hipEventCreate", [&] { hipEvent_t e; return hipEventCreateWithFlags(&e, hipEventDisableTiming); }},
      {"hipStreamCreate", [&] { hipStream_t s; return hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }},
      {"hipIpcGetMemHandle", [&] { hipIpcMemHandle_t h; return hipIpcGetMemHandle(&h, keep2); }},
      {"hipStreamSynchronize other stream", [&] { return hipStreamSynchronize(b); }},
      {"hipDeviceSynchronize (expected to wait)", [&] { return hipDeviceSynchronize(); }},
  };
  for (auto& [name, call] : probes) {
    *flag = 0;
    hipLaunchKernelGGL(spin, dim3(8), dim3(64), 0, a, dflag, uint64_t(200000000));  // 2 s
    CHECK(hipGetLastError());
    std::this_thread::sleep_for(std::chrono::milliseconds(20));  // the kernel is running now
    const auto t0 = std::chrono::steady_clock::now();
    const hipError_t e = call();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *flag = 1;
    CHECK(hipStreamSynchronize(a));
    CHECK(hipStreamSynchronize(b));
    std::printf("{\"call\": \"%s\", \"ms\": %.3f, \"waited_for_kernel\": %s, \"status\": \"%s\"}\n", name.c_str(), ms,
                ms > 1000.0 ? "true" : "false", hipGetErrorString(e));
    std::fflush(stdout);
  }
  return 0;
}
