// Flag hand-off latency between two workgroups of one GPU (the threshold round's critical
// path is a chain of such hand-offs): workgroup 0 stores flag = i, workgroup 1 waits for it
// and answers ack = i, workgroup 0 waits for the ack; iters round trips, timed with
// s_memrealtime (100 MHz). Variants:
//   mode 0: system-scope relaxed store / load, fine-grained memory (the slab flags)
//   mode 1: mode 0 + a system-scope release fence before each store (publish_flags)
//   mode 2: mode 1 + a system-scope acquire after each observed flag
//   mode 3: agent-scope relaxed store / load, coarse-grained memory (control words)
//   mode 4: mode 0 with a 1 KiB write-through payload stored before each flag
// Output: one JSON line per mode, us per one-way hand-off.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/flag_latency tools/flag_latency.hip && /tmp/flag_latency
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <int MODE>
__global__ void pingpong(uint32_t* w, uint32_t* payload, int iters, uint64_t* out) {
  constexpr int scope = MODE == 3 ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_SYSTEM;
  uint32_t* mine = w + (blockIdx.x == 0 ? 0 : 64);
  uint32_t* theirs = w + (blockIdx.x == 0 ? 64 : 0);
  const uint64_t limit = __builtin_amdgcn_s_memrealtime() + 200000000ull;  // 2 s: every wave exits
  uint64_t t0 = 0;
  bool ok = true;
  for (int i = 1; i <= iters && ok; ++i) {
    if (i == 2 && threadIdx.x == 0) t0 = __builtin_amdgcn_s_memrealtime();
    const bool first = blockIdx.x == 0;
    if (!first) {  // wait, then answer
      if (threadIdx.x == 0) {
        while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, scope) != static_cast<uint32_t>(i)) {
          if (__builtin_amdgcn_s_memrealtime() > limit) { ok = false; break; }
        }
        if (MODE == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      }
    }
    __syncthreads();
    if (MODE == 4) {
      __builtin_nontemporal_store(static_cast<uint32_t>(i), payload + blockIdx.x * 256 + threadIdx.x);
    }
    if (threadIdx.x == 0) {
      if (MODE == 1 || MODE == 2 || MODE == 4) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(mine, static_cast<uint32_t>(i), __ATOMIC_RELAXED, scope);
    }
    if (first && threadIdx.x == 0) {
      while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, scope) != static_cast<uint32_t>(i)) {
        if (__builtin_amdgcn_s_memrealtime() > limit) { ok = false; break; }
      }
      if (MODE == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = ok ? __builtin_amdgcn_s_memrealtime() - t0 : 0;
}

template <int MODE>
int run(uint32_t* fine, uint32_t* coarse, uint32_t* payload, uint64_t* out, int iters) {
  uint32_t* w = MODE == 3 ? coarse : fine;
  CHECK(hipMemset(w, 0, 512));
  hipLaunchKernelGGL(pingpong<MODE>, dim3(2), dim3(256), 0, 0, w, payload, iters, out);
  CHECK(hipDeviceSynchronize());
  uint64_t t = 0;
  CHECK(hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost));
  const double us = t / 100.0 / (2.0 * (iters - 1));
  std::printf("{\"mode\": %d, \"iters\": %d, \"us_one_way\": %.3f}\n", MODE, iters, t ? us : -1.0);
  return 0;
}

int main() {
  uint32_t *fine = nullptr, *coarse = nullptr, *payload = nullptr;
  uint64_t* out = nullptr;
  CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), 4096, hipDeviceMallocFinegrained));
  CHECK(hipMalloc(&coarse, 4096));
  CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&payload), 8192, hipDeviceMallocFinegrained));
  CHECK(hipMalloc(&out, 8));
  const int iters = 2000;
  if (run<0>(fine, coarse, payload, out, iters) || run<1>(fine, coarse, payload, out, iters) ||
      run<2>(fine, coarse, payload, out, iters) || run<3>(fine, coarse, payload, out, iters) ||
      run<4>(fine, coarse, payload, out, iters))
    return 1;
  return 0;
}
