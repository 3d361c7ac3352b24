// Probe of the copy-engine (SDMA) primitives the SDMA bucket allreduce needs, on one MI355X:
//   1. a same-device copy forced onto an SDMA engine (hsa_amd_memory_async_copy_on_engine,
//      force_copy_on_sdma) - HIP's hipMemcpyAsync uses a blit KERNEL for device-to-device
//      copies whatever GPU_BLIT_ENGINE_TYPE says (profiles/round4/README.md);
//   2. stream ordering without the host: the copy depends on an HSA signal that a one-lane
//      kernel on the HIP stream releases, and a chained 4-byte copy writes an epoch flag into
//      device memory that the stream then waits for with hipStreamWaitValue32 (the command
//      processor polls; no CU spins);
//   3. copy bandwidth on 1 / 2 / 4 / 8 engines.
// Build: hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.cc -lhsa-runtime64 -o build/sdma_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)
#define HSACHK(x)                                                                  \
  do {                                                                             \
    hsa_status_t s_ = (x);                                                         \
    if (s_ != HSA_STATUS_SUCCESS) {                                                \
      const char* m_ = nullptr;                                                    \
      hsa_status_string(s_, &m_);                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, m_ ? m_ : "?");                         \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ void release_kernel(int64_t* p) {
  if (threadIdx.x == 0) __hip_atomic_store(p, int64_t{0}, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static hsa_status_t find_gpu(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  auto* v = static_cast<std::vector<hsa_agent_t>*>(data);
  if (t == HSA_DEVICE_TYPE_GPU) v->push_back(a);
  return HSA_STATUS_SUCCESS;
}

int main() {
  HIPCHK(hipSetDevice(0));
  HIPCHK(hipFree(nullptr));
  HSACHK(hsa_init());
  std::vector<hsa_agent_t> gpus;
  HSACHK(hsa_iterate_agents(find_gpu, &gpus));
  if (gpus.empty()) return 1;
  hsa_agent_t g = gpus[0];
  uint32_t mask = 0;
  HSACHK(hsa_amd_memory_copy_engine_status(g, g, &mask));
  std::vector<hsa_amd_sdma_engine_id_t> engines;
  for (int b = 0; b < 16; ++b)
    if (mask & (1u << b)) engines.push_back(static_cast<hsa_amd_sdma_engine_id_t>(1u << b));
  std::printf("{\"gpus\": %zu, \"engine_mask\": %u, \"engines\": %zu}\n", gpus.size(), mask, engines.size());
  if (engines.empty()) return 1;

  const size_t bytes = size_t{256} << 20;
  char *a = nullptr, *b = nullptr;
  uint32_t *flag = nullptr, *epoch_src = nullptr;
  HIPCHK(hipMalloc(&a, bytes));
  HIPCHK(hipMalloc(&b, bytes));
  HIPCHK(hipMalloc(&flag, 64));
  HIPCHK(hipMalloc(&epoch_src, 64));
  HIPCHK(hipMemset(a, 0x5a, bytes));
  HIPCHK(hipMemset(b, 0, bytes));
  HIPCHK(hipMemset(flag, 0, 64));
  const uint32_t epoch = 7;
  HIPCHK(hipMemcpy(epoch_src, &epoch, 4, hipMemcpyHostToDevice));
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // 2. ordering: sleep kernel -> release -> [SDMA copy -> SDMA flag copy] -> stream waits flag
  hsa_signal_t start, done, done2;
  HSACHK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &start));
  HSACHK(hsa_signal_create(1, 0, nullptr, &done));
  HSACHK(hsa_signal_create(1, 0, nullptr, &done2));
  volatile hsa_signal_value_t* startp = nullptr;
  HSACHK(hsa_amd_signal_value_pointer(start, &startp));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HSACHK(hsa_amd_memory_async_copy_on_engine(b, g, a, g, bytes, 1, &start, done, engines[0], true));
  HSACHK(hsa_amd_memory_async_copy_on_engine(flag, g, epoch_src, g, 4, 1, &done, done2, engines[0], true));
  HIPCHK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(release_kernel, dim3(1), dim3(64), 0, s, const_cast<int64_t*>(reinterpret_cast<volatile int64_t*>(startp)));
  HIPCHK(hipStreamWaitValue32(s, flag, epoch, hipStreamWaitValueEq, 0xffffffffu));
  HIPCHK(hipEventRecord(e1, s));
  HIPCHK(hipStreamSynchronize(s));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned char> h(4096);
  HIPCHK(hipMemcpy(h.data(), b + bytes - 4096, 4096, hipMemcpyDeviceToHost));
  bool ok = true;
  for (unsigned char c : h) ok = ok && c == 0x5a;
  std::printf("{\"test\": \"ordered\", \"ms\": %.4f, \"GBps\": %.1f, \"data_ok\": %s, \"done\": %ld}\n", ms,
              bytes / (ms * 1e6), ok ? "true" : "false", static_cast<long>(hsa_signal_load_relaxed(done)));

  // 3. bandwidth on k engines (the buffer split in k parts, one per engine), host-timed
  for (size_t k : {size_t{1}, size_t{2}, size_t{4}, size_t{8}, engines.size()}) {
    if (k > engines.size()) continue;
    const size_t part = bytes / k;
    hsa_signal_t sig;
    HSACHK(hsa_signal_create(static_cast<hsa_signal_value_t>(k), 0, nullptr, &sig));
    const int iters = 5;
    double best = 1e9;
    for (int it = 0; it < iters; ++it) {
      hsa_signal_store_relaxed(sig, static_cast<hsa_signal_value_t>(k));
      auto t0 = std::chrono::steady_clock::now();
      for (size_t e = 0; e < k; ++e)
        HSACHK(hsa_amd_memory_async_copy_on_engine(b + e * part, g, a + e * part, g, part, 0, nullptr, sig,
                                                   engines[e], true));
      hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_EQ, 0, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
      const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      best = t < best ? t : best;
    }
    std::printf("{\"test\": \"bandwidth\", \"engines\": %zu, \"best_ms\": %.4f, \"GBps\": %.1f}\n", k, best,
                bytes / (best * 1e6));
    hsa_signal_destroy(sig);
  }
  return 0;
}
