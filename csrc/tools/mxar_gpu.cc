// The GPU half of the native worker: linked only into the `mxar-gpu` executable (the `mxar`
// executable is host-only and leaves make_gpu_worker unresolved - a weak declaration in
// mxar_main.cc). `mxar-gpu worker [port sourceDataSize] --device k` is the reference's
// worker (AllreduceWorker.scala:272-301) with its rounds on GPU k: an XgmiRoundPlane
// (csrc/hip/xgmi_plane.h) under a PlaneWorkerActor, the demo source data[i] = i + iteration
// produced by the fill_iota kernel - no Python anywhere in the round path.
#include "../core/delay.h"
#include "../core/env.h"
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <vector>
#include <stdexcept>
#include <string>

#include "../hip/device_plane.h"
#include "../hip/xgmi_comm.h"
#include "../hip/xgmi_plane.h"
#include "../runtime/round_plane.h"
#include "gpu_worker.h"

namespace mxar {


namespace {
// Round inputs of the iota source: a few device buffers reused round after round. A buffer
// comes back when the plane drops the round's input (after the round's completion word: the
// kernel has read it), so its next fill cannot overwrite data a round still reads. Fills run
// on a stream of the source's own, not the plane's: a small round's kernel stays resident on
// the plane stream between rounds (xgmi_plane.cc launch_resident), and a fill queued behind
// it would not run until it left; the plane waits for the fill's stream instead.
struct InputPool {
  std::mutex mu;
  std::vector<void*> free;
  ~InputPool() {
    for (void* p : free) (void)hipFree(p);
  }
};
}  // namespace

GpuWorkerParts make_gpu_worker(const GpuWorkerOptions& g) {
  // dtype: 0 float32 (the reference's element type), 1 bfloat16, 2 float16 - the plane's
  // element type and the source's (the kernel sums in fp32 and rounds once)
  const int device = g.device, size = g.size, max_peers = g.max_peers, max_lag = g.max_lag, grid = g.grid;
  const double timeout_s = g.timeout_s;
  const int64_t min_chunk = g.min_chunk;
  const bool static_source = g.static_source || g.has_value;
  const int dtype = g.dtype;
  const double delay_us = g.source_delay_us;
  XgmiPlaneOptions o;
  o.device = device;
  o.dtype = static_cast<DType>(dtype);
  o.capacity = size;
  o.max_peers = max_peers;
  o.max_lag = max_lag;
  o.grid = grid;
  o.timeout_s = timeout_s;
  o.min_chunk = min_chunk;
  o.lag_wait_us = g.lag_wait_us;
  GpuWorkerParts p;
  auto plane = make_xgmi_plane(o);
  p.plane = plane;
  hipStream_t s = nullptr;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    throw std::runtime_error("mxar-gpu: no stream on device " + std::to_string(device));
  auto src_stream = std::shared_ptr<void>(s, [](void* q) { (void)hipStreamDestroy(static_cast<hipStream_t>(q)); });
  if (const char* path = study_env("MXAR_PLANE_STAMPS")) {
    // study knob: phase stamps of this worker's round kernels (kPhaseSlots u64 per workgroup,
    // s_memrealtime - one clock for every process on the GPU), the last round's written as one
    // JSON line to `path` when the job ends (tools/phase_profile.py reads the same layout)
    constexpr int64_t kSlots = 2048;
    uint64_t* buf = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&buf), kSlots * 8 * sizeof(uint64_t)) != hipSuccess ||
        hipMemset(buf, 0, kSlots * 8 * sizeof(uint64_t)) != hipSuccess)
      throw std::runtime_error("mxar-gpu: stamps buffer");
    plane->set_phase_stamps(buf, kSlots);
    const std::string out = path;
    p.at_exit = [buf, out, device]() {
      std::vector<uint64_t> h(kSlots * 8);
      (void)hipSetDevice(device);
      if (hipMemcpy(h.data(), buf, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return;
      if (FILE* f = std::fopen(out.c_str(), "a")) {
        std::fprintf(f, "{\"pid\": %d, \"stamps\": [", static_cast<int>(getpid()));
        bool first = true;
        for (int64_t w = 0; w < kSlots; ++w) {
          if (h[w * 8] == 0) continue;
          std::fprintf(f, "%s[", first ? "" : ",");
          for (int k = 0; k < 8; ++k) std::fprintf(f, "%s%llu", k ? "," : "", static_cast<unsigned long long>(h[w * 8 + k]));
          std::fprintf(f, "]");
          first = false;
        }
        std::fprintf(f, "]}\n");
        std::fclose(f);
      }
    };
  }
  const size_t bytes = static_cast<size_t>(size) * dtype_size(o.dtype);
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("mxar-gpu: no device " + std::to_string(device));
  if (static_source) {
    // --source static: data[i] = i, filled once - the same buffer every round (the bench's
    // tensor dataSource; isolates the engine from the per-round fill)
    void* mem = nullptr;
    if (hipMalloc(&mem, bytes) != hipSuccess) throw std::runtime_error("mxar-gpu: hipMalloc failed");
    if (g.has_value)
      launch_fill_affine(mem, size, 0.0, g.source_value, o.dtype, s);
    else
      launch_fill_iota(mem, size, 0.0, o.dtype, s);
    if (hipStreamSynchronize(s) != hipSuccess) throw std::runtime_error("mxar-gpu: source fill failed");
    std::shared_ptr<void> owner(mem, [](void* q) { (void)hipFree(q); });
    auto payload = std::make_shared<DevicePayload>(owner, 0, static_cast<size_t>(size), device, nullptr, nullptr, dtype);
    p.source = [payload, delay_us](const AllReduceInputRequest&) {
      precise_delay_us(delay_us);
      return AllReduceInput{payload};
    };
    return p;
  }
  // the demo source (AllreduceWorker.scala:272-301): data[i] = i + iteration, produced by the
  // fill_iota kernel on the plane's stream into a pooled buffer
  auto pool = std::make_shared<InputPool>();
  const DType dt = o.dtype;
  p.source = [device, size, s, src_stream, bytes, pool, dt, dtype, delay_us](const AllReduceInputRequest& r) {
    precise_delay_us(delay_us);
    void* mem = nullptr;
    {
      std::lock_guard<std::mutex> g(pool->mu);
      if (!pool->free.empty()) {
        mem = pool->free.back();
        pool->free.pop_back();
      }
    }
    if (mem == nullptr && hipMalloc(&mem, bytes) != hipSuccess) throw std::runtime_error("mxar-gpu: hipMalloc failed");
    launch_fill_iota(mem, size, static_cast<double>(r.iteration), dt, s);
    std::shared_ptr<void> owner(mem, [pool](void* q) {
      std::lock_guard<std::mutex> g(pool->mu);
      pool->free.push_back(q);
    });
    return AllReduceInput{std::make_shared<DevicePayload>(owner, 0, static_cast<size_t>(size), device, s, nullptr, dtype)};
  };
  return p;
}

}  // namespace mxar
