// The GPU half of the native worker: linked only into the `mxar-gpu` executable (the `mxar`
// executable is host-only and leaves make_gpu_worker unresolved - a weak declaration in
// mxar_main.cc). `mxar-gpu worker [port sourceDataSize] --device k` is the reference's
// worker (AllreduceWorker.scala:272-301) with its rounds on GPU k: an XgmiRoundPlane
// (csrc/hip/xgmi_plane.h) under a PlaneWorkerActor, the demo source data[i] = i + iteration
// produced by the fill_iota kernel - no Python anywhere in the round path.
#include <hip/hip_runtime.h>

#include <memory>
#include <stdexcept>
#include <string>

#include "../hip/device_plane.h"
#include "../hip/xgmi_comm.h"
#include "../hip/xgmi_plane.h"
#include "../runtime/round_plane.h"
#include "gpu_worker.h"

namespace mxar {


GpuWorkerParts make_gpu_worker(int device, int size, int max_peers, int max_lag, int grid, double timeout_s,
                               int64_t min_chunk) {
  XgmiPlaneOptions o;
  o.device = device;
  o.dtype = DType::F32;
  o.capacity = size;
  o.max_peers = max_peers;
  o.max_lag = max_lag;
  o.grid = grid;
  o.timeout_s = timeout_s;
  o.min_chunk = min_chunk;
  GpuWorkerParts p;
  p.plane = make_xgmi_plane(o);
  hipStream_t s = nullptr;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
    throw std::runtime_error("mxar-gpu: cannot create a stream on device " + std::to_string(device));
  // every round's input: a stream-ordered buffer filled by the fill_iota kernel, released
  // (stream-ordered) once the plane no longer holds it; the ready event orders the round
  p.source = [device, size, s](const AllReduceInputRequest& r) {
    void* mem = nullptr;
    if (hipMallocAsync(&mem, static_cast<size_t>(size) * sizeof(float), s) != hipSuccess)
      throw std::runtime_error("mxar-gpu: hipMallocAsync failed");
    launch_fill_iota(mem, size, static_cast<double>(r.iteration), DType::F32, s);
    std::shared_ptr<void> owner(mem, [s](void* q) { (void)hipFreeAsync(q, s); });
    return AllReduceInput{std::make_shared<DevicePayload>(owner, 0, static_cast<size_t>(size), device, s,
                                                          record_ready(s), 0)};
  };
  return p;
}

}  // namespace mxar
