// Hook between the native worker executable (mxar_main.cc) and its GPU round engine
// (mxar_gpu.cc). make_gpu_worker is weak: only `mxar-gpu` links the definition.
#pragma once
#include <functional>
#include <memory>

#include "../runtime/allreduce_actors.h"
#include "../runtime/round_plane.h"

namespace mxar {

struct GpuWorkerParts {
  std::shared_ptr<RoundPlane> plane;  // an XgmiRoundPlane on the chosen device
  DataSource source;                  // data[i] = i + iteration, produced on the device
  std::function<void()> at_exit;      // after the job (MXAR_PLANE_STAMPS: write the last round's stamps)
};

GpuWorkerParts make_gpu_worker(int device, int size, int max_peers, int max_lag, int grid, double timeout_s,
                               int64_t min_chunk, bool static_source, int dtype)
    __attribute__((weak));

}  // namespace mxar
