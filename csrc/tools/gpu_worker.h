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

struct GpuWorkerOptions {
  int device = 0, size = 10, max_peers = 8, max_lag = 4, grid = 0;
  double timeout_s = 60.0;
  int64_t min_chunk = 0;
  bool static_source = false;  // the same buffer every round (data[i] = i, or source_value)
  bool has_value = false;      // --source-value V: a static source holding V everywhere
  double source_value = 0.0;
  double source_delay_us = 0.0;  // --source-delay-us D: every fetch waits D us first (a straggler)
  double lag_wait_us = -1.0;     // --lag-wait-us W: XgmiPlaneOptions::lag_wait_us
  int dtype = 0;
};

GpuWorkerParts make_gpu_worker(const GpuWorkerOptions& g) __attribute__((weak));

}  // namespace mxar
