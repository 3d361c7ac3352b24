// LoopbackRoundPlane: the RoundPlane contract (round_plane.h) in host memory, for the
// workers of one process - the CPU twin of XgmiRoundPlane (csrc/hip/xgmi_plane.*).
//
// What it is for: PlaneWorkerActor (the reference worker at round granularity,
// plane_worker.h) runs unchanged on a machine without a GPU - CPU tests of the round
// engine's control logic (stash before Init, epochs, catch-up, cold rounds, out-of-order
// sinks), sanitizer builds, and `mxar-worker --plane loopback` demos.
//
// Model of one round r (per membership epoch), mirroring the threshold kernel's rules
// (csrc/hip/xgmi_threshold.hip) at block granularity:
//   * a worker's round becomes ACTIVE when its previous round completed (the GPU plane's
//     stream order); an active, non-cold round contributes the worker's input;
//   * owner j reduces its block once its own round is active and exactly the first
//     f32(thReduce * P) contributions (arrival order) are in, or with everything present
//     when its round is forced / cold; every chunk of the block then counts that many;
//   * worker i's round completes once f32(thComplete * P * nch) reduced chunks exist,
//     taking the first that many in reduction order; a forced or cold round completes at
//     once with what is reduced (its own block excluded when only the force reduced it);
//     chunks not taken are zeros with count 0;
//   * force(r) forces this worker's rounds <= r; a worker launching round r forces every
//     peer whose progress is behind r - (maxLag + 1) (the lag gate's FORCE request).
// Completions are delivered on the plane's own thread, in launch order.
//
// Descriptor: "loop1 hub=<name> id=<n>". Every worker of one job names the same hub; the
// planes of a hub must live in one process.
#pragma once

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "round_plane.h"

namespace mxar {

class LoopbackHub;

struct LoopbackPlaneStats {
  uint64_t launches = 0, cold = 0, forced_rounds = 0, peer_forces = 0, completed = 0;
};

class LoopbackRoundPlane final : public RoundPlane {
 public:
  explicit LoopbackRoundPlane(const std::string& hub);
  ~LoopbackRoundPlane() override;
  const char* name() const override { return "loopback"; }
  std::string descriptor() const override { return desc_; }
  void set_done(DoneFn fn) override;
  void configure(const PlaneConfig& cfg) override;
  void launch(int round, const Payload& input, bool cold) override;
  void force(int round) override;
  void drain() override;
  int chunks() const override { return nch_; }
  LoopbackPlaneStats stats() const;

 private:
  friend class LoopbackHub;
  struct Pending {
    int round = 0;
    Payload input;
    bool cold = false;
    bool active = false;
    bool done = false;
    RoundResult res;
  };
  void deliver_loop();

  std::shared_ptr<LoopbackHub> hub_;
  std::string desc_;
  uint64_t uid_ = 0;
  PlaneConfig cfg_;
  bool configured_ = false;
  int nch_ = 0;
  // below: guarded by the hub's mutex
  std::deque<Pending> q_;
  int forced_upto_ = -1;
  int progress_ = -1;  // last completed round of this epoch
  LoopbackPlaneStats st_;
  // delivery
  std::condition_variable cv_, cv_idle_;
  bool stop_ = false;
  std::mutex done_mu_;
  DoneFn done_;
  std::thread th_;
};

std::shared_ptr<LoopbackRoundPlane> make_loopback_plane(const std::string& hub);

}  // namespace mxar
