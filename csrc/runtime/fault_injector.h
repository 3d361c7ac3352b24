// Fault-injection transport decorator: an ActorRef that forwards to a target
// ref but can drop, duplicate or delay messages, selected by message kind, round range and
// probability (seeded, reproducible). The reference only injects faults by hand in its spec
// (omitting / delaying messages, AllreduceSpec.scala:358-529); this makes straggler, loss and
// reordering scenarios scriptable for whole clusters: hand the master a FaultyRef in the
// MemberUp of a worker and every message to that worker (peers' scatters and reduces, the
// master's Init/Start) goes through the injector.
#pragma once

#include <atomic>
#include <mutex>
#include <random>
#include <set>
#include <string>

#include "actor_system.h"

namespace mxar {

struct FaultPolicy {
  double drop = 0.0;        // probability of dropping a selected message
  double duplicate = 0.0;   // probability of delivering a selected message twice
  int delay_ms = 0;         // delay every selected message (reorders it after later ones)
  double delay_prob = 1.0;  // probability that a selected message is delayed
  std::set<std::string> kinds;  // message names ("ScatterBlock", ...); empty = all
  int round_lo = INT32_MIN, round_hi = INT32_MAX;  // only messages of these rounds
  uint64_t seed = 1;
};

struct FaultStats {
  uint64_t seen = 0, forwarded = 0, dropped = 0, duplicated = 0, delayed = 0;
};

class FaultyRef final : public ActorRefBase {
 public:
  FaultyRef(ActorSystem* sys, ActorRef target, FaultPolicy policy);
  void tell(Message msg, ActorRef sender) override;
  std::string path() const override { return target_->path(); }
  bool is_remote() const override { return target_->is_remote(); }
  const ActorRef& target() const { return target_; }
  FaultStats stats();
  void set_enabled(bool on) { enabled_ = on; }

 private:
  bool selected(const Message& m) const;
  ActorSystem* sys_;
  ActorRef target_;
  FaultPolicy p_;
  std::mutex mu_;
  std::mt19937_64 rng_;
  FaultStats st_;
  std::atomic<bool> enabled_{true};
};

int message_round(const Message& m);  // -1 for messages without a round

}  // namespace mxar
