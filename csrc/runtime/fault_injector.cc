#include "fault_injector.h"

#include <chrono>

namespace mxar {

int message_round(const Message& m) {
  if (auto* s = std::get_if<ScatterBlock>(&m)) return s->round;
  if (auto* r = std::get_if<ReduceBlock>(&m)) return r->round;
  if (auto* c = std::get_if<CompleteAllreduce>(&m)) return c->round;
  if (auto* st = std::get_if<StartAllreduce>(&m)) return st->round;
  return -1;
}

FaultyRef::FaultyRef(ActorSystem* sys, ActorRef target, FaultPolicy policy)
    : sys_(sys), target_(std::move(target)), p_(std::move(policy)), rng_(p_.seed) {}

bool FaultyRef::selected(const Message& m) const {
  if (!p_.kinds.empty() && !p_.kinds.count(message_name(m))) return false;
  const int r = message_round(m);
  const bool ranged = p_.round_lo != INT32_MIN || p_.round_hi != INT32_MAX;
  if (r < 0) return !ranged;  // a round filter selects round-carrying messages only
  return r >= p_.round_lo && r <= p_.round_hi;
}

void FaultyRef::tell(Message msg, ActorRef sender) {
  bool drop = false, dup = false, delay = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    ++st_.seen;
    if (enabled_.load() && selected(msg)) {
      std::uniform_real_distribution<double> u(0.0, 1.0);
      drop = u(rng_) < p_.drop;
      dup = !drop && u(rng_) < p_.duplicate;
      delay = !drop && p_.delay_ms > 0 && u(rng_) < p_.delay_prob;
    }
    if (drop) ++st_.dropped;
    if (dup) ++st_.duplicated;
    if (delay) ++st_.delayed;
    if (!drop) ++st_.forwarded;
  }
  if (drop) return;
  if (delay) {
    // The timer delivers with no sender; keep the original sender by wrapping nothing -
    // the protocol never replies to senders, so only ordering changes.
    sys_->schedule_once(std::chrono::milliseconds(p_.delay_ms), target_, msg);
    if (dup) sys_->schedule_once(std::chrono::milliseconds(p_.delay_ms), target_, std::move(msg));
    return;
  }
  if (dup) target_->tell(msg, sender);
  target_->tell(std::move(msg), std::move(sender));
}

FaultStats FaultyRef::stats() {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

}  // namespace mxar
