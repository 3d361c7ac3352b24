#include "master_core.h"

#include <algorithm>

#include "log.h"
#include "trace.h"

namespace mxar {

// MemberUp -> register (AllreduceMaster.scala:38-48, 70-82)
void MasterCore::on_member_up(int handle) {
  for (auto& [id, h] : workers_)
    if (h == handle) return;  // already registered
  // id = workers.size in the reference (:75-76); after a removal that id can collide
  // with a live worker, so take the first free id instead.
  int id = 0;
  while (workers_.count(id)) ++id;
  workers_[id] = handle;
  MXAR_LOG(INFO, "master", "----current size = " << workers_.size());
  if (p_.resumeOnJoin && round_ >= 0 && !finished_) {  // a join mid-job: everyone resumes here
    MXAR_LOG(INFO, "master", "----worker joined at round " << round_ << ": re-initialising "
                                                           << workers_.size() << " workers there");
    stats_.join_reinits++;
    init_workers(resume_round());
    if (!external_idle()) start_allreduce();
    return;
  }
  const int need = round_ < 0 ? std::max(p_.initWorkers, f32_threshold_count(p_.thAllreduce, p_.totalWorkers))
                              : f32_threshold_count(p_.thAllreduce, p_.totalWorkers);
  if (static_cast<int>(workers_.size()) >= need) {
    MXAR_LOG(INFO, "master", "----" << workers_.size() << " (out of " << p_.totalWorkers << ") workers are up");
    init_workers();
    round_ = std::max(0, p_.startRound);
    last_reported_ = round_ - 1;
    finished_ = false;
    if (p_.externalRounds) {  // the client starts the first round
      awaiting_ = true;
      started_ = false;
      return;
    }
    start_allreduce();
  }
}

MasterCore::StartResult MasterCore::on_external_start(int round, std::string* why) {
  auto refuse = [&](std::string r) {
    if (why) *why = std::move(r);
    return StartResult::Refused;
  };
  if (!p_.externalRounds) return refuse("master is not in externalRounds mode");
  if (round_ < 0 || workers_.empty()) return refuse("workers are not initialised");
  if (finished_) return refuse("job finished");
  if (round > p_.maxRound) return refuse("round beyond maxRound " + std::to_string(p_.maxRound));
  if (started_ ? round <= round_ : round < round_)
    return refuse("round " + std::to_string(round) + " is not after round " + std::to_string(round_));
  if (!awaiting_) {  // round_ in flight: queue one start behind its barrier
    if (queued_ >= 0) return refuse("round " + std::to_string(queued_) + " is already queued");
    queued_ = round;
    return StartResult::Queued;
  }
  round_ = round;
  awaiting_ = false;
  started_ = true;
  start_allreduce();
  return StartResult::Started;
}

// Terminated (AllreduceMaster.scala:50-56)
void MasterCore::on_terminated(int handle) {
  bool removed = false;
  for (auto it = workers_.begin(); it != workers_.end(); ++it) {
    if (it->second == handle) {
      MXAR_LOG(INFO, "master", "----worker " << it->first << " is terminated, removing it from the set");
      workers_.erase(it);
      stats_.removed++;
      removed = true;
      break;
    }
  }
  if (removed && p_.reinitOnLoss && round_ >= 0 && !finished_ && !workers_.empty()) {
    // the survivors become a new epoch that resumes at the current round (its partial
    // completions belong to the old epoch and are discarded)
    MXAR_LOG(WARNING, "master", "----re-initialising the " << workers_.size() << " surviving workers at round "
                                                             << round_);
    stats_.loss_reinits++;
    init_workers(resume_round());
    if (!external_idle()) start_allreduce();
    return;
  }
  // With liveBarrier the round may now be complete.
  if (p_.liveBarrier && round_ >= 0 && !finished_ &&
      static_cast<float>(numComplete_) >= barrier_base() * p_.thAllreduce && numComplete_ > 0) {
    on_complete(-1, -1);
  }
}

float MasterCore::barrier_base() const {
  if (p_.liveBarrier || p_.reinitOnLoss)
    return static_cast<float>(std::min<int>(p_.totalWorkers, static_cast<int>(workers_.size())));
  return static_cast<float>(p_.totalWorkers);
}

// CompleteAllreduce (AllreduceMaster.scala:58-67)
void MasterCore::on_complete(int srcId, int round, int64_t epoch) {
  if (epoch >= 0 && epoch != epoch_ && round >= 0) {  // sent before the last re-init
    stats_.stale_completes++;
    return;
  }
  if (srcId >= 0) {
    MXAR_LOG(INFO, "master", "----Node " << srcId << " completes allreduce round " << round);
    if (Tracer::get().enabled())
      trace_instant("master", "complete r" + std::to_string(round), "{\"worker\":" + std::to_string(srcId) + "}");
    stats_.completes++;
    if (round != round_ || (p_.externalRounds && (awaiting_ || !started_))) {
      stats_.stale_completes++;
      fx_->complete_seen(srcId, round, false);
      return;
    }
    numComplete_ += 1;
    fx_->complete_seen(srcId, round, true);
  }
  // numComplete >= totalWorkers * thAllreduce : float compare, not truncated (:62)
  volatile float need = barrier_base() * p_.thAllreduce;
  if (static_cast<float>(numComplete_) >= need && !(p_.externalRounds && awaiting_)) advance();
}

void MasterCore::advance() {
  if (last_reported_ < round_) {
    last_reported_ = round_;
    fx_->round_completed(round_, epoch_);
  }
  if (p_.externalRounds && round_ < p_.maxRound) {  // the client's next start, or wait for it
    if (queued_ > round_) {
      const int r = queued_;
      queued_ = -1;
      round_ = r;
      start_allreduce();
      fx_->queued_start_done(r, true, "");
      return;
    }
    awaiting_ = true;
    return;
  }
  if (p_.externalRounds && queued_ >= 0) {  // cannot happen (queued <= maxRound), kept safe
    fx_->queued_start_done(queued_, false, "job finished");
    queued_ = -1;
  }
  if (round_ < p_.maxRound) {
    MXAR_LOG(INFO, "master", "----" << numComplete_ << " (out of " << p_.totalWorkers
                                    << ") workers complete round " << round_);
    round_ += 1;
    start_allreduce();
  } else if (!finished_) {
    finished_ = true;
    MXAR_LOG(INFO, "master", "----All " << (p_.maxRound + 1) << " rounds complete");
    fx_->finished(p_.maxRound + 1);
  }
}

// Round deadline: a round that has not reached the barrier roundTimeoutMs after
// its start is advanced anyway - the coordinator-level counterpart of the workers' maxLag
// catch-up (stragglers then force-complete it when the next Start arrives).
void MasterCore::on_round_timeout(int64_t epoch, int round) {
  if (epoch != epoch_ || round != round_ || finished_ || round_ < 0 || awaiting_) return;  // already advanced
  stats_.round_timeouts++;
  MXAR_LOG(WARNING, "master", "----Round " << round << " timed out with " << numComplete_ << " of "
                                             << workers_.size() << " completions; advancing");
  advance();
}

// init_workers (AllreduceMaster.scala:84-89)
void MasterCore::init_workers(int startRound) {
  if (queued_ >= 0) {  // a new membership epoch: the client re-drives from its InitWorkers
    fx_->queued_start_done(queued_, false, "workers re-initialised");
    queued_ = -1;
  }
  // re-number densely 0..P-1 in id order
  std::map<int, int> dense;
  int k = 0;
  for (auto& [id, h] : workers_) dense[k++] = h;
  workers_.swap(dense);
  if (epoch_ > 0)  // skip past every device round epoch the previous membership epoch could use
    round_base_ += static_cast<uint32_t>(std::max(0, round_ - epoch_start_round_ + 1)) + 1u;
  epoch_start_round_ = startRound;
  ++epoch_;
  stats_.inits++;
  for (auto& [idx, h] : workers_) {
    MXAR_LOG(INFO, "master", "----Init worker " << idx << " (epoch " << epoch_ << ")");
    InitParams p;
    p.destId = idx;
    p.numPeers = static_cast<int>(workers_.size());
    p.thReduce = p_.thReduce;
    p.thComplete = p_.thComplete;
    p.maxLag = p_.maxLag;
    p.dataSize = p_.dataSize;
    p.maxChunkSize = p_.maxChunkSize;
    p.epoch = epoch_;
    p.startRound = startRound;
    p.roundBase = round_base_;
    fx_->send_init(h, p, workers_);
  }
  InitParams p;
  p.numPeers = static_cast<int>(workers_.size());
  p.thReduce = p_.thReduce;
  p.thComplete = p_.thComplete;
  p.maxLag = p_.maxLag;
  p.dataSize = p_.dataSize;
  p.maxChunkSize = p_.maxChunkSize;
  p.epoch = epoch_;
  p.startRound = startRound;
  p.roundBase = round_base_;
  fx_->workers_initialized(p, workers_);
}

// startAllreduce (AllreduceMaster.scala:91-97)
void MasterCore::start_allreduce() {
  MXAR_LOG(INFO, "master", "----Start allreduce round " << round_);
  trace_instant("master", "start r" + std::to_string(round_));
  numComplete_ = 0;
  stats_.rounds_started++;
  for (auto& [idx, h] : workers_) fx_->send_start(h, round_);
  if (p_.roundTimeoutMs > 0) fx_->arm_round_timer(epoch_, round_, p_.roundTimeoutMs);
}

}  // namespace mxar
