// Coordinator state machine: membership -> ids, InitWorkers broadcast, round barrier.
//
//   reference: src/main/scala/sample/cluster/allreduce/AllreduceMaster.scala:15-98
//
// Kept: init trigger at (totalWorkers * thAllreduce).toInt registered workers (truncated,
// :42) and advance when numComplete >= totalWorkers * thAllreduce (float compare, NOT
// truncated, :62) - the asymmetry is protocol-visible; rounds 0..maxRound
// run (maxRound + 1 rounds); every MemberUp past the threshold re-initialises everyone
// at round 0 (now epoch-tagged).
// Fixed: all state changes happen on the coordinator's own turn; ids are
// re-numbered densely 0..P-1 at every (re-)init so removals cannot collide (Q3);
// optional barrier on live membership (Q4, `liveBarrier`); a finished notification
// after maxRound (Q15).
#pragma once

#include <algorithm>

#include <functional>
#include <map>
#include <string>
#include <vector>

#include "worker_core.h"

namespace mxar {

struct MasterParams {
  int totalWorkers = 2;
  float thAllreduce = 1.f;
  float thReduce = 0.9f;
  float thComplete = 0.8f;
  int maxLag = 1;
  int dataSize = 10;
  int maxRound = 100;
  int maxChunkSize = 2;
  bool liveBarrier = false;
  int startRound = 0;  // resume point (checkpoint/resume)
  int roundTimeoutMs = 0;  // > 0: advance a round that misses the barrier this long
  // Extension: when a registered worker terminates, re-initialise the
  // survivors as a new membership epoch that resumes at the current round, and count the
  // barrier over live workers. The reference only re-initialises on MemberUp, so a lost
  // worker leaves its peers waiting on rounds that can never complete (Q4).
  bool reinitOnLoss = false;
  // Extension: a worker that joins while rounds are running (e.g. a restarted one) is taken
  // in by re-initialising everyone at the CURRENT round. The reference restarts the whole
  // job at round 0 on every MemberUp past the threshold (Q2).
  bool resumeOnJoin = false;
  // Extension: rounds are driven from outside (the control bridge,
  // csrc/runtime/control_bridge.h). After init and after every barrier the master waits
  // for an external StartAllreduce(r) instead of starting round + 1 itself, i.e. the
  // client plays AllreduceMaster.scala:58-67,91-97 while this master keeps membership,
  // ids and InitWorkers.
  bool externalRounds = false;
  // Extension: the FIRST initialisation waits for at least this many registered workers
  // (0: the reference's totalWorkers * thAllreduce, AllreduceMaster.scala:42). Below
  // thAllreduce = 1 the reference starts the job with the first workers up and restarts it
  // at round 0 when the next one joins; a deployment that knows its size asks for it here.
  int initWorkers = 0;
};

class MasterEffects {
 public:
  virtual ~MasterEffects() = default;
  // `ids` maps worker id -> handle for the whole membership (the InitWorkers.workers map).
  virtual void send_init(int handle, const InitParams& p, const std::map<int, int>& ids) = 0;
  virtual void send_start(int handle, int round) = 0;
  virtual void finished(int rounds) = 0;
  // Called once per round that reached the barrier (the checkpoint hook).
  virtual void round_completed(int /*round*/, int64_t /*epoch*/) {}
  // Ask the host to call MasterCore::on_round_timeout(epoch, round) after `ms`.
  virtual void arm_round_timer(int64_t /*epoch*/, int /*round*/, int /*ms*/) {}
  // Called once per (re-)initialisation, after every worker got its InitWorkers.
  virtual void workers_initialized(const InitParams& /*p*/, const std::map<int, int>& /*ids*/) {}
  // Called for every CompleteAllreduce the barrier counted (counted = round matched).
  virtual void complete_seen(int /*srcId*/, int /*round*/, bool /*counted*/) {}
  // externalRounds: a queued start ran at the barrier (started) or was dropped (a re-init or
  // the end of the job made it invalid; `why` says which).
  virtual void queued_start_done(int /*round*/, bool /*started*/, const std::string& /*why*/) {}
};

struct MasterStats {
  uint64_t inits = 0, rounds_started = 0, completes = 0, stale_completes = 0, removed = 0, round_timeouts = 0,
           loss_reinits = 0, join_reinits = 0;
};

class MasterCore {
 public:
  MasterCore(MasterEffects* fx, MasterParams p) : fx_(fx), p_(p) {}

  void on_member_up(int handle);
  void on_terminated(int handle);
  // epoch < 0: untagged (accepted); otherwise completions of another epoch are stale
  void on_complete(int srcId, int round, int64_t epoch = -1);
  void on_round_timeout(int64_t epoch, int round);
  // externalRounds: start round `round`. Started now while the master is waiting (workers
  // initialised, previous round at its barrier or none started yet); while a round is in
  // flight ONE later start is queued and runs the moment the barrier is reached (the client
  // keeps its round trip off the critical path; rounds still never overlap). Needs
  // round > the last round started (== startRound allowed first) and round <= maxRound.
  enum class StartResult { Started, Queued, Refused };
  StartResult on_external_start(int round, std::string* why);
  bool awaiting_start() const { return awaiting_; }
  int queued_start() const { return queued_; }

  int round() const { return round_; }
  int num_complete() const { return numComplete_; }
  int64_t epoch() const { return epoch_; }
  uint32_t round_base() const { return round_base_; }
  bool finished() const { return finished_; }
  const std::map<int, int>& workers() const { return workers_; }  // id -> handle
  const MasterParams& params() const { return p_; }
  const MasterStats& stats() const { return stats_; }

 private:
  void init_workers() { init_workers(std::max(0, p_.startRound)); }
  void init_workers(int startRound);
  void start_allreduce();
  void advance();
  float barrier_base() const;
  // externalRounds and no round in flight: a re-init must not start a round by itself
  bool external_idle() const { return p_.externalRounds && (awaiting_ || !started_); }
  // Where a mid-job re-init resumes: the current round, unless it already passed its barrier
  // while the client has not started the next one (then workers begin at the next round, so a
  // completed round is never force-completed a second time).
  int resume_round() const { return p_.externalRounds && awaiting_ && started_ ? round_ + 1 : round_; }

  MasterEffects* fx_;
  MasterParams p_;
  std::map<int, int> workers_;  // id -> handle (AllreduceMaster.scala:26)
  int round_ = -1;              // :29
  int numComplete_ = 0;         // :30
  int64_t epoch_ = 0;
  // Device round epochs of plane workers (InitWorkers.roundBase): every epoch's rounds map
  // above all rounds any earlier epoch started, so flags left in a reused arena are stale.
  uint32_t round_base_ = 0;
  int epoch_start_round_ = 0;
  int last_reported_ = -1;
  bool finished_ = false;
  bool awaiting_ = false;  // externalRounds: waiting for the client's next StartAllreduce
  bool started_ = false;   // externalRounds: round_ has been started in this epoch
  int queued_ = -1;        // externalRounds: start queued behind the round in flight (-1 none)
  MasterStats stats_;
};

}  // namespace mxar
