// Actor shells that host the protocol cores on the actor runtime.
//   WorkerActor  <- class AllreduceWorker (AllreduceWorker.scala:9-270)
//   MasterActor  <- class AllreduceMaster (AllreduceMaster.scala:15-98)
// The shells only translate between ActorRefs and the cores' integer ids; all
// protocol decisions live in WorkerCore / MasterCore.
#pragma once

#include <mutex>

#include <functional>
#include <memory>

#include "../core/master_core.h"
#include "../core/worker_core.h"
#include "actor_system.h"
#include "control_bridge.h"

namespace mxar {

using DataSource = std::function<AllReduceInput(const AllReduceInputRequest&)>;
using DataSink = std::function<void(const AllReduceOutput&)>;

class WorkerActor final : public Actor, public WorkerEffects {
 public:
  WorkerActor(DataSource source, DataSink sink, std::shared_ptr<DataPlane> plane = nullptr);
  void receive(Envelope& env, ActorContext& ctx) override;
  std::string kind() const override { return "worker"; }

  // WorkerEffects
  void to_peer(int peer, ScatterBlock&& m) override;
  void to_peer(int peer, ReduceBlock&& m) override;
  void to_master(CompleteAllreduce&& m) override;
  void to_self(WorkerMsg&& m) override;
  AllReduceInput fetch(const AllReduceInputRequest& req) override;
  void sink(AllReduceOutput&& out) override;

  const WorkerCore& core() const { return core_; }

 private:
  template <class M>
  void send_peer(int peer, M&& m);
  DataSource source_;
  DataSink sink_;
  WorkerCore core_;
  std::map<int, ActorRef> peers_;
  ActorRef master_;
  ActorContext* ctx_ = nullptr;
};

class MasterActor final : public Actor, public MasterEffects {
 public:
  using FinishedCallback = std::function<void(int rounds)>;
  using RoundCallback = std::function<void(int round, int64_t epoch)>;  // checkpoint hook
  MasterActor(MasterParams p, FinishedCallback on_finished = nullptr, RoundCallback on_round = nullptr);
  // Stops the control bridge: its threads hold references to it, so without an explicit
  // stop it would outlive the master (control_bridge.h, "Threads and lifetime").
  ~MasterActor() override;
  void receive(Envelope& env, ActorContext& ctx) override;
  std::string kind() const override { return "master"; }

  // MasterEffects
  void send_init(int handle, const InitParams& p, const std::map<int, int>& ids) override;
  void send_start(int handle, int round) override;
  void finished(int rounds) override;
  void round_completed(int round, int64_t epoch) override;
  void arm_round_timer(int64_t epoch, int round, int ms) override;
  void workers_initialized(const InitParams& p, const std::map<int, int>& ids) override;
  void complete_seen(int srcId, int round, bool counted) override;
  void queued_start_done(int round, bool started, const std::string& why) override;

  // Control bridge (csrc/runtime/control_bridge.h): events go out to its clients, its
  // BridgeCommands come in. Set before the master receives its first message.
  void set_bridge(std::shared_ptr<ControlBridge> b) { bridge_ = std::move(b); }
  const std::shared_ptr<ControlBridge>& bridge() const { return bridge_; }

  const MasterCore& core() const { return core_; }
  // steady_clock (CLOCK_MONOTONIC = Python's perf_counter) seconds at which each round
  // reached the barrier - recorded natively, so timing a job needs no callback per round
  std::vector<double> round_stamps() const;

 private:
  int handle_of(const ActorRef& ref, bool create);
  MasterCore core_;
  std::vector<ActorRef> handles_;
  std::vector<std::string> metas_;  // per handle: MemberUp.meta (plane descriptor or "")
  FinishedCallback on_finished_;
  RoundCallback on_round_;
  ActorContext* ctx_ = nullptr;
  std::shared_ptr<ControlBridge> bridge_;
  uint64_t queued_client_ = 0;  // bridge client whose StartAllreduce is queued
  mutable std::mutex stamp_mu_;
  std::vector<double> stamps_;
};

}  // namespace mxar
