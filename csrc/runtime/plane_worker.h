// PlaneWorkerActor: the reference's AllreduceWorker (AllreduceWorker.scala:9-270) at round
// granularity over a RoundPlane (round_plane.h). The master protocol is unchanged -
// InitWorkers, StartAllreduce(r), CompleteAllreduce(id, r) - and so are the user hooks
// (dataSource per round, dataSink per completed round); the per-chunk ScatterBlock /
// ReduceBlock traffic is the plane's job (one xGMI launch per round on MI355X).
//
// Handler map (reference -> here):
//   InitWorkers  (:37-82)   -> plane.configure(): block ranges, chunks, thresholds, maxLag,
//                              every peer's plane descriptor (InitWorkers.planes: the IPC
//                              handles of their HBM arenas) and the round-epoch base
//   StartAllreduce (:84-104)-> maxRound = max(...); forced catch-up of every round
//                              < maxRound - maxLag (plane.force for rounds in flight, a
//                              cold launch for rounds never started); then fetch + launch
//                              every round up to maxRound (dataSource, :171-178)
//   complete / flush (:180-192, :253-268) -> the plane's completion: dataSink(output with
//                              the real per-chunk counts), CompleteAllreduce to the master,
//                              round advances past every completed round
// Kept from WorkerCore: messages before Init are stashed, newer-epoch messages
// stashed and older ones dropped (Q2).
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <vector>

#include "../core/worker_core.h"
#include "actor_system.h"
#include "allreduce_actors.h"
#include "round_plane.h"

namespace mxar {

struct PlaneWorkerStats {
  uint64_t start_in = 0, rounds_launched = 0, cold_rounds = 0, forced_completions = 0, rounds_completed = 0;
  uint64_t complete_out = 0, stale_dropped = 0, stashed = 0, plane_errors = 0, inits = 0;
  // rounds a StartAllreduce jumped ahead to because a newer one was already in the mailbox
  uint64_t starts_coalesced = 0;
};

class PlaneWorkerActor final : public Actor {
 public:
  PlaneWorkerActor(DataSource source, DataSink sink, std::shared_ptr<RoundPlane> plane);
  ~PlaneWorkerActor() override;
  void receive(Envelope& env, ActorContext& ctx) override;
  // a stopped worker (PoisonPill, downed) abandons its rounds in flight at once: its round
  // kernel would otherwise wait out its deadline for peers that moved on without it, holding
  // its hardware queue (and a resident kernel) meanwhile
  void post_stop(ActorContext&) override { plane_->abort(0x7fffffff); }
  // The newest StartAllreduce enqueued (epoch, round): a worker that fell behind its mailbox
  // (a slow dataSource) catches up to it at once instead of fetching every queued round -
  // the GPU analogue of the reference's future-round message making a laggard StartAllreduce
  // (AllreduceWorker.scala:123-126), which on the device is the peers' FORCE word.
  void on_enqueue(const Message& m) override;
  std::string kind() const override { return "plane-worker"; }

  int id() const { return id_; }
  int round() const { return round_; }
  int max_round() const { return maxRound_; }
  int launched() const { return launched_; }
  int64_t epoch() const { return cfg_.epoch; }
  int peers() const { return cfg_.peers; }
  bool initialized() const { return id_ >= 0; }
  const PlaneWorkerStats& stats() const { return stats_; }
  RoundLatency round_latency() const;
  const std::shared_ptr<RoundPlane>& plane() const { return plane_; }

 private:
  void on_init(const InitWorkers& m, ActorContext& ctx);
  void on_start(const StartAllreduce& m);
  void on_done(PlaneRoundDone& d);

  DataSource source_;
  DataSink sink_;
  std::shared_ptr<RoundPlane> plane_;
  PlaneConfig cfg_;
  ActorRef master_;
  ActorRef self_;
  int id_ = -1;
  int round_ = -1, maxRound_ = -1, launched_ = -1;
  std::set<int> completed_;
  std::atomic<uint64_t> announced_{0};  // (epoch low 32 bits << 32) | round of the newest Start enqueued
  std::map<int, uint64_t> t0_;
  mutable std::mutex lat_mu_;  // lat_ms_: round_latency() may be called from another thread
  std::vector<double> lat_ms_;
  size_t lat_pos_ = 0;
  uint64_t lat_count_ = 0;
  PlaneWorkerStats stats_;
};

}  // namespace mxar
