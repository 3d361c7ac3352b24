#include "plane_worker.h"

#include <algorithm>

#include "../core/log.h"
#include "../core/trace.h"

namespace mxar {

PlaneWorkerActor::PlaneWorkerActor(DataSource source, DataSink sink, std::shared_ptr<RoundPlane> plane)
    : source_(std::move(source)), sink_(std::move(sink)), plane_(std::move(plane)) {
  if (!plane_) throw std::invalid_argument("PlaneWorkerActor needs a RoundPlane");
}

PlaneWorkerActor::~PlaneWorkerActor() {
  // rounds still in flight are abandoned before the plane may call back into nothing
  try {
    plane_->abort(0x7fffffff);
    plane_->drain();
  } catch (const std::exception& e) {
    MXAR_LOG(ERROR, "worker", "----plane drain at shutdown failed: " << e.what());
  }
  plane_->set_done(nullptr);
}

void PlaneWorkerActor::receive(Envelope& env, ActorContext& ctx) {
  if (!self_) {
    self_ = ctx.self();
    // the plane's completion thread posts each finished round to this worker's mailbox
    std::weak_ptr<ActorRefBase> weak = self_;
    plane_->set_done([weak](RoundResult&& r) {
      if (auto s = weak.lock()) {
        PlaneRoundDone d;
        d.epoch = r.epoch;
        d.output = AllReduceOutput{std::move(r.data), std::move(r.count), r.round};
        d.error = r.error;
        d.cold = r.cold;
        s->tell(Message(std::move(d)), nullptr);
      }
    });
  }
  if (auto* init = std::get_if<InitWorkers>(&env.msg)) {
    on_init(*init, ctx);
    ctx.unstash_all();  // replay what arrived before Init
  } else if (auto* st = std::get_if<StartAllreduce>(&env.msg)) {
    if (!initialized() || st->epoch > cfg_.epoch) {  // before Init / a newer epoch's Init in flight
      stats_.stashed++;
      MXAR_LOG(WARNING, "worker", "----Actor is not initialized (stashing StartAllreduce " << st->round << ")");
      ctx.stash(std::move(env));
    } else if (st->epoch < cfg_.epoch) {
      stats_.stale_dropped++;
    } else {
      on_start(*st);
    }
  } else if (auto* d = std::get_if<PlaneRoundDone>(&env.msg)) {
    on_done(*d);
  } else if (std::holds_alternative<ScatterBlock>(env.msg) || std::holds_alternative<ReduceBlock>(env.msg)) {
    // a peer using the actor data path: the planes of one job must agree
    MXAR_LOG(ERROR, "worker", "----plane worker received a ScatterBlock/ReduceBlock message: every worker of a "
                              "plane job must use a plane (dropped)");
    stats_.stale_dropped++;
  }
}

// InitWorkers (AllreduceWorker.scala:37-82)
void PlaneWorkerActor::on_init(const InitWorkers& m, ActorContext&) {
  const int P = static_cast<int>(m.workers.size());
  if (P <= 0 || m.destId < 0 || m.destId >= P) throw ProtocolError("InitWorkers with a bad destId / no peers");
  if (static_cast<int>(m.planes.size()) != P)
    throw ProtocolError("InitWorkers carries " + std::to_string(m.planes.size()) + " plane descriptors for " +
                        std::to_string(P) + " workers: every worker of a plane job must announce a plane");
  PlaneConfig c;
  c.id = m.destId;
  c.peers = P;
  c.thReduce = m.thReduce;
  c.thComplete = m.thComplete;
  c.maxLag = m.maxLag;
  c.dataSize = m.dataSize;
  c.maxChunkSize = m.maxChunkSize;
  c.epoch = m.epoch;
  c.startRound = std::max(0, m.startRound);
  c.roundBase = m.roundBase;
  c.descriptors = m.planes;
  plane_->configure(c);  // drains the previous epoch's rounds first (their results are dropped)
  cfg_ = c;
  master_ = m.master;
  id_ = c.id;
  round_ = c.startRound;
  maxRound_ = round_ - 1;
  launched_ = round_ - 1;
  completed_.clear();
  t0_.clear();
  stats_.inits++;
  MXAR_LOG(INFO, "worker", "----Actor id = " << id_ << " (epoch " << m.epoch << ", plane " << plane_->name() << ")");
  MXAR_LOG(INFO, "worker", "----Number of peers = " << P);
  MXAR_LOG(INFO, "worker", "----Thresholds: thReduce = " << m.thReduce << ", thComplete = " << m.thComplete
                                                          << ", maxLag = " << m.maxLag);
}

void PlaneWorkerActor::on_enqueue(const Message& m) {
  const auto* st = std::get_if<StartAllreduce>(&m);
  if (st == nullptr || st->round < 0) return;
  const uint64_t v = (static_cast<uint64_t>(static_cast<uint32_t>(st->epoch)) << 32) | static_cast<uint32_t>(st->round);
  uint64_t cur = announced_.load(std::memory_order_relaxed);
  while (v > cur && !announced_.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}

// StartAllreduce (AllreduceWorker.scala:84-104)
void PlaneWorkerActor::on_start(const StartAllreduce& m) {
  stats_.start_in++;
  MXAR_LOG(INFO, "worker", "----Start allreduce round " << m.round);
  maxRound_ = std::max(maxRound_, m.round);
  // a newer StartAllreduce of this epoch already waits in the mailbox: take its round now (it
  // is a no-op when its turn comes), so a worker slower than the master catches up in one step
  const uint64_t ann = announced_.load(std::memory_order_relaxed);
  if (static_cast<uint32_t>(ann >> 32) == static_cast<uint32_t>(cfg_.epoch)) {
    const int newest = static_cast<int>(static_cast<uint32_t>(ann));
    if (newest > maxRound_) {
      stats_.starts_coalesced += static_cast<uint64_t>(newest - maxRound_);
      maxRound_ = newest;
    }
  }
  const int target = maxRound_ - cfg_.maxLag;  // every round < target must complete now
  if (round_ < target) {
    // forced catch-up (:91-97): rounds in flight stop waiting, rounds never started are
    // completed cold - with what the peers delivered, nothing of our own
    MXAR_LOG(INFO, "worker", "----Catch up: force-completing rounds " << round_ << ".." << target - 1);
    trace_instant("worker", "forced catch-up r" + std::to_string(round_) + ".." + std::to_string(target - 1),
                  "{\"worker\":" + std::to_string(id_) + "}");
    stats_.forced_completions += static_cast<uint64_t>(target - round_);
    plane_->force(target - 1);
    while (launched_ < target - 1) {
      ++launched_;
      plane_->launch(launched_, nullptr, true);
      stats_.cold_rounds++;
      stats_.rounds_launched++;
    }
  }
  while (launched_ < maxRound_) {  // fetch + scatter every round up to maxRound (:98-102)
    const int r = launched_ + 1;
    MXAR_LOG(INFO, "worker", "fetch " << r);
    t0_[r] = Tracer::now_ns();
    AllReduceInput in;
    {
      TraceScope span("worker", [&] {
        return std::make_pair(std::string("fetch r" + std::to_string(r)),
                              std::string("{\"worker\":" + std::to_string(id_) + "}"));
      });
      in = source_(AllReduceInputRequest{r});
    }
    if (payload_size(in.data) != static_cast<size_t>(cfg_.dataSize))  // AllreduceWorker.scala:174-176
      throw ProtocolError("Input data size " + std::to_string(payload_size(in.data)) +
                          " is different from initialization time " + std::to_string(cfg_.dataSize) + "!");
    {
      TraceScope span("worker", [&] {
        return std::make_pair(std::string("launch r" + std::to_string(r)),
                              std::string("{\"worker\":" + std::to_string(id_) + "}"));
      });
      plane_->launch(r, in.data, false);
    }
    launched_ = r;
    stats_.rounds_launched++;
  }
}

// complete + flush (AllreduceWorker.scala:180-192, 253-268)
void PlaneWorkerActor::on_done(PlaneRoundDone& d) {
  if (d.epoch != cfg_.epoch) {  // a round of a previous membership epoch, drained at re-init
    stats_.stale_dropped++;
    return;
  }
  const int r = d.output.iteration;
  if (d.error) {
    stats_.plane_errors++;
    MXAR_LOG(ERROR, "worker", "----plane error word " << d.error << " in round " << r << " at worker " << id_);
  }
  if (auto it = t0_.find(r); it != t0_.end()) {
    const double ms = (Tracer::now_ns() - it->second) / 1e6;
    std::lock_guard<std::mutex> g(lat_mu_);
    if (lat_ms_.size() < 4096)
      lat_ms_.push_back(ms);
    else
      lat_ms_[lat_pos_] = ms;
    lat_pos_ = (lat_pos_ + 1) % 4096;
    ++lat_count_;
    t0_.erase(it);
  }
  MXAR_LOG(INFO, "worker", "----Flushing round " << r << " (" << payload_size(d.output.data) << " elements)");
  {
    TraceScope span("worker", [&] {
      return std::make_pair(std::string("sink r" + std::to_string(r)),
                            std::string("{\"worker\":" + std::to_string(id_) + "}"));
    });
    if (sink_) sink_(d.output);
  }
  stats_.rounds_completed++;
  stats_.complete_out++;
  if (master_) master_->tell(CompleteAllreduce{id_, r, cfg_.epoch}, self_);
  completed_.insert(r);
  while (completed_.count(round_)) {
    completed_.erase(round_);
    ++round_;
  }
}

RoundLatency PlaneWorkerActor::round_latency() const {
  RoundLatency r;
  std::vector<double> v;
  {
    std::lock_guard<std::mutex> g(lat_mu_);
    r.count = lat_count_;
    v = lat_ms_;
  }
  if (v.empty()) return r;
  std::sort(v.begin(), v.end());
  auto q = [&](double p) { return v[std::min(v.size() - 1, static_cast<size_t>(p * (v.size() - 1) + 0.5))]; };
  r.p50_ms = q(0.5);
  r.p99_ms = q(0.99);
  r.max_ms = v.back();
  double s = 0;
  for (double x : v) s += x;
  r.mean_ms = s / v.size();
  return r;
}

}  // namespace mxar
