#include "allreduce_actors.h"

#include <sstream>

#include <chrono>

#include "../core/log.h"

namespace mxar {

// ------------------------------------------------------------------------ worker
WorkerActor::WorkerActor(DataSource source, DataSink sink, std::shared_ptr<DataPlane> plane)
    : source_(std::move(source)), sink_(std::move(sink)), core_(this, std::move(plane)) {}

void WorkerActor::receive(Envelope& env, ActorContext& ctx) {
  ctx_ = &ctx;
  struct Visitor {
    WorkerActor* w;
    Envelope& env;
    ActorContext& ctx;
    void operator()(InitWorkers& m) {
      InitParams p;
      p.destId = m.destId;
      p.numPeers = static_cast<int>(m.workers.size());
      p.thReduce = m.thReduce;
      p.thComplete = m.thComplete;
      p.maxLag = m.maxLag;
      p.dataSize = m.dataSize;
      p.maxChunkSize = m.maxChunkSize;
      p.epoch = m.epoch;
      p.startRound = m.startRound;
      w->peers_ = m.workers;
      w->master_ = m.master;
      w->core_.on_init(p);
      ctx.unstash_all();  // replay what arrived before Init
    }
    void operator()(StartAllreduce& m) {
      if (!w->core_.on_start(m)) {
        MXAR_LOG(WARNING, "worker", "----Actor is not initialized (stashing StartAllreduce " << m.round << ")");
        ctx.stash(std::move(env));
      }
    }
    void operator()(ScatterBlock& m) {
      if (!w->core_.on_scatter(m)) {
        MXAR_LOG(WARNING, "worker", "----Have not initialized! (stashing ScatterBlock)");
        ctx.stash(std::move(env));
      }
    }
    void operator()(ReduceBlock& m) {
      if (!w->core_.on_reduce(m)) {
        MXAR_LOG(WARNING, "worker", "----Have not initialized! (stashing ReduceBlock)");
        ctx.stash(std::move(env));
      }
    }
    void operator()(Terminated& m) {
      // AllreduceWorker.scala:153-158 (dead code there: the worker never watches)
      for (auto it = w->peers_.begin(); it != w->peers_.end(); ++it) {
        if (it->second == m.ref) {
          MXAR_LOG(WARNING, "worker", "----peer " << it->first << " terminated");
          it->second = ctx.system().dead_letters();
        }
      }
    }
    void operator()(CompleteAllreduce&) {}
    void operator()(MemberUp&) {}
    void operator()(AllreduceFinished&) {}
    void operator()(PoisonPill&) {}
    void operator()(TextMessage&) {}
    void operator()(RoundTimeout&) {}
    void operator()(PlaneRoundDone&) {}
    void operator()(BridgeCommand&) {}
  };
  std::visit(Visitor{this, env, ctx}, env.msg);
  ctx_ = nullptr;
}

template <class M>
void WorkerActor::send_peer(int peer, M&& m) {
  auto it = peers_.find(peer);
  ActorRef self = ctx_ ? ctx_->self() : nullptr;
  if (it == peers_.end() || !it->second) {
    MXAR_LOG(WARNING, "worker", "----no actor for peer " << peer << ", message dropped");
    if (ctx_) ctx_->system().dead_letters()->tell(Message(std::forward<M>(m)), self);
    return;
  }
  it->second->tell(Message(std::forward<M>(m)), self);
}

void WorkerActor::to_peer(int peer, ScatterBlock&& m) { send_peer(peer, std::move(m)); }
void WorkerActor::to_peer(int peer, ReduceBlock&& m) { send_peer(peer, std::move(m)); }

void WorkerActor::to_master(CompleteAllreduce&& m) {
  ActorRef self = ctx_ ? ctx_->self() : nullptr;
  if (master_) master_->tell(Message(std::move(m)), self);
}

void WorkerActor::to_self(WorkerMsg&& m) {
  ActorRef self = ctx_->self();
  std::visit([&](auto&& x) { self->tell(Message(std::move(x)), self); }, std::move(m));
}

AllReduceInput WorkerActor::fetch(const AllReduceInputRequest& req) { return source_(req); }

void WorkerActor::sink(AllReduceOutput&& out) {
  if (sink_) sink_(out);
}

// ------------------------------------------------------------------------ master
MasterActor::~MasterActor() {
  if (bridge_) bridge_->stop();
}

MasterActor::MasterActor(MasterParams p, FinishedCallback on_finished, RoundCallback on_round)
    : core_(this, p), on_finished_(std::move(on_finished)), on_round_(std::move(on_round)) {}

int MasterActor::handle_of(const ActorRef& ref, bool create) {
  for (size_t i = 0; i < handles_.size(); ++i)
    if (handles_[i] == ref) return static_cast<int>(i);
  if (!create) return -1;
  handles_.push_back(ref);
  metas_.emplace_back();
  return static_cast<int>(handles_.size() - 1);
}

void MasterActor::receive(Envelope& env, ActorContext& ctx) {
  ctx_ = &ctx;
  if (auto* up = std::get_if<MemberUp>(&env.msg)) {
    MXAR_LOG(INFO, "master", "----Detect member " << (up->address.empty() ? up->ref->path() : up->address) << " up");
    if (up->role == "worker" && up->ref) {
      ctx.watch(up->ref);  // AllreduceMaster.scala:74
      const int h = handle_of(up->ref, true);
      if (!up->meta.empty()) metas_[h] = up->meta;
      core_.on_member_up(h);
    }
  } else if (auto* t = std::get_if<Terminated>(&env.msg)) {
    MXAR_LOG(INFO, "master", "----" << (t->ref ? t->ref->path() : "?") << " is terminated, removing it from the set");
    int h = handle_of(t->ref, false);
    if (h >= 0) core_.on_terminated(h);
  } else if (auto* c = std::get_if<CompleteAllreduce>(&env.msg)) {
    core_.on_complete(c->srcId, c->round, c->epoch);
  } else if (auto* rt = std::get_if<RoundTimeout>(&env.msg)) {
    core_.on_round_timeout(rt->epoch, rt->round);
  } else if (auto* bc = std::get_if<BridgeCommand>(&env.msg)) {
    if (bridge_ && bc->kind == BridgeCommand::Start) {
      std::string why;
      const std::string r = std::to_string(bc->round);
      switch (core_.on_external_start(bc->round, &why)) {
        case MasterCore::StartResult::Started:
          bridge_->reply(bc->client, "{\"type\":\"Accepted\",\"cmd\":\"StartAllreduce\",\"round\":" + r + "}");
          break;
        case MasterCore::StartResult::Queued:
          queued_client_ = bc->client;
          bridge_->reply(bc->client, "{\"type\":\"Queued\",\"cmd\":\"StartAllreduce\",\"round\":" + r + "}");
          break;
        case MasterCore::StartResult::Refused:
          bridge_->reply(bc->client, "{\"type\":\"Error\",\"cmd\":\"StartAllreduce\",\"round\":" + r +
                                         ",\"reason\":\"" + json_escape(why) + "\"}");
          break;
      }
    } else if (bridge_) {
      std::ostringstream o;
      o << "{\"type\":\"Status\",\"round\":" << core_.round() << ",\"epoch\":" << core_.epoch()
        << ",\"workers\":" << core_.workers().size() << ",\"numComplete\":" << core_.num_complete()
        << ",\"awaiting\":" << (core_.awaiting_start() ? "true" : "false") << ",\"queued\":" << core_.queued_start()
        << ",\"finished\":" << (core_.finished() ? "true" : "false") << "}";
      bridge_->reply(bc->client, o.str());
    }
  }
  ctx_ = nullptr;
}

void MasterActor::workers_initialized(const InitParams& p, const std::map<int, int>& ids) {
  if (!bridge_) return;
  std::ostringstream o;
  o << "{\"type\":\"InitWorkers\",\"epoch\":" << p.epoch << ",\"workers\":[";
  bool first = true;
  for (auto& [id, h] : ids) {
    o << (first ? "" : ",") << id;
    first = false;
  }
  o << "],\"thReduce\":" << p.thReduce << ",\"thComplete\":" << p.thComplete << ",\"maxLag\":" << p.maxLag
    << ",\"dataSize\":" << p.dataSize << ",\"maxChunkSize\":" << p.maxChunkSize
    << ",\"startRound\":" << p.startRound << ",\"maxRound\":" << core_.params().maxRound
    << ",\"externalRounds\":"
    << (core_.params().externalRounds ? "true" : "false") << "}";
  bridge_->set_init_line(o.str());
  bridge_->publish(o.str());
}

void MasterActor::queued_start_done(int round, bool started, const std::string& why) {
  if (!bridge_) return;
  const std::string r = std::to_string(round);
  bridge_->reply(queued_client_,
                 started ? "{\"type\":\"Accepted\",\"cmd\":\"StartAllreduce\",\"round\":" + r + "}"
                         : "{\"type\":\"Error\",\"cmd\":\"StartAllreduce\",\"round\":" + r +
                               ",\"reason\":\"queued start dropped: " + json_escape(why) + "\"}");
}

void MasterActor::complete_seen(int srcId, int round, bool counted) {
  if (!bridge_) return;
  bridge_->publish("{\"type\":\"CompleteAllreduce\",\"srcId\":" + std::to_string(srcId) +
                   ",\"round\":" + std::to_string(round) + ",\"counted\":" + (counted ? "true" : "false") + "}");
}

void MasterActor::arm_round_timer(int64_t epoch, int round, int ms) {
  ctx_->system().schedule_once(std::chrono::milliseconds(ms), ctx_->self(), RoundTimeout{epoch, round});
}

void MasterActor::send_init(int handle, const InitParams& p, const std::map<int, int>& ids) {
  InitWorkers m;
  for (auto& [id, h] : ids) m.workers[id] = handles_[h];
  m.master = ctx_->self();
  m.destId = p.destId;
  m.thReduce = p.thReduce;
  m.thComplete = p.thComplete;
  m.maxLag = p.maxLag;
  m.dataSize = p.dataSize;
  m.maxChunkSize = p.maxChunkSize;
  m.epoch = p.epoch;
  m.startRound = p.startRound;
  m.roundBase = p.roundBase;
  bool any_plane = false;
  for (auto& [id, h] : ids) any_plane = any_plane || !metas_[h].empty();
  if (any_plane)
    for (auto& [id, h] : ids) m.planes[id] = metas_[h];
  handles_[handle]->tell(Message(std::move(m)), ctx_->self());
}

void MasterActor::send_start(int handle, int round) {
  handles_[handle]->tell(StartAllreduce{round, core_.epoch()}, ctx_->self());
}

void MasterActor::finished(int rounds) {
  if (bridge_) bridge_->publish("{\"type\":\"AllreduceFinished\",\"rounds\":" + std::to_string(rounds) + "}");
  if (on_finished_) on_finished_(rounds);
}

void MasterActor::round_completed(int round, int64_t epoch) {
  {
    std::lock_guard<std::mutex> g(stamp_mu_);
    if (stamps_.size() < (size_t{1} << 22))
      stamps_.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count());
  }
  if (bridge_)
    bridge_->publish("{\"type\":\"RoundComplete\",\"round\":" + std::to_string(round) +
                     ",\"epoch\":" + std::to_string(epoch) + ",\"numComplete\":" +
                     std::to_string(core_.num_complete()) + "}");
  if (on_round_) on_round_(round, epoch);
}

std::vector<double> MasterActor::round_stamps() const {
  std::lock_guard<std::mutex> g(stamp_mu_);
  return stamps_;
}

}  // namespace mxar
