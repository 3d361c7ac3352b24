#include "loopback_plane.h"

#include <algorithm>
#include <climits>
#include <map>
#include <random>
#include <sstream>
#include <vector>

#include "../core/data_buffer.h"
#include "../core/log.h"

namespace mxar {

// The shared state of one hub: per membership epoch, the registered planes and the
// contributions / reduced blocks of every round still in flight. One mutex guards the hub
// and the per-plane round queues of every plane attached to it.
class LoopbackHub {
 public:
  struct RoundState {
    std::vector<int> arrivals;                // contributor ids, arrival order
    std::vector<std::vector<float>> contrib;  // [P]
    std::vector<int> reduce_seq;              // [P] order in which blocks got reduced, -1 = not yet
    std::vector<int> reduce_cnt;              // [P] contributions summed into the block
    std::vector<char> forced_reduce;          // [P] reduced only because its owner was forced
    std::vector<std::vector<float>> block;    // [P] reduced block
    int next_seq = 0;
  };
  struct Epoch {
    int P = 0;
    int dataSize = 0;
    int maxLag = 0;
    int64_t block = 0, chunk = 0;
    int nch = 0;
    int min_reduce = 1, min_complete = 0;
    std::vector<LoopbackRoundPlane*> planes;
    std::map<int, RoundState> rounds;
  };

  explicit LoopbackHub(std::string name) : name_(std::move(name)) {}
  const std::string& name() const { return name_; }

  static std::shared_ptr<LoopbackHub> get(const std::string& name) {
    static std::mutex mu;
    static std::map<std::string, std::weak_ptr<LoopbackHub>> hubs;
    std::lock_guard<std::mutex> g(mu);
    auto& w = hubs[name];
    if (auto h = w.lock()) return h;
    auto h = std::make_shared<LoopbackHub>(name);
    w = h;
    return h;
  }

  std::mutex mu;
  std::condition_variable cv;  // a round became deliverable somewhere in this hub
  std::map<int64_t, Epoch> epochs;

  // ---- everything below runs under `mu` ----
  RoundState& state(Epoch& E, int r) {
    RoundState& R = E.rounds[r];
    if (static_cast<int>(R.contrib.size()) != E.P) {
      R.contrib.assign(E.P, {});
      R.reduce_seq.assign(E.P, -1);
      R.reduce_cnt.assign(E.P, 0);
      R.forced_reduce.assign(E.P, 0);
      R.block.assign(E.P, {});
    }
    return R;
  }

  static LoopbackRoundPlane::Pending* find(LoopbackRoundPlane* p, int r) {
    for (auto& x : p->q_)
      if (x.round == r) return &x;
    return nullptr;
  }

  // A round of plane p becomes active: it contributes (unless cold) and asks peers more
  // than maxLag + 1 rounds behind to force-complete (the kernel's lag-gate FORCE request).
  void activate(Epoch& E, LoopbackRoundPlane* p, LoopbackRoundPlane::Pending& x, std::deque<int>& work) {
    x.active = true;
    const int id = p->cfg_.id;
    if (!x.cold) {
      RoundState& R = state(E, x.round);
      R.contrib[id] = x.input ? x.input->to_host() : std::vector<float>(E.dataSize, 0.f);
      R.contrib[id].resize(E.dataSize, 0.f);
      R.arrivals.push_back(id);
      x.input.reset();
    }
    work.push_back(x.round);
    const int behind = x.round - (E.maxLag + 1);
    for (int k = 0; k < E.P; ++k) {
      LoopbackRoundPlane* q = E.planes[k];
      if (q == nullptr || q == p || q->progress_ >= behind || q->forced_upto_ >= behind) continue;
      q->forced_upto_ = behind;
      q->st_.peer_forces++;
      for (auto& y : q->q_)
        if (y.active && !y.done && y.round <= behind) work.push_back(y.round);
    }
  }

  void reduce_block(Epoch& E, RoundState& R, int j, int take, bool forced_only) {
    const int64_t b0 = static_cast<int64_t>(j) * E.block;
    const int64_t len = std::max<int64_t>(0, std::min<int64_t>(E.block, E.dataSize - b0));
    std::vector<float> s(static_cast<size_t>(len), 0.f);
    for (int a = 0; a < take && a < static_cast<int>(R.arrivals.size()); ++a) {
      const std::vector<float>& v = R.contrib[R.arrivals[a]];
      for (int64_t t = 0; t < len; ++t) s[t] += v[b0 + t];
    }
    R.block[j] = std::move(s);
    R.reduce_seq[j] = R.next_seq++;
    R.reduce_cnt[j] = take;
    R.forced_reduce[j] = forced_only ? 1 : 0;
  }

  void complete(Epoch& E, RoundState& R, LoopbackRoundPlane* p, LoopbackRoundPlane::Pending& x, bool forced,
                int64_t epoch, std::deque<int>& work) {
    const int id = p->cfg_.id;
    std::vector<int> order;
    for (int j = 0; j < E.P; ++j)
      if (R.reduce_seq[j] >= 0) order.push_back(j);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return R.reduce_seq[a] < R.reduce_seq[b]; });
    const int limit = forced ? INT_MAX : E.min_complete;
    std::vector<float> out(static_cast<size_t>(E.dataSize), 0.f);
    std::vector<int> counts(static_cast<size_t>(E.P) * E.nch, 0);
    int taken = 0;
    for (int j : order) {
      if (forced && j == id && R.forced_reduce[j]) continue;  // reduced by the force: flushed after
      const int64_t b0 = static_cast<int64_t>(j) * E.block;
      const int64_t len = static_cast<int64_t>(R.block[j].size());
      for (int c = 0; c < E.nch && taken < limit; ++c, ++taken) {
        const int64_t c0 = static_cast<int64_t>(c) * E.chunk;
        const int64_t c1 = std::min<int64_t>(len, c0 + E.chunk);
        for (int64_t t = c0; t < c1; ++t) out[b0 + t] = R.block[j][t];
        counts[static_cast<size_t>(j) * E.nch + c] = R.reduce_cnt[j];
      }
    }
    x.done = true;
    x.res.epoch = epoch;
    x.res.round = x.round;
    x.res.cold = x.cold;
    x.res.data = make_host_payload(std::move(out));
    x.res.count = std::move(counts);
    if (forced) p->st_.forced_rounds++;
    p->st_.completed++;
    p->progress_ = std::max(p->progress_, x.round);
    // stream order: the next launched round of this plane starts now
    for (auto& y : p->q_)
      if (!y.active) {
        activate(E, p, y, work);
        break;
      } else if (!y.done) {
        break;
      }
  }

  void evaluate(Epoch& E, int r, int64_t epoch, std::deque<int>& work) {
    RoundState& R = state(E, r);
    for (bool changed = true; changed;) {
      changed = false;
      for (int j = 0; j < E.P; ++j) {  // owners' reduces
        if (R.reduce_seq[j] >= 0 || E.planes[j] == nullptr) continue;
        LoopbackRoundPlane::Pending* x = find(E.planes[j], r);
        if (x == nullptr || !x->active) continue;
        const bool forced = x->cold || E.planes[j]->forced_upto_ >= r;
        const int present = static_cast<int>(R.arrivals.size());
        if (present >= E.min_reduce) {
          reduce_block(E, R, j, E.min_reduce, false);
        } else if (forced) {
          reduce_block(E, R, j, present, true);
        } else {
          continue;
        }
        changed = true;
      }
      int reduced = 0;
      for (int j = 0; j < E.P; ++j) reduced += R.reduce_seq[j] >= 0 ? E.nch : 0;
      for (int i = 0; i < E.P; ++i) {  // completions
        LoopbackRoundPlane* p = E.planes[i];
        if (p == nullptr) continue;
        LoopbackRoundPlane::Pending* x = find(p, r);
        if (x == nullptr || !x->active || x->done) continue;
        const bool forced = x->cold || p->forced_upto_ >= r;
        if (reduced >= E.min_complete || forced) {
          complete(E, R, p, *x, reduced < E.min_complete, epoch, work);
          changed = true;
        }
      }
    }
  }

  void run(int64_t epoch, std::deque<int>& work) {
    auto it = epochs.find(epoch);
    if (it == epochs.end()) return;
    Epoch& E = it->second;
    while (!work.empty()) {
      const int r = work.front();
      work.pop_front();
      evaluate(E, r, epoch, work);
    }
    // rounds every worker has completed are no longer needed
    int low = INT_MAX;
    for (LoopbackRoundPlane* p : E.planes) low = p == nullptr ? INT_MIN : std::min(low, p->progress_);
    for (auto r = E.rounds.begin(); r != E.rounds.end() && r->first <= low;) r = E.rounds.erase(r);
    cv.notify_all();
  }

 private:
  std::string name_;
};

namespace {

std::map<std::string, std::string> parse_kv(const std::string& s, std::string* tag) {
  std::istringstream is(s);
  std::map<std::string, std::string> kv;
  is >> *tag;
  std::string t;
  while (is >> t) {
    const auto e = t.find('=');
    if (e != std::string::npos) kv[t.substr(0, e)] = t.substr(e + 1);
  }
  return kv;
}

}  // namespace

LoopbackRoundPlane::LoopbackRoundPlane(const std::string& hub) : hub_(LoopbackHub::get(hub)) {
  if (hub.empty() || hub.find(' ') != std::string::npos)
    throw std::invalid_argument("loopback plane: the hub name must be a non-empty word");
  std::random_device rd;
  uid_ = (static_cast<uint64_t>(rd()) << 32) ^ rd();
  std::ostringstream os;
  os << "loop1 hub=" << hub << " id=" << uid_;
  desc_ = os.str();
  th_ = std::thread([this] { deliver_loop(); });
}

LoopbackRoundPlane::~LoopbackRoundPlane() {
  try {
    force(INT_MAX - 1);
    drain();
  } catch (...) {
  }
  {
    std::lock_guard<std::mutex> g(hub_->mu);
    if (configured_) {
      auto it = hub_->epochs.find(cfg_.epoch);
      if (it != hub_->epochs.end()) {
        auto& pl = it->second.planes;
        if (cfg_.id < static_cast<int>(pl.size()) && pl[cfg_.id] == this) pl[cfg_.id] = nullptr;
        if (std::all_of(pl.begin(), pl.end(), [](LoopbackRoundPlane* p) { return p == nullptr; }))
          hub_->epochs.erase(it);
      }
    }
    stop_ = true;
  }
  hub_->cv.notify_all();
  if (th_.joinable()) th_.join();
}

void LoopbackRoundPlane::set_done(DoneFn fn) {
  std::lock_guard<std::mutex> g(done_mu_);
  done_ = std::move(fn);
}

void LoopbackRoundPlane::configure(const PlaneConfig& cfg) {
  if (cfg.peers < 1) throw ProtocolError("loopback plane: no peers");
  if (cfg.dataSize <= 0) throw ProtocolError("loopback plane: dataSize must be > 0");
  if (cfg.maxChunkSize <= 0) throw ProtocolError("maxChunkSize must be > 0");
  if (static_cast<int>(cfg.descriptors.size()) != cfg.peers)
    throw ProtocolError("InitWorkers.planes must hold one descriptor per worker");
  for (const auto& [k, d] : cfg.descriptors) {
    std::string tag;
    const auto kv = parse_kv(d, &tag);
    if (tag != "loop1" || kv.count("hub") == 0 || kv.at("hub") != hub_->name())
      throw ProtocolError("loopback plane (hub " + hub_->name() + "): worker " + std::to_string(k) +
                          " announced '" + d + "' - every worker of a job must use the same loopback hub");
  }
  if (configured_) {  // the previous epoch's rounds finish (forced) first
    force(INT_MAX - 1);
    drain();
  }
  std::deque<int> work;
  std::lock_guard<std::mutex> g(hub_->mu);
  if (configured_) {
    auto it = hub_->epochs.find(cfg_.epoch);
    if (it != hub_->epochs.end()) {
      auto& pl = it->second.planes;
      if (cfg_.id < static_cast<int>(pl.size()) && pl[cfg_.id] == this) pl[cfg_.id] = nullptr;
      if (std::all_of(pl.begin(), pl.end(), [](LoopbackRoundPlane* p) { return p == nullptr; }))
        hub_->epochs.erase(it);
    }
  }
  const int P = cfg.peers;
  LoopbackHub::Epoch& E = hub_->epochs[cfg.epoch];
  const int64_t block = f32_ceil_div(cfg.dataSize, P);  // AllreduceWorker.scala:211-214
  const int nch = static_cast<int>(std::max<int64_t>(1, (block + cfg.maxChunkSize - 1) / cfg.maxChunkSize));
  if (E.P == 0) {
    E.P = P;
    E.dataSize = cfg.dataSize;
    E.maxLag = cfg.maxLag;
    E.block = block;
    E.chunk = cfg.maxChunkSize;
    E.nch = nch;
    E.min_reduce = std::max(1, f32_threshold_count(cfg.thReduce, P));
    E.min_complete = f32_threshold_chunks(cfg.thComplete, P, nch);
    E.planes.assign(P, nullptr);
  } else if (E.P != P || E.dataSize != cfg.dataSize || E.chunk != cfg.maxChunkSize) {
    throw ProtocolError("loopback plane: workers of epoch " + std::to_string(cfg.epoch) + " disagree on the geometry");
  }
  if (cfg.id < 0 || cfg.id >= P) throw ProtocolError("loopback plane: bad worker id");
  E.planes[cfg.id] = this;
  cfg_ = cfg;
  nch_ = nch;
  configured_ = true;
  forced_upto_ = cfg.startRound - 1;
  progress_ = cfg.startRound - 1;
  q_.clear();
  hub_->run(cfg.epoch, work);
}

void LoopbackRoundPlane::launch(int round, const Payload& input, bool cold) {
  if (!configured_) throw ProtocolError("loopback plane: launch before configure (InitWorkers)");
  if (!cold && (!input || static_cast<int>(input->size()) != cfg_.dataSize))
    throw ProtocolError("loopback plane: input must hold dataSize elements");
  std::deque<int> work;
  std::lock_guard<std::mutex> g(hub_->mu);
  if (!q_.empty() && round != q_.back().round + 1) throw ProtocolError("loopback plane: rounds must be launched in order");
  Pending x;
  x.round = round;
  x.input = cold ? nullptr : input;
  x.cold = cold;
  q_.push_back(std::move(x));
  st_.launches++;
  if (cold) st_.cold++;
  const bool ready = std::all_of(q_.begin(), std::prev(q_.end()), [](const Pending& y) { return y.done; });
  auto it = hub_->epochs.find(cfg_.epoch);
  if (ready && it != hub_->epochs.end()) hub_->activate(it->second, this, q_.back(), work);
  hub_->run(cfg_.epoch, work);
}

void LoopbackRoundPlane::force(int round) {
  if (!configured_) return;
  std::deque<int> work;
  std::lock_guard<std::mutex> g(hub_->mu);
  if (round <= forced_upto_) return;
  forced_upto_ = round;
  for (auto& y : q_)
    if (y.active && !y.done && y.round <= round) work.push_back(y.round);
  hub_->run(cfg_.epoch, work);
}

void LoopbackRoundPlane::drain() {
  std::unique_lock<std::mutex> lk(hub_->mu);
  cv_idle_.wait(lk, [&] { return q_.empty(); });
}

LoopbackPlaneStats LoopbackRoundPlane::stats() const {
  std::lock_guard<std::mutex> g(hub_->mu);
  return st_;
}

void LoopbackRoundPlane::deliver_loop() {
  for (;;) {
    RoundResult res;
    {
      std::unique_lock<std::mutex> lk(hub_->mu);
      hub_->cv.wait(lk, [&] { return stop_ || (!q_.empty() && q_.front().done); });
      if (q_.empty() || !q_.front().done) {
        if (stop_) return;
        continue;
      }
      res = std::move(q_.front().res);
    }
    {
      std::lock_guard<std::mutex> g(done_mu_);
      if (done_) done_(std::move(res));
    }
    {
      std::lock_guard<std::mutex> g(hub_->mu);
      q_.pop_front();
    }
    cv_idle_.notify_all();
  }
}

std::shared_ptr<LoopbackRoundPlane> make_loopback_plane(const std::string& hub) {
  return std::make_shared<LoopbackRoundPlane>(hub);
}

}  // namespace mxar
