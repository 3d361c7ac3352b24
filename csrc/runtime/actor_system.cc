#include "../core/env.h"
#include "actor_system.h"

#include <algorithm>
#include <cstdlib>
#include <thread>

#include "../core/log.h"

namespace mxar {

namespace {
std::atomic<uint64_t> g_uid{1};

// The dispatcher thread's run-next slot (ActorSystem::lifo_): set while the thread runs an
// actor turn of `tl_sys`; a cell that turn schedules waits in `tl_next`.
thread_local ActorSystem* tl_sys = nullptr;
thread_local bool tl_in_turn = false;
thread_local std::shared_ptr<ActorCell> tl_next;

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

// Timed condition-variable waits go through system_clock deadlines: libstdc++ implements
// steady_clock waits with pthread_cond_clockwait, which ThreadSanitizer (GCC 11) does not
// intercept - it would miss the unlock inside the wait and report phantom double locks.
// A system_clock deadline uses pthread_cond_timedwait, which every sanitizer models.
template <class Pred>
bool cv_wait_for(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, std::chrono::milliseconds d,
                 Pred pred) {
  const auto deadline = std::chrono::system_clock::now() + d;
  while (!pred()) {
    if (cv.wait_until(lk, deadline) == std::cv_status::timeout) return pred();
  }
  return true;
}
}

ActorRefBase::ActorRefBase() : uid_(g_uid.fetch_add(1)) {}

const char* message_name(const Message& m) {
  static const char* names[] = {"InitWorkers",    "StartAllreduce", "ScatterBlock",
                                "ReduceBlock",    "CompleteAllreduce", "MemberUp",
                                "Terminated",     "AllreduceFinished", "PoisonPill",
                                "TextMessage",    "RoundTimeout",      "PlaneRoundDone",
                                "BridgeCommand"};
  static_assert(sizeof(names) / sizeof(names[0]) == std::variant_size_v<Message>, "one name per message");
  return names[m.index()];
}

// ------------------------------------------------------------------------ context
ActorRef ActorContext::self() const { return cell_->ref(); }

void ActorContext::watch(const ActorRef& ref) {
  if (!ref) return;
  auto* local = dynamic_cast<LocalActorRef*>(ref.get());
  if (!local) {  // remote refs: the cluster layer's failure detector reports them
    if (ref->is_remote())
      if (auto h = sys_->remote_watch_hook()) h(ref, self(), true);
    return;
  }
  auto c = local->cell();
  ActorRef me = self();
  if (!c || c->stopped()) {
    me->tell(Terminated{ref}, nullptr);
    return;
  }
  std::lock_guard<std::mutex> g(c->mu_);
  c->watchers_.insert(me);
}

void ActorContext::unwatch(const ActorRef& ref) {
  auto* local = dynamic_cast<LocalActorRef*>(ref.get());
  if (!local) {
    if (ref && ref->is_remote())
      if (auto h = sys_->remote_watch_hook()) h(ref, self(), false);
    return;
  }
  auto c = local->cell();
  if (!c) return;
  std::lock_guard<std::mutex> g(c->mu_);
  c->watchers_.erase(self());
}

// stash / unstash run inside the actor's own turn: the cell's consumer-private queues
void ActorContext::stash(Envelope env) { cell_->stash_.push_back(std::move(env)); }

void ActorContext::unstash_all() {
  // Stashed messages go back to the FRONT of the mailbox, in their original order
  // (Akka's Stash.unstashAll semantics).
  const auto n = static_cast<int64_t>(cell_->stash_.size());
  if (n == 0) return;
  cell_->pending_.fetch_add(n);
  while (!cell_->stash_.empty()) {
    cell_->front_.push_front(std::move(cell_->stash_.back()));
    cell_->stash_.pop_back();
  }
}

void ActorContext::stop_self() { cell_->stop_requested_ = true; }

// ------------------------------------------------------------------------ refs
void LocalActorRef::tell(Message msg, ActorRef sender) {
  auto c = cell_.lock();
  if (!c || c->stopped()) {
    sys_->dead_letters()->tell(std::move(msg), std::move(sender));
    return;
  }
  c->enqueue(Envelope{std::move(msg), std::move(sender)});
}

void ProbeRef::tell(Message msg, ActorRef sender) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(Envelope{std::move(msg), std::move(sender)});
  }
  cv_.notify_all();
}

std::optional<Envelope> ProbeRef::receive(std::chrono::milliseconds timeout) {
  if (sys_->deterministic()) {
    sys_->run_until_idle();
    std::lock_guard<std::mutex> g(mu_);
    if (q_.empty()) return std::nullopt;
    Envelope e = std::move(q_.front());
    q_.pop_front();
    return e;
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (!cv_wait_for(cv_, lk, timeout, [&] { return !q_.empty(); })) return std::nullopt;
  Envelope e = std::move(q_.front());
  q_.pop_front();
  return e;
}

size_t ProbeRef::pending() {
  if (sys_->deterministic()) sys_->run_until_idle();
  std::lock_guard<std::mutex> g(mu_);
  return q_.size();
}

void ProbeRef::clear() {
  std::lock_guard<std::mutex> g(mu_);
  q_.clear();
}

void DeadLetterRef::tell(Message msg, ActorRef sender) {
  count_.fetch_add(1);
  sys_->note_dead_letter(msg, sender);
}

// ------------------------------------------------------------------------ mailbox
MpscMailbox::MpscMailbox() {
  head_ = new Node;
  tail_.store(head_, std::memory_order_relaxed);
}

MpscMailbox::~MpscMailbox() {
  Envelope e;
  while (pop(e)) {
  }
  delete head_;
}

// Per-thread node cache: a dispatcher thread frees the nodes of the mail it consumes and
// allocates nodes for the mail its actors send, so nodes cycle within a thread without
// touching the allocator (glibc's per-thread cache holds only 7 blocks per size; a round's
// burst of Scatter/Reduce messages overflowed it into the locked arena bins).
struct MpscMailbox::NodeCache {
  std::vector<Node*> free;
  ~NodeCache() {
    for (Node* n : free) delete n;
  }
  static NodeCache& local() {
    thread_local NodeCache c;
    return c;
  }
};

MpscMailbox::Node* MpscMailbox::alloc_node() {
  auto& c = NodeCache::local().free;
  if (c.empty()) return new Node;
  Node* n = c.back();
  c.pop_back();
  n->next.store(nullptr, std::memory_order_relaxed);
  return n;
}

void MpscMailbox::free_node(Node* n) {
  auto& c = NodeCache::local().free;
  if (c.size() >= 1024) {
    delete n;
    return;
  }
  n->env = Envelope{};  // drop the payload / sender references now
  c.push_back(n);
}

void MpscMailbox::push(Envelope&& e) {
  Node* n = alloc_node();
  n->env = std::move(e);
  Node* prev = tail_.exchange(n, std::memory_order_acq_rel);
  prev->next.store(n, std::memory_order_release);  // the consumer may now reach n
}

bool MpscMailbox::pop(Envelope& out) {
  Node* h = head_;
  Node* next = h->next.load(std::memory_order_acquire);
  if (next == nullptr) return false;  // empty, or a push between its exchange and its link
  out = std::move(next->env);
  head_ = next;  // next becomes the stub
  free_node(h);
  return true;
}

// ------------------------------------------------------------------------ cell
ActorCell::ActorCell(ActorSystem* sys, std::unique_ptr<Actor> actor, std::string path)
    : sys_(sys), actor_(std::move(actor)), path_(std::move(path)) {}

void ActorCell::enqueue(Envelope env) {
  // count first (seq_cst), then push, then try to schedule: a dispatcher that clears
  // scheduled_ and then reads pending_ sees this message whenever our schedule() lost
  pending_.fetch_add(1);
  actor_->on_enqueue(env.msg);
  mailbox_.push(std::move(env));
  sys_->schedule(shared_from_this());
}

bool ActorCell::has_mail() { return pending_.load() > 0; }

size_t ActorCell::process(size_t n) {
  ActorContext ctx(sys_, this);
  if (!started_.exchange(true)) {
    try {
      actor_->pre_start(ctx);
    } catch (...) {
      sys_->record_exception(std::current_exception());
    }
  }
  size_t done = 0;
  while (done < n && !stopped_) {
    Envelope env;
    if (!front_.empty()) {
      env = std::move(front_.front());
      front_.pop_front();
    } else if (!mailbox_.pop(env)) {
      break;  // empty (or a push not linked yet: pending_ keeps the cell scheduled)
    }
    pending_.fetch_sub(1);
    ++done;
    if (std::holds_alternative<PoisonPill>(env.msg)) {
      do_stop();
      break;
    }
    ctx.sender_ = env.sender;
    try {
      actor_->receive(env, ctx);
    } catch (const std::exception& e) {
      // Supervision: "resume" - the actor keeps its state (the reference's default
      // restart would reset an initialised worker to id = -1).
      sys_->note_failure(path_, e.what());
      sys_->record_exception(std::current_exception());
    } catch (...) {
      sys_->note_failure(path_, "unknown exception");
      sys_->record_exception(std::current_exception());
    }
    if (stop_requested_) {
      do_stop();
      break;
    }
    // A cell this turn put in the run-next slot waits for the turn to end. When the turn goes
    // on (more mail), it goes to the run queue for an idle thread instead: a straggling worker
    // whose handler blocks in its dataSource for 2 ms per message held the master - scheduled
    // by the worker's CompleteAllreduce - for two or three such messages, stalling every fast
    // worker's round with it (profiles/round6/README.md section 6).
    if (tl_next && tl_sys == sys_ && done < n && pending_.load() > 0) {
      std::shared_ptr<ActorCell> next = std::move(tl_next);
      tl_next.reset();
      sys_->enqueue(next);
    }
  }
  return done;
}

void ActorCell::do_stop() {
  if (stopped_.exchange(true)) return;
  ActorContext ctx(sys_, this);
  try {
    actor_->post_stop(ctx);
  } catch (...) {
  }
  std::set<ActorRef> w;
  {
    std::lock_guard<std::mutex> g(mu_);
    w.swap(watchers_);
  }
  std::deque<Envelope> rest;
  rest.swap(front_);
  for (Envelope e; mailbox_.pop(e);) rest.push_back(std::move(e));
  pending_.fetch_sub(static_cast<int64_t>(rest.size()));
  ActorRef me = ref();
  for (auto& e : rest) sys_->dead_letters()->tell(std::move(e.msg), e.sender);
  for (auto& watcher : w) watcher->tell(Terminated{me}, me);
  sys_->remove_cell(path_);
}

// ------------------------------------------------------------------------ system
ActorSystem::ActorSystem(std::string name, Mode mode, int threads, int throughput)
    : name_(std::move(name)), mode_(mode), throughput_(std::max(1, throughput)) {
  dead_letters_ = std::make_shared<DeadLetterRef>(this);
  virtual_now_ = std::chrono::steady_clock::time_point{};
  if (mode_ == Mode::Threaded) {
    // A dispatcher thread that ran out of work polls the run queue for MXAR_DISPATCH_SPIN_US
    // (default 50 us) before it sleeps on the condition variable: a protocol round is a chain
    // of actor hops (Start -> worker, plane done -> worker, Complete -> master), and a futex
    // wake-up per hop costs more than the hop itself.
    spin_us_ = 50;
    if (const char* e = std::getenv("MXAR_DISPATCH_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
    if (const char* e = study_env("MXAR_DISPATCH_LIFO")) lifo_ = std::atoi(e) != 0;
    if (const char* e = study_env("MXAR_DISPATCH_SPINNERS")) max_spinners_ = std::max(1, std::atoi(e));
    int n = threads > 0 ? threads : std::max(2u, std::min(8u, std::thread::hardware_concurrency()));
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { worker_loop(); });
    timer_thread_ = std::thread([this] { timer_loop(); });
  }
}

ActorSystem::~ActorSystem() { shutdown(); }

void ActorSystem::shutdown() {
  if (shutdown_.exchange(true)) return;
  rq_cv_.notify_all();
  timer_cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  if (timer_thread_.joinable()) timer_thread_.join();
  std::map<std::string, std::shared_ptr<ActorCell>> cells;
  {
    std::lock_guard<std::mutex> g(reg_mu_);
    cells.swap(cells_);
    refs_.clear();
  }
  for (auto& [p, c] : cells) {
    ActorContext ctx(this, c.get());
    if (!c->stopped_.exchange(true)) {
      try {
        c->actor_->post_stop(ctx);
      } catch (...) {
      }
    }
  }
  std::lock_guard<std::mutex> g(rq_mu_);
  runq_.clear();
}

ActorRef ActorSystem::actor_of(std::unique_ptr<Actor> actor, std::string name) {
  std::string path;
  std::shared_ptr<ActorCell> cell;
  ActorRef ref;
  {
    std::lock_guard<std::mutex> g(reg_mu_);
    if (name.empty()) name = "$" + std::to_string(++name_counter_);
    path = "/user/" + name;
    if (cells_.count(path)) throw std::runtime_error("actor name [" + name + "] is not unique!");
    cell = std::make_shared<ActorCell>(this, std::move(actor), path);
    ref = std::make_shared<LocalActorRef>(cell, path, this);
    cell->ref_ = ref;
    cells_[path] = cell;
    refs_[path] = ref;
  }
  // pre_start runs on the actor's first turn; schedule one so it happens promptly.
  if (mode_ == Mode::Threaded) schedule(cell);
  return ref;
}

std::shared_ptr<ProbeRef> ActorSystem::make_probe(std::string name) {
  std::lock_guard<std::mutex> g(reg_mu_);
  if (name.empty()) name = "testActor" + std::to_string(++name_counter_);
  auto p = std::make_shared<ProbeRef>("/system/" + name, this);
  refs_[p->path()] = p;
  return p;
}

ActorRef ActorSystem::lookup(const std::string& path) {
  std::lock_guard<std::mutex> g(reg_mu_);
  auto it = refs_.find(path);
  return it == refs_.end() ? nullptr : it->second;
}

void ActorSystem::stop(const ActorRef& ref) {
  if (ref) ref->tell(PoisonPill{}, nullptr);
}

void ActorSystem::remove_cell(const std::string& path) {
  std::lock_guard<std::mutex> g(reg_mu_);
  cells_.erase(path);
  refs_.erase(path);
}

void ActorSystem::schedule(const std::shared_ptr<ActorCell>& cell) {
  if (cell->scheduled_.exchange(true)) return;
  if (lifo_ && tl_in_turn && tl_sys == this) {
    // scheduled by an actor turn on this dispatcher: run it next here; a cell already in the
    // slot goes to the run queue (for any idle thread to take)
    std::shared_ptr<ActorCell> prev = std::move(tl_next);
    tl_next = cell;
    if (!prev) return;
    return enqueue(prev);
  }
  enqueue(cell);
}

void ActorSystem::enqueue(const std::shared_ptr<ActorCell>& cell) {
  size_t queued;
  {
    std::lock_guard<std::mutex> g(rq_mu_);
    runq_.push_back(cell);
    queued = runq_.size();
    runq_len_.store(queued, std::memory_order_release);
  }
  // A spinning dispatcher takes the cell without a wake-up: the futex syscall of notify_one
  // would sit on the sender's critical path (every hop of a protocol round). No lost wake-up:
  // a spinner decrements spinning_ BEFORE it locks rq_mu_ and tests the queue, so either it
  // sees this push under the lock, or the push came later and this load sees it gone.
  // (One spinner per queued cell: with fewer, a sleeper is woken so that cells queued
  // back to back - a Start to every worker - still run in parallel.)
  if (static_cast<size_t>(spinning_.load(std::memory_order_seq_cst)) < queued) rq_cv_.notify_one();
}

void ActorSystem::record_exception(std::exception_ptr e) {
  if (mode_ != Mode::Deterministic) return;
  std::lock_guard<std::mutex> g(exc_mu_);
  if (!pending_exc_) pending_exc_ = e;
}

size_t ActorSystem::run_until_idle(size_t max_messages) {
  if (mode_ != Mode::Deterministic) throw std::runtime_error("run_until_idle needs a deterministic system");
  size_t total = 0;
  while (total < max_messages) {
    std::shared_ptr<ActorCell> cell;
    {
      std::lock_guard<std::mutex> g(rq_mu_);
      if (runq_.empty()) break;
      cell = runq_.front();
      runq_.pop_front();
      runq_len_.store(runq_.size(), std::memory_order_release);
    }
    cell->scheduled_.store(false);
    total += cell->process(1);  // one message per turn: fair round-robin interleaving
    if (!cell->stopped() && cell->has_mail()) schedule(cell);
    std::exception_ptr e;
    {
      std::lock_guard<std::mutex> g(exc_mu_);
      std::swap(e, pending_exc_);
    }
    if (e) std::rethrow_exception(e);
  }
  delivered_.fetch_add(total, std::memory_order_relaxed);
  return total;
}

void ActorSystem::worker_loop() {
  tl_sys = this;
  while (true) {
    std::shared_ptr<ActorCell> cell;
    if (tl_next) {  // the run-next slot: still counted busy since the turn that filled it
      cell = std::move(tl_next);
      tl_next.reset();
    } else {
      // Idle spin, by at most max_spinners_ threads at a time (the rest sleep at once: a cell
      // queued back to back with another wakes one of them): pause-based polling (a hop costs
      // ~0.1 us to notice), yielding the core every ~32 polls so that an oversubscribed host
      // still runs everyone.
      // (A thread over the cap counts in spinning_ until it decrements, which it does before
      // it locks rq_mu_ and tests the queue: it takes a cell schedule() did not wake anyone for.)
      if (spin_us_ > 0 && runq_len_.load(std::memory_order_acquire) == 0) {
        if (spinning_.fetch_add(1, std::memory_order_seq_cst) < max_spinners_) {
          const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us_);
          for (unsigned i = 1; runq_len_.load(std::memory_order_acquire) == 0 && !shutdown_.load() &&
                               std::chrono::steady_clock::now() < until;
               ++i) {
            if ((i & 31) == 0) {
              std::this_thread::yield();
            } else {
              for (int k = 0; k < 8; ++k) cpu_relax();
            }
          }
        }
        spinning_.fetch_sub(1, std::memory_order_seq_cst);
      }
      std::unique_lock<std::mutex> lk(rq_mu_);
      rq_cv_.wait(lk, [&] { return shutdown_.load() || !runq_.empty(); });
      if (shutdown_) return;
      cell = runq_.front();
      runq_.pop_front();
      runq_len_.store(runq_.size(), std::memory_order_release);
      ++busy_;
    }
    tl_in_turn = true;
    size_t n = cell->process(static_cast<size_t>(throughput_));
    tl_in_turn = false;
    cell->scheduled_.store(false);
    // Re-check after clearing the flag: a message may have arrived in between (to the run
    // queue, not the run-next slot: a busy actor must not monopolise this thread).
    if (!cell->stopped() && cell->has_mail()) schedule(cell);
    delivered_.fetch_add(n, std::memory_order_relaxed);
    if (tl_next && shutdown_.load()) {
      // shutting down: the slot's cell goes back to the queue (cleared by shutdown())
      std::shared_ptr<ActorCell> c = std::move(tl_next);
      tl_next.reset();
      enqueue(c);
    }
    if (!tl_next) {
      std::lock_guard<std::mutex> g(rq_mu_);
      --busy_;
      if (busy_ == 0 && runq_.empty()) idle_cv_.notify_all();
    }
  }
}

bool ActorSystem::await_idle(std::chrono::milliseconds timeout) {
  if (mode_ == Mode::Deterministic) {
    run_until_idle();
    return true;
  }
  std::unique_lock<std::mutex> lk(rq_mu_);
  return cv_wait_for(idle_cv_, lk, timeout, [&] { return busy_ == 0 && runq_.empty(); });
}

// ------------------------------------------------------------------------ timers
uint64_t ActorSystem::schedule_once(std::chrono::milliseconds delay, ActorRef target, Message msg) {
  auto shared = std::make_shared<Message>(std::move(msg));
  std::lock_guard<std::mutex> g(timer_mu_);
  const auto now = mode_ == Mode::Deterministic ? virtual_now_ : std::chrono::steady_clock::now();
  Timer t{++timer_seq_, now + delay, std::chrono::milliseconds(0), std::move(target),
          [shared] { return *shared; }};
  timers_.push_back(std::move(t));
  timer_cv_.notify_all();
  return timer_seq_;
}

uint64_t ActorSystem::schedule_repeated(std::chrono::milliseconds initial, std::chrono::milliseconds period,
                                        ActorRef target, std::function<Message()> make) {
  std::lock_guard<std::mutex> g(timer_mu_);
  const auto now = mode_ == Mode::Deterministic ? virtual_now_ : std::chrono::steady_clock::now();
  timers_.push_back(Timer{++timer_seq_, now + initial, period, std::move(target), std::move(make)});
  timer_cv_.notify_all();
  return timer_seq_;
}

void ActorSystem::cancel(uint64_t id) {
  std::lock_guard<std::mutex> g(timer_mu_);
  timers_.erase(std::remove_if(timers_.begin(), timers_.end(), [&](const Timer& t) { return t.id == id; }),
                timers_.end());
}

void ActorSystem::fire_due_timers_locked(std::chrono::steady_clock::time_point now,
                                         std::vector<std::pair<ActorRef, Message>>& out) {
  std::sort(timers_.begin(), timers_.end(), [](const Timer& a, const Timer& b) {
    return a.due < b.due || (a.due == b.due && a.id < b.id);
  });
  std::vector<Timer> keep;
  for (auto& t : timers_) {
    if (t.due <= now) {
      out.emplace_back(t.target, t.make());
      if (t.period.count() > 0) {
        t.due += t.period;
        keep.push_back(std::move(t));
      }
    } else {
      keep.push_back(std::move(t));
    }
  }
  timers_.swap(keep);
}

void ActorSystem::advance_time(std::chrono::milliseconds dt) {
  if (mode_ != Mode::Deterministic) throw std::runtime_error("advance_time needs a deterministic system");
  const auto target = virtual_now_ + dt;
  while (true) {
    std::vector<std::pair<ActorRef, Message>> fire;
    {
      std::lock_guard<std::mutex> g(timer_mu_);
      // fire timers one due-instant at a time so periodic timers interleave correctly
      std::chrono::steady_clock::time_point next = target;
      for (auto& t : timers_) next = std::min(next, t.due);
      if (next > target || timers_.empty()) {
        virtual_now_ = target;
        break;
      }
      virtual_now_ = next;
      fire_due_timers_locked(virtual_now_, fire);
      if (fire.empty()) {
        virtual_now_ = target;
        break;
      }
    }
    for (auto& [ref, msg] : fire) ref->tell(std::move(msg), nullptr);
    run_until_idle();
  }
}

void ActorSystem::timer_loop() {
  std::unique_lock<std::mutex> lk(timer_mu_);
  while (!shutdown_) {
    auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
    for (auto& t : timers_) next = std::min(next, t.due);
    const auto wait = std::chrono::duration_cast<std::chrono::microseconds>(next - std::chrono::steady_clock::now());
    if (wait.count() > 0) timer_cv_.wait_until(lk, std::chrono::system_clock::now() + wait);
    if (shutdown_) break;
    std::vector<std::pair<ActorRef, Message>> fire;
    fire_due_timers_locked(std::chrono::steady_clock::now(), fire);
    lk.unlock();
    for (auto& [ref, msg] : fire) ref->tell(std::move(msg), nullptr);
    lk.lock();
  }
}

// ------------------------------------------------------------------------ stats
SystemStats ActorSystem::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  SystemStats s = stats_;
  s.delivered = delivered_.load(std::memory_order_relaxed);
  s.dead_letters = dead_letters_->count();
  return s;
}

void ActorSystem::note_dead_letter(const Message& m, const ActorRef& sender) {
  uint64_t n;
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    n = ++dead_letters_logged_;
  }
  if (n <= 5)  // application.conf:23 log-dead-letters = 5
    MXAR_LOG(INFO, name_, "Message [" << message_name(m) << "] from " << (sender ? sender->path() : "noSender")
                                      << " was not delivered. [" << n << "] dead letters encountered.");
}

void ActorSystem::note_failure(const std::string& path, const std::string& what) {
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.actor_failures++;
  }
  MXAR_LOG(ERROR, name_, "actor " << path << " failed: " << what << " (resuming)");
}

}  // namespace mxar
