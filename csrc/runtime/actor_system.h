// Lightweight actor runtime: mailboxes, dispatcher, DeathWatch, stash, timers, dead
// letters and test probes. Replaces the parts of Akka the reference relies on
// (SURVEY §1 layer L0, build.sbt:15-27): `Actor`, `ActorRef.!`, per-sender FIFO,
// `context.watch` / `Terminated`, and the TestKit `testActor`.
//
// Two execution modes:
//   * Threaded      - a pool of dispatcher threads; an actor is scheduled when mail
//                     arrives and processes up to `throughput` messages per turn
//                     (Akka's default dispatcher model). Used by clusters and CLIs.
//   * Deterministic - no threads; the host calls run_until_idle() and actors are
//                     stepped round-robin one message at a time. Message order is then
//                     a pure function of the program, which the conformance tests need
//                     (test T1 only passes under "batch then drain").
// Per (sender, receiver) FIFO holds in both modes: one mailbox per actor, a lock-free
// multi-producer / single-consumer queue (MpscMailbox): a tell() is one atomic exchange
// plus one release store, never a lock, and the dispatcher thread that holds the actor's
// turn is the only consumer.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../core/protocol.h"

namespace mxar {

class ActorSystem;
class ActorCell;

struct Envelope {
  Message msg;
  ActorRef sender;
};

class ActorRefBase : public std::enable_shared_from_this<ActorRefBase> {
 public:
  ActorRefBase();
  virtual ~ActorRefBase() = default;
  virtual void tell(Message msg, ActorRef sender) = 0;
  virtual std::string path() const = 0;
  virtual bool is_remote() const { return false; }
  virtual bool is_probe() const { return false; }
  uint64_t uid() const { return uid_; }

 private:
  uint64_t uid_;
};

class ActorContext;

class Actor {
 public:
  virtual ~Actor() = default;
  virtual void pre_start(ActorContext&) {}
  virtual void receive(Envelope& env, ActorContext& ctx) = 0;
  virtual void post_stop(ActorContext&) {}
  virtual std::string kind() const { return "actor"; }
  // Called on the SENDER's thread as a message is enqueued (before the push): a hint an actor
  // may record with atomics only (it may run concurrently with receive()). PlaneWorkerActor
  // notes the newest StartAllreduce in its mailbox here.
  virtual void on_enqueue(const Message&) {}
};

class ActorContext {
 public:
  ActorContext(ActorSystem* sys, ActorCell* cell) : sys_(sys), cell_(cell) {}
  ActorRef self() const;
  const ActorRef& sender() const { return sender_; }
  ActorSystem& system() const { return *sys_; }
  void watch(const ActorRef& ref);
  void unwatch(const ActorRef& ref);
  void stash(Envelope env);
  void unstash_all();
  void stop_self();

 private:
  friend class ActorCell;
  ActorSystem* sys_;
  ActorCell* cell_;
  ActorRef sender_;
};

// Local actor reference.
class LocalActorRef final : public ActorRefBase {
 public:
  explicit LocalActorRef(std::weak_ptr<ActorCell> cell, std::string path, ActorSystem* sys)
      : cell_(std::move(cell)), path_(std::move(path)), sys_(sys) {}
  void tell(Message msg, ActorRef sender) override;
  std::string path() const override { return path_; }
  std::shared_ptr<ActorCell> cell() const { return cell_.lock(); }

 private:
  std::weak_ptr<ActorCell> cell_;
  std::string path_;
  ActorSystem* sys_;
};

// TestKit-style probe: every message sent to it is queued for the test to inspect.
class ProbeRef final : public ActorRefBase {
 public:
  ProbeRef(std::string path, ActorSystem* sys) : path_(std::move(path)), sys_(sys) {}
  void tell(Message msg, ActorRef sender) override;
  std::string path() const override { return path_; }
  bool is_probe() const override { return true; }
  // Deterministic mode: drains the system first, then pops (nullopt when empty).
  // Threaded mode: waits up to `timeout` for a message.
  std::optional<Envelope> receive(std::chrono::milliseconds timeout);
  size_t pending();
  void clear();

 private:
  std::string path_;
  ActorSystem* sys_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Envelope> q_;
};

// Sink for messages to stopped / unknown actors (application.conf:23 log-dead-letters = 5).
class DeadLetterRef final : public ActorRefBase {
 public:
  explicit DeadLetterRef(ActorSystem* sys) : sys_(sys) {}
  void tell(Message msg, ActorRef sender) override;
  std::string path() const override { return "/deadLetters"; }
  uint64_t count() const { return count_.load(); }

 private:
  ActorSystem* sys_;
  std::atomic<uint64_t> count_{0};
};

// Unbounded MPSC queue (D. Vyukov's stub-node list). Producers swap the tail and link the
// previous node; the single consumer walks from the stub. A push whose link is not yet
// visible reads as "empty" for a moment - the cell's `pending_` count (raised before the
// push) keeps such a cell scheduled, so no message is ever stranded.
class MpscMailbox {
 public:
  MpscMailbox();
  ~MpscMailbox();
  MpscMailbox(const MpscMailbox&) = delete;
  MpscMailbox& operator=(const MpscMailbox&) = delete;
  void push(Envelope&& e);  // any thread
  bool pop(Envelope& out);  // the consumer only

 private:
  struct Node {
    std::atomic<Node*> next{nullptr};
    Envelope env;
  };
  struct NodeCache;
  static Node* alloc_node();
  static void free_node(Node* n);
  alignas(64) std::atomic<Node*> tail_;
  alignas(64) Node* head_;
};

class ActorCell : public std::enable_shared_from_this<ActorCell> {
 public:
  ActorCell(ActorSystem* sys, std::unique_ptr<Actor> actor, std::string path);
  void enqueue(Envelope env);
  // Processes up to n messages; returns how many were processed.
  size_t process(size_t n);
  bool has_mail();
  const std::string& path() const { return path_; }
  ActorRef ref() const { return ref_.lock(); }
  Actor* actor() { return actor_.get(); }
  bool stopped() const { return stopped_.load(); }

 private:
  friend class ActorSystem;
  friend class ActorContext;
  void do_stop();
  ActorSystem* sys_;
  std::unique_ptr<Actor> actor_;
  std::string path_;
  std::weak_ptr<ActorRefBase> ref_;
  std::mutex mu_;  // watchers_ only (the mail path takes no lock)
  MpscMailbox mailbox_;
  // Consumer-private (the actor's own turn): unstashed messages, delivered before the
  // mailbox (Akka's Stash.unstashAll prepends), and the stash itself.
  std::deque<Envelope> front_;
  std::deque<Envelope> stash_;
  // Messages pushed or unstashed and not yet taken; raised BEFORE a push, so a dispatcher
  // that releases the cell and then reads it cannot miss a concurrent tell().
  std::atomic<int64_t> pending_{0};
  std::set<ActorRef> watchers_;
  std::atomic<bool> scheduled_{false};
  std::atomic<bool> stopped_{false};
  std::atomic<bool> started_{false};
  bool stop_requested_ = false;
};

struct SystemStats {
  uint64_t delivered = 0;
  uint64_t dead_letters = 0;
  uint64_t actor_failures = 0;
};

class ActorSystem {
 public:
  enum class Mode { Threaded, Deterministic };

  ActorSystem(std::string name, Mode mode, int threads = 0, int throughput = 64);
  ~ActorSystem();
  ActorSystem(const ActorSystem&) = delete;
  ActorSystem& operator=(const ActorSystem&) = delete;

  const std::string& name() const { return name_; }
  Mode mode() const { return mode_; }
  bool deterministic() const { return mode_ == Mode::Deterministic; }

  // Creates "/user/<name>" (a unique name is generated when empty).
  ActorRef actor_of(std::unique_ptr<Actor> actor, std::string name = "");
  std::shared_ptr<ProbeRef> make_probe(std::string name = "");
  ActorRef dead_letters() const { return dead_letters_; }
  ActorRef lookup(const std::string& path);
  void stop(const ActorRef& ref);

  // Deterministic mode: run until no actor has mail (or max_messages processed).
  // Rethrows the first exception an actor raised while processing.
  size_t run_until_idle(size_t max_messages = SIZE_MAX);
  // Deterministic mode virtual clock: advance and fire due timers.
  void advance_time(std::chrono::milliseconds dt);

  // Timers (both modes). Returns a handle for cancel().
  uint64_t schedule_once(std::chrono::milliseconds delay, ActorRef target, Message msg);
  uint64_t schedule_repeated(std::chrono::milliseconds initial, std::chrono::milliseconds period,
                             ActorRef target, std::function<Message()> make);
  void cancel(uint64_t timer);

  // Threaded mode: block until no actor has mail and no message is being processed.
  bool await_idle(std::chrono::milliseconds timeout);
  void shutdown();
  bool terminated() const { return shutdown_.load(); }

  SystemStats stats();
  void note_dead_letter(const Message& m, const ActorRef& sender);

  // DeathWatch for remote refs is delegated to the cluster layer (csrc/cluster).
  using RemoteWatchHook = std::function<void(const ActorRef& target, const ActorRef& watcher, bool watch)>;
  void set_remote_watch_hook(RemoteWatchHook h) {
    std::lock_guard<std::mutex> g(hook_mu_);
    remote_watch_ = std::move(h);
  }
  RemoteWatchHook remote_watch_hook() {
    std::lock_guard<std::mutex> g(hook_mu_);
    return remote_watch_;
  }
  void note_failure(const std::string& path, const std::string& what);

  // Called by cells/refs.
  void schedule(const std::shared_ptr<ActorCell>& cell);
  void enqueue(const std::shared_ptr<ActorCell>& cell);  // run queue + wake-up (no run-next slot)
  void remove_cell(const std::string& path);
  void record_exception(std::exception_ptr e);

 private:
  void worker_loop();
  void timer_loop();
  void fire_due_timers_locked(std::chrono::steady_clock::time_point now,
                              std::vector<std::pair<ActorRef, Message>>& out);

  struct Timer {
    uint64_t id;
    std::chrono::steady_clock::time_point due;
    std::chrono::milliseconds period{0};
    ActorRef target;
    std::function<Message()> make;
  };

  std::string name_;
  Mode mode_;
  int throughput_;
  std::shared_ptr<DeadLetterRef> dead_letters_;

  std::mutex reg_mu_;
  std::map<std::string, std::shared_ptr<ActorCell>> cells_;
  std::map<std::string, ActorRef> refs_;
  uint64_t name_counter_ = 0;

  std::mutex rq_mu_;
  std::condition_variable rq_cv_;
  std::condition_variable idle_cv_;
  std::deque<std::shared_ptr<ActorCell>> runq_;
  std::atomic<size_t> runq_len_{0};  // runq_.size(), readable without rq_mu_ (idle spin)
  int spin_us_ = 0;                  // idle dispatcher threads poll this long before sleeping
  // dispatcher threads in their idle spin: schedule() skips the condition variable's futex
  // wake while one of them will see the run queue anyway
  std::atomic<int> spinning_{0};
  // run-next slot (MXAR_DISPATCH_LIFO, default on): a cell scheduled by an actor turn on a
  // dispatcher thread runs next on THAT thread, without a run-queue hop - a protocol round's
  // Complete -> master -> Start chain stays on one warm thread (Go's runnext)
  bool lifo_ = true;
  int max_spinners_ = 2;     // MXAR_DISPATCH_SPINNERS: dispatcher threads spinning at once
  int busy_ = 0;
  std::vector<std::thread> threads_;
  std::atomic<bool> shutdown_{false};

  std::mutex timer_mu_;
  std::condition_variable timer_cv_;
  std::vector<Timer> timers_;
  uint64_t timer_seq_ = 0;
  std::thread timer_thread_;
  std::chrono::steady_clock::time_point virtual_now_;

  std::mutex exc_mu_;
  std::exception_ptr pending_exc_;

  std::mutex stats_mu_;
  SystemStats stats_;
  std::atomic<uint64_t> delivered_{0};  // per-turn count without stats_mu_
  std::mutex hook_mu_;
  RemoteWatchHook remote_watch_;
  uint64_t dead_letters_logged_ = 0;
};

}  // namespace mxar
