// Host-runtime stress program for sanitizer builds (ThreadSanitizer / AddressSanitizer):
// the threaded actor system, the TCP cluster layer and the full master/worker protocol,
// with fault injection, exactly as the CLIs run them - but in one process without Python,
// so the sanitizer sees every thread. Exit 0 = all rounds exact and clean shutdown.
//
//   build + run: python tools/sanitize.py --sanitize thread
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../cluster/cluster_node.h"
#include "../core/log.h"
#include "../runtime/allreduce_actors.h"
#include "../runtime/akka_endpoint.h"
#include "../runtime/control_bridge.h"
#include "../runtime/fault_injector.h"
#include "../runtime/loopback_plane.h"
#include "../runtime/plane_worker.h"

using namespace mxar;

static bool wait_until(const std::function<bool()>& pred, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < timeout_s) {
    if (pred()) return true;
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  return false;
}

// In-process threaded cluster with reordering faults; exact thresholds.
static int run_local(int P, int N, int C, int rounds) {
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 4);
  std::atomic<bool> done{false};
  MasterParams mp{P, 1.f, 1.f, 1.f, 3, N, rounds - 1, C, false};
  ActorRef master = sys->actor_of(std::make_unique<MasterActor>(mp, [&](int) { done = true; }), "master");
  std::mutex mu;
  std::vector<std::vector<std::vector<float>>> outs(P);
  std::vector<ActorRef> refs;
  for (int k = 0; k < P; ++k) {
    DataSource src = [N, k](const AllReduceInputRequest& r) {
      std::vector<float> v(N);
      for (int i = 0; i < N; ++i) v[i] = static_cast<float>((i + r.iteration) * (k + 1));
      return AllReduceInput{make_host_payload(std::move(v))};
    };
    DataSink sink = [&, k](const AllReduceOutput& o) {
      std::lock_guard<std::mutex> g(mu);
      if (static_cast<int>(outs[k].size()) <= o.iteration) outs[k].resize(o.iteration + 1);
      outs[k][o.iteration] = o.data->to_host();
    };
    ActorRef w = sys->actor_of(std::make_unique<WorkerActor>(src, sink), "worker" + std::to_string(k));
    FaultPolicy fp;
    fp.delay_ms = 2;
    fp.delay_prob = 0.3;
    fp.kinds = {"ScatterBlock", "ReduceBlock"};
    fp.seed = 11 + k;
    refs.push_back(std::make_shared<FaultyRef>(sys.get(), w, fp));
  }
  for (auto& r : refs) master->tell(MemberUp{r, "worker", ""}, nullptr);
  const bool ok = wait_until([&] { return done.load(); }, 60);
  sys->await_idle(std::chrono::milliseconds(5000));
  sys->shutdown();
  if (!ok) {
    std::fprintf(stderr, "local cluster did not finish\n");
    return 1;
  }
  const float tri = P * (P + 1) / 2.f;
  for (int k = 0; k < P; ++k)
    for (int r = 0; r < rounds; ++r)
      for (int i = 0; i < N; ++i)
        if (std::fabs(outs[k][r][i] - (i + r) * tri) > 1e-3f) {
          std::fprintf(stderr, "bad sum worker %d round %d idx %d\n", k, r, i);
          return 1;
        }
  return 0;
}

// The control bridge (csrc/runtime/control_bridge.h): an external driver thread runs every
// round through a socket, pipelined (one StartAllreduce queued behind the round in flight),
// while churn threads connect, half-send and vanish - bridge reader / acceptor / reaper
// threads, the master's publishes and client fds all under the sanitizer.
static int connect_to(int port) {
  int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  ::inet_pton(AF_INET, "127.0.0.1", &a.sin_addr);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    ::close(fd);
    return -1;
  }
  return fd;
}

static int run_bridge(int P, int N, int C, int rounds) {
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 4);
  std::atomic<bool> done{false};
  MasterParams mp{P, 1.f, 1.f, 1.f, 1, N, rounds - 1, C, false};
  mp.externalRounds = true;
  auto actor = std::make_unique<MasterActor>(mp, [&](int) { done = true; });
  auto bridge = ControlBridge::start("127.0.0.1", 0);
  actor->set_bridge(bridge);
  ActorRef master = sys->actor_of(std::move(actor), "master");
  bridge->attach(master, master->path());
  const int port = bridge->port();
  std::atomic<int> sinks{0};
  for (int k = 0; k < P; ++k) {
    DataSource src = [N](const AllReduceInputRequest& r) {
      std::vector<float> v(N, static_cast<float>(r.iteration));
      return AllReduceInput{make_host_payload(std::move(v))};
    };
    DataSink sink = [&](const AllReduceOutput&) { sinks++; };
    ActorRef w = sys->actor_of(std::make_unique<WorkerActor>(src, sink), "worker" + std::to_string(k));
    master->tell(MemberUp{w, "worker", ""}, nullptr);
  }
  std::atomic<bool> stop_churn{false};
  std::vector<std::thread> churn;
  for (int t = 0; t < 3; ++t)
    churn.emplace_back([&, t] {
      for (int i = 0; !stop_churn.load(); ++i) {
        int fd = connect_to(port);
        if (fd < 0) continue;
        char b[32];
        (void)!::recv(fd, b, sizeof(b), 0);
        if ((i + t) % 2) (void)!::send(fd, "{\"type\":\"Sta", 12, MSG_NOSIGNAL);
        ::close(fd);
      }
    });
  int completed = 0;
  std::string err;
  {
    int fd = -1;
    for (int i = 0; i < 100 && fd < 0; ++i) fd = connect_to(port);
    std::string buf;
    auto line = [&]() -> std::map<std::string, std::string> {
      for (;;) {
        if (auto nl = buf.find('\n'); nl != std::string::npos) {
          std::string l = buf.substr(0, nl);
          buf.erase(0, nl + 1);
          std::map<std::string, std::string> kv;
          if (!parse_flat_json(l, kv)) kv["type"] = l.find("InitWorkers") != std::string::npos ? "InitWorkers" : "?";
          return kv;
        }
        char tmp[4096];
        ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
        if (n <= 0) return {{"type", "EOF"}};
        buf.append(tmp, static_cast<size_t>(n));
      }
    };
    auto start = [&](int r) {
      std::string l = "{\"type\":\"StartAllreduce\",\"round\":" + std::to_string(r) + "}\n";
      (void)!::send(fd, l.data(), l.size(), MSG_NOSIGNAL);
    };
    std::map<std::string, std::string> m;
    do m = line(); while (m["type"] != "InitWorkers" && m["type"] != "EOF");
    int next = 0;
    start(next++);
    start(next++);
    while (completed < rounds) {
      m = line();
      if (m["type"] == "EOF" || m["type"] == "Error") {
        err = "bridge driver got " + m["type"] + " " + m["reason"];
        break;
      }
      if (m["type"] == "RoundComplete") ++completed;
      if (m["type"] == "Accepted" && std::stoi(m["round"]) == next - 1 && next < rounds) start(next++);
    }
    ::close(fd);
  }
  stop_churn = true;
  for (auto& t : churn) t.join();
  const bool ok = err.empty() && wait_until([&] { return done.load(); }, 30);
  sys->await_idle(std::chrono::milliseconds(5000));
  sys->shutdown();
  bridge.reset();
  if (!ok) {
    std::fprintf(stderr, "bridge-driven job failed: %s (rounds %d)\n", err.c_str(), completed);
    return 1;
  }
  if (sinks.load() != P * rounds) {
    std::fprintf(stderr, "bridge-driven job: %d outputs, want %d\n", sinks.load(), P * rounds);
    return 1;
  }
  return 0;
}

// Bridge teardown: (1) a client that connects and never reads while the master
// runs rounds on its own - its queue overflows and it is dropped, the rounds never stall on
// its socket; (2) the system shuts down while another client floods StartAllreduce, with
// the master holding the ONLY reference to the bridge, so the master (and the bridge's
// owner reference) can die inside a reader's tell().
static int run_bridge_teardown(int P, int N, int C, int rounds) {
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 4);
  std::atomic<bool> done{false};
  MasterParams mp{P, 1.f, 1.f, 1.f, 1, N, rounds - 1, C, false};
  auto actor = std::make_unique<MasterActor>(mp, [&](int) { done = true; });
  int port = 0;
  {
    auto bridge = ControlBridge::start("127.0.0.1", 0);
    bridge->set_max_queued_bytes(4096);
    actor->set_bridge(bridge);
    port = bridge->port();
    ActorRef master = sys->actor_of(std::move(actor), "master");
    bridge->attach(master, master->path());
    int lazy = connect_to(port);  // connects, never reads
    if (lazy >= 0) {
      int small = 4096;
      ::setsockopt(lazy, SOL_SOCKET, SO_RCVBUF, &small, sizeof(small));
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    for (int k = 0; k < P; ++k) {
      DataSource src = [N](const AllReduceInputRequest& r) {
        std::vector<float> v(N, static_cast<float>(r.iteration));
        return AllReduceInput{make_host_payload(std::move(v))};
      };
      ActorRef w = sys->actor_of(std::make_unique<WorkerActor>(src, [](const AllReduceOutput&) {}),
                                 "worker" + std::to_string(k));
      master->tell(MemberUp{w, "worker", ""}, nullptr);
    }
    const bool ok = wait_until([&] { return done.load(); }, 60);
    if (lazy >= 0) ::close(lazy);
    if (!ok) {
      std::fprintf(stderr, "bridge teardown: rounds stalled behind a client that never reads\n");
      sys->shutdown();
      return 1;
    }
  }  // from here the master actor owns the only reference to the bridge
  std::atomic<bool> stop_flood{false};
  std::thread flood([&] {
    int fd = connect_to(port);
    if (fd < 0) return;
    const std::string l = "{\"type\":\"StartAllreduce\",\"round\":1}\n{\"type\":\"Status\"}\n";
    while (!stop_flood.load())
      if (::send(fd, l.data(), l.size(), MSG_NOSIGNAL) <= 0) break;
    ::close(fd);
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(50));
  sys->shutdown();  // drops the master -> ~MasterActor stops the bridge mid-flood
  stop_flood = true;
  flood.join();
  return 0;
}

// The round engine on host memory: master + P PlaneWorkerActors over LoopbackRoundPlanes
// (plane completion threads, hub mutex, actor mailboxes all live under the sanitizer).
static int run_plane(int P, int N, int C, int rounds) {
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 4);
  std::atomic<bool> done{false};
  MasterParams mp{P, 1.f, 1.f, 1.f, 1, N, rounds - 1, C, false};
  ActorRef master = sys->actor_of(std::make_unique<MasterActor>(mp, [&](int) { done = true; }), "master");
  std::mutex mu;
  std::vector<std::vector<std::vector<float>>> outs(P);
  std::vector<std::shared_ptr<LoopbackRoundPlane>> planes;
  std::vector<ActorRef> refs;
  for (int k = 0; k < P; ++k) {
    DataSource src = [N, k](const AllReduceInputRequest& r) {
      std::vector<float> v(N);
      for (int i = 0; i < N; ++i) v[i] = static_cast<float>((i + r.iteration) * (k + 1));
      return AllReduceInput{make_host_payload(std::move(v))};
    };
    DataSink sink = [&, k](const AllReduceOutput& o) {
      std::lock_guard<std::mutex> g(mu);
      if (static_cast<int>(outs[k].size()) <= o.iteration) outs[k].resize(o.iteration + 1);
      outs[k][o.iteration] = o.data->to_host();
    };
    planes.push_back(make_loopback_plane("stress"));
    refs.push_back(sys->actor_of(std::make_unique<PlaneWorkerActor>(src, sink, planes.back()), "pw" + std::to_string(k)));
  }
  for (int k = 0; k < P; ++k) master->tell(MemberUp{refs[k], "worker", "", planes[k]->descriptor()}, nullptr);
  const bool ok = wait_until([&] { return done.load(); }, 60);
  for (auto& p : planes) p->drain();
  sys->await_idle(std::chrono::milliseconds(5000));
  sys->shutdown();
  if (!ok) {
    std::fprintf(stderr, "plane cluster did not finish\n");
    return 1;
  }
  const float tri = P * (P + 1) / 2.f;
  for (int k = 0; k < P; ++k)
    for (int r = 0; r < rounds; ++r)
      for (int i = 0; i < N; ++i)
        if (std::fabs(outs[k][r][i] - (i + r) * tri) > 1e-3f) {
          std::fprintf(stderr, "plane: bad sum worker %d round %d idx %d\n", k, r, i);
          return 1;
        }
  return 0;
}

// Three nodes over TCP on 127.0.0.1: master node + two worker nodes.
static int run_tcp(int rounds) {
  const int N = 10, C = 2;
  auto msys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 2);
  std::atomic<bool> done{false};
  MasterParams mp{2, 1.f, 1.f, 1.f, 1, N, rounds - 1, C, false};
  ActorRef master = msys->actor_of(std::make_unique<MasterActor>(mp, [&](int) { done = true; }), "master");
  ClusterConfig mc;
  mc.port = 0;
  mc.roles = {"master"};
  mc.heartbeat_interval_s = 0.05;
  auto mnode = ClusterNode::start(msys, mc);
  mnode->subscribe(master);
  const std::string seed = mnode->address();
  std::vector<std::shared_ptr<ActorSystem>> wsys;
  std::vector<std::shared_ptr<ClusterNode>> wnodes;
  std::atomic<int> outputs{0};
  for (int k = 0; k < 2; ++k) {
    auto s = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 2);
    DataSource src = [N](const AllReduceInputRequest& r) {
      std::vector<float> v(N);
      for (int i = 0; i < N; ++i) v[i] = static_cast<float>(i + r.iteration);
      return AllReduceInput{make_host_payload(std::move(v))};
    };
    DataSink sink = [&](const AllReduceOutput&) { outputs++; };
    s->actor_of(std::make_unique<WorkerActor>(src, sink), "worker");
    ClusterConfig wc;
    wc.port = 0;
    wc.roles = {"worker"};
    wc.seed_nodes = {seed};
    wc.heartbeat_interval_s = 0.05;
    wnodes.push_back(ClusterNode::start(s, wc));
    wsys.push_back(s);
  }
  const bool ok = wait_until([&] { return done.load() && outputs.load() >= 2 * rounds; }, 60);
  for (auto& n : wnodes) n->leave();
  for (auto& n : wnodes) n->shutdown();
  mnode->shutdown();
  for (auto& s : wsys) s->shutdown();
  msys->shutdown();
  if (!ok) {
    std::fprintf(stderr, "tcp cluster did not finish (outputs %d)\n", outputs.load());
    return 1;
  }
  return 0;
}

// Lock-free mailbox under contention: producer threads tell numbered messages to one actor
// that stashes everything while "closed" and unstashes when a TextMessage opens it; every
// message must arrive exactly once and in order per producer (Akka's per-pair FIFO).
namespace {
class SeqActor final : public Actor {
 public:
  SeqActor(int producers, std::atomic<int>* total, std::atomic<int>* bad)
      : next_(producers, 0), total_(total), bad_(bad) {}
  void receive(Envelope& env, ActorContext& ctx) override {
    if (auto* t = std::get_if<TextMessage>(&env.msg)) {
      closed_ = t->text == "close";
      if (!closed_) ctx.unstash_all();
      return;
    }
    auto* c = std::get_if<CompleteAllreduce>(&env.msg);
    if (c == nullptr) return;
    if (closed_) {
      ctx.stash(std::move(env));
      return;
    }
    if (c->round != next_[c->srcId]) bad_->fetch_add(1);
    next_[c->srcId] = c->round + 1;
    total_->fetch_add(1);
  }

 private:
  std::vector<int> next_;
  bool closed_ = false;
  std::atomic<int>* total_;
  std::atomic<int>* bad_;
};
}  // namespace

static int run_mailbox(int producers, int per) {
  auto sys = std::make_shared<ActorSystem>("MailboxStress", ActorSystem::Mode::Threaded, 4);
  std::atomic<int> total{0}, bad{0};
  ActorRef a = sys->actor_of(std::make_unique<SeqActor>(producers, &total, &bad), "seq");
  std::vector<std::thread> ts;
  for (int k = 0; k < producers; ++k)
    ts.emplace_back([&, k] {
      for (int i = 0; i < per; ++i) a->tell(CompleteAllreduce{k, i, 0}, nullptr);
    });
  std::thread toggler([&] {  // close / open the actor while the producers run
    for (int i = 0; i < 200; ++i) {
      a->tell(TextMessage{i % 2 == 0 ? "close" : "open"}, nullptr);
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    a->tell(TextMessage{"open"}, nullptr);
  });
  for (auto& t : ts) t.join();
  toggler.join();
  const bool ok = wait_until([&] { return total.load() == producers * per; }, 60.0);
  sys->shutdown();
  if (!ok || bad.load() != 0) {
    std::fprintf(stderr, "mailbox: %d of %d delivered, %d out of order\n", total.load(), producers * per, bad.load());
    return 1;
  }
  return 0;
}

// The akka.tcp front-end (csrc/runtime/akka_endpoint.h): a driver associates and runs every
// round with Java-serialized StartAllreduce by ActorSelection, counting CompleteAllreduce;
// churn threads associate and vanish, send garbage or a frame without a handshake; the
// system shuts down with the driver still associated (the endpoint's stop hook) - the
// endpoint's acceptor / reader / writer threads and the bridge's taps under the sanitizer.
static int run_akka(int P, int N, int C, int rounds) {
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 4);
  std::atomic<bool> done{false};
  MasterParams mp{P, 1.f, 1.f, 1.f, 1, N, rounds - 1, C, false};
  mp.externalRounds = true;
  auto actor = std::make_unique<MasterActor>(mp, [&](int) { done = true; });
  auto bridge = ControlBridge::start("127.0.0.1", 0);
  actor->set_bridge(bridge);
  ActorRef master = sys->actor_of(std::move(actor), "master");
  bridge->attach(master, master->path());
  AkkaEndpoint::Options ao;
  ao.heartbeat_s = 0.002;  // heartbeats race the replies on every writer
  auto ep = AkkaEndpoint::start(bridge, ao);
  const int port = ep->port();
  for (int k = 0; k < P; ++k) {
    DataSource src = [N](const AllReduceInputRequest& r) {
      std::vector<float> v(N, static_cast<float>(r.iteration));
      return AllReduceInput{make_host_payload(std::move(v))};
    };
    ActorRef w = sys->actor_of(std::make_unique<WorkerActor>(src, [](const AllReduceOutput&) {}),
                               "worker" + std::to_string(k));
    master->tell(MemberUp{w, "worker", ""}, nullptr);
  }
  auto send_frame = [](int fd, const std::string& pdu) {
    std::string f(4, '\0');
    for (int k = 0; k < 4; ++k) f[static_cast<size_t>(k)] = static_cast<char>(pdu.size() >> (24 - 8 * k));
    f += pdu;
    (void)!::send(fd, f.data(), f.size(), MSG_NOSIGNAL);
  };
  auto read_frame = [](int fd, std::string& body) {
    char h[4];
    size_t got = 0;
    while (got < 4) {
      ssize_t n = ::recv(fd, h + got, 4 - got, 0);
      if (n <= 0) return false;
      got += static_cast<size_t>(n);
    }
    size_t len = 0;
    for (char c : h) len = len << 8 | static_cast<uint8_t>(c);
    body.resize(len);
    got = 0;
    while (got < len) {
      ssize_t n = ::recv(fd, body.data() + got, len - got, 0);
      if (n <= 0) return false;
      got += static_cast<size_t>(n);
    }
    return true;
  };
  akka::Address me;
  me.system = "Driver";
  me.host = "127.0.0.1";
  me.port = 1;
  std::atomic<bool> stop_churn{false};
  std::vector<std::thread> churn;
  for (int t = 0; t < 3; ++t)
    churn.emplace_back([&, t] {
      for (int i = 0; !stop_churn.load(); ++i) {
        int fd = connect_to(port);
        if (fd < 0) continue;
        if ((i + t) % 3 == 0) {
          send_frame(fd, akka::encode_associate(me, 7, ""));
          std::string b;
          (void)read_frame(fd, b);
        } else if ((i + t) % 3 == 1) {
          send_frame(fd, akka::encode_payload_pdu("x"));
        } else {
          (void)!::send(fd, "\xff\xff\xff\xff", 4, MSG_NOSIGNAL);
        }
        ::close(fd);
      }
    });
  std::string err;
  int completed = 0;
  int fd = -1;
  for (int i = 0; i < 100 && fd < 0; ++i) fd = connect_to(port);
  send_frame(fd, akka::encode_associate(me, 42, ""));
  const std::string self = me.str() + "/user/driver";
  auto start = [&](int r) {
    akka::JavaObject o;
    o.class_name = "sample.cluster.allreduce.StartAllreduce";
    o.suid = ep->suid_start();
    o.fields = {{'I', "round", r, 0.0}};
    akka::SerializedMsg inner;
    inner.serializer = akka::kJavaSerializer;
    inner.bytes = akka::java_serialize(o);
    akka::Envelope e;
    e.has_envelope = true;
    e.recipient = ep->address() + "/";
    e.msg.serializer = akka::kContainerSerializer;
    e.msg.bytes = akka::encode_selection(inner, {{1, "user"}, {1, "master"}}, false);
    e.has_sender = true;
    e.sender = self;
    send_frame(fd, akka::encode_payload_pdu(akka::encode_container(e)));
  };
  std::string body;
  int seen = 0;
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  start(0);
  while (completed < rounds && std::chrono::steady_clock::now() < deadline) {
    if (!read_frame(fd, body)) {
      err = "driver association closed";
      break;
    }
    akka::Pdu pdu;
    akka::Envelope env;
    akka::JavaObject o;
    if (!akka::decode_pdu(body, pdu)) {
      err = "undecodable PDU";
      break;
    }
    if (!pdu.is_payload || !akka::decode_container(pdu.payload, env) || !env.has_envelope) continue;
    if (env.recipient != self || !akka::java_deserialize(env.msg.bytes, o) || o.fields.size() != 2) {
      err = "unexpected message to " + env.recipient;
      break;
    }
    const int round = static_cast<int>(o.fields[0].i);  // fields in stream order: round, srcId
    if (round != completed) continue;
    if (++seen == P) {
      seen = 0;
      if (++completed < rounds) start(completed);
    }
  }
  stop_churn = true;
  for (auto& t : churn) t.join();
  const bool ok = err.empty() && completed == rounds && wait_until([&] { return done.load(); }, 30);
  const auto st = ep->stats();
  sys->await_idle(std::chrono::milliseconds(5000));
  sys->shutdown();  // the master's bridge stop runs the endpoint's stop: the driver is told
  std::string bye;
  akka::Pdu last;
  bool told = false;
  while (read_frame(fd, bye))
    if (akka::decode_pdu(bye, last) && !last.is_payload && last.command == akka::kShuttingDown) told = true;
  ::close(fd);
  bridge.reset();
  ep.reset();
  if (!ok || !told || st.starts != static_cast<uint64_t>(rounds)) {
    std::fprintf(stderr, "akka-driven job failed: %s (rounds %d, starts %llu, shutdown notice %d)\n", err.c_str(),
                 completed, static_cast<unsigned long long>(st.starts), told);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  Logger::get().set_level(LogLevel::ERROR);
  const std::string only = argc > 1 ? argv[1] : "";
  int rc = 0;
  if (only.empty() || only == "mailbox") rc = run_mailbox(6, 20000);
  if (rc == 0 && (only.empty() || only == "local")) rc = run_local(4, 37, 3, 30);
  if (rc == 0 && (only.empty() || only == "local2")) rc = run_local(3, 9, 2, 30);
  if (rc == 0 && (only.empty() || only == "tcp")) rc = run_tcp(20);
  if (rc == 0 && (only.empty() || only == "plane")) rc = run_plane(3, 41, 4, 40);
  if (rc == 0 && (only.empty() || only == "bridge")) rc = run_bridge(3, 23, 4, 60);
  if (rc == 0 && (only.empty() || only == "bridge_teardown")) rc = run_bridge_teardown(3, 23, 4, 400);
  if (rc == 0 && (only.empty() || only == "akka")) rc = run_akka(3, 23, 4, 60);
  std::printf(rc == 0 ? "runtime_stress: OK\n" : "runtime_stress: FAILED\n");
  return rc;
}
