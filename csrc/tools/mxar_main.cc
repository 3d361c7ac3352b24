// mxar: native (Python-free) master / worker executables of the actor runtime - the
// reference's AllreduceMaster.main (AllreduceMaster.scala:101-137) and AllreduceWorker.main
// (AllreduceWorker.scala:272-301), same positional arguments and defaults, on the C++
// actor system + TCP cluster layer (csrc/runtime, csrc/cluster).
//
//   mxar master [port totalWorkers dataSize maxChunkSize] [options]
//       defaults 2551 2 totalWorkers*5 2; thAllreduce 1, thReduce 0.9, thComplete 0.8,
//       maxLag 1, maxRound 100 (AllreduceMaster.scala:105-114). Exits once round maxRound
//       completed (the reference idles forever).
//   mxar worker [port sourceDataSize] [options]
//       defaults 2553 10; data source data[i] = i + iteration (AllreduceWorker.scala:285-291);
//       the sink logs every completed round; exits when the master leaves the cluster.
//   options: --host H  --seeds addr[,addr]  --th-allreduce F --th-reduce F --th-complete F
//            --max-lag N --max-round N --round-timeout-ms N --loglevel L --quiet
//   seeds default to the reference's application.conf:14-16 (127.0.0.1:2551, :2552).
//   mxar-gpu worker ... --device K   (the same executable linked with csrc/tools/mxar_gpu.cc)
//       the worker's rounds run on GPU K: an XgmiRoundPlane under a PlaneWorkerActor, the
//       source filled on the device. Workers on one node exchange through the xGMI arena.
#include <functional>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>
#include <map>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <numeric>
#include <optional>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../cluster/cluster_node.h"
#include "../core/log.h"
#include "../core/output_check.h"
#include "../runtime/akka_endpoint.h"
#include "../runtime/allreduce_actors.h"
#include "../runtime/plane_worker.h"
#include "gpu_worker.h"

using namespace mxar;


namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop = true; }

// The node and the actor system were shut down explicitly; leave without running the
// destructors of the objects still referenced from transport / actor state (the OS reclaims
// sockets and memory), so a departed peer can never hold the exit.
[[noreturn]] void exit_now(int rc) {
  std::fflush(nullptr);
  std::_Exit(rc);
}

struct Options {
  std::vector<std::string> positional;
  std::string host = "127.0.0.1";
  std::vector<std::string> seeds;
  float th_allreduce = 1.f, th_reduce = 0.9f, th_complete = 0.8f;  // AllreduceMaster.scala:105-107
  int bridge_port = -1;                 // --bridge PORT (control bridge, docs/BRIDGE.md)
  bool external_rounds = false;         // --external-rounds
  int akka_port = -1;                   // --akka-port PORT (akka.tcp endpoint, docs/AKKA_WIRE.md)
  std::string akka_package = "sample.cluster.allreduce", akka_cookie;
  int64_t akka_suid_start = 0, akka_suid_complete = 0;
  bool lockstep = false;                // drive: start the next round only after the barrier
  int max_lag = 1, max_round = 100, round_timeout_ms = 0;          // :108-109
  int init_workers = 0;  // --init-workers N: the first init waits for N workers (MasterParams.initWorkers)
  std::string loglevel = "INFO";
  bool quiet = false;
  int device = -1;  // worker: >= 0 runs the rounds on this GPU (mxar-gpu)
  int max_peers = 8, plane_max_lag = 4, grid = 0;
  double plane_timeout_s = 60.0;
  int64_t min_chunk = 0;  // --min-chunk N: one flag per chunk of >= N elements (0: 1 KiB)
  bool static_source = false;  // --source static: the same input every round (default iota: i + iteration)
  int dtype = 0;     // --dtype fp32|bf16|fp16 (GPU worker element type)
  int spin_us = -1;  // --spin-us N: dispatcher idle spin + cluster reader socket poll (-1: built-in defaults)
  bool has_value = false;    // --source-value V: static source, V everywhere (the straggler bench: 1, 2, 4, ...)
  double source_value = 0.0;
  double source_delay_us = 0.0;  // --source-delay-us D: every fetch waits D us (a straggling dataSource)
  double lag_wait_us = -1.0;     // --lag-wait-us W: a round waits at most W us for a lagging peer
  int check_chunk = 0;           // --check-chunk C: check the last output (power-of-two sources, maxChunkSize C)
};

// --spin-us: how long an idle actor dispatcher and a cluster reader keep polling before they
// sleep. A GPU round leaves every host thread idle for the kernel's duration; past the spin
// they sleep, and each hop of the next round (Complete, Start: two TCP frames, two actor
// turns) then pays a wake-up. 500 us covers a 256 MiB round: native 64 MiB rounds 176-198 ->
// 152-160 us, the in-process engine's time (profiles/round3/native_spin_ab.jsonl). Costs a
// core per spinning thread while rounds run. An explicit MXAR_* environment variable wins.
void apply_spin(int us) {
  if (us < 0) return;
  const std::string v = std::to_string(us);
  setenv("MXAR_DISPATCH_SPIN_US", v.c_str(), 0);
  setenv("MXAR_TCP_SPIN_US", v.c_str(), 0);
}

[[noreturn]] void usage(const char* msg) {
  std::fprintf(stderr,
               "%s\nusage: mxar master [port totalWorkers dataSize maxChunkSize] [options]\n"
               "       mxar worker [port sourceDataSize] [options]\n"
               "options: --host H --seeds a[,b] --th-allreduce F --th-reduce F --th-complete F --max-lag N\n"
               "         --max-round N --round-timeout-ms N --init-workers N --loglevel L --quiet\n"
               "master control bridge (docs/BRIDGE.md): --bridge PORT [--external-rounds]\n"
               "master akka.tcp endpoint (docs/AKKA_WIRE.md): --akka-port PORT [--akka-package P --akka-cookie C\n"
               "                              --akka-suid-start N --akka-suid-complete N]\n"
               "       mxar drive [host:]bridgePort [rounds] [--lockstep]   (bridge client)\n"
               "worker on a GPU (mxar-gpu): --device K [--max-peers N --plane-max-lag N --grid N --plane-timeout S\n"
               "                              --min-chunk N --source iota|static --dtype fp32|bf16|fp16\n"
               "                              --source-value V --source-delay-us D --lag-wait-us W --check-chunk C]\n"
               "host threads: --spin-us N (dispatcher + socket polling; GPU workers default 500)\n",
               msg);
  std::exit(2);
}

Options parse(int argc, char** argv) {
  Options o;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) usage(("missing value for " + a).c_str());
      return argv[++i];
    };
    if (a == "--host") o.host = val();
    else if (a == "--seeds") {
      std::stringstream ss(val());
      std::string s;
      while (std::getline(ss, s, ',')) o.seeds.push_back(s);
    } else if (a == "--th-allreduce") o.th_allreduce = std::stof(val());
    else if (a == "--th-reduce") o.th_reduce = std::stof(val());
    else if (a == "--th-complete") o.th_complete = std::stof(val());
    else if (a == "--max-lag") o.max_lag = std::stoi(val());
    else if (a == "--max-round") o.max_round = std::stoi(val());
    else if (a == "--round-timeout-ms") o.round_timeout_ms = std::stoi(val());
    else if (a == "--init-workers") o.init_workers = std::stoi(val());
    else if (a == "--bridge") o.bridge_port = std::stoi(val());
    else if (a == "--external-rounds") o.external_rounds = true;
    else if (a == "--akka-port") o.akka_port = std::stoi(val());
    else if (a == "--akka-package") o.akka_package = val();
    else if (a == "--akka-cookie") o.akka_cookie = val();
    else if (a == "--akka-suid-start") o.akka_suid_start = std::stoll(val());
    else if (a == "--akka-suid-complete") o.akka_suid_complete = std::stoll(val());
    else if (a == "--lockstep") o.lockstep = true;
    else if (a == "--loglevel") o.loglevel = val();
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--device") o.device = std::stoi(val());
    else if (a == "--max-peers") o.max_peers = std::stoi(val());
    else if (a == "--plane-max-lag") o.plane_max_lag = std::stoi(val());
    else if (a == "--grid") o.grid = std::stoi(val());
    else if (a == "--plane-timeout") o.plane_timeout_s = std::stod(val());
    else if (a == "--min-chunk") o.min_chunk = std::stoll(val());
    else if (a == "--spin-us") o.spin_us = std::stoi(val());
    else if (a == "--dtype") {
      const std::string v = val();
      if (v != "fp32" && v != "bf16" && v != "fp16") usage("--dtype must be fp32, bf16 or fp16");
      o.dtype = v == "fp32" ? 0 : v == "bf16" ? 1 : 2;
    }
    else if (a == "--source") {
      const std::string v = val();
      if (v != "iota" && v != "static") usage("--source must be iota or static");
      o.static_source = v == "static";
    }
    else if (a == "--source-value") {
      o.has_value = true;
      o.source_value = std::stod(val());
    }
    else if (a == "--source-delay-us") o.source_delay_us = std::stod(val());
    else if (a == "--lag-wait-us") o.lag_wait_us = std::stod(val());
    else if (a == "--check-chunk") o.check_chunk = std::stoi(val());
    else if (a.rfind("--", 0) == 0) usage(("unknown option " + a).c_str());
    else o.positional.push_back(a);
  }
  if (o.seeds.empty())  // application.conf:14-16
    o.seeds = {"mxar.tcp://ClusterSystem@127.0.0.1:2551", "mxar.tcp://ClusterSystem@127.0.0.1:2552"};
  return o;
}

int pos_int(const Options& o, size_t k, int def) { return o.positional.size() > k ? std::stoi(o.positional[k]) : def; }

void set_level(const std::string& l) {
  static const char* names[] = {"TRACE", "DEBUG", "INFO", "WARNING", "ERROR", "OFF"};
  for (int i = 0; i < 6; ++i)
    if (l == names[i]) Logger::get().set_level(static_cast<LogLevel>(i));
}

[[noreturn]] void run_master(const Options& o) {
  const int port = pos_int(o, 0, 2551);
  const int total = pos_int(o, 1, 2);
  const int data_size = pos_int(o, 2, total * 5);
  const int chunk = pos_int(o, 3, 2);
  MasterParams mp;
  mp.totalWorkers = total;
  mp.thAllreduce = o.th_allreduce;
  mp.thReduce = o.th_reduce;
  mp.thComplete = o.th_complete;
  mp.maxLag = o.max_lag;
  mp.dataSize = data_size;
  mp.maxRound = o.max_round;
  mp.maxChunkSize = chunk;
  mp.roundTimeoutMs = o.round_timeout_ms;
  mp.externalRounds = o.external_rounds;
  mp.initWorkers = o.init_workers;
  apply_spin(o.spin_us);
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 2);
  std::atomic<int> finished{-1};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<double> stamps;  // completion time of every round (master thread only)
  stamps.reserve(static_cast<size_t>(o.max_round) + 1);
  auto on_round = [&stamps](int, int64_t) {
    stamps.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count());
  };
  auto master_actor = std::make_unique<MasterActor>(mp, [&](int rounds) { finished = rounds; }, on_round);
  std::shared_ptr<ControlBridge> bridge;
  if (o.bridge_port >= 0 || o.akka_port >= 0) {  // the akka.tcp endpoint is a front-end of the bridge
    bridge = ControlBridge::start(o.host, o.bridge_port >= 0 ? o.bridge_port : 0);
    master_actor->set_bridge(bridge);
  }
  ActorRef master = sys->actor_of(std::move(master_actor), "master");
  std::shared_ptr<AkkaEndpoint> akka_ep;
  if (bridge) {
    bridge->attach(master, master->path());
    std::printf("[mxar master] control bridge on %s:%d%s\n", o.host.c_str(), bridge->port(),
                o.external_rounds ? " (external rounds)" : "");
    if (o.akka_port >= 0) {
      AkkaEndpoint::Options ao;
      ao.host = o.host;
      ao.port = o.akka_port;
      ao.package = o.akka_package;
      ao.cookie = o.akka_cookie;
      ao.suid_start = o.akka_suid_start;
      ao.suid_complete = o.akka_suid_complete;
      akka_ep = AkkaEndpoint::start(bridge, ao);
      std::printf("[mxar master] akka.tcp endpoint %s serves %s\n", akka_ep->address().c_str(),
                  akka_ep->master_path().c_str());
    }
  }
  ClusterConfig cc;
  cc.host = o.host;
  cc.port = port;
  cc.roles = {"master"};
  cc.seed_nodes = o.seeds;
  auto node = ClusterNode::start(sys, cc);
  node->subscribe(master);
  std::printf("[mxar master] %s totalWorkers=%d dataSize=%d maxChunkSize=%d th=(%.2f, %.2f, %.2f) maxLag=%d "
              "maxRound=%d\n",
              node->address().c_str(), total, data_size, chunk, o.th_allreduce, o.th_reduce, o.th_complete,
              o.max_lag, o.max_round);
  std::fflush(stdout);
  while (!g_stop && finished.load() < 0) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (finished.load() >= 0) {
    std::printf("[mxar master] finished %d rounds in %.3f s\n", finished.load(), s);
    if (stamps.size() > 2) {  // steady state: the intervals between consecutive round completions
      std::vector<double> iv;
      for (size_t i = 1; i < stamps.size(); ++i) iv.push_back((stamps[i] - stamps[i - 1]) * 1e6);
      std::sort(iv.begin(), iv.end());
      const double rate = static_cast<double>(stamps.size() - 1) / (stamps.back() - stamps.front());
      std::printf("{\"rounds\": %zu, \"steady_rounds_per_s\": %.1f, \"round_interval_p50_us\": %.1f, "
                  "\"round_interval_p99_us\": %.1f}\n",
                  stamps.size(), rate, iv[iv.size() / 2], iv[std::min(iv.size() - 1, iv.size() * 99 / 100)]);
    }
  }
  std::fflush(stdout);
  node->leave();
  std::this_thread::sleep_for(std::chrono::milliseconds(200));  // let the Leave / Removed frames go out
  if (akka_ep) akka_ep->stop();  // DISASSOCIATE_SHUTTING_DOWN to its clients
  node->shutdown();
  sys->shutdown();
  exit_now(finished.load() >= 0 ? 0 : 1);
}

const PlaneWorkerActor* plane_actor(const ActorRef& ref) {
  auto* l = dynamic_cast<LocalActorRef*>(ref.get());
  auto c = l ? l->cell() : nullptr;
  return c ? dynamic_cast<const PlaneWorkerActor*>(c->actor()) : nullptr;
}
int plane_worker_peers(const ActorRef& ref) {
  const PlaneWorkerActor* w = plane_actor(ref);
  return w ? w->peers() : 0;
}
PlaneWorkerStats plane_worker_stats(const ActorRef& ref) {
  const PlaneWorkerActor* w = plane_actor(ref);
  return w ? w->stats() : PlaneWorkerStats{};
}

[[noreturn]] void run_worker(const Options& o) {
  const int port = pos_int(o, 0, 2553);
  const int size = pos_int(o, 1, 10);
  apply_spin(o.spin_us >= 0 ? o.spin_us : o.device >= 0 ? 500 : -1);  // a GPU worker polls through its rounds
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 2);
  DataSource src = [size](const AllReduceInputRequest& r) {  // AllreduceWorker.scala:285-291
    std::vector<float> v(size);
    for (int i = 0; i < size; ++i) v[i] = static_cast<float>(i + r.iteration);
    return AllReduceInput{make_host_payload(std::move(v))};
  };
  std::atomic<int> rounds{0};
  const bool quiet = o.quiet;
  // quiet: the newest output is kept (a reference, no copy) and checked once at the end, so a
  // timed run reports the sum of its own last round (benchmarks/sections.py native_deployment);
  // every round's sink time and count totals are kept for the summary line
  std::mutex last_mu;
  std::optional<AllReduceOutput> last;
  std::vector<double> sink_t;
  uint64_t count_sum = 0, count_n = 0, count_zero = 0;
  DataSink sink = [&rounds, quiet, &last_mu, &last, &sink_t, &count_sum, &count_n,
                   &count_zero](const AllReduceOutput& out) {  // AllreduceWorker.scala:295-297
    rounds++;
    if (quiet) {
      const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
      std::lock_guard<std::mutex> g(last_mu);
      if (!last || out.iteration >= last->iteration) last = out;
      if (sink_t.size() < (size_t{1} << 22)) sink_t.push_back(t);
      for (int c : out.count) {
        count_sum += static_cast<uint64_t>(c > 0 ? c : 0);
        count_zero += c == 0 ? 1 : 0;
      }
      count_n += out.count.size();
    }
    if (!quiet) {  // quiet: no copy back of a device output either
      const std::vector<float> d = out.data->to_host();
      const double sum = std::accumulate(d.begin(), d.end(), 0.0);
      std::printf("[mxar worker] round %d sum %.1f head", out.iteration, sum);
      for (size_t i = 0; i < d.size() && i < 6; ++i) std::printf(" %g", d[i]);
      std::printf("\n");
      std::fflush(stdout);
    }
  };
  ClusterConfig cc;
  std::function<void()> gpu_at_exit;
  ActorRef plane_worker;
  if (o.device >= 0) {  // the round engine on a GPU: one threshold-kernel launch per round
    if (make_gpu_worker == nullptr) usage("--device needs the GPU build of this executable: mxar-gpu");
    GpuWorkerOptions go;
    go.device = o.device;
    go.size = size;
    go.max_peers = o.max_peers;
    go.max_lag = o.plane_max_lag;
    go.grid = o.grid;
    go.timeout_s = o.plane_timeout_s;
    go.min_chunk = o.min_chunk;
    go.static_source = o.static_source;
    go.has_value = o.has_value;
    go.source_value = o.source_value;
    go.source_delay_us = o.source_delay_us;
    go.lag_wait_us = o.lag_wait_us;
    go.dtype = o.dtype;
    GpuWorkerParts g = make_gpu_worker(go);
    cc.meta = g.plane->descriptor();  // relayed by the master in InitWorkers.planes
    gpu_at_exit = g.at_exit;
    plane_worker = sys->actor_of(std::make_unique<PlaneWorkerActor>(g.source, sink, g.plane), "worker");
  } else {
    sys->actor_of(std::make_unique<WorkerActor>(src, sink), "worker");
  }
  cc.host = o.host;
  cc.port = port;
  cc.roles = {"worker"};
  cc.seed_nodes = o.seeds;
  auto node = ClusterNode::start(sys, cc);
  std::printf("[mxar worker] %s sourceDataSize=%d\n", node->address().c_str(), size);
  std::fflush(stdout);
  bool saw_master = false;
  while (!g_stop) {
    bool master_up = false;
    for (const MemberInfo& m : node->members())
      if (m.has_role("master") && m.status == MemberStatus::Up && !node->is_unreachable(m.address)) master_up = true;
    // a short-lived master can join and leave between two polls: a completed round also
    // proves it was there
    if (master_up || rounds.load() > 0) saw_master = true;
    if (saw_master && !master_up) break;  // the master left: the job is over
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  if (gpu_at_exit) gpu_at_exit();
  {
    std::lock_guard<std::mutex> g(last_mu);
    std::string check = "null", check_detail = "null";
    int last_round = -1;
    if (last) {
      const std::vector<float> d = last->data->to_host();
      const double sum = std::accumulate(d.begin(), d.end(), 0.0);
      std::printf("[mxar worker] last round %d sum %.1f\n", last->iteration, sum);
      last_round = last->iteration;
      if (o.check_chunk > 0 && !last->count.empty()) {
        const int peers = plane_worker ? plane_worker_peers(plane_worker) : 0;
        const OutputCheck c = check_power_of_two_output(d, last->count, peers, o.check_chunk);
        check = c.ok ? "true" : "false";
        if (!c.ok) {
          std::printf("[mxar worker] check failed: %lld of %lld chunks\n", static_cast<long long>(c.bad_chunks),
                      static_cast<long long>(c.chunks));
          char b[256];
          std::snprintf(b, sizeof(b),
                        "{\"bad_chunks\": %lld, \"chunks\": %lld, \"peers\": %d, \"block\": %d, \"chunk\": %d, "
                        "\"count\": %d, \"value\": %g, \"distinct\": %d}",
                        static_cast<long long>(c.bad_chunks), static_cast<long long>(c.chunks), peers, c.first_block,
                        c.first_chunk, c.first_count, static_cast<double>(c.first_value), c.first_distinct);
          check_detail = b;
        }
      }
      last.reset();
    }
    if (quiet && sink_t.size() > 4) {
      // the worker's own round period: intervals between consecutive sink calls, the first
      // tenth left out (warm-up)
      std::vector<double> iv;
      for (size_t i = std::max<size_t>(1, sink_t.size() / 10); i < sink_t.size(); ++i)
        iv.push_back((sink_t[i] - sink_t[i - 1]) * 1e6);
      std::sort(iv.begin(), iv.end());
      double mean = 0;
      for (double x : iv) mean += x;
      mean /= static_cast<double>(iv.size());
      PlaneWorkerStats ps{};
      if (plane_worker) ps = plane_worker_stats(plane_worker);
      std::printf("{\"worker_summary\": {\"rounds\": %zu, \"last_round\": %d, \"period_p50_us\": %.2f, "
                  "\"period_p99_us\": %.2f, \"period_mean_us\": %.2f, \"count_mean\": %.4f, \"count_zero_frac\": %.4f, "
                  "\"forced\": %llu, \"cold\": %llu, \"coalesced\": %llu, \"plane_errors\": %llu, \"validated\": %s, "
                  "\"check_detail\": %s}}\n",
                  sink_t.size(), last_round, iv[iv.size() / 2], iv[std::min(iv.size() - 1, iv.size() * 99 / 100)], mean,
                  count_n ? static_cast<double>(count_sum) / static_cast<double>(count_n) : 0.0,
                  count_n ? static_cast<double>(count_zero) / static_cast<double>(count_n) : 0.0,
                  static_cast<unsigned long long>(ps.forced_completions), static_cast<unsigned long long>(ps.cold_rounds),
                  static_cast<unsigned long long>(ps.starts_coalesced), static_cast<unsigned long long>(ps.plane_errors),
                  check.c_str(), check_detail.c_str());
    }
  }
  std::printf("[mxar worker] %d rounds completed\n", rounds.load());
  std::fflush(stdout);
  node->leave();
  std::this_thread::sleep_for(std::chrono::milliseconds(100));  // let the Leave frame go out
  node->shutdown();
  sys->shutdown();  // destroys the plane worker: its plane aborts and drains, the GPU is idle
  if (o.device >= 0) {  // run the atexit handlers: the HIP runtime and a profiler flush there
    std::fflush(nullptr);
    std::exit(0);
  }
  exit_now(0);
}

}  // namespace

// `mxar drive [host:]port [rounds] [--lockstep]`: a Python-free control-bridge client
// (docs/BRIDGE.md) that plays AllreduceMaster's round loop (AllreduceMaster.scala:58-67,
// 91-97) against a master started with --bridge PORT --external-rounds. Pipelined by default
// (the next start is queued while a round runs). Prints one JSON summary line.
[[noreturn]] void run_drive(const Options& o) {
  if (o.positional.empty()) usage("drive: missing [host:]port");
  std::string host = o.host, hp = o.positional[0];
  if (auto c = hp.rfind(':'); c != std::string::npos) {
    host = hp.substr(0, c);
    hp = hp.substr(c + 1);
  }
  const int port = std::stoi(hp);
  const int want = pos_int(o, 1, -1);  // -1: through maxRound (from InitWorkers' job)
  int fd = -1;
  for (int attempt = 0; attempt < 300 && fd < 0 && !g_stop; ++attempt) {  // the master may still be starting
    fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    ::inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      ::close(fd);
      fd = -1;
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
  }
  if (fd < 0) throw std::runtime_error("drive: cannot connect to " + host + ":" + hp);
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  std::string buf;
  auto next_line = [&]() -> std::map<std::string, std::string> {
    for (;;) {
      if (auto nl = buf.find('\n'); nl != std::string::npos) {
        std::string line = buf.substr(0, nl);
        buf.erase(0, nl + 1);
        std::map<std::string, std::string> kv;
        if (!parse_flat_json(line, kv)) {  // InitWorkers carries an array: pull its scalars by hand
          kv.clear();
          for (const char* k : {"type", "startRound", "maxRound", "epoch"}) {
            auto at = line.find(std::string("\"") + k + "\":");
            if (at == std::string::npos) continue;
            at += std::strlen(k) + 3;
            auto end = line.find_first_of(",}", at);
            std::string v = line.substr(at, end - at);
            if (!v.empty() && v.front() == '"') v = v.substr(1, v.size() - 2);
            kv[k] = v;
          }
        }
        if (kv["type"] == "Error") throw std::runtime_error("drive: bridge refused: " + line);
        return kv;
      }
      char tmp[65536];
      ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
      if (n <= 0) throw std::runtime_error("drive: bridge closed the connection");
      buf.append(tmp, static_cast<size_t>(n));
    }
  };
  auto send_start = [&](int r) {
    const std::string l = "{\"type\":\"StartAllreduce\",\"round\":" + std::to_string(r) + "}\n";
    if (::send(fd, l.data(), l.size(), MSG_NOSIGNAL) != static_cast<ssize_t>(l.size()))
      throw std::runtime_error("drive: send failed");
  };
  std::map<std::string, std::string> m;
  do m = next_line(); while (m["type"] != "InitWorkers");
  const int first = std::stoi(m["startRound"]);
  const int max_round = std::stoi(m["maxRound"]);
  const int last = want > 0 ? std::min(max_round, first + want - 1) : max_round;
  std::vector<double> stamps;
  int completed = 0, next = first;
  bool finished = false;
  send_start(next++);
  if (!o.lockstep && next <= last) send_start(next++);  // one queued behind the first
  while (!finished && !g_stop) {
    m = next_line();
    const std::string& t = m["type"];
    if (t == "RoundComplete") {
      stamps.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count());
      ++completed;
      if (completed >= last - first + 1) break;
      if (o.lockstep) send_start(next++);
    } else if (t == "Accepted" && !o.lockstep) {  // round r started: queue r + 1 behind it
      if (std::stoi(m["round"]) == next - 1 && next <= last) send_start(next++);
    } else if (t == "AllreduceFinished") {
      finished = true;
    } else if (t == "InitWorkers") {
      throw std::runtime_error("drive: workers re-initialised (epoch " + m["epoch"] + ")");
    }
  }
  ::close(fd);
  double rate = 0, p50 = 0;
  if (stamps.size() > 2) {
    std::vector<double> iv;
    for (size_t i = 1; i < stamps.size(); ++i) iv.push_back((stamps[i] - stamps[i - 1]) * 1e6);
    std::sort(iv.begin(), iv.end());
    rate = static_cast<double>(stamps.size() - 1) / (stamps.back() - stamps.front());
    p50 = iv[iv.size() / 2];
  }
  std::printf("{\"driver\": \"%s\", \"rounds\": %d, \"rounds_per_s\": %.1f, \"round_interval_p50_us\": %.1f}\n",
              o.lockstep ? "bridge lock-step" : "bridge pipelined", completed, rate, p50);
  std::fflush(stdout);
  exit_now(completed > 0 ? 0 : 1);
}

int main(int argc, char** argv) {
  if (argc < 2) usage("missing role");
  std::signal(SIGINT, on_signal);
  std::signal(SIGTERM, on_signal);
  const std::string role = argv[1];
  const Options o = parse(argc, argv);
  set_level(o.loglevel);
  try {
    if (role == "master") run_master(o);
    if (role == "worker") run_worker(o);
    if (role == "drive") run_drive(o);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mxar %s: %s\n", role.c_str(), e.what());
    exit_now(1);
  }
  usage(("unknown role " + role).c_str());
}
