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
#include <algorithm>
#include <atomic>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../cluster/cluster_node.h"
#include "../core/log.h"
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
  int max_lag = 1, max_round = 100, round_timeout_ms = 0;          // :108-109
  std::string loglevel = "INFO";
  bool quiet = false;
  int device = -1;  // worker: >= 0 runs the rounds on this GPU (mxar-gpu)
  int max_peers = 8, plane_max_lag = 4, grid = 0;
  double plane_timeout_s = 60.0;
};

[[noreturn]] void usage(const char* msg) {
  std::fprintf(stderr,
               "%s\nusage: mxar master [port totalWorkers dataSize maxChunkSize] [options]\n"
               "       mxar worker [port sourceDataSize] [options]\n"
               "options: --host H --seeds a[,b] --th-allreduce F --th-reduce F --th-complete F --max-lag N\n"
               "         --max-round N --round-timeout-ms N --loglevel L --quiet\n"
               "master control bridge (docs/BRIDGE.md): --bridge PORT [--external-rounds]\n"
               "worker on a GPU (mxar-gpu): --device K [--max-peers N --plane-max-lag N --grid N --plane-timeout S]\n",
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
    else if (a == "--bridge") o.bridge_port = std::stoi(val());
    else if (a == "--external-rounds") o.external_rounds = true;
    else if (a == "--loglevel") o.loglevel = val();
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--device") o.device = std::stoi(val());
    else if (a == "--max-peers") o.max_peers = std::stoi(val());
    else if (a == "--plane-max-lag") o.plane_max_lag = std::stoi(val());
    else if (a == "--grid") o.grid = std::stoi(val());
    else if (a == "--plane-timeout") o.plane_timeout_s = std::stod(val());
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
  if (o.bridge_port >= 0) {
    bridge = ControlBridge::start(o.host, o.bridge_port);
    master_actor->set_bridge(bridge);
  }
  ActorRef master = sys->actor_of(std::move(master_actor), "master");
  if (bridge) {
    bridge->attach(master, master->path());
    std::printf("[mxar master] control bridge on %s:%d%s\n", o.host.c_str(), bridge->port(),
                o.external_rounds ? " (external rounds)" : "");
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
  node->shutdown();
  sys->shutdown();
  exit_now(finished.load() >= 0 ? 0 : 1);
}

[[noreturn]] void run_worker(const Options& o) {
  const int port = pos_int(o, 0, 2553);
  const int size = pos_int(o, 1, 10);
  auto sys = std::make_shared<ActorSystem>("ClusterSystem", ActorSystem::Mode::Threaded, 2);
  DataSource src = [size](const AllReduceInputRequest& r) {  // AllreduceWorker.scala:285-291
    std::vector<float> v(size);
    for (int i = 0; i < size; ++i) v[i] = static_cast<float>(i + r.iteration);
    return AllReduceInput{make_host_payload(std::move(v))};
  };
  std::atomic<int> rounds{0};
  const bool quiet = o.quiet;
  DataSink sink = [&rounds, quiet](const AllReduceOutput& out) {  // AllreduceWorker.scala:295-297
    rounds++;
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
  if (o.device >= 0) {  // the round engine on a GPU: one threshold-kernel launch per round
    if (make_gpu_worker == nullptr) usage("--device needs the GPU build of this executable: mxar-gpu");
    GpuWorkerParts g = make_gpu_worker(o.device, size, o.max_peers, o.plane_max_lag, o.grid, o.plane_timeout_s);
    cc.meta = g.plane->descriptor();  // relayed by the master in InitWorkers.planes
    sys->actor_of(std::make_unique<PlaneWorkerActor>(g.source, sink, g.plane), "worker");
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
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mxar %s: %s\n", role.c_str(), e.what());
    exit_now(1);
  }
  usage(("unknown role " + role).c_str());
}
