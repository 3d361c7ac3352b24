// Cluster extension of an ActorSystem: remote actor refs over TCP, membership, failure
// detection and remote DeathWatch. Replaces akka-remote + akka-cluster as used by the
// reference (application.conf:1-34, AllreduceMaster.scala:32-82):
//
//   * Transport  - one outbound TCP connection per (this node -> peer node); every frame
//                  to a peer goes through it under one lock, so per sender/receiver-pair
//                  FIFO holds (the reference's tests rely on it, AllreduceSpec.scala:520).
//   * Membership - nodes join through `seed_nodes`; the first seed joins itself and
//                  starts the cluster (Akka's rule). The leader - the smallest address
//                  among reachable members, so every node computes the same one - admits
//                  joiners (Welcome + MemberUp broadcast) and removes failed members.
//                  Subscribers get MemberUp for every current and future member
//                  (InitialStateAsEvents); for a "worker" member the event carries the ref
//                  of its "/user/worker" actor (the reference's resolveOne,
//                  AllreduceMaster.scala:72-73).
//   * Failure detection - heartbeats every `heartbeat_interval`; a member silent for
//                  `acceptable_heartbeat_pause` is unreachable; the leader downs it after
//                  `auto_down_unreachable_after` (application.conf:20, 10 s). Removal
//                  delivers Terminated(ref) to every local watcher of a ref on that node
//                  (DeathWatch, AllreduceMaster.scala:50-56,74).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../runtime/actor_system.h"
#include "codec.h"
#include "shm_ring.h"

namespace mxar {

struct ClusterConfig {
  std::string host = "127.0.0.1";
  int port = 2551;  // 0 = pick a free port
  std::vector<std::string> roles;
  std::vector<std::string> seed_nodes;  // "mxar.tcp://Sys@host:port" (akka.tcp:// accepted)
  double heartbeat_interval_s = 1.0;
  double acceptable_heartbeat_pause_s = 3.0;
  double auto_down_unreachable_after_s = 10.0;  // < 0 disables auto-down
  double connect_timeout_s = 2.0;
  std::string worker_path = "/user/worker";
  // Announced with the join and delivered in every MemberUp of this member (a GPU worker's
  // plane descriptor: the master relays it to the peers in InitWorkers.planes).
  std::string meta;
};

struct ClusterStats {
  uint64_t frames_out = 0, frames_in = 0, bytes_out = 0, bytes_in = 0;
  uint64_t connects = 0, connect_failures = 0, send_failures = 0, undeliverable = 0, decode_errors = 0;
  uint64_t members_up = 0, members_removed = 0, heartbeats_in = 0;
  uint64_t shm_links_out = 0, shm_links_in = 0;  // same-host connections on the shared-memory ring
};

class ClusterNode;

class RemoteActorRef final : public ActorRefBase {
 public:
  RemoteActorRef(std::weak_ptr<ClusterNode> node, std::string address, std::string path)
      : node_(std::move(node)), address_(std::move(address)), path_(std::move(path)) {}
  void tell(Message msg, ActorRef sender) override;
  std::string path() const override { return address_ + path_; }
  bool is_remote() const override { return true; }
  const std::string& address() const { return address_; }
  const std::string& local_path() const { return path_; }

 private:
  std::weak_ptr<ClusterNode> node_;
  std::string address_, path_;
};

class ClusterNode : public std::enable_shared_from_this<ClusterNode>, public RefCodec {
 public:
  static std::shared_ptr<ClusterNode> start(std::shared_ptr<ActorSystem> sys, ClusterConfig cfg);
  ~ClusterNode() override;

  const std::string& address() const { return address_; }
  int port() const { return port_; }
  const ClusterConfig& config() const { return cfg_; }

  // Ref for a full path "mxar.tcp://Sys@host:port/user/x" (cached: one object per path,
  // so ref identity comparisons hold). Local paths resolve to the local actor.
  ActorRef resolve(const std::string& full);
  void subscribe(const ActorRef& subscriber);
  void unsubscribe(const ActorRef& subscriber);
  std::vector<MemberInfo> members();
  std::string leader();
  bool joined() const { return joined_.load(); }
  bool is_unreachable(const std::string& address);
  // Graceful leave (the leader removes us), then stop the transport.
  void leave();
  void shutdown();
  ClusterStats stats();

  // Transport entry point used by RemoteActorRef::tell.
  void send(const std::string& address, const std::string& path, const Message& m, const ActorRef& sender);

  // RefCodec
  std::string encode_ref(const ActorRef& r) const override;
  ActorRef decode_ref(const std::string& s) override;

 private:
  ClusterNode(std::shared_ptr<ActorSystem> sys, ClusterConfig cfg);
  void listen();
  void accept_loop();
  void reader_loop(int fd);
  void ticker_loop();
  void handle_frame(const uint8_t* p, size_t n);
  bool send_frame(const std::string& address, const std::vector<uint8_t>& payload);
  void broadcast(const std::vector<uint8_t>& payload, const std::string& except = "");
  std::vector<uint8_t> frame_member_event(MemberEventKind k, const MemberInfo& m);
  void on_member_up(const MemberInfo& m);
  void on_member_removed(const std::string& address);
  void deliver_local(const std::string& path, Message m, const ActorRef& sender);
  void watch_remote(const ActorRef& target, const ActorRef& watcher, bool on);
  MemberUp member_up_event(const MemberInfo& m);
  void close_connection(const std::string& address);

  struct OutConn {
    int fd = -1;
    std::mutex mu;
    // same-host fast path: the ring offered on this connection (ShmOffer), live once the peer
    // acked it and ShmSwitch went out - every later frame goes through the ring
    std::unique_ptr<ShmRing> ring;
    bool ring_live = false;
    bool ring_tried = false;
  };
  bool same_host(const std::string& address) const;
  void on_shm_ack(const std::string& from, const std::string& name, bool ok);

  std::weak_ptr<ActorSystem> sys_;
  ClusterConfig cfg_;
  std::string address_;
  int port_ = 0;
  int listen_fd_ = -1;
  uint64_t uid_ = 0;
  std::atomic<bool> stopping_{false};
  std::atomic<bool> joined_{false};
  std::atomic<bool> leaving_{false};  // leave() was called: never (re-)join
  std::thread accept_thread_, ticker_thread_;
  std::mutex readers_mu_;
  std::vector<std::thread> readers_;
  std::vector<int> reader_fds_;

  std::mutex conn_mu_;
  std::map<std::string, std::shared_ptr<OutConn>> conns_;

  std::mutex mem_mu_;
  std::map<std::string, MemberInfo> members_;  // address -> info (Up members)
  std::map<std::string, std::chrono::steady_clock::time_point> last_seen_;
  std::map<std::string, std::chrono::steady_clock::time_point> unreachable_since_;
  std::set<ActorRef> subscribers_;
  std::map<std::string, std::vector<std::pair<ActorRef, ActorRef>>> watches_;  // address -> (target, watcher)

  std::mutex ref_mu_;
  std::map<std::string, ActorRef> ref_cache_;

  std::mutex stats_mu_;
  ClusterStats stats_;
  uint64_t hb_seq_ = 0;
};

std::string normalize_address(const std::string& a);

}  // namespace mxar
