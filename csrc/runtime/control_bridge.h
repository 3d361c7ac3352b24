// Control bridge: the master's round protocol over a language-neutral line protocol.
//
// SURVEY §7.5 item 3 ("existing Akka client can drive it"): the bridge carries the
// reference's CONTROL messages with the reference's names and field names as JSON lines over
// TCP, so any client needs only a socket and a JSON printer
// (examples/akka_bridge/BridgeDriver.scala). An Akka client that speaks only akka.tcp uses
// the bridge's Akka front-end instead (csrc/runtime/akka_endpoint.h, docs/AKKA_WIRE.md).
// Payloads never cross either: data stays on the workers' planes (HBM / xGMI).
//
// The client plays the round driver of AllreduceMaster.scala:58-67,91-97; the master
// (MasterParams.externalRounds) keeps membership, dense ids and InitWorkers (:38-56,84-89).
//
//   client -> bridge   {"type":"StartAllreduce","round":r}      start round r
//                      {"type":"Status"}                         one Status reply
//   bridge -> client   {"type":"Hello","protocol":"mxar-bridge/1",...}         on connect
//                      {"type":"InitWorkers","epoch":e,"workers":[0,..],"thReduce":..,
//                       "thComplete":..,"maxLag":..,"dataSize":..,"maxChunkSize":..,
//                       "startRound":..}                          every (re-)init
//                      {"type":"CompleteAllreduce","srcId":i,"round":r,"counted":b}
//                      {"type":"RoundComplete","round":r,"epoch":e,"numComplete":n}
//                      {"type":"AllreduceFinished","rounds":n}
//                      {"type":"Accepted","cmd":"StartAllreduce","round":r}
//                      {"type":"Error","cmd":...,"reason":"..."}  (to the sender only)
//                      {"type":"Status","round":..,"epoch":..,"workers":..,
//                       "numComplete":..,"awaiting":b,"finished":b}
//
// Events go to every connected client; Accepted / Error / Status only to the sender.
// A client that connects late first gets Hello, then the last InitWorkers line.
//
// Threads and lifetime: one acceptor thread, and per client a reader and a writer thread.
// Every thread holds a strong reference to the bridge, so the bridge is never destroyed
// while one of its own threads still runs (a reader's tell() may be the call that drops
// the master - and with it the master's reference). Whoever owns the bridge calls stop()
// (MasterActor's destructor does): threads then exit and release their references.
// publish() / reply() never block on a socket: each client has a bounded outbound queue
// drained by its writer thread; a client whose queue overflows (it stopped reading) is
// disconnected instead of stalling the master actor that publishes round events.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "actor_system.h"

namespace mxar {

// Flat JSON object -> key/value strings (strings unescaped, numbers/bools/null verbatim).
// Nested values are rejected. Returns false on malformed input.
bool parse_flat_json(const std::string& line, std::map<std::string, std::string>& out);
std::string json_escape(const std::string& s);

class ControlBridge : public std::enable_shared_from_this<ControlBridge> {
 public:
  // Listen on host:port (port 0 = any free port; see port()).
  static std::shared_ptr<ControlBridge> start(const std::string& host, int port);
  ~ControlBridge();
  ControlBridge(const ControlBridge&) = delete;
  ControlBridge& operator=(const ControlBridge&) = delete;

  // Commands from clients go to `master` as BridgeCommand messages.
  void attach(ActorRef master, std::string master_path);
  int port() const { return port_; }
  // Send one line to every client (events) / to one client (replies).
  void publish(const std::string& line);
  void reply(uint64_t client, const std::string& line);
  // Remember the latest InitWorkers line for clients that connect later.
  void set_init_line(std::string line);
  size_t clients() const;
  // In-process front-ends (csrc/runtime/akka_endpoint.h) speak other wire formats: a tap gets
  // every event line and the replies addressed to its id (it must not block), submit()
  // forwards a command as a client's would (false without a master). on_stop() hooks run in
  // stop(), before the clients are dropped.
  using Tap = std::function<void(const std::string& line)>;
  uint64_t add_tap(Tap tap);
  void remove_tap(uint64_t id);
  bool submit(const BridgeCommand& cmd);
  void on_stop(std::function<void()> hook);
  // Outbound queue cap per client (bytes, default kMaxQueuedBytes); tests lower it.
  void set_max_queued_bytes(size_t b) { max_queued_.store(b); }
  void stop();

 private:
  // Outbound bytes a client may have queued before it is dropped (a control line is < 1 KiB,
  // so this is thousands of rounds of events a client has not read).
  static constexpr size_t kMaxQueuedBytes = 4u << 20;

  struct Client {
    ~Client();  // closes fd: only once no publisher can still be writing to it
    uint64_t id;
    int fd = -1;
    std::mutex wmu;               // guards out / queued
    std::condition_variable wcv;  // writer wake-up
    std::deque<std::string> out;  // lines waiting for the writer
    size_t queued = 0;            // bytes in `out`
    std::thread reader, writer;
    std::atomic<bool> dead{false};
    void kill();  // mark dead, wake the writer, unblock the reader (idempotent)
  };
  ControlBridge() = default;
  void accept_loop(std::shared_ptr<ControlBridge> self);
  void read_loop(std::shared_ptr<ControlBridge> self, std::shared_ptr<Client> c);
  void write_loop(std::shared_ptr<ControlBridge> self, std::shared_ptr<Client> c);
  // Queue one line for a client (never blocks on the socket); false if the client is gone.
  bool write_line(Client& c, const std::string& line);
  void reap();

  int lfd_ = -1;
  int wake_[2] = {-1, -1};
  int port_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<size_t> max_queued_{kMaxQueuedBytes};
  std::thread acceptor_;
  mutable std::mutex mu_;
  std::vector<std::shared_ptr<Client>> clients_;
  uint64_t next_id_ = 1;
  ActorRef master_;
  std::string master_path_;
  std::string init_line_;
  std::vector<std::pair<uint64_t, Tap>> taps_;
  std::vector<std::function<void()>> stop_hooks_;
};

}  // namespace mxar
