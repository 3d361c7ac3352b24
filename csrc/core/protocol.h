// Wire protocol of the threshold allreduce: the five actor messages and the three
// user-I/O records of the reference, with identical fields and field order.
//
//   reference: src/main/scala/sample/cluster/allreduce/AllreduceMessage.scala:7-20
//              src/main/scala/sample/cluster/allreduce/DataWrapper.scala:3-7
//
// Payloads (`value`, `data`) are reference-counted immutable float32 chunks. A payload
// is host memory or device (HBM) memory; the protocol cores never touch the bytes
// themselves, they hand payloads to a DataPlane (host loops or HIP kernels).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <variant>
#include <vector>

namespace mxar {

// ---------------------------------------------------------------------------------
// Payload storage
// ---------------------------------------------------------------------------------
class PayloadStorage {
 public:
  virtual ~PayloadStorage() = default;
  virtual bool on_device() const = 0;
  // Pointer to the first float (host pointer, or device pointer when on_device()).
  virtual const float* data() const = 0;
  virtual size_t size() const = 0;
  // Blocking copy to host (device payloads synchronise on their ready event).
  virtual std::vector<float> to_host() const = 0;
  // Element type: 0 = float32 (every host payload, the reference's Array[Float]),
  // 1 = bfloat16, 2 = float16 (device payloads of the xGMI round engine). size() counts
  // elements of this type; to_host() converts to float32.
  virtual int dtype() const { return 0; }
};
using Payload = std::shared_ptr<const PayloadStorage>;

class HostPayload final : public PayloadStorage {
 public:
  explicit HostPayload(std::vector<float> v) : v_(std::move(v)) {}
  bool on_device() const override { return false; }
  const float* data() const override { return v_.data(); }
  size_t size() const override { return v_.size(); }
  std::vector<float> to_host() const override { return v_; }
  const std::vector<float>& vec() const { return v_; }

 private:
  std::vector<float> v_;
};

inline Payload make_host_payload(std::vector<float> v) {
  return std::make_shared<HostPayload>(std::move(v));
}
inline size_t payload_size(const Payload& p) { return p ? p->size() : 0; }

// ---------------------------------------------------------------------------------
// Actor references (opaque to the protocol cores; implemented by the runtime)
// ---------------------------------------------------------------------------------
class ActorRefBase;
using ActorRef = std::shared_ptr<ActorRefBase>;

// ---------------------------------------------------------------------------------
// Messages (AllreduceMessage.scala)
// ---------------------------------------------------------------------------------
struct InitWorkers {  // AllreduceMessage.scala:7-16
  std::map<int, ActorRef> workers;
  ActorRef master;
  int destId = 0;
  float thReduce = 1.f;
  float thComplete = 1.f;
  int maxLag = 0;
  int dataSize = 0;
  int maxChunkSize = 1024;
  // Extension (not in the reference): membership epoch, bumped by the master on every
  // (re-)initialisation so late messages of an older epoch can be told apart.
  int64_t epoch = 0;
  // Extension: first round of this epoch - 0 normally, the checkpointed
  // round when a job resumes (workers start there instead of replaying earlier rounds).
  int startRound = 0;
  // Extension (data plane A): every worker's plane descriptor as it announced
  // it at registration (MemberUp.meta) - for the xGMI round engine the IPC handle of its
  // HBM arena - so each worker maps its peers' slabs from InitWorkers alone. Empty when the
  // workers use the actor data path (ScatterBlock / ReduceBlock messages).
  std::map<int, std::string> planes;
  // Extension: device round-epoch base of this membership epoch. Round r of the epoch is
  // device epoch roundBase + (r - startRound) + 1; the master keeps the bases increasing
  // across re-initialisations, so flags an older epoch left in a reused arena are never
  // mistaken for this epoch's.
  uint32_t roundBase = 0;
};

// Extension: the round messages carry the membership epoch of the
// InitWorkers they belong to, as a trailing field (the reference's field order is kept).
// A worker drops messages of an older epoch and stashes messages of a newer one until its
// own re-init arrives, so traffic in flight across a re-initialisation can never land in
// the new epoch's buffers.
struct StartAllreduce {  // AllreduceMessage.scala:17
  int round = 0;
  int64_t epoch = 0;
};

struct ScatterBlock {  // AllreduceMessage.scala:18
  Payload value;
  int srcId = 0;
  int destId = 0;
  int chunkId = 0;
  int round = 0;
  int64_t epoch = 0;
};

struct ReduceBlock {  // AllreduceMessage.scala:19
  Payload value;
  int srcId = 0;
  int destId = 0;
  int chunkId = 0;
  int round = 0;
  int count = 0;
  int64_t epoch = 0;
};

struct CompleteAllreduce {  // AllreduceMessage.scala:20
  int srcId = 0;
  int round = 0;
  int64_t epoch = 0;
};

// ---------------------------------------------------------------------------------
// User I/O records (DataWrapper.scala)
// ---------------------------------------------------------------------------------
struct AllReduceInputRequest {  // DataWrapper.scala:3
  int iteration = 0;
};
struct AllReduceInput {  // DataWrapper.scala:5
  Payload data;
};
struct AllReduceOutput {  // DataWrapper.scala:7
  Payload data;
  // The reference always reports Array(0) (AllreduceWorker.scala:191).
  // We report the real per-chunk contribution counts of every block, concatenated in
  // block order (a superset: element 0 is still a valid count).
  std::vector<int> count;
  int iteration = 0;
};

// ---------------------------------------------------------------------------------
// Runtime / cluster control messages (Akka library messages in the reference)
// ---------------------------------------------------------------------------------
struct MemberUp {  // akka.cluster.ClusterEvent.MemberUp (AllreduceMaster.scala:38)
  ActorRef ref;  // the member's "/user/worker" actor, already resolved
  std::string role;
  std::string address;
  // Extension: metadata the member announced when it joined (ClusterConfig.meta); a GPU
  // worker's plane descriptor, relayed by the master in InitWorkers.planes.
  std::string meta;
};
struct Terminated {  // akka.actor.Terminated (AllreduceMaster.scala:50)
  ActorRef ref;
};
// Emitted by the master when maxRound has completed (the reference idles).
struct AllreduceFinished {
  int rounds = 0;
};
struct PoisonPill {};
// Generic string message for tests and for the TCP control plane's tooling.
struct TextMessage {
  std::string text;
};
// The master's round deadline (scheduled to itself, mxar.allreduce.round-timeout): the
// round `round` of membership epoch `epoch` has not reached the barrier in time.
struct RoundTimeout {
  int64_t epoch = 0;
  int round = 0;
};
// A round of a plane worker (csrc/runtime/plane_worker.h) finished on its data plane; posted
// by the plane's completion thread to the worker's own mailbox. `output` is the reference's
// AllReduceOutput (dataSink), `error` the plane's error word (0 = healthy), `cold` marks a
// round force-completed before it ever started.
struct PlaneRoundDone {
  int64_t epoch = 0;
  AllReduceOutput output;
  uint32_t error = 0;
  bool cold = false;
};

// A command from a control-bridge client (csrc/runtime/control_bridge.h) to the master:
// Start = the reference's StartAllreduce(round) issued by an external round driver,
// Status = one Status reply. Local to a node (never encoded).
struct BridgeCommand {
  enum Kind { Start, Status } kind = Status;
  int round = 0;
  uint64_t client = 0;  // bridge client that receives the reply
};

using Message = std::variant<InitWorkers, StartAllreduce, ScatterBlock, ReduceBlock,
                             CompleteAllreduce, MemberUp, Terminated, AllreduceFinished,
                             PoisonPill, TextMessage, RoundTimeout, PlaneRoundDone, BridgeCommand>;

const char* message_name(const Message& m);

}  // namespace mxar
