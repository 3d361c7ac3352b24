// RoundPlane: the data plane of a round-granular worker (PlaneWorkerActor) - the whole
// scatter / threshold-reduce / broadcast / threshold-complete exchange of one allreduce
// round runs inside the plane, as ONE launch, instead of as P x C ScatterBlock and C x P
// ReduceBlock actor messages (AllreduceWorker.scala:194-251). The actor keeps the
// reference's control protocol: InitWorkers / StartAllreduce in, CompleteAllreduce out,
// dataSource / dataSink per round, forced catch-up when StartAllreduce runs ahead.
//
// Implementations:
//   XgmiRoundPlane     (csrc/hip/xgmi_plane.*)  - HBM arena exported over IPC, one
//                      threshold-kernel launch per round over xGMI peer stores (MI355X)
//   LoopbackRoundPlane (loopback_plane.*)       - host memory + one thread per plane, same
//                      round semantics; in-process clusters on a CPU (tests, sanitizers)
//
// Semantics every plane implements for round r (reference order):
//   * the own input block chunks go to their owners, a chunk is reduced from exactly the
//     first f32(thReduce * P) contributions (what was queued at the round's start first,
//     then the own one, then later arrivals), the reduced chunk goes to every worker;
//   * the round completes with the first f32(thComplete * P * nch) reduced chunks; the
//     rest are zeros with count 0 (AllReduceOutput.count = per-chunk contribution counts);
//   * force(r) makes every round <= r stop waiting and complete with what has arrived
//     (catch-up); a `cold` round (stale before it was started) contributes nothing;
//   * a plane never runs more than maxLag rounds ahead of a peer's progress: the peer is
//     asked to force-complete instead.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <string>

#include "../core/protocol.h"

namespace mxar {

struct PlaneConfig {
  int id = 0;
  int peers = 0;
  float thReduce = 1.f, thComplete = 1.f;
  int maxLag = 0;
  int dataSize = 0;
  int maxChunkSize = 1;
  int64_t epoch = 0;
  int startRound = 0;
  uint32_t roundBase = 0;
  std::map<int, std::string> descriptors;  // InitWorkers.planes: every worker's descriptor
};

struct RoundResult {
  int64_t epoch = 0;
  int round = 0;
  Payload data;            // dataSize elements (plane dtype)
  std::vector<int> count;  // [peers][chunks] contributions per output chunk
  uint32_t error = 0;
  bool cold = false;
};

class RoundPlane {
 public:
  using DoneFn = std::function<void(RoundResult&&)>;
  virtual ~RoundPlane() = default;
  virtual const char* name() const = 0;
  // What the worker announces at registration (MemberUp.meta); peers map it in configure().
  virtual std::string descriptor() const = 0;
  // Called from the plane's completion thread, once per launched round, in launch order.
  virtual void set_done(DoneFn fn) = 0;
  // (Re-)initialise for a membership epoch: finishes every round in flight first.
  virtual void configure(const PlaneConfig& cfg) = 0;
  // Enqueue round `round` (asynchronous). `input` holds dataSize elements; ignored (may be
  // null) for a cold round.
  virtual void launch(int round, const Payload& input, bool cold) = 0;
  // Rounds <= `round` stop waiting and complete with what has arrived.
  virtual void force(int round) = 0;
  // Rounds <= `round` are abandoned (re-initialisation, shutdown): like force(), and a
  // round that has not started exchanging yet delivers nothing instead of waiting for a
  // peer that may never come back (its result is dropped as an older epoch anyway).
  virtual void abort(int round) { force(round); }
  // Block until every launched round has completed (and its done callback ran).
  virtual void drain() = 0;
  // Chunks per block of the current configuration (AllReduceOutput.count has peers x this).
  virtual int chunks() const = 0;
};

}  // namespace mxar
