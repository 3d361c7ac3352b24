// Protocol state machine of one allreduce worker, independent of transport and of
// where the bytes live.
//
//   reference: src/main/scala/sample/cluster/allreduce/AllreduceWorker.scala:9-270
//
// Behaviour contract, kept exactly for every configuration in which the
// reference works:
//   * float32 thresholds evaluated like the JVM, `==` triggers that fire exactly once;
//   * scatter/broadcast fan-out in rotated order (i + id) % P, self included;
//   * out-of-order round completion, outdated-message dropping, future-round
//     self-trigger (Start(r) then the message re-enqueued at the mailbox tail);
//   * forced catch-up when the master runs more than maxLag rounds ahead.
// Deliberate fixes (each documented in docs/PROTOCOL.md):
//   * messages that arrive before Init are stashed, not busy re-enqueued;
//   * scatter sends each destination its own chunk count;
//   * short tail blocks are padded instead of indexing out of bounds;
//   * malformed messages are dropped with an error instead of crashing the actor.
#pragma once

#include <functional>
#include <map>
#include <set>
#include <string>
#include <variant>
#include <vector>

#include "data_buffer.h"
#include "protocol.h"
#include "trace.h"

namespace mxar {

struct InitParams {
  int destId = 0;
  int numPeers = 0;
  float thReduce = 1.f;
  float thComplete = 1.f;
  int maxLag = 0;
  int dataSize = 0;
  int maxChunkSize = 1024;
  int64_t epoch = 0;
  int startRound = 0;
  uint32_t roundBase = 0;  // device round-epoch base (InitWorkers.roundBase; plane workers)
};

// Messages the worker core can emit to a peer or to itself.
using WorkerMsg = std::variant<StartAllreduce, ScatterBlock, ReduceBlock>;

// Side effects of the core, provided by whoever hosts it (actor runtime, engine, test).
class WorkerEffects {
 public:
  virtual ~WorkerEffects() = default;
  virtual void to_peer(int peer, ScatterBlock&& m) = 0;
  virtual void to_peer(int peer, ReduceBlock&& m) = 0;
  virtual void to_master(CompleteAllreduce&& m) = 0;
  // Self-send: appended to the tail of the own mailbox (AllreduceWorker.scala:124-125).
  virtual void to_self(WorkerMsg&& m) = 0;
  virtual AllReduceInput fetch(const AllReduceInputRequest& req) = 0;  // dataSource
  virtual void sink(AllReduceOutput&& out) = 0;                        // dataSink
};

struct RoundLatency {  // fetch of round r -> its completion, over the last 4096 rounds
  uint64_t count = 0;
  double p50_ms = 0, p99_ms = 0, mean_ms = 0, max_ms = 0;
};

struct WorkerStats {
  uint64_t scatter_in = 0, reduce_in = 0, start_in = 0;
  uint64_t scatter_out = 0, reduce_out = 0, complete_out = 0;
  uint64_t bytes_out = 0, bytes_in = 0;
  uint64_t outdated_dropped = 0, future_requeued = 0, stashed = 0;
  uint64_t forced_completions = 0, rounds_completed = 0, reductions = 0;
  uint64_t duplicate_arrivals = 0, malformed_dropped = 0, stale_epoch_dropped = 0;
};

class WorkerCore {
 public:
  WorkerCore(WorkerEffects* fx, std::shared_ptr<DataPlane> plane);

  bool initialized() const { return id_ >= 0; }
  void on_init(const InitParams& p);
  // The three handlers return false when the core is not initialised, or when the message
  // belongs to a newer membership epoch than the last Init: the host must stash it and
  // replay it after the next Init. Messages of an older epoch are dropped.
  bool on_start(const StartAllreduce& m);
  bool on_scatter(const ScatterBlock& m);
  bool on_reduce(const ReduceBlock& m);

  // Introspection (tests, metrics, checkpoint of control state)
  int id() const { return id_; }
  int round() const { return round_; }
  int max_round() const { return maxRound_; }
  int max_scattered() const { return maxScattered_; }
  const std::set<int>& completed() const { return completed_; }
  int num_peers() const { return P_; }
  const BlockLayout& layout() const { return layout_; }
  int my_num_chunks() const { return myNumChunks_; }
  int max_num_chunks() const { return maxNumChunks_; }
  const DataBuffer& scatter_buf() const { return scatterBuf_; }
  const DataBuffer& reduce_buf() const { return reduceBuf_; }
  const WorkerStats& stats() const { return stats_; }
  RoundLatency round_latency() const;
  const InitParams& params() const { return params_; }
  std::string describe() const;

 private:
  void fetch(int round);
  void scatter();
  void broadcast(const Payload& v, int chunkId, int round, int count);
  std::pair<Payload, int> reduce(int row, int chunkId);
  void complete(int completedRound, int row);
  void flush(int completedRound, int row);
  bool outdated(int r) const { return r < round_ || completed_.count(r) > 0; }
  int epoch_gate(int64_t e);

  WorkerEffects* fx_;
  std::shared_ptr<DataPlane> plane_;
  InitParams params_;
  int id_ = -1;
  int P_ = 0;
  int round_ = -1, maxRound_ = -1, maxScattered_ = -1;
  std::set<int> completed_;
  Payload data_;
  BlockLayout layout_;
  int myBlockSize_ = 0, maxBlockSize_ = 0, myNumChunks_ = 0, maxNumChunks_ = 0;
  DataBuffer scatterBuf_, reduceBuf_;
  // per physical row, per block owner: count carried by the ReduceBlock (for Output.count)
  std::vector<int> reduceCounts_;
  WorkerStats stats_;
  std::map<int, uint64_t> round_t0_;
  std::vector<double> lat_ms_;
  size_t lat_pos_ = 0;
  uint64_t lat_count_ = 0;
};

}  // namespace mxar
