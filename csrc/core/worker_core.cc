#include "worker_core.h"

#include <algorithm>
#include <sstream>

#include "log.h"

namespace mxar {

namespace {
std::string dump(const Payload& p) {
  std::ostringstream os;
  os << "[";
  if (p) {
    std::vector<float> h = p->to_host();
    for (size_t i = 0; i < h.size() && i < 64; ++i) os << (i ? ", " : "") << h[i];
    if (h.size() > 64) os << ", ...(" << h.size() << ")";
  }
  os << "]";
  return os.str();
}
}  // namespace

WorkerCore::WorkerCore(WorkerEffects* fx, std::shared_ptr<DataPlane> plane)
    : fx_(fx), plane_(plane ? std::move(plane) : HostPlane::instance()) {}

// InitWorkers handler (AllreduceWorker.scala:37-82)
void WorkerCore::on_init(const InitParams& p) {
  if (p.numPeers <= 0) throw ProtocolError("InitWorkers with no peers");
  if (p.destId < 0 || p.destId >= p.numPeers)
    throw ProtocolError("InitWorkers destId " + std::to_string(p.destId) + " outside 0.." +
                        std::to_string(p.numPeers - 1));
  if (p.maxChunkSize <= 0) throw ProtocolError("InitWorkers maxChunkSize must be > 0");
  if (p.maxLag < 0) throw ProtocolError("InitWorkers maxLag must be >= 0");
  params_ = p;
  id_ = p.destId;
  P_ = p.numPeers;
  round_ = std::max(0, p.startRound);  // clear round info to start over (at the resume round)
  maxRound_ = round_ - 1;
  maxScattered_ = round_ - 1;
  completed_.clear();
  data_ = plane_->zeros(static_cast<size_t>(p.dataSize));

  layout_ = BlockLayout(p.dataSize, P_, p.maxChunkSize);
  myBlockSize_ = layout_.block_size(id_);
  maxBlockSize_ = layout_.max_block_size();
  myNumChunks_ = layout_.num_chunks(id_);
  maxNumChunks_ = maxBlockSize_ == 0 ? 0 : f32_ceil_div(maxBlockSize_, p.maxChunkSize);

  const int rows = p.maxLag + 1;
  scatterBuf_.counters = ArrivalCounters(rows, P_, myNumChunks_, p.thReduce);
  scatterBuf_.slab = plane_->make_slab(rows, P_, static_cast<size_t>(myBlockSize_));
  scatterBuf_.dataSize = myBlockSize_;
  scatterBuf_.maxChunkSize = p.maxChunkSize;

  // Reduce buffer: the reference requires (thComplete * P * maxNumChunks).toInt chunks,
  // which can never be reached when tail blocks have fewer chunks. Keep the
  // reference formula whenever all blocks have the same chunk count (every config in
  // which the reference works), otherwise count the chunks that actually exist.
  int minChunks = -1;
  if (!layout_.uniform_chunks())
    minChunks = f32_threshold_count(p.thComplete, layout_.total_chunks());
  reduceBuf_.counters = ArrivalCounters(rows, P_, maxNumChunks_, p.thComplete, minChunks);
  reduceBuf_.slab = plane_->make_slab(rows, P_, static_cast<size_t>(maxBlockSize_));
  reduceBuf_.dataSize = maxBlockSize_;
  reduceBuf_.maxChunkSize = p.maxChunkSize;
  reduceCounts_.assign(static_cast<size_t>(rows) * P_ * std::max(maxNumChunks_, 0), 0);

  MXAR_LOG(INFO, "worker", "----Actor id = " << id_ << " (epoch " << p.epoch << ")");
  MXAR_LOG(INFO, "worker", "----Number of peers = " << P_);
  MXAR_LOG(INFO, "worker", "----Thresholds: thReduce = " << p.thReduce << ", thComplete = "
                                                          << p.thComplete << ", maxLag = " << p.maxLag);
  MXAR_LOG(INFO, "worker", "----Size of scatter buffer: " << rows << " x " << P_ << " x " << myBlockSize_);
  MXAR_LOG(INFO, "worker", "----Size of reduce buffer: " << rows << " x " << P_ << " x " << maxBlockSize_);
}

// StartAllreduce handler (AllreduceWorker.scala:84-104)
// Membership-epoch gate: 1 = handle, 0 = drop (older epoch), -1 = stash
// (newer epoch: this worker's own re-init is still in flight).
int WorkerCore::epoch_gate(int64_t e) {
  if (e == params_.epoch) return 1;
  if (e > params_.epoch) {
    stats_.stashed++;
    return -1;
  }
  stats_.stale_epoch_dropped++;
  return 0;
}

bool WorkerCore::on_start(const StartAllreduce& s) {
  if (!initialized()) {
    stats_.stashed++;
    return false;
  }
  if (const int g = epoch_gate(s.epoch); g <= 0) return g == 0;
  stats_.start_in++;
  MXAR_LOG(INFO, "worker", "----Start allreduce round " << s.round);
  maxRound_ = std::max(maxRound_, s.round);
  while (round_ < maxRound_ - params_.maxLag) {  // fell behind too much: forced catch-up
    for (int k = 0; k < myNumChunks_; ++k) {
      auto [v, c] = reduce(0, k);
      broadcast(v, k, round_, c);
    }
    stats_.forced_completions++;
    trace_instant("worker", "forced catch-up r" + std::to_string(round_), "{\"worker\":" + std::to_string(id_) + "}");
    MXAR_LOG(INFO, "worker", "----Catch up: force-completing round " << round_);
    complete(round_, 0);
  }
  while (maxScattered_ < maxRound_) {
    fetch(maxScattered_ + 1);
    scatter();
    maxScattered_ += 1;
  }
  for (auto it = completed_.begin(); it != completed_.end();)
    it = (*it < round_) ? completed_.erase(it) : std::next(it);
  return true;
}

// ScatterBlock handler (AllreduceWorker.scala:106-127)
bool WorkerCore::on_scatter(const ScatterBlock& s) {
  if (!initialized()) {
    stats_.stashed++;
    return false;
  }
  if (const int g = epoch_gate(s.epoch); g <= 0) return g == 0;
  stats_.scatter_in++;
  stats_.bytes_in += payload_size(s.value) * sizeof(float);
  MXAR_LOG(TRACE, "worker", "----receive scattered data from round " << s.round << ": value = "
                                << dump(s.value) << ", srcId = " << s.srcId << ", destId = " << s.destId
                                << ", chunkId=" << s.chunkId << ", current round = " << round_);
  if (s.destId != id_ || s.srcId < 0 || s.srcId >= P_ || s.chunkId < 0 ||
      s.chunkId >= myNumChunks_ ||
      static_cast<size_t>(s.chunkId) * params_.maxChunkSize + payload_size(s.value) >
          static_cast<size_t>(myBlockSize_)) {
    // The reference asserts (AllreduceWorker.scala:112) and the actor restarts, losing
    // its state; we drop the malformed message and keep going.
    stats_.malformed_dropped++;
    MXAR_LOG(ERROR, "worker", "----Malformed ScatterBlock dropped (src " << s.srcId << ", dest "
                                  << s.destId << ", chunk " << s.chunkId << ", len "
                                  << payload_size(s.value) << ") at worker " << id_);
    return true;
  }
  if (outdated(s.round)) {
    stats_.outdated_dropped++;
    MXAR_LOG(WARNING, "worker", "----Outdated scattered data (round " << s.round << ", current " << round_ << ")");
  } else if (s.round <= maxRound_) {
    const int row = s.round - round_;
    if (!scatterBuf_.counters.mark_src(row, s.srcId, s.chunkId)) stats_.duplicate_arrivals++;
    scatterBuf_.store(s.value, row, s.srcId, s.chunkId);
    if (scatterBuf_.counters.reach_threshold(row, s.chunkId)) {
      MXAR_LOG(DEBUG, "worker", "----receive " << scatterBuf_.counters.count(row, s.chunkId)
                                    << " scattered data (numPeers = " << P_ << "), chunkId =" << s.chunkId
                                    << " for round " << s.round << ", start reducing");
      auto [v, c] = reduce(row, s.chunkId);
      broadcast(v, s.chunkId, s.round, c);
    }
  } else {
    stats_.future_requeued++;
    fx_->to_self(StartAllreduce{s.round, params_.epoch});
    fx_->to_self(ScatterBlock(s));
  }
  return true;
}

// ReduceBlock handler (AllreduceWorker.scala:129-150)
bool WorkerCore::on_reduce(const ReduceBlock& r) {
  if (!initialized()) {
    stats_.stashed++;
    return false;
  }
  if (const int g = epoch_gate(r.epoch); g <= 0) return g == 0;
  stats_.reduce_in++;
  stats_.bytes_in += payload_size(r.value) * sizeof(float);
  MXAR_LOG(TRACE, "worker", "----Receive reduced data from round " << r.round << ": value = " << dump(r.value)
                                << ", srcId = " << r.srcId << ", destId = " << r.destId
                                << ", chunkId=" << r.chunkId);
  const bool too_big = payload_size(r.value) > static_cast<size_t>(params_.maxChunkSize);
  if (too_big || r.destId != id_ || r.srcId < 0 || r.srcId >= P_ || r.chunkId < 0 ||
      r.chunkId >= maxNumChunks_ ||
      static_cast<size_t>(r.chunkId) * params_.maxChunkSize + payload_size(r.value) >
          static_cast<size_t>(maxBlockSize_)) {
    // AllreduceWorker.scala:135-136 asserts; see on_scatter.
    stats_.malformed_dropped++;
    MXAR_LOG(ERROR, "worker", "----Malformed ReduceBlock dropped (src " << r.srcId << ", dest " << r.destId
                                  << ", chunk " << r.chunkId << ", len " << payload_size(r.value)
                                  << (too_big ? ", larger than maxChunkSize" : "") << ") at worker " << id_);
    return true;
  }
  if (outdated(r.round)) {
    stats_.outdated_dropped++;
    MXAR_LOG(WARNING, "worker", "----Outdated reduced data (round " << r.round << ", current " << round_ << ")");
  } else if (r.round <= maxRound_) {
    const int row = r.round - round_;
    if (!reduceBuf_.counters.mark_src(row, r.srcId, r.chunkId)) stats_.duplicate_arrivals++;
    reduceBuf_.store(r.value, row, r.srcId, r.chunkId);
    const size_t ci = (static_cast<size_t>(reduceBuf_.counters.phys(row)) * P_ + r.srcId) * maxNumChunks_ + r.chunkId;
    reduceCounts_[ci] = r.count;
    if (reduceBuf_.counters.reach_round_threshold(row)) {
      MXAR_LOG(DEBUG, "worker", "----Receive enough reduced data (numPeers = " << P_ << ") for round "
                                    << r.round << ", complete");
      complete(r.round, row);
    }
  } else {
    stats_.future_requeued++;
    fx_->to_self(StartAllreduce{r.round, params_.epoch});
    fx_->to_self(ReduceBlock(r));
  }
  return true;
}

// fetch (AllreduceWorker.scala:171-178)
void WorkerCore::fetch(int round) {
  MXAR_LOG(INFO, "worker", "fetch " << round);
  round_t0_[round] = Tracer::now_ns();
  TraceScope span("worker", [&] {
    return std::make_pair(std::string("fetch r" + std::to_string(round)),
                          std::string("{\"worker\":" + std::to_string(id_) + "}"));
  });
  AllReduceInput in = fx_->fetch(AllReduceInputRequest{round});
  if (payload_size(in.data) != static_cast<size_t>(params_.dataSize))
    throw ProtocolError("Input data size " + std::to_string(payload_size(in.data)) +
                        " is different from initialization time " + std::to_string(params_.dataSize) + "!");
  data_ = plane_->adopt(std::move(in.data));  // e.g. upload a host input to HBM once
}

// flush (AllreduceWorker.scala:180-192)
void WorkerCore::flush(int completedRound, int row) {
  const int phys = reduceBuf_.counters.phys(row);
  Payload out = reduceBuf_.slab->flush(phys, static_cast<size_t>(params_.dataSize));
  MXAR_LOG(TRACE, "worker", "----Flushing " << dump(out) << " at completed round " << completedRound);
  MXAR_LOG(INFO, "worker", "----Flushing round " << completedRound << " (" << payload_size(out) << " floats)");
  std::vector<int> counts(reduceCounts_.begin() + static_cast<size_t>(phys) * P_ * maxNumChunks_,
                          reduceCounts_.begin() + static_cast<size_t>(phys + 1) * P_ * maxNumChunks_);
  fx_->sink(AllReduceOutput{std::move(out), std::move(counts), completedRound});
}

// scatter (AllreduceWorker.scala:194-209)
void WorkerCore::scatter() {
  TraceScope span("worker", [&] {
    return std::make_pair(std::string("scatter r" + std::to_string(maxScattered_ + 1)),
                          std::string("{\"worker\":" + std::to_string(id_) + "}"));
  });
  const int r = maxScattered_ + 1;
  const int C = params_.maxChunkSize;
  for (int i = 0; i < P_; ++i) {
    const int idx = (i + id_) % P_;
    const int bstart = layout_.start[idx];
    const int len = layout_.block_size(idx);
    // each destination gets its OWN chunk count. The reference iterates
    // myNumChunks for every destination, which duplicates or omits tail chunks when
    // block chunk counts differ; for equal counts both loops are identical.
    const int nchunks = layout_.num_chunks(idx);
    for (int k = 0; k < nchunks; ++k) {
      const int cs = std::min(k * C, len - 1);
      const int ce = std::min((k + 1) * C - 1, len - 1);
      Payload chunk = plane_->slice(data_, static_cast<size_t>(bstart + cs), static_cast<size_t>(ce - cs + 1));
      MXAR_LOG(TRACE, "worker", "----send msg " << dump(chunk) << " from " << id_ << " to " << idx
                                    << ", chunkId: " << k);
      stats_.scatter_out++;
      stats_.bytes_out += payload_size(chunk) * sizeof(float);
      fx_->to_peer(idx, ScatterBlock{std::move(chunk), id_, idx, k, r, params_.epoch});
    }
  }
}

// broadcast (AllreduceWorker.scala:230-238)
void WorkerCore::broadcast(const Payload& v, int chunkId, int round, int count) {
  MXAR_LOG(DEBUG, "worker", "----Start broadcasting");
  for (int i = 0; i < P_; ++i) {
    const int idx = (i + id_) % P_;
    MXAR_LOG(TRACE, "worker", "----Broadcast data:" << dump(v) << ", src: " << id_ << ", dest: " << idx
                                  << ", chunkId: " << chunkId << ", round: " << round);
    stats_.reduce_out++;
    stats_.bytes_out += payload_size(v) * sizeof(float);
    fx_->to_peer(idx, ReduceBlock{v, id_, idx, chunkId, round, count, params_.epoch});
  }
}

// reduce (AllreduceWorker.scala:240-251): sums ALL peer slots (missing ones are zero)
std::pair<Payload, int> WorkerCore::reduce(int row, int chunkId) {
  MXAR_LOG(DEBUG, "worker", "----Start reducing");
  const int count = scatterBuf_.counters.count(row, chunkId);
  const size_t len = scatterBuf_.chunk_len(chunkId);
  const int phys = scatterBuf_.counters.phys(row);
  stats_.reductions++;
  Payload v = scatterBuf_.slab->reduce(phys, static_cast<size_t>(chunkId) * params_.maxChunkSize, len);
  return {std::move(v), count};
}

// complete (AllreduceWorker.scala:253-268)
void WorkerCore::complete(int completedRound, int row) {
  MXAR_LOG(DEBUG, "worker", "----Complete allreduce round " << completedRound);
  TraceScope span("worker", [&] {
    return std::make_pair(std::string("complete r" + std::to_string(completedRound)),
                          std::string("{\"worker\":" + std::to_string(id_) + "}"));
  });
  if (auto it = round_t0_.find(completedRound); it != round_t0_.end()) {
    const double ms = (Tracer::now_ns() - it->second) / 1e6;
    if (lat_ms_.size() < 4096)
      lat_ms_.push_back(ms);
    else
      lat_ms_[lat_pos_] = ms;
    lat_pos_ = (lat_pos_ + 1) % 4096;
    ++lat_count_;
    round_t0_.erase(it);
  }
  flush(completedRound, row);
  data_ = plane_->zeros(0);
  stats_.complete_out++;
  stats_.rounds_completed++;
  fx_->to_master(CompleteAllreduce{id_, completedRound, params_.epoch});
  completed_.insert(completedRound);
  if (round_ == completedRound) {
    do {
      round_ += 1;
      const size_t recycled = static_cast<size_t>(reduceBuf_.counters.phys(0));
      scatterBuf_.up();
      reduceBuf_.up();
      // the recycled row's reported contribution counts start over with its data
      const size_t per_row = static_cast<size_t>(P_) * std::max(maxNumChunks_, 0);
      std::fill(reduceCounts_.begin() + recycled * per_row, reduceCounts_.begin() + (recycled + 1) * per_row, 0);
    } while (completed_.count(round_));
  }
}

RoundLatency WorkerCore::round_latency() const {
  RoundLatency r;
  r.count = lat_count_;
  if (lat_ms_.empty()) return r;
  std::vector<double> v = lat_ms_;
  std::sort(v.begin(), v.end());
  auto q = [&](double p) { return v[std::min(v.size() - 1, static_cast<size_t>(p * (v.size() - 1) + 0.5))]; };
  r.p50_ms = q(0.5);
  r.p99_ms = q(0.99);
  r.max_ms = v.back();
  double s = 0;
  for (double x : v) s += x;
  r.mean_ms = s / v.size();
  return r;
}

std::string WorkerCore::describe() const {
  std::ostringstream os;
  os << "WorkerCore(id=" << id_ << ", P=" << P_ << ", round=" << round_ << ", maxRound=" << maxRound_
     << ", maxScattered=" << maxScattered_ << ", completed={";
  bool first = true;
  for (int c : completed_) {
    os << (first ? "" : ",") << c;
    first = false;
  }
  os << "}, plane=" << plane_->name() << ")";
  return os.str();
}

}  // namespace mxar
