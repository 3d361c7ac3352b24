// Temporal lag-ring buffer of the worker: (maxLag+1) rows x peers x blockSize float
// slots plus per-(row, chunk) arrival counters.
//
//   reference: src/main/scala/sample/cluster/allreduce/buffer/DataBuffer.scala:3-82
//
// The reference keeps data and counters in one JVM object and re-allocates a row on
// every rotation (DataBuffer.scala:63-67). Here the two concerns are split:
//   * ArrivalCounters  - host-side control state (counters, thresholds, ring offset);
//                        the state machine branches on it, so it stays on the host.
//   * Slab             - the data rows. HostSlab uses one contiguous host allocation;
//                        the HIP DevicePlane (csrc/hip/device_plane.*) keeps the same
//                        [row][peer][block] layout in HBM. Rotation is a memset of the
//                        recycled row, never an allocation.
// The physical row of round r is always r mod rows (offset tracks round), so remote
// writers can address a row without knowing the receiver's offset.
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "protocol.h"

namespace mxar {

// ---- float32 arithmetic exactly as the JVM evaluates it -------
// (threshold * peerSize).toInt and (threshold * peerSize * numChunks).toInt: float32
// products evaluated left to right, truncated toward zero. A double evaluation differs
// in 215 (th, P, C) cases (e.g. th=0.04, P=5, C=5: float32 gives 0, double gives 1).
int f32_threshold_count(float threshold, int peers);
int f32_threshold_chunks(float threshold, int peers, int numChunks);
// math.ceil(1f * a / b).toInt (float32 division, then ceil); exact integer ceil-div
// beyond 2^24 where float32 can no longer represent a.
int f32_ceil_div(int64_t a, int64_t b);

// ---- block partitioning (AllreduceWorker.scala:211-228) ----------------------------
struct BlockLayout {
  int dataSize = 0;
  int peers = 0;
  int maxChunkSize = 1;
  std::vector<int> start;  // size peers (padded with dataSize)
  std::vector<int> end;
  int step = 0;

  BlockLayout() = default;
  BlockLayout(int dataSize, int peers, int maxChunkSize);
  int block_size(int idx) const { return end[idx] - start[idx]; }
  int num_chunks(int idx) const;  // ceil(blockSize / maxChunkSize), float32 like reference
  int max_block_size() const { return block_size(0); }
  int total_chunks() const;
  bool uniform_chunks() const;
};

// ---- arrival counters -----------------------------------------------------------------
class ArrivalCounters {
 public:
  ArrivalCounters() = default;
  // rows = maxLag + 1 (the worker passes maxLag+1, AllreduceWorker.scala:62,70)
  ArrivalCounters(int rows, int peers, int numChunks, float threshold, int minChunksOverride = -1);

  int phys(int row) const { return (row + offset_) % rows_; }
  void add(int row, int chunk);
  int count(int row, int chunk) const { return counts_[idx(row, chunk)]; }
  // DataBuffer.reachThreshold: exact equality -> fires exactly once per (row, chunk).
  bool reach_threshold(int row, int chunk) const { return count(row, chunk) == minRequired_; }
  // DataBuffer.reachRoundThreshold: sum over chunks == minChunksRequired (exact).
  bool reach_round_threshold(int row) const;
  int round_total(int row) const;
  // Rotate: the old row 0 becomes the (cleared) new last row. Returns its physical id.
  int up();
  void clear();

  int rows() const { return rows_; }
  int peers() const { return peers_; }
  int num_chunks() const { return numChunks_; }
  int min_required() const { return minRequired_; }
  int min_chunks_required() const { return minChunksRequired_; }
  int offset() const { return offset_; }
  std::vector<int> row_counts(int row) const;

  // Duplicate-arrival telemetry (the reference double-counts silently).
  bool mark_src(int row, int src, int chunk);  // returns true if (row,src,chunk) was new

 private:
  size_t idx(int row, int chunk) const {
    return static_cast<size_t>(phys(row)) * numChunks_ + chunk;
  }
  int rows_ = 0, peers_ = 0, numChunks_ = 0;
  float threshold_ = 1.f;
  int minRequired_ = 0, minChunksRequired_ = 0;
  int offset_ = 0;
  std::vector<int> counts_;
  std::vector<uint8_t> seen_;  // rows x peers x chunks
};

// ---- data slabs ------------------------------------------------------------------------
// Abstract slab of rows x peers x slotSize floats. Row arguments are PHYSICAL rows.
class Slab {
 public:
  virtual ~Slab() = default;
  virtual void store(const Payload& v, int physRow, int src, size_t offset) = 0;
  // Element-wise sum over all peers of [offset, offset+len) -> new payload.
  // Summation order is peer 0..P-1 in float32 (AllreduceWorker.scala:245-249).
  virtual Payload reduce(int physRow, size_t offset, size_t len) = 0;
  // Concatenate the peer slots of a row and truncate to n (AllreduceWorker.scala:180-192).
  virtual Payload flush(int physRow, size_t n) = 0;
  virtual void clear_row(int physRow) = 0;
  size_t slot_size() const { return slot_; }
  int peers() const { return peers_; }
  int rows() const { return rows_; }

 protected:
  int rows_ = 0, peers_ = 0;
  size_t slot_ = 0;
};

// Factory + payload helpers for a given memory space.
class DataPlane {
 public:
  virtual ~DataPlane() = default;
  virtual const char* name() const = 0;
  virtual std::unique_ptr<Slab> make_slab(int rows, int peers, size_t slotSize) = 0;
  // Zero-copy or copied sub-range of a payload (scatter chunking).
  virtual Payload slice(const Payload& p, size_t start, size_t len) = 0;
  // Payload of n zeros (the reference initialises data with zeros).
  virtual Payload zeros(size_t n) = 0;
  // Bring a payload into this plane's memory space (identity when it already lives there).
  virtual Payload adopt(Payload p) { return p; }
};

class HostSlab final : public Slab {
 public:
  HostSlab(int rows, int peers, size_t slot);
  void store(const Payload& v, int physRow, int src, size_t offset) override;
  Payload reduce(int physRow, size_t offset, size_t len) override;
  Payload flush(int physRow, size_t n) override;
  void clear_row(int physRow) override;
  const float* row_ptr(int physRow, int src) const {
    return buf_.data() + (static_cast<size_t>(physRow) * peers_ + src) * slot_;
  }

 private:
  std::vector<float> buf_;
};

class HostPlane final : public DataPlane {
 public:
  const char* name() const override { return "host"; }
  std::unique_ptr<Slab> make_slab(int rows, int peers, size_t slotSize) override {
    return std::make_unique<HostSlab>(rows, peers, slotSize);
  }
  Payload slice(const Payload& p, size_t start, size_t len) override;
  Payload zeros(size_t n) override { return make_host_payload(std::vector<float>(n, 0.f)); }
  static std::shared_ptr<HostPlane> instance();
};

// Full DataBuffer = counters + slab, as the worker uses it.
struct DataBuffer {
  ArrivalCounters counters;
  std::unique_ptr<Slab> slab;
  int dataSize = 0;
  int maxChunkSize = 1;

  void store(const Payload& v, int row, int src, int chunk);
  // DataBuffer.get(row, chunkId) length: min(dataSize, (chunk+1)*C) - chunk*C
  size_t chunk_len(int chunk) const;
  void up();
};

class ProtocolError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

}  // namespace mxar
