#include "data_buffer.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace mxar {

// volatile stores keep the compiler from contracting / widening the float products:
// the JVM evaluates (threshold * peerSize) in float32, then (* numChunks) in float32.
int f32_threshold_count(float threshold, int peers) {
  volatile float p = threshold * static_cast<float>(peers);
  return static_cast<int>(p);
}

int f32_threshold_chunks(float threshold, int peers, int numChunks) {
  volatile float p = threshold * static_cast<float>(peers);
  volatile float q = p * static_cast<float>(numChunks);
  return static_cast<int>(q);
}

int f32_ceil_div(int64_t a, int64_t b) {
  if (b <= 0) throw ProtocolError("ceil_div by non-positive divisor");
  if (a < (int64_t{1} << 24) && b < (int64_t{1} << 24)) {
    volatile float q = static_cast<float>(a) / static_cast<float>(b);
    return static_cast<int>(std::ceil(static_cast<double>(q)));
  }
  return static_cast<int>((a + b - 1) / b);
}

// ---------------------------------------------------------------------------------
BlockLayout::BlockLayout(int n, int p, int c) : dataSize(n), peers(p), maxChunkSize(c) {
  if (p <= 0) throw ProtocolError("BlockLayout: peers must be > 0");
  if (c <= 0) throw ProtocolError("BlockLayout: maxChunkSize must be > 0");
  if (n < 0) throw ProtocolError("BlockLayout: negative dataSize");
  // stepSize = ceil(dataSize * 1f / peers.size)   (AllreduceWorker.scala:212)
  step = n == 0 ? 0 : f32_ceil_div(n, p);
  start.assign(p, n);
  end.assign(p, n);
  // Array.range(0, dataSize, stepSize): may hold fewer than P entries - the
  // missing tail blocks are padded as empty [n, n) instead of indexing out of bounds.
  int k = 0;
  if (step > 0)
    for (int64_t s = 0; s < n && k < p; s += step) start[k++] = static_cast<int>(s);
  for (int i = 0; i < p; ++i) {
    // range(idx): last peer ends at dataSize, others at the next range start
    end[i] = (i >= p - 1) ? n : start[i + 1];
    if (end[i] < start[i]) end[i] = start[i];
  }
}

int BlockLayout::num_chunks(int idx) const {
  int bs = block_size(idx);
  return bs == 0 ? 0 : f32_ceil_div(bs, maxChunkSize);
}

int BlockLayout::total_chunks() const {
  int t = 0;
  for (int i = 0; i < peers; ++i) t += num_chunks(i);
  return t;
}

bool BlockLayout::uniform_chunks() const {
  int c0 = num_chunks(0);
  for (int i = 1; i < peers; ++i)
    if (num_chunks(i) != c0) return false;
  return true;
}

// ---------------------------------------------------------------------------------
ArrivalCounters::ArrivalCounters(int rows, int peers, int numChunks, float threshold,
                                 int minChunksOverride)
    : rows_(rows), peers_(peers), numChunks_(numChunks), threshold_(threshold) {
  if (rows <= 0) throw ProtocolError("ArrivalCounters: rows must be > 0");
  minRequired_ = f32_threshold_count(threshold, peers);
  minChunksRequired_ = minChunksOverride >= 0 ? minChunksOverride
                                              : f32_threshold_chunks(threshold, peers, numChunks);
  // with th*P < 1 the reference's `==` test can never fire (count starts at
  // 0 and the first store makes it 1). We require at least one arrival instead.
  if (minRequired_ < 1) minRequired_ = 1;
  if (minChunksRequired_ < 1 && numChunks > 0) minChunksRequired_ = 1;
  counts_.assign(static_cast<size_t>(rows) * std::max(numChunks, 0), 0);
  seen_.assign(static_cast<size_t>(rows) * peers * std::max(numChunks, 0), 0);
}

void ArrivalCounters::add(int row, int chunk) {
  if (row < 0 || row >= rows_ || chunk < 0 || chunk >= numChunks_)
    throw ProtocolError("ArrivalCounters::add out of range (row " + std::to_string(row) +
                        ", chunk " + std::to_string(chunk) + ")");
  counts_[idx(row, chunk)] += 1;
}

bool ArrivalCounters::reach_round_threshold(int row) const {
  return round_total(row) == minChunksRequired_;
}

int ArrivalCounters::round_total(int row) const {
  int s = 0;
  const size_t base = static_cast<size_t>(phys(row)) * numChunks_;
  for (int i = 0; i < numChunks_; ++i) s += counts_[base + i];
  return s;
}

int ArrivalCounters::up() {
  offset_ = (offset_ + 1) % rows_;
  const int recycled = (offset_ + rows_ - 1) % rows_;
  std::fill(counts_.begin() + static_cast<size_t>(recycled) * numChunks_,
            counts_.begin() + static_cast<size_t>(recycled + 1) * numChunks_, 0);
  const size_t per_row = static_cast<size_t>(peers_) * numChunks_;
  std::fill(seen_.begin() + recycled * per_row, seen_.begin() + (recycled + 1) * per_row, 0);
  return recycled;
}

void ArrivalCounters::clear() {
  std::fill(counts_.begin(), counts_.end(), 0);
  std::fill(seen_.begin(), seen_.end(), 0);
  offset_ = 0;
}

std::vector<int> ArrivalCounters::row_counts(int row) const {
  std::vector<int> out(numChunks_);
  const size_t base = static_cast<size_t>(phys(row)) * numChunks_;
  for (int i = 0; i < numChunks_; ++i) out[i] = counts_[base + i];
  return out;
}

bool ArrivalCounters::mark_src(int row, int src, int chunk) {
  if (src < 0 || src >= peers_ || chunk < 0 || chunk >= numChunks_) return true;
  const size_t i = (static_cast<size_t>(phys(row)) * peers_ + src) * numChunks_ + chunk;
  const bool fresh = seen_[i] == 0;
  seen_[i] = 1;
  return fresh;
}

// ---------------------------------------------------------------------------------
HostSlab::HostSlab(int rows, int peers, size_t slot) {
  rows_ = rows;
  peers_ = peers;
  slot_ = slot;
  buf_.assign(static_cast<size_t>(rows) * peers * slot, 0.f);
}

void HostSlab::store(const Payload& v, int physRow, int src, size_t offset) {
  const size_t n = payload_size(v);
  if (physRow < 0 || physRow >= rows_ || src < 0 || src >= peers_ || offset + n > slot_)
    throw ProtocolError("HostSlab::store out of range (src " + std::to_string(src) +
                        ", offset " + std::to_string(offset) + ", len " + std::to_string(n) +
                        ", slot " + std::to_string(slot_) + ")");
  if (n == 0) return;
  float* dst = buf_.data() + (static_cast<size_t>(physRow) * peers_ + src) * slot_ + offset;
  if (v->on_device()) {
    std::vector<float> h = v->to_host();
    std::memcpy(dst, h.data(), n * sizeof(float));
  } else {
    std::memcpy(dst, v->data(), n * sizeof(float));
  }
}

Payload HostSlab::reduce(int physRow, size_t offset, size_t len) {
  std::vector<float> out(len, 0.f);
  if (offset + len > slot_) throw ProtocolError("HostSlab::reduce out of range");
  for (int i = 0; i < peers_; ++i) {
    const float* s = row_ptr(physRow, i) + offset;
    for (size_t j = 0; j < len; ++j) out[j] += s[j];
  }
  return make_host_payload(std::move(out));
}

Payload HostSlab::flush(int physRow, size_t n) {
  std::vector<float> out(n, 0.f);
  size_t transferred = 0;
  for (int i = 0; i < peers_ && transferred < n; ++i) {
    const size_t c = std::min(n - transferred, slot_);
    std::memcpy(out.data() + transferred, row_ptr(physRow, i), c * sizeof(float));
    transferred += c;
  }
  return make_host_payload(std::move(out));
}

void HostSlab::clear_row(int physRow) {
  auto b = buf_.begin() + static_cast<size_t>(physRow) * peers_ * slot_;
  std::fill(b, b + static_cast<size_t>(peers_) * slot_, 0.f);
}

Payload HostPlane::slice(const Payload& p, size_t start, size_t len) {
  if (start + len > payload_size(p)) throw ProtocolError("HostPlane::slice out of range");
  if (p->on_device()) {
    std::vector<float> h = p->to_host();
    return make_host_payload(std::vector<float>(h.begin() + start, h.begin() + start + len));
  }
  const float* d = p->data();
  return make_host_payload(std::vector<float>(d + start, d + start + len));
}

std::shared_ptr<HostPlane> HostPlane::instance() {
  static std::shared_ptr<HostPlane> inst = std::make_shared<HostPlane>();
  return inst;
}

// ---------------------------------------------------------------------------------
void DataBuffer::store(const Payload& v, int row, int src, int chunk) {
  // DataBuffer.store: arraycopy into slot[src] at chunk*C, then count += 1
  const int phys = counters.phys(row);
  slab->store(v, phys, src, static_cast<size_t>(chunk) * maxChunkSize);
  counters.add(row, chunk);
}

size_t DataBuffer::chunk_len(int chunk) const {
  const int64_t endPos = std::min<int64_t>(dataSize, int64_t(chunk + 1) * maxChunkSize);
  const int64_t len = endPos - int64_t(chunk) * maxChunkSize;
  return len > 0 ? static_cast<size_t>(len) : 0;
}

void DataBuffer::up() {
  const int recycled = counters.up();
  slab->clear_row(recycled);
}

}  // namespace mxar
