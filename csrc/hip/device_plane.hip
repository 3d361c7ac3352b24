// DevicePlane implementation (see device_plane.h).
#include "device_plane.h"

#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>

#include "xgmi_comm.h"

namespace mxar {

// ------------------------------------------------------------------ events
ReadyEvent record_ready(hipStream_t s) {
  hipEvent_t e = nullptr;
  hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  hip_check(hipEventRecord(e, s), "hipEventRecord");
  return ReadyEvent(static_cast<void*>(e), [](void* p) { (void)hipEventDestroy(static_cast<hipEvent_t>(p)); });
}

void DevicePayload::wait_host() const {
  if (ready_)
    hip_check(hipEventSynchronize(static_cast<hipEvent_t>(ready_.get())), "hipEventSynchronize");
  else if (stream_)
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

std::vector<float> DevicePayload::to_host() const {
  std::vector<float> h(n_);
  if (n_ == 0) return h;
  wait_host();
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (dtype_ == 0) {
    hip_check(hipMemcpy(h.data(), data(), n_ * sizeof(float), hipMemcpyDeviceToHost), "hipMemcpy D2H");
    return h;
  }
  std::vector<uint16_t> raw(n_);
  hip_check(hipMemcpy(raw.data(), bytes(), n_ * 2, hipMemcpyDeviceToHost), "hipMemcpy D2H");
  for (size_t i = 0; i < n_; ++i) {
    if (dtype_ == 1) {  // bfloat16: the high half of a float32
      const uint32_t b = static_cast<uint32_t>(raw[i]) << 16;
      std::memcpy(&h[i], &b, 4);
    } else {  // float16
      h[i] = static_cast<float>(__builtin_bit_cast(_Float16, raw[i]));
    }
  }
  return h;
}

// ------------------------------------------------------------------ pool
static size_t size_class(size_t bytes) {
  size_t c = 256;
  while (c < bytes) c <<= 1;
  return c;
}

DevicePool::~DevicePool() {
  *alive_ = false;
  std::lock_guard<std::mutex> g(mu_);
  (void)hipSetDevice(device_);
  for (auto& [cls, v] : free_)
    for (void* p : v) (void)hipFree(p);
  free_.clear();
}

std::shared_ptr<void> DevicePool::get(size_t bytes) {
  const size_t cls = size_class(std::max<size_t>(bytes, 1));
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = free_.find(cls);
    if (it != free_.end() && !it->second.empty()) {
      p = it->second.back();
      it->second.pop_back();
      cached_ -= cls;
    }
  }
  if (!p) {
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipMalloc(&p, cls), "hipMalloc(pool)");
  }
  std::weak_ptr<bool> alive = alive_;
  DevicePool* self = this;
  return std::shared_ptr<void>(p, [self, alive, cls](void* q) {
    auto a = alive.lock();
    if (a && *a)
      self->put(q, cls);
    else
      (void)hipFree(q);
  });
}

void DevicePool::put(void* p, size_t cls) {
  std::lock_guard<std::mutex> g(mu_);
  free_[cls].push_back(p);
  cached_ += cls;
}

size_t DevicePool::cached_bytes() {
  std::lock_guard<std::mutex> g(mu_);
  return cached_;
}

// ------------------------------------------------------------------ plane
DevicePlane::DevicePlane(int device) : device_(device), pool_(device) {
  hip_check(hipSetDevice(device_), "hipSetDevice");
  // A blocking stream: it is implicitly ordered with the legacy default stream, which is
  // where torch code that hands tensors to sources/sinks runs by default.
  hip_check(hipStreamCreate(&stream_), "hipStreamCreate");
}

DevicePlane::~DevicePlane() {
  (void)hipSetDevice(device_);
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    {
      std::lock_guard<std::mutex> g(pending_mu_);
      pending_.clear();
    }
    (void)hipStreamDestroy(stream_);
  }
}

void DevicePlane::synchronize() {
  hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  prune();
}

void DevicePlane::prune() {
  std::lock_guard<std::mutex> g(pending_mu_);
  size_t k = 0;
  for (auto& e : pending_)
    if (hipEventQuery(static_cast<hipEvent_t>(e.second.get())) != hipSuccess) pending_[k++] = std::move(e);
  pending_.resize(k);
}

void DevicePlane::wait_for(const Payload& p) {
  auto* d = dynamic_cast<const DevicePayload*>(p.get());
  if (!d || d->stream() == stream_ || !d->ready()) return;
  hip_check(hipStreamWaitEvent(stream_, static_cast<hipEvent_t>(d->ready().get()), 0), "hipStreamWaitEvent");
}

void DevicePlane::hold(const Payload& p) {
  auto* d = dynamic_cast<const DevicePayload*>(p.get());
  if (d && d->stream() == stream_) return;  // own memory is stream-ordered already
  // host payloads too: an asynchronous H2D copy reads them after this call returns
  ReadyEvent e = record_ready(stream_);
  std::lock_guard<std::mutex> g(pending_mu_);
  pending_.emplace_back(p, std::move(e));
  if (pending_.size() > 256) {
    size_t k = 0;
    for (auto& x : pending_)
      if (hipEventQuery(static_cast<hipEvent_t>(x.second.get())) != hipSuccess) pending_[k++] = std::move(x);
    pending_.resize(k);
  }
}

Payload DevicePlane::alloc(size_t n) {
  return std::make_shared<DevicePayload>(pool_.get(n * sizeof(float)), 0, n, device_, stream_);
}

Payload DevicePlane::zeros(size_t n) {
  auto mem = pool_.get(n * sizeof(float));
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (n) hip_check(hipMemsetAsync(mem.get(), 0, n * sizeof(float), stream_), "hipMemsetAsync");
  return std::make_shared<DevicePayload>(std::move(mem), 0, n, device_, stream_, record_ready(stream_));
}

Payload DevicePlane::to_device(const Payload& p) {
  if (!p) return zeros(0);
  auto* d = dynamic_cast<const DevicePayload*>(p.get());
  if (d && d->device() == device_) return p;
  const size_t n = p->size();
  auto mem = pool_.get(n * sizeof(float));
  hip_check(hipSetDevice(device_), "hipSetDevice");
  if (n) {
    if (p->on_device()) {  // another device: peer copy
      wait_for(p);
      hip_check(hipMemcpyAsync(mem.get(), p->data(), n * sizeof(float), hipMemcpyDefault, stream_), "hipMemcpyAsync");
      hold(p);
      d2d_bytes += n * sizeof(float);
    } else {
      // host payloads are immutable: keep this one alive until the stream has copied it
      // instead of draining the stream (the old per-store hipStreamSynchronize)
      hip_check(hipMemcpyAsync(mem.get(), p->data(), n * sizeof(float), hipMemcpyHostToDevice, stream_),
                "hipMemcpyAsync H2D");
      hold(p);
      h2d_bytes += n * sizeof(float);
    }
  }
  return std::make_shared<DevicePayload>(std::move(mem), 0, n, device_, stream_, record_ready(stream_));
}

Payload DevicePlane::adopt(Payload p) { return to_device(p); }

Payload DevicePlane::slice(const Payload& p, size_t start, size_t len) {
  if (start + len > payload_size(p)) throw ProtocolError("DevicePlane::slice out of range");
  Payload dp = to_device(p);
  auto* d = static_cast<const DevicePayload*>(dp.get());
  return std::make_shared<DevicePayload>(d->memory(), d->offset() + start, len, d->device(), d->stream(),
                                         d->ready());
}

std::unique_ptr<Slab> DevicePlane::make_slab(int rows, int peers, size_t slotSize) {
  return std::make_unique<DeviceSlab>(this, rows, peers, slotSize);
}

std::shared_ptr<DevicePlane> make_device_plane(int device) { return std::make_shared<DevicePlane>(device); }

// ------------------------------------------------------------------ slab
DeviceSlab::DeviceSlab(DevicePlane* plane, int rows, int peers, size_t slot) : plane_(plane) {
  rows_ = rows;
  peers_ = peers;
  slot_ = slot;
  const size_t bytes = static_cast<size_t>(rows) * peers * slot * sizeof(float);
  hip_check(hipSetDevice(plane->device()), "hipSetDevice");
  void* p = nullptr;
  hip_check(hipMalloc(&p, std::max<size_t>(bytes, 16)), "hipMalloc(slab)");
  mem_ = std::shared_ptr<void>(p, [](void* q) { (void)hipFree(q); });
  if (bytes) hip_check(hipMemsetAsync(p, 0, bytes, plane->stream()), "hipMemsetAsync(slab)");
}

void DeviceSlab::store(const Payload& v, int physRow, int src, size_t offset) {
  const size_t n = payload_size(v);
  if (physRow < 0 || physRow >= rows_ || src < 0 || src >= peers_ || offset + n > slot_)
    throw ProtocolError("DeviceSlab::store out of range (src " + std::to_string(src) + ", offset " +
                        std::to_string(offset) + ", len " + std::to_string(n) + ", slot " + std::to_string(slot_) +
                        ")");
  if (n == 0) return;
  float* dst = row_ptr(physRow, src) + offset;
  hip_check(hipSetDevice(plane_->device()), "hipSetDevice");
  if (v->on_device()) {
    plane_->wait_for(v);
    hip_check(hipMemcpyAsync(dst, v->data(), n * sizeof(float), hipMemcpyDefault, plane_->stream()),
              "hipMemcpyAsync(store)");
    plane_->hold(v);
    plane_->d2d_bytes += n * sizeof(float);
  } else {
    hip_check(hipMemcpyAsync(dst, v->data(), n * sizeof(float), hipMemcpyHostToDevice, plane_->stream()),
              "hipMemcpyAsync(store H2D)");
    plane_->hold(v);  // immutable host payload, alive until the copy ran (no stream drain)
    plane_->h2d_bytes += n * sizeof(float);
  }
}

Payload DeviceSlab::reduce(int physRow, size_t offset, size_t len) {
  if (offset + len > slot_) throw ProtocolError("DeviceSlab::reduce out of range");
  Payload out = plane_->alloc(len);
  hip_check(hipSetDevice(plane_->device()), "hipSetDevice");
  const float* base = row_ptr(physRow, 0) + offset;
  // K1: fp32 sum over the P peer slots in peer order 0..P-1 (bit-identical to the host loop).
  if (((reinterpret_cast<uintptr_t>(base) | (slot_ * sizeof(float))) & 15) == 0) {
    launch_reduce_slots(base, static_cast<int64_t>(slot_), peers_, const_cast<float*>(out->data()),
                        static_cast<int64_t>(len), DType::F32, 1.f, plane_->stream());
  } else {
    // unaligned chunk start: stage the P rows at an aligned pitch, then reduce
    const size_t ld = (len + 3) / 4 * 4;
    Payload stage = plane_->alloc(ld * peers_);
    for (int i = 0; i < peers_; ++i)
      hip_check(hipMemcpyAsync(const_cast<float*>(stage->data()) + i * ld, row_ptr(physRow, i) + offset,
                               len * sizeof(float), hipMemcpyDeviceToDevice, plane_->stream()),
                "hipMemcpyAsync(stage)");
    launch_reduce_slots(stage->data(), static_cast<int64_t>(ld), peers_, const_cast<float*>(out->data()),
                        static_cast<int64_t>(len), DType::F32, 1.f, plane_->stream());
    plane_->hold(stage);
  }
  ++plane_->kernels;
  auto* d = static_cast<const DevicePayload*>(out.get());
  return std::make_shared<DevicePayload>(d->memory(), 0, len, plane_->device(), plane_->stream(),
                                         record_ready(plane_->stream()));
}

Payload DeviceSlab::flush(int physRow, size_t n) {
  // the P reduce slots of a row are contiguous ([peer][slot]), so the concatenation
  // truncated to n is one copy of the row's first n floats
  Payload out = plane_->alloc(n);
  hip_check(hipSetDevice(plane_->device()), "hipSetDevice");
  if (n) {
    const size_t avail = static_cast<size_t>(peers_) * slot_;
    const size_t c = std::min(n, avail);
    hip_check(hipMemcpyAsync(const_cast<float*>(out->data()), row_ptr(physRow, 0), c * sizeof(float),
                             hipMemcpyDeviceToDevice, plane_->stream()),
              "hipMemcpyAsync(flush)");
    if (c < n)
      hip_check(hipMemsetAsync(const_cast<float*>(out->data()) + c, 0, (n - c) * sizeof(float), plane_->stream()),
                "hipMemsetAsync(flush tail)");
  }
  auto* d = static_cast<const DevicePayload*>(out.get());
  return std::make_shared<DevicePayload>(d->memory(), 0, n, plane_->device(), plane_->stream(),
                                         record_ready(plane_->stream()));
}

void DeviceSlab::clear_row(int physRow) {
  hip_check(hipSetDevice(plane_->device()), "hipSetDevice");
  hip_check(hipMemsetAsync(row_ptr(physRow, 0), 0, static_cast<size_t>(peers_) * slot_ * sizeof(float),
                           plane_->stream()),
            "hipMemsetAsync(clear_row)");
}

}  // namespace mxar
