// DevicePlane: the worker protocol's data (DataBuffer slabs, message payloads, input and
// output vectors) resident in MI355X HBM. Reference data paths it replaces:
//   DataBuffer.store / get / up      (buffer/DataBuffer.scala:35-67)  -> DeviceSlab (copy
//                                     into [row][peer][slot] HBM, hipMemsetAsync rotation)
//   AllreduceWorker.reduce           (AllreduceWorker.scala:240-251)  -> reduce_slots kernel
//   getDataBlock / chunk slicing     (:200-204, :216-221)            -> zero-copy views
//   flush                            (:180-192)                      -> one device copy
// Every operation of a plane is ordered on the plane's own HIP stream; payload memory
// comes from a per-device caching pool (no hipMalloc on the message path). Payloads are
// handed to Python as torch tensors through DLPack (zero copy) and torch tensors are
// accepted as payloads through `__dlpack__` (zero copy, ordered on the plane stream).
#pragma once

#include <hip/hip_runtime_api.h>

#include <map>
#include <atomic>
#include <memory>
#include <mutex>
#include <vector>

#include "../core/data_buffer.h"

namespace mxar {

class DevicePool {
 public:
  explicit DevicePool(int device) : device_(device) {}
  ~DevicePool();
  // Returns a block of at least `bytes` (rounded to a power-of-two class >= 256 B).
  std::shared_ptr<void> get(size_t bytes);
  size_t cached_bytes();
  int device() const { return device_; }

 private:
  void put(void* p, size_t cls);
  int device_;
  std::mutex mu_;
  std::map<size_t, std::vector<void*>> free_;
  size_t cached_ = 0;
  std::shared_ptr<bool> alive_ = std::make_shared<bool>(true);
};

// Completion marker of the operation that produced a payload (a hipEvent recorded on the
// producing stream). Consumers on other streams wait on it; views share it.
using ReadyEvent = std::shared_ptr<void>;
ReadyEvent record_ready(hipStream_t s);

// Device payload: a float view [offset, offset + n) of a refcounted device allocation.
class DevicePayload final : public PayloadStorage {
 public:
  // offset and n in elements of `dtype` (0 = float32, 1 = bfloat16, 2 = float16)
  DevicePayload(std::shared_ptr<void> mem, size_t offset, size_t n, int device, hipStream_t stream,
                ReadyEvent ready = nullptr, int dtype = 0)
      : mem_(std::move(mem)), off_(offset), n_(n), device_(device), stream_(stream), ready_(std::move(ready)),
        dtype_(dtype) {}
  bool on_device() const override { return true; }
  // first element (typed as float for the protocol's float32 payloads; see dtype())
  const float* data() const override {
    return reinterpret_cast<const float*>(static_cast<const char*>(mem_.get()) + off_ * elem_bytes());
  }
  const void* bytes() const { return static_cast<const char*>(mem_.get()) + off_ * elem_bytes(); }
  size_t size() const override { return n_; }
  int dtype() const override { return dtype_; }
  size_t elem_bytes() const { return dtype_ == 0 ? 4 : 2; }
  std::vector<float> to_host() const override;
  int device() const { return device_; }
  const std::shared_ptr<void>& memory() const { return mem_; }
  size_t offset() const { return off_; }
  hipStream_t stream() const { return stream_; }
  const ReadyEvent& ready() const { return ready_; }
  // Block the host until the producing operation finished.
  void wait_host() const;
  // Pooled round outputs (xgmi_plane.cc): a buffer whose memory was handed to another stream
  // (a torch tensor view, or a native consumer enqueuing GPU work on its own stream) is
  // returned to the pool only behind the default stream; one never exported is reused at
  // once on the producer's stream. to_py marks it; native consumers call mark_exported().
  void set_export_flag(std::shared_ptr<std::atomic<bool>> f) { exported_ = std::move(f); }
  void mark_exported() const {
    if (exported_) exported_->store(true, std::memory_order_relaxed);
  }

 private:
  std::shared_ptr<std::atomic<bool>> exported_;
  std::shared_ptr<void> mem_;
  size_t off_, n_;
  int device_;
  hipStream_t stream_;
  ReadyEvent ready_;
  int dtype_ = 0;
};

class DevicePlane;

class DeviceSlab final : public Slab {
 public:
  DeviceSlab(DevicePlane* plane, int rows, int peers, size_t slot);
  void store(const Payload& v, int physRow, int src, size_t offset) override;
  Payload reduce(int physRow, size_t offset, size_t len) override;
  Payload flush(int physRow, size_t n) override;
  void clear_row(int physRow) override;

 private:
  float* row_ptr(int physRow, int src) const {
    return static_cast<float*>(mem_.get()) + (static_cast<size_t>(physRow) * peers_ + src) * slot_;
  }
  DevicePlane* plane_;
  std::shared_ptr<void> mem_;
};

class DevicePlane final : public DataPlane, public std::enable_shared_from_this<DevicePlane> {
 public:
  explicit DevicePlane(int device);
  ~DevicePlane() override;
  const char* name() const override { return "device"; }
  std::unique_ptr<Slab> make_slab(int rows, int peers, size_t slotSize) override;
  Payload slice(const Payload& p, size_t start, size_t len) override;
  Payload zeros(size_t n) override;
  Payload adopt(Payload p) override;

  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  DevicePool& pool() { return pool_; }
  Payload alloc(size_t n);
  // Host or device payload -> device payload owned by this plane (copy if needed).
  Payload to_device(const Payload& p);
  void synchronize();
  // Order this plane's stream after the producer of `p` (no-op for own / host payloads).
  void wait_for(const Payload& p);
  // Keep `p` alive until the work just enqueued on this stream has finished with it.
  void hold(const Payload& p);
  // bytes moved host->device / device->device through this plane, kernel launches
  uint64_t h2d_bytes = 0, d2d_bytes = 0, kernels = 0;

 private:
  void prune();
  int device_;
  hipStream_t stream_ = nullptr;
  DevicePool pool_;
  std::mutex pending_mu_;
  std::vector<std::pair<Payload, ReadyEvent>> pending_;
};

std::shared_ptr<DevicePlane> make_device_plane(int device);

}  // namespace mxar
