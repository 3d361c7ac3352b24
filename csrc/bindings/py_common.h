// Shared helpers for the Python bindings: payload <-> numpy conversion, message
// <-> Python object conversion, and GIL-safe holders for Python callables.
#pragma once

#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <mutex>
#include <optional>

#include "../core/protocol.h"
#include "../runtime/allreduce_actors.h"

namespace py = pybind11;

namespace mxar {

// A Python callable that may be destroyed from a non-Python thread.
struct PyCallable {
  py::object fn;
  explicit PyCallable(py::object f) : fn(std::move(f)) {}
  ~PyCallable() {
    if (!Py_IsInitialized()) {
      fn.release();  // interpreter gone: leak rather than crash
      return;
    }
    py::gil_scoped_acquire g;
    fn = py::object();
  }
};

Payload payload_from_py(const py::handle& obj);
py::object payload_to_py(const Payload& p);
py::object message_to_py(const Message& m);
Message message_from_py(const py::handle& obj);

// Hook so the HIP part of the module can turn device payloads into torch tensors
// (DLPack) and accept torch CUDA tensors as payloads.
using DevicePayloadToPy = py::object (*)(const Payload&);
using PyToDevicePayload = Payload (*)(const py::handle&);  // returns nullptr if not a device tensor
void register_device_payload_hooks(DevicePayloadToPy to_py, PyToDevicePayload from_py);
// Plane workers: a device tensor of ANY supported dtype (float32 / bfloat16 / float16),
// zero-copy, ordered after its producer by an event on torch's current stream (no host
// synchronisation). nullptr if `obj` is not a device tensor.
void register_typed_payload_hook(PyToDevicePayload from_py);
Payload typed_payload_from_py(const py::handle& obj);

// dataSource / dataSink that run without Python: plane_worker() takes them as they are, so a
// round's fetch and flush take no GIL (hip.tensor_source: a persistent device buffer;
// last_output_sink: keeps the newest AllReduceOutput for the caller to read).
struct NativeSource {
  DataSource fn;
};
struct LastOutput {
  std::mutex mu;
  std::optional<AllReduceOutput> out;
  uint64_t rounds = 0;
  // record = true: every round's (iteration, steady-clock seconds at the sink) and its
  // per-chunk counts folded into totals (the straggler bench's per-worker round period and
  // mean count, without Python on the round path)
  bool record = false;
  std::vector<std::pair<int, double>> stamps;
  uint64_t count_sum = 0, count_n = 0, count_zero = 0;
};
struct NativeSink {
  DataSink fn;
  std::shared_ptr<LastOutput> keep;
};

}  // namespace mxar
