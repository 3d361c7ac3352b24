// Python bindings of the HIP data plane. Device buffers cross the boundary as raw
// addresses (torch `tensor.data_ptr()`) and streams as `torch.cuda.Stream.cuda_stream`,
// so the native module does not link against libtorch; torch is imported first and its
// bundled libamdhip64 (same SONAME) is the one HIP runtime of the process.
#include "../core/delay.h"
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>
#include <vector>

#include "../bindings/py_common.h"
#include "device_plane.h"
#include "sdma_comm.h"
#include "xgmi_comm.h"
#include "xgmi_plane.h"
#include "residency.h"

namespace py = pybind11;

namespace mxar {

// ---------------------------------------------------------------------------------
// DLPack (ABI v0, "dltensor" capsules): zero-copy device payload <-> torch tensor
// ---------------------------------------------------------------------------------
namespace {
struct DLDevice {
  int32_t device_type;
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLFloat = 2;
constexpr uint8_t kDLBfloat = 4;

struct ExportCtx {
  Payload keep;
  int64_t shape[1];
  int64_t strides[1];
};

void export_deleter(DLManagedTensor* m) {
  delete static_cast<ExportCtx*>(m->manager_ctx);  // drops the payload ref (C++ only: no GIL)
  delete m;
}

void capsule_destructor(PyObject* cap) {
  if (PyCapsule_IsValid(cap, "dltensor")) {  // never consumed
    auto* m = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap, "dltensor"));
    if (m && m->deleter) m->deleter(m);
  }
}

py::object device_payload_to_py(const Payload& p) {
  auto* d = dynamic_cast<const DevicePayload*>(p.get());
  if (!d) return py::none();
  d->wait_host();  // torch consumes it on its own stream
  d->mark_exported();  // a pooled round output returns to its pool behind torch's stream
  auto* ctx = new ExportCtx{p, {static_cast<int64_t>(p->size())}, {1}};
  auto* mt = new DLManagedTensor{};
  mt->dl_tensor.data = const_cast<void*>(d->bytes());
  mt->dl_tensor.device = DLDevice{kDLROCM, d->device()};
  mt->dl_tensor.ndim = 1;
  mt->dl_tensor.dtype = d->dtype() == 1   ? DLDataType{kDLBfloat, 16, 1}
                        : d->dtype() == 2 ? DLDataType{kDLFloat, 16, 1}
                                          : DLDataType{kDLFloat, 32, 1};
  mt->dl_tensor.shape = ctx->shape;
  mt->dl_tensor.strides = ctx->strides;
  mt->dl_tensor.byte_offset = 0;
  mt->manager_ctx = ctx;
  mt->deleter = export_deleter;
  py::capsule cap(mt, "dltensor", capsule_destructor);
  return py::module_::import("torch.utils.dlpack").attr("from_dlpack")(cap);
}

Payload py_to_device_payload(const py::handle& obj) {
  if (!py::hasattr(obj, "__dlpack__") || !py::hasattr(obj, "is_cuda")) return nullptr;
  if (!obj.attr("is_cuda").cast<bool>()) return nullptr;  // CPU tensors take the numpy path
  py::object t = obj.attr("detach")().attr("float")().attr("contiguous")().attr("reshape")(-1);
  // order: the producer ran on torch's current stream; make it complete before the
  // worker's plane stream (a different stream) reads the memory
  py::module_::import("torch.cuda").attr("current_stream")(t.attr("device")).attr("synchronize")();
  py::object cap = t.attr("__dlpack__")();
  auto* mt = static_cast<DLManagedTensor*>(PyCapsule_GetPointer(cap.ptr(), "dltensor"));
  if (!mt) throw py::error_already_set();
  PyCapsule_SetName(cap.ptr(), "used_dltensor");
  const int64_t n = mt->dl_tensor.ndim > 0 ? mt->dl_tensor.shape[0] : 1;
  char* data = static_cast<char*>(mt->dl_tensor.data) + mt->dl_tensor.byte_offset;
  std::shared_ptr<void> mem(data, [mt](void*) {
    if (!mt->deleter) return;
    if (Py_IsInitialized()) {
      py::gil_scoped_acquire g;
      mt->deleter(mt);
    } else {
      mt->deleter(mt);
    }
  });
  return std::make_shared<DevicePayload>(std::move(mem), 0, static_cast<size_t>(n), mt->dl_tensor.device.device_id,
                                         nullptr, nullptr);
}
// Plane-worker inputs: the tensor's own dtype, zero copy (the payload keeps a reference to
// the tensor), ordered after its producer by an event on torch's current stream when that
// stream still has work in flight. This runs once per round on the dataSource path, so the
// torch objects it needs are looked up once.
struct TorchRefs {
  py::object tensor_type, f32, bf16, f16, raw_stream;
};
const TorchRefs& torch_refs() {
  static TorchRefs* r = [] {
    py::module_ torch = py::module_::import("torch");
    auto* t = new TorchRefs{torch.attr("Tensor"), torch.attr("float32"), torch.attr("bfloat16"),
                            torch.attr("float16"), py::none()};
    py::object c = torch.attr("_C");
    if (py::hasattr(c, "_cuda_getCurrentRawStream")) t->raw_stream = c.attr("_cuda_getCurrentRawStream");
    return t;
  }();
  return *r;
}

Payload py_to_device_payload_typed(const py::handle& obj) {
  const TorchRefs& T = torch_refs();
  if (!py::isinstance(obj, T.tensor_type)) return nullptr;
  py::object t = py::reinterpret_borrow<py::object>(obj);
  if (!t.attr("is_cuda").cast<bool>()) return nullptr;
  const py::object dt = t.attr("dtype");
  int code = -1;
  if (dt.is(T.f32)) code = 0;
  else if (dt.is(T.bf16)) code = 1;
  else if (dt.is(T.f16)) code = 2;
  if (code < 0) throw py::type_error("plane input must be float32, bfloat16 or float16");
  if (!t.attr("is_contiguous")().cast<bool>()) t = t.attr("contiguous")();
  const uintptr_t ptr = t.attr("data_ptr")().cast<uintptr_t>();
  const int64_t n = t.attr("numel")().cast<int64_t>();
  const int dev = t.attr("get_device")().cast<int>();
  uintptr_t cs = 0;
  if (!T.raw_stream.is_none())
    cs = T.raw_stream(dev).cast<uintptr_t>();
  else
    cs = py::module_::import("torch").attr("cuda").attr("current_stream")(dev).attr("cuda_stream").cast<uintptr_t>();
  auto* hold = new py::object(std::move(t));  // released with the GIL when the plane drops the input
  std::shared_ptr<void> mem(reinterpret_cast<void*>(ptr), [hold](void*) {
    if (Py_IsInitialized()) {
      py::gil_scoped_acquire g;
      delete hold;
    } else {
      hold->release();
      delete hold;
    }
  });
  // the producer's stream idle: nothing to order after (and no marker that could queue behind
  // another worker's spinning round in a shared hardware queue)
  const hipStream_t ps = reinterpret_cast<hipStream_t>(cs);
  ReadyEvent ready = hipStreamQuery(ps) == hipSuccess ? nullptr : record_ready(ps);
  (void)hipGetLastError();
  return std::make_shared<DevicePayload>(std::move(mem), 0, static_cast<size_t>(n), dev, nullptr, std::move(ready),
                                         code);
}
}  // namespace

// dataSource over one persistent device tensor, without Python per round: each fetch returns
// the same buffer, ordered after the work queued on the stream that was torch's current
// stream at creation (an event only if that stream is busy, as the per-round import does).
// That stream must outlive the source (torch's default / current streams do).
NativeSource tensor_source(py::object obj, double delay_us) {
  const TorchRefs& T = torch_refs();
  if (!py::isinstance(obj, T.tensor_type) || !obj.attr("is_cuda").cast<bool>())
    throw py::type_error("tensor_source needs a GPU tensor");
  if (!obj.attr("is_contiguous")().cast<bool>()) throw py::value_error("tensor_source needs a contiguous tensor");
  const py::object dt = obj.attr("dtype");
  const int code = dt.is(T.f32) ? 0 : dt.is(T.bf16) ? 1 : dt.is(T.f16) ? 2 : -1;
  if (code < 0) throw py::type_error("plane input must be float32, bfloat16 or float16");
  const uintptr_t ptr = obj.attr("data_ptr")().cast<uintptr_t>();
  const size_t n = obj.attr("numel")().cast<size_t>();
  const int dev = obj.attr("get_device")().cast<int>();
  const uintptr_t cs = !T.raw_stream.is_none()
                           ? T.raw_stream(dev).cast<uintptr_t>()
                           : py::module_::import("torch").attr("cuda").attr("current_stream")(dev).attr("cuda_stream").cast<uintptr_t>();
  auto holder = std::make_shared<PyCallable>(obj);  // keeps the tensor alive; released with the GIL
  std::shared_ptr<void> mem(holder, reinterpret_cast<void*>(ptr));
  const hipStream_t ps = reinterpret_cast<hipStream_t>(cs);
  return NativeSource{[mem, n, dev, code, ps, delay_us](const AllReduceInputRequest&) -> AllReduceInput {
    precise_delay_us(delay_us);  // a straggling source (0: none)
    ReadyEvent ready = hipStreamQuery(ps) == hipSuccess ? nullptr : record_ready(ps);
    (void)hipGetLastError();
    return AllReduceInput{std::make_shared<DevicePayload>(mem, 0, n, dev, nullptr, std::move(ready), code)};
  }};
}

static hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
static const void* as_cptr(uintptr_t p) { return reinterpret_cast<const void*>(p); }
static void* as_ptr(uintptr_t p) { return reinterpret_cast<void*>(p); }

void bind_hip(py::module_& m) {
  py::module_ h = m.def_submodule("hip", "HIP/CDNA4 data plane (gfx950)");
  register_device_payload_hooks(&device_payload_to_py, &py_to_device_payload);
  register_typed_payload_hook(&py_to_device_payload_typed);
  h.def("tensor_source", &tensor_source, py::arg("tensor"), py::arg("delay_us") = 0.0,
        "dataSource for a plane worker: the same GPU tensor every round, no Python (GIL) per round; "
        "delay_us: each fetch first waits this long on the worker's thread (a straggler)");

  // the device budget of spinning workgroups (residency.h)
  struct ResidencyToken {
    std::shared_ptr<void> t;
  };
  py::class_<ResidencyToken>(h, "ResidencyToken").def("release", [](ResidencyToken& k) { k.t.reset(); });
  h.def("residency_reserve",
        [](int device, int wgs, const std::string& who) { return ResidencyToken{Residency::get().reserve(device, wgs, who)}; },
        py::arg("device"), py::arg("wgs"), py::arg("who"),
        "reserve spinning workgroups on a device (released with the token); raises with the budget named");
  h.def("residency_state", [](int device) {
    py::dict d;
    d["capacity"] = Residency::get().capacity(device);
    d["used"] = Residency::get().used(device);
    py::list hs;
    for (const ResidencyHolder& x : Residency::get().holders(device)) hs.append(py::make_tuple(x.who, x.wgs));
    d["holders"] = hs;
    return d;
  }, py::arg("device"));

  py::class_<DevicePlane, DataPlane, std::shared_ptr<DevicePlane>>(h, "DevicePlane")
      .def_property_readonly("device", &DevicePlane::device)
      .def("synchronize", [](DevicePlane& p) {
        py::gil_scoped_release r;
        p.synchronize();
      })
      .def_property_readonly("stream", [](DevicePlane& p) { return reinterpret_cast<uintptr_t>(p.stream()); })
      .def_property_readonly("cached_bytes", [](DevicePlane& p) { return p.pool().cached_bytes(); })
      .def_readonly("h2d_bytes", &DevicePlane::h2d_bytes)
      .def_readonly("d2d_bytes", &DevicePlane::d2d_bytes)
      .def_readonly("kernels", &DevicePlane::kernels);
  h.def("device_plane", &make_device_plane, py::arg("device") = 0,
        "DataPlane whose slabs and payloads live in HBM of `device` (worker protocol on the GPU)");

  h.def("shared_launch_rule", &shared_launch_rule, py::arg("ranks_here"), py::arg("default_grid"),
        "workgroups per rank at most when several logical ranks share one default-grid launch (0: no cap)");
  h.def("size_grid_rule", &size_grid_rule, py::arg("bytes"), py::arg("grid"), py::arg("world"), py::arg("oneshot"),
        py::arg("full_at") = int64_t{512} << 20, py::arg("cap") = 256,
        "workgroups a default-grid launch of `bytes` (all ranks of the launch) uses (XgmiComm::launch_grid)");
  py::enum_<DType>(h, "DType").value("F32", DType::F32).value("BF16", DType::BF16).value("F16", DType::F16);

  py::class_<XgmiPlaneStats>(h, "XgmiPlaneStats")
      .def_readonly("launches", &XgmiPlaneStats::launches)
      .def_readonly("cold", &XgmiPlaneStats::cold)
      .def_readonly("forced", &XgmiPlaneStats::forced)
      .def_readonly("bytes", &XgmiPlaneStats::bytes)
      .def_readonly("completed", &XgmiPlaneStats::completed)
      .def_readonly("coarsened", &XgmiPlaneStats::coarsened)
      .def_readonly("pool_grown", &XgmiPlaneStats::pool_grown)
      .def_readonly("resident_pool_misses", &XgmiPlaneStats::resident_pool_misses)
      .def_readonly("resident_rounds", &XgmiPlaneStats::resident_rounds)
      .def_readonly("resident_launches", &XgmiPlaneStats::resident_launches)
      .def_readonly("resident_parks", &XgmiPlaneStats::resident_parks)
      .def_readonly("group_rounds", &XgmiPlaneStats::group_rounds)
      .def_readonly("group_launches", &XgmiPlaneStats::group_launches)
      .def_readonly("group_size", &XgmiPlaneStats::group_size)
      .def_readonly("peer_maps", &XgmiPlaneStats::peer_maps);
  py::class_<XgmiRoundPlane, RoundPlane, std::shared_ptr<XgmiRoundPlane>>(h, "XgmiRoundPlane")
      .def_property_readonly("stats", &XgmiRoundPlane::stats)
      .def("debug_state", &XgmiRoundPlane::debug_state,
           "diagnostics: door / resident / group words, the device go word and control words (JSON)")
      .def_property_readonly("arena_bytes", &XgmiRoundPlane::arena_bytes)
      .def_property_readonly("chunk_elems", &XgmiRoundPlane::chunk_elems)
      .def_property_readonly("block_elems", &XgmiRoundPlane::block_elems)
      .def_property_readonly("device", [](const XgmiRoundPlane& p) { return p.options().device; })
      .def_property_readonly("stream", [](const XgmiRoundPlane& p) { return reinterpret_cast<uintptr_t>(p.stream()); })
      .def(
          "set_phase_stamps",
          [](XgmiRoundPlane& p, uintptr_t buf, int64_t slots) { p.set_phase_stamps(reinterpret_cast<uint64_t*>(buf), slots); },
          py::arg("buf"), py::arg("slots"),
          "per-workgroup phase stamps of this plane's round kernels (kPhaseSlots u64 each; 0 = off)")
      .def("drain", [](XgmiRoundPlane& p) {
        py::gil_scoped_release r;
        p.drain();
      });
  h.def(
      "xgmi_plane",
      [](int device, DType dtype, int64_t capacity, int max_peers, int max_lag, int grid, double timeout_s,
         bool order_ref, bool high_priority, bool order_release, int spin_us, bool split, int64_t min_chunk,
         double lag_wait_us, bool residency_external) {
        XgmiPlaneOptions o;
        o.device = device;
        o.dtype = dtype;
        o.capacity = capacity;
        o.max_peers = max_peers;
        o.max_lag = max_lag;
        o.grid = grid;
        o.timeout_s = timeout_s;
        o.order_ref = order_ref;
        o.high_priority = high_priority;
        o.order_release = order_release;
        o.spin_us = spin_us;
        o.split = split;
        o.min_chunk = min_chunk;
        o.lag_wait_us = lag_wait_us;
        o.residency_external = residency_external;
        py::gil_scoped_release r;
        return make_xgmi_plane(o);
      },
      py::arg("device") = 0, py::arg("dtype") = DType::F32, py::arg("capacity"), py::arg("max_peers") = 8,
      py::arg("max_lag") = 4, py::arg("grid") = 0, py::arg("timeout_s") = 60.0, py::arg("order_ref") = true,
      py::arg("high_priority") = true, py::arg("order_release") = true, py::arg("spin_us") = 1000, py::arg("split") = true,
      py::arg("min_chunk") = 0, py::arg("lag_wait_us") = -1.0, py::arg("residency_external") = false,
      "RoundPlane of the protocol engine on MI355X: an HBM arena exported over IPC, one threshold-kernel launch "
      "per round (csrc/hip/xgmi_plane.h)");
  py::enum_<Algo>(h, "Algo").value("Auto", Algo::Auto).value("TwoShot", Algo::TwoShot).value("OneShot", Algo::OneShot).value("Ring", Algo::Ring).value("LL", Algo::LL).value("RingNative", Algo::RingNative);
  py::enum_<Coll>(h, "Coll")
      .value("AllToAll", Coll::AllToAll)
      .value("AllGather", Coll::AllGather)
      .value("ReduceScatter", Coll::ReduceScatter);

  py::class_<CommStats>(h, "CommStats")
      .def_readonly("calls", &CommStats::calls)
      .def_readonly("launches", &CommStats::launches)
      .def_readonly("bytes", &CommStats::bytes)
      .def_readonly("oneshot", &CommStats::oneshot)
      .def_readonly("twoshot", &CommStats::twoshot)
      .def_readonly("ring", &CommStats::ring)
      .def_readonly("threshold", &CommStats::threshold)
      .def_readonly("ll", &CommStats::ll)
      .def_readonly("coll", &CommStats::coll)
      .def_readonly("adamw", &CommStats::adamw)
      .def_readonly("stream_switches", &CommStats::stream_switches);

  py::class_<AdamW>(h, "AdamW")
      .def(py::init<>())
      .def_readwrite("lr", &AdamW::lr)
      .def_readwrite("beta1", &AdamW::beta1)
      .def_readwrite("beta2", &AdamW::beta2)
      .def_readwrite("eps", &AdamW::eps)
      .def_readwrite("weight_decay", &AdamW::weight_decay)
      .def_readwrite("step", &AdamW::step);

  h.def("sdma_diagnose", &sdma_diagnose, py::arg("device") = 0);
  h.def("sdma_copy_probe", &sdma_copy_probe, py::arg("device"), py::arg("dst"), py::arg("src"), py::arg("bytes"),
        py::arg("engine") = 0, py::arg("iters") = 10, py::arg("nengines") = 1, py::call_guard<py::gil_scoped_release>());
  h.def("pci_location", &pci_location, py::arg("device"));
  py::class_<SdmaComm>(h, "SdmaComm")
      .def(py::init<int, int, int, int64_t, int, int, double>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("slot_bytes"), py::arg("grid") = 32, py::arg("engines_per_peer") = 0, py::arg("timeout_s") = 20.0)
      .def("handle", [](const SdmaComm& c) { return py::bytes(c.handle()); })
      .def("connect", [](SdmaComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (auto& b : hs) v.emplace_back(static_cast<std::string>(b));
        c.connect(v);
      })
      .def("connect_local", &SdmaComm::connect_local)
      .def("allreduce",
           [](SdmaComm& c, uintptr_t in, uintptr_t out, int64_t n, DType dt, uintptr_t stream, float scale) {
             py::gil_scoped_release r;
             c.allreduce(reinterpret_cast<const void*>(in), reinterpret_cast<void*>(out), n, dt,
                         reinterpret_cast<hipStream_t>(stream), scale);
           },
           py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("dtype"), py::arg("stream") = 0, py::arg("scale") = 1.0f,
           "out = scale x sum over ranks of inp; cross-rank copies on the SDMA engines (sdma_comm.h)")
      .def_static(
          "allreduce_local",
          [](const std::vector<SdmaComm*>& comms, const std::vector<uintptr_t>& ins, const std::vector<uintptr_t>& outs,
             int64_t n, DType dt, uintptr_t stream, float scale) {
            std::vector<const void*> i(ins.size());
            std::vector<void*> o(outs.size());
            for (size_t k = 0; k < ins.size(); ++k) i[k] = reinterpret_cast<const void*>(ins[k]);
            for (size_t k = 0; k < outs.size(); ++k) o[k] = reinterpret_cast<void*>(outs[k]);
            py::gil_scoped_release r;
            SdmaComm::allreduce_local(comms, i, o, n, dt, reinterpret_cast<hipStream_t>(stream), scale);
          },
          py::arg("comms"), py::arg("inputs"), py::arg("outputs"), py::arg("n"), py::arg("dtype"), py::arg("stream") = 0,
          py::arg("scale") = 1.0f)
      .def("error", &SdmaComm::error)
      .def("clear_error", &SdmaComm::clear_error)
      .def("debug_state", &SdmaComm::debug_state)
      .def_property("grid", &SdmaComm::grid, &SdmaComm::set_grid)
      .def_property("pieces", &SdmaComm::pieces, &SdmaComm::set_pieces,
                    "pipeline pieces per block (0 = one per 64 MiB of the block, 2..8)")
      .def_property_readonly("engines", &SdmaComm::engines)
      .def_property_readonly("engines_per_peer", &SdmaComm::engines_per_peer)
      .def_property_readonly("slot_bytes", &SdmaComm::slot_bytes)
      .def_property_readonly("rank", &SdmaComm::rank)
      .def_property_readonly("world", &SdmaComm::world)
      .def_property_readonly("stats", [](const SdmaComm& c) {
        const SdmaStats& s = c.stats();
        py::dict d;
        d["calls"] = s.calls;
        d["copies"] = s.copies;
        d["bytes"] = s.bytes;
        d["host_waits"] = s.host_waits;
        return d;
      });
  py::class_<XgmiComm>(h, "XgmiComm")
      .def(py::init<int, int, int, int64_t, int, double, int>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("slot_bytes"), py::arg("grid") = 0, py::arg("timeout_s") = 20.0, py::arg("threshold_rows") = 0)
      .def("ipc_handle", [](const XgmiComm& c) { return py::bytes(c.ipc_handle()); })
      .def("connect", [](XgmiComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (auto& b : hs) v.emplace_back(static_cast<std::string>(b));
        c.connect(v);
      })
      .def("connect_local", &XgmiComm::connect_local)
      .def(
          "allreduce",
          [](XgmiComm& c, uintptr_t in, uintptr_t out, int64_t n, DType dt, uintptr_t stream, Algo algo,
             float scale) {
            py::gil_scoped_release r;
            c.allreduce(as_cptr(in), as_ptr(out), n, dt, as_stream(stream), algo, scale);
          },
          py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("dtype"), py::arg("stream") = 0,
          py::arg("algo") = Algo::Auto, py::arg("scale") = 1.0f)
      .def(
          "allreduce_threshold",
          [](XgmiComm& c, uintptr_t in, uintptr_t out, int64_t n, DType dt, uintptr_t stream, float thr, float thc,
             uintptr_t counts, float scale, bool rescale) {
            py::gil_scoped_release r;
            c.allreduce_threshold(as_cptr(in), as_ptr(out), n, dt, as_stream(stream), thr, thc,
                                  reinterpret_cast<int32_t*>(counts), scale, rescale);
          },
          py::arg("inp"), py::arg("out"), py::arg("n"), py::arg("dtype"), py::arg("stream") = 0,
          py::arg("th_reduce") = 1.0f, py::arg("th_complete") = 1.0f, py::arg("counts") = 0, py::arg("scale") = 1.0f,
          py::arg("rescale") = false)
      .def_static(
          "allreduce_threshold_local",
          [](const std::vector<XgmiComm*>& comms, const std::vector<uintptr_t>& ins, const std::vector<uintptr_t>& outs,
             int64_t n, DType dt, uintptr_t stream, float thr, float thc, uintptr_t counts, float scale,
             bool rescale) {
            std::vector<const void*> i;
            std::vector<void*> o;
            for (auto p : ins) i.push_back(as_cptr(p));
            for (auto p : outs) o.push_back(as_ptr(p));
            py::gil_scoped_release r;
            XgmiComm::allreduce_threshold_local(comms, i, o, n, dt, as_stream(stream), thr, thc,
                                                reinterpret_cast<int32_t*>(counts), scale, rescale);
          },
          py::arg("comms"), py::arg("inputs"), py::arg("outputs"), py::arg("n"), py::arg("dtype"),
          py::arg("stream") = 0, py::arg("th_reduce") = 1.0f, py::arg("th_complete") = 1.0f, py::arg("counts") = 0,
          py::arg("scale") = 1.0f, py::arg("rescale") = false)
      .def("resolve", &XgmiComm::resolve, py::arg("n"), py::arg("dtype"), py::arg("algo") = Algo::Auto,
           py::arg("ranks_in_launch") = 1, "the kernel a call of `algo` over n elements runs (Auto resolved)")
      .def("threshold_chunks", &XgmiComm::threshold_chunks, py::arg("n"), py::arg("dtype"),
           py::arg("ranks_in_launch") = 1)
      .def("set_straggler", &XgmiComm::set_straggler, py::arg("rank"), py::arg("us"))
      .def("set_read_delay", &XgmiComm::set_read_delay, py::arg("rank"), py::arg("us"))
      .def("set_forward_delay", &XgmiComm::set_forward_delay, py::arg("rank"), py::arg("us"))
      .def_property_readonly("threshold_rows", &XgmiComm::threshold_rows)
      .def_property_readonly("slab_address", &XgmiComm::slab_address)
      .def_property("size_grid", &XgmiComm::size_grid, &XgmiComm::set_size_grid)
      .def(
          "barrier",
          [](XgmiComm& c, uintptr_t stream) {
            py::gil_scoped_release r;
            c.barrier(as_stream(stream));
          },
          py::arg("stream") = 0)
      .def_static(
          "allreduce_local",
          [](const std::vector<XgmiComm*>& comms, const std::vector<uintptr_t>& ins, const std::vector<uintptr_t>& outs,
             int64_t n, DType dt, uintptr_t stream, Algo algo, float scale) {
            std::vector<const void*> i;
            std::vector<void*> o;
            for (auto p : ins) i.push_back(as_cptr(p));
            for (auto p : outs) o.push_back(as_ptr(p));
            py::gil_scoped_release r;
            XgmiComm::allreduce_local(comms, i, o, n, dt, as_stream(stream), algo, scale);
          },
          py::arg("comms"), py::arg("inputs"), py::arg("outputs"), py::arg("n"), py::arg("dtype"),
          py::arg("stream") = 0, py::arg("algo") = Algo::Auto, py::arg("scale") = 1.0f)
      .def(
          "step_adamw",
          [](XgmiComm& c, uintptr_t grads, uintptr_t params, int64_t n, DType dt, uintptr_t stream, uintptr_t mp,
             uintptr_t m1, uintptr_t m2, const AdamW& hp, float scale) {
            AdamShard st{reinterpret_cast<float*>(mp), reinterpret_cast<float*>(m1), reinterpret_cast<float*>(m2)};
            py::gil_scoped_release r;
            c.step_adamw(as_cptr(grads), as_ptr(params), n, dt, as_stream(stream), st, hp, scale);
          },
          py::arg("grads"), py::arg("params"), py::arg("n"), py::arg("dtype"), py::arg("stream"), py::arg("master"),
          py::arg("exp_avg"), py::arg("exp_avg_sq"), py::arg("hyper"), py::arg("scale") = 1.0f)
      .def_static(
          "step_adamw_local",
          [](const std::vector<XgmiComm*>& comms, const std::vector<uintptr_t>& grads,
             const std::vector<uintptr_t>& params, int64_t n, DType dt, uintptr_t stream,
             const std::vector<std::tuple<uintptr_t, uintptr_t, uintptr_t>>& states, const AdamW& hp, float scale) {
            std::vector<const void*> g;
            std::vector<void*> p;
            std::vector<AdamShard> st;
            for (auto x : grads) g.push_back(as_cptr(x));
            for (auto x : params) p.push_back(as_ptr(x));
            for (auto& [a, b, c] : states)
              st.push_back({reinterpret_cast<float*>(a), reinterpret_cast<float*>(b), reinterpret_cast<float*>(c)});
            py::gil_scoped_release r;
            XgmiComm::step_adamw_local(comms, g, p, n, dt, as_stream(stream), st, hp, scale);
          },
          py::arg("comms"), py::arg("grads"), py::arg("params"), py::arg("n"), py::arg("dtype"), py::arg("stream"),
          py::arg("states"), py::arg("hyper"), py::arg("scale") = 1.0f)
      .def("block_elems", &XgmiComm::block_elems, py::arg("n"), py::arg("dtype"))
      .def(
          "collective",
          [](XgmiComm& c, Coll op, uintptr_t in, uintptr_t out, int64_t m, DType dt, uintptr_t stream, float scale) {
            py::gil_scoped_release r;
            c.collective(op, as_cptr(in), as_ptr(out), m, dt, as_stream(stream), scale);
          },
          py::arg("op"), py::arg("inp"), py::arg("out"), py::arg("m"), py::arg("dtype"), py::arg("stream") = 0,
          py::arg("scale") = 1.0f)
      .def_static(
          "collective_local",
          [](const std::vector<XgmiComm*>& comms, Coll op, const std::vector<uintptr_t>& ins,
             const std::vector<uintptr_t>& outs, int64_t m, DType dt, uintptr_t stream, float scale) {
            std::vector<const void*> i;
            std::vector<void*> o;
            for (auto p : ins) i.push_back(as_cptr(p));
            for (auto p : outs) o.push_back(as_ptr(p));
            py::gil_scoped_release r;
            XgmiComm::collective_local(comms, op, i, o, m, dt, as_stream(stream), scale);
          },
          py::arg("comms"), py::arg("op"), py::arg("inputs"), py::arg("outputs"), py::arg("m"), py::arg("dtype"),
          py::arg("stream") = 0, py::arg("scale") = 1.0f)
      .def_static(
          "barrier_local",
          [](const std::vector<XgmiComm*>& comms, uintptr_t stream) {
            py::gil_scoped_release r;
            XgmiComm::barrier_group(comms, as_stream(stream));
          },
          py::arg("comms"), py::arg("stream") = 0)
      .def_property_readonly("probe_max_bytes", &XgmiComm::probe_max_bytes)
      .def(
          "probe_push",
          [](XgmiComm& c, uintptr_t src, int64_t bytes, uint32_t mask, int grid, uintptr_t stream, int mode) {
            py::gil_scoped_release r;
            c.probe_push(as_cptr(src), bytes, mask, grid, as_stream(stream), mode);
          },
          py::arg("src"), py::arg("bytes"), py::arg("peer_mask"), py::arg("grid"), py::arg("stream") = 0,
          py::arg("mode") = 0,
          "bring-up probe (no flags), every peer in peer_mask: mode 0 write-through push into its S slot, 1 plain "
          "stores into its coarse-grained probe buffer + a system release, 2 pull (remote loads of its S slot)")
      .def("probe_coarse_handle", [](XgmiComm& c) { return py::bytes(c.probe_coarse_handle()); })
      .def("probe_coarse_connect", [](XgmiComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (auto& b : hs) v.emplace_back(static_cast<std::string>(b));
        c.probe_coarse_connect(v);
      })
      .def(
          "probe_pingpong",
          [](XgmiComm& c, int peer, int iters, uint32_t nonce, bool fenced, uintptr_t out, uintptr_t stream) {
            py::gil_scoped_release r;
            c.probe_pingpong(peer, iters, nonce, fenced, reinterpret_cast<uint64_t*>(out), as_stream(stream));
          },
          py::arg("peer"), py::arg("iters"), py::arg("nonce"), py::arg("fenced"), py::arg("out"),
          py::arg("stream") = 0, "bring-up probe: flag round trips with peer; the leader writes ticks to out[0]")
      .def("error", &XgmiComm::error)
      .def("ctl_words", &XgmiComm::ctl_words)
      .def("clear_error", &XgmiComm::clear_error)
      .def("reset_local", [](XgmiComm& c) {
        py::gil_scoped_release r;
        c.reset_local();
      })
      .def("arm_solo_rehearsal", [](XgmiComm& c) {
        py::gil_scoped_release r;
        c.arm_solo_rehearsal();
      }, "one-rank traffic rehearsal only: peers' flags into this slab read as reached (xgmi_comm.h)")
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("world", &XgmiComm::world)
      .def_property_readonly("device", &XgmiComm::device)
      .def_property("grid", &XgmiComm::grid, &XgmiComm::set_grid)
      .def_property("oneshot_max_bytes", &XgmiComm::oneshot_max_bytes, &XgmiComm::set_oneshot_max_bytes)
      .def_property("ll_auto_max_bytes", &XgmiComm::ll_auto_max_bytes, &XgmiComm::set_ll_auto_max_bytes)
      .def_property_readonly("ll_max_bytes", &XgmiComm::ll_max_bytes)
      .def_property_readonly("slot_bytes", &XgmiComm::slot_bytes)
      .def_property_readonly("slab_bytes", &XgmiComm::slab_bytes)
      .def_property_readonly("alloc_bytes", &XgmiComm::alloc_bytes)
      .def_property_readonly("connected", &XgmiComm::connected)
      .def_property_readonly("stats", &XgmiComm::stats)
      .def_property("fence", &XgmiComm::fence, &XgmiComm::set_fence)
      .def_property("units_per_wg", &XgmiComm::units_per_wg, &XgmiComm::set_units_per_wg)
      .def_property("ring_depth", &XgmiComm::ring_depth, &XgmiComm::set_ring_depth)
      .def("set_timeout", &XgmiComm::set_timeout)
      .def(
          "set_phase_stamps",
          [](XgmiComm& c, uintptr_t buf, int64_t slots) { c.set_phase_stamps(reinterpret_cast<uint64_t*>(buf), slots); },
          py::arg("buf"), py::arg("slots"),
          "study knob: per-workgroup phase stamps of the two-shot / ring kernels (0 = off)");

  h.def(
      "reduce_slots",
      [](uintptr_t slots, int64_t stride, int nslots, uintptr_t out, int64_t n, DType dt, float scale, uintptr_t s) {
        launch_reduce_slots(as_cptr(slots), stride, nslots, as_ptr(out), n, dt, scale, as_stream(s));
      },
      py::arg("slots"), py::arg("slot_stride"), py::arg("nslots"), py::arg("out"), py::arg("n"), py::arg("dtype"),
      py::arg("scale") = 1.0f, py::arg("stream") = 0);
  h.def(
      "fill_iota",
      [](uintptr_t dst, int64_t n, double off, DType dt, uintptr_t s) {
        launch_fill_iota(as_ptr(dst), n, off, dt, as_stream(s));
      },
      py::arg("dst"), py::arg("n"), py::arg("offset"), py::arg("dtype"), py::arg("stream") = 0);
  h.def(
      "clock_probe",
      [](uintptr_t out, int samples, uint64_t interval_ticks, uintptr_t s) {
        launch_clock_probe(reinterpret_cast<uint64_t*>(out), samples, interval_ticks, as_stream(s));
      },
      py::arg("out"), py::arg("samples"), py::arg("interval_ticks"), py::arg("stream") = 0,
      "study tool: one wave samples (s_memtime, s_memrealtime) every interval_ticks (100 MHz) into out[2 * samples]");
  h.def(
      "fill_uniform",
      [](uintptr_t dst, int64_t n, uint64_t seed, DType dt, uintptr_t s) {
        launch_fill_uniform(as_ptr(dst), n, seed, dt, as_stream(s));
      },
      py::arg("dst"), py::arg("n"), py::arg("seed"), py::arg("dtype"), py::arg("stream") = 0);
  h.def(
      "cast",
      [](uintptr_t src, DType di, uintptr_t dst, DType d_o, int64_t n, uintptr_t s) {
        launch_cast(as_cptr(src), di, as_ptr(dst), d_o, n, as_stream(s));
      },
      py::arg("src"), py::arg("dtype_in"), py::arg("dst"), py::arg("dtype_out"), py::arg("n"), py::arg("stream") = 0);
  h.def(
      "bucket_copy",
      [](uintptr_t table, int count, uintptr_t bucket, DType dt, bool pack, int64_t total, uintptr_t s) {
        launch_bucket_copy(reinterpret_cast<const uint64_t*>(table), count, as_ptr(bucket), dt, pack, total,
                           as_stream(s));
      },
      py::arg("table"), py::arg("count"), py::arg("bucket"), py::arg("dtype"), py::arg("pack"), py::arg("total"),
      py::arg("stream") = 0);
  h.def(
      "copy",
      [](uintptr_t src, uintptr_t dst, int64_t bytes, uintptr_t s) { launch_copy(as_cptr(src), as_ptr(dst), bytes, as_stream(s)); },
      py::arg("src"), py::arg("dst"), py::arg("bytes"), py::arg("stream") = 0);
  h.def("set_copy_variant", &set_copy_variant);
  h.def("set_reduce_variant", &set_reduce_variant);
  // Stream-ordering events for the gradient reducer. scope: 0 = HIP default (system-scope
  // release when recorded), 1 = device-scope release, 2 = no system fence. Timing disabled.
  h.def(
      "event_create",
      [](int scope) {
        unsigned flags = hipEventDisableTiming;
        if (scope == 1) flags |= hipEventReleaseToDevice;
        if (scope == 2) flags |= hipEventDisableSystemFence;
        hipEvent_t e = nullptr;
        hip_check(hipEventCreateWithFlags(&e, flags), "hipEventCreateWithFlags");
        return reinterpret_cast<uintptr_t>(e);
      },
      py::arg("scope") = 1);
  h.def("event_destroy", [](uintptr_t e) { (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(e)); });
  h.def("event_record", [](uintptr_t e, uintptr_t s) {
    hip_check(hipEventRecord(reinterpret_cast<hipEvent_t>(e), as_stream(s)), "hipEventRecord");
  });
  h.def("stream_wait_event", [](uintptr_t s, uintptr_t e) {
    hip_check(hipStreamWaitEvent(as_stream(s), reinterpret_cast<hipEvent_t>(e), 0), "hipStreamWaitEvent");
  });
  // A stream whose kernels run only on `cus` of the device's CUs, spread evenly over the CU
  // numbering (every XCD gets its share): a collective overlapped with compute then occupies
  // a fixed slice of the GPU instead of a workgroup on every CU (ddp.py `cuN:` schedules).
  // exclude=True gives the complement - the compute stream of a CU split (ddp.py
  // compute_stream_excluding), whose GEMM tiles then never share a CU with the collective.
  h.def(
      "stream_create_cu_mask",
      [](int device, int cus, bool exclude) {
        hip_check(hipSetDevice(device), "hipSetDevice");
        int total = 0;
        hip_check(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, device), "CU count");
        if (cus < 1 || cus > total) throw std::invalid_argument("stream_create_cu_mask: cus must be in [1, CU count]");
        std::vector<uint32_t> mask(static_cast<size_t>((total + 31) / 32), 0u);
        for (int i = 0; i < cus; ++i) {
          const int cu = static_cast<int>(static_cast<int64_t>(i) * total / cus);
          mask[static_cast<size_t>(cu / 32)] |= 1u << (cu % 32);
        }
        if (exclude) {  // every CU BUT those: the compute side of a CU split
          for (int cu = 0; cu < total; ++cu) mask[static_cast<size_t>(cu / 32)] ^= 1u << (cu % 32);
        }
        hipStream_t st = nullptr;
        hip_check(hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(mask.size()), mask.data()),
                  "hipExtStreamCreateWithCUMask");
        return reinterpret_cast<uintptr_t>(st);
      },
      py::arg("device"), py::arg("cus"), py::arg("exclude") = false,
      "stream on `cus` CUs spread over the device (exclude=True: on every CU but those)");
  h.def("stream_destroy", [](uintptr_t s) { (void)hipStreamDestroy(reinterpret_cast<hipStream_t>(s)); });
  h.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    return n;
  });
  // Topology of a device pair: (can_access_peer, link type, hop count). Link types are
  // HSA_AMD_LINK_INFO_TYPE_* (4 = xGMI, 2 = PCIe); (-1, -1) when the runtime does not say.
  h.def(
      "link_info",
      [](int a, int b) {
        int can = 0;
        if (a != b) (void)hipDeviceCanAccessPeer(&can, a, b);
        uint32_t type = 0, hops = 0;
        const bool ok = a != b && hipExtGetLinkTypeAndHopCount(a, b, &type, &hops) == hipSuccess;
        (void)hipGetLastError();
        return py::make_tuple(a == b ? true : can != 0, ok ? static_cast<int>(type) : -1,
                              ok ? static_cast<int>(hops) : -1);
      },
      py::arg("a"), py::arg("b"));
  h.attr("MAX_RANKS") = kMaxRanks;
}

}  // namespace mxar
