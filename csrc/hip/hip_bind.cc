// Python bindings of the HIP data plane. Device buffers cross the boundary as raw
// addresses (torch `tensor.data_ptr()`) and streams as `torch.cuda.Stream.cuda_stream`,
// so the native module does not link against libtorch; torch is imported first and its
// bundled libamdhip64 (same SONAME) is the one HIP runtime of the process.
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <vector>

#include "xgmi_comm.h"

namespace py = pybind11;

namespace mxar {

static hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
static const void* as_cptr(uintptr_t p) { return reinterpret_cast<const void*>(p); }
static void* as_ptr(uintptr_t p) { return reinterpret_cast<void*>(p); }

void bind_hip(py::module_& m) {
  py::module_ h = m.def_submodule("hip", "HIP/CDNA4 data plane (gfx950)");

  py::enum_<DType>(h, "DType").value("F32", DType::F32).value("BF16", DType::BF16);
  py::enum_<Algo>(h, "Algo").value("Auto", Algo::Auto).value("TwoShot", Algo::TwoShot).value("OneShot", Algo::OneShot);

  py::class_<CommStats>(h, "CommStats")
      .def_readonly("calls", &CommStats::calls)
      .def_readonly("launches", &CommStats::launches)
      .def_readonly("bytes", &CommStats::bytes)
      .def_readonly("oneshot", &CommStats::oneshot)
      .def_readonly("twoshot", &CommStats::twoshot);

  py::class_<XgmiComm>(h, "XgmiComm")
      .def(py::init<int, int, int, int64_t, int, double>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("slot_bytes"), py::arg("grid") = 0, py::arg("timeout_s") = 20.0)
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
      .def_static(
          "barrier_local",
          [](const std::vector<XgmiComm*>& comms, uintptr_t stream) {
            py::gil_scoped_release r;
            XgmiComm::barrier_group(comms, as_stream(stream));
          },
          py::arg("comms"), py::arg("stream") = 0)
      .def("error", &XgmiComm::error)
      .def("clear_error", &XgmiComm::clear_error)
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("world", &XgmiComm::world)
      .def_property_readonly("device", &XgmiComm::device)
      .def_property("grid", &XgmiComm::grid, &XgmiComm::set_grid)
      .def_property("oneshot_max_bytes", &XgmiComm::oneshot_max_bytes, &XgmiComm::set_oneshot_max_bytes)
      .def_property_readonly("slot_bytes", &XgmiComm::slot_bytes)
      .def_property_readonly("slab_bytes", &XgmiComm::slab_bytes)
      .def_property_readonly("connected", &XgmiComm::connected)
      .def_property_readonly("stats", &XgmiComm::stats)
      .def_property("fence", &XgmiComm::fence, &XgmiComm::set_fence)
      .def("set_timeout", &XgmiComm::set_timeout);

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
  h.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    return n;
  });
  h.attr("MAX_RANKS") = kMaxRanks;
}

}  // namespace mxar
