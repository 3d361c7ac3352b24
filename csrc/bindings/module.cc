// Python module `akka_allreduce_1_amd._C`: protocol messages, protocol cores, the actor
// runtime, the TCP cluster transport and (csrc/hip) the HIP/CDNA4 data plane.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <mutex>
#include <atomic>
#include <condition_variable>
#include <thread>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <optional>
#include <sstream>

#include "../core/data_buffer.h"
#include "../core/log.h"
#include "../core/trace.h"
#include "../core/master_core.h"
#include "../core/worker_core.h"
#include "../runtime/actor_system.h"
#include "../runtime/allreduce_actors.h"
#include "../runtime/fault_injector.h"
#include "../runtime/loopback_plane.h"
#include "../runtime/plane_geometry.h"
#include "../runtime/plane_worker.h"
#include "py_common.h"

namespace py = pybind11;
using namespace mxar;

namespace mxar {
void bind_cluster(py::module_& m);  // csrc/bindings/cluster_bind.cc
void bind_hip(py::module_& m);      // csrc/hip/hip_bind.cc
void bind_akka(py::module_& m);     // csrc/bindings/akka_bind.cc
}  // namespace mxar

namespace mxar {

static DevicePayloadToPy g_dev_to_py = nullptr;
static PyToDevicePayload g_py_to_dev = nullptr;

void register_device_payload_hooks(DevicePayloadToPy to_py, PyToDevicePayload from_py) {
  g_dev_to_py = to_py;
  g_py_to_dev = from_py;
}

static PyToDevicePayload g_py_to_dev_typed = nullptr;
void register_typed_payload_hook(PyToDevicePayload from_py) { g_py_to_dev_typed = from_py; }

Payload typed_payload_from_py(const py::handle& obj) {
  if (g_py_to_dev_typed) {
    Payload d = g_py_to_dev_typed(obj);
    if (d) return d;
  }
  return payload_from_py(obj);
}

Payload payload_from_py(const py::handle& obj) {
  if (obj.is_none()) return make_host_payload({});
  if (g_py_to_dev) {
    Payload d = g_py_to_dev(obj);
    if (d) return d;
  }
  auto arr = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(obj);
  if (!arr) throw py::type_error("payload must be a float sequence, numpy array or tensor");
  std::vector<float> v(static_cast<size_t>(arr.size()));
  if (!v.empty()) std::memcpy(v.data(), arr.data(), v.size() * sizeof(float));
  return make_host_payload(std::move(v));
}

py::object payload_to_py(const Payload& p) {
  if (!p) return py::array_t<float>(0);
  if (p->on_device()) {
    if (g_dev_to_py) return g_dev_to_py(p);
    std::vector<float> h = p->to_host();
    py::array_t<float> a(h.size());
    if (!h.empty()) std::memcpy(a.mutable_data(), h.data(), h.size() * sizeof(float));
    return std::move(a);
  }
  py::array_t<float> a(p->size());
  if (p->size()) std::memcpy(a.mutable_data(), p->data(), p->size() * sizeof(float));
  return std::move(a);
}

py::object message_to_py(const Message& m) {
  return std::visit([](const auto& x) -> py::object { return py::cast(x); }, m);
}

Message message_from_py(const py::handle& obj) {
  if (py::isinstance<InitWorkers>(obj)) return obj.cast<InitWorkers>();
  if (py::isinstance<StartAllreduce>(obj)) return obj.cast<StartAllreduce>();
  if (py::isinstance<ScatterBlock>(obj)) return obj.cast<ScatterBlock>();
  if (py::isinstance<ReduceBlock>(obj)) return obj.cast<ReduceBlock>();
  if (py::isinstance<CompleteAllreduce>(obj)) return obj.cast<CompleteAllreduce>();
  if (py::isinstance<MemberUp>(obj)) return obj.cast<MemberUp>();
  if (py::isinstance<Terminated>(obj)) return obj.cast<Terminated>();
  if (py::isinstance<AllreduceFinished>(obj)) return obj.cast<AllreduceFinished>();
  if (py::isinstance<PoisonPill>(obj)) return obj.cast<PoisonPill>();
  if (py::isinstance<TextMessage>(obj)) return obj.cast<TextMessage>();
  if (py::isinstance<RoundTimeout>(obj)) return obj.cast<RoundTimeout>();
  if (py::isinstance<py::str>(obj)) return TextMessage{obj.cast<std::string>()};
  throw py::type_error("not a protocol message: " + std::string(py::str(py::type::of(obj))));
}

}  // namespace mxar

namespace {

bool payload_eq(const Payload& a, const Payload& b) {
  if (payload_size(a) != payload_size(b)) return false;
  if (!a || !b) return true;
  std::vector<float> x = a->to_host(), y = b->to_host();
  return x == y;
}

std::string vec_str(const Payload& p) {
  std::ostringstream os;
  os << "[";
  if (p) {
    auto h = p->to_host();
    for (size_t i = 0; i < h.size() && i < 16; ++i) os << (i ? ", " : "") << h[i];
    if (h.size() > 16) os << ", ...";
  }
  os << "]";
  return os.str();
}

// Source/sink adapters that call into Python with the GIL held.
DataSource make_source(py::object fn) {
  auto holder = std::make_shared<PyCallable>(std::move(fn));
  return [holder](const AllReduceInputRequest& req) -> AllReduceInput {
    py::gil_scoped_acquire g;
    py::object r = holder->fn(req);
    if (py::isinstance<AllReduceInput>(r)) return r.cast<AllReduceInput>();
    return AllReduceInput{payload_from_py(r)};
  };
}

DataSink make_sink(py::object fn) {
  if (fn.is_none()) return nullptr;
  auto holder = std::make_shared<PyCallable>(std::move(fn));
  return [holder](const AllReduceOutput& out) {
    py::gil_scoped_acquire g;
    holder->fn(out);
  };
}

// dataSource of a plane worker: a device tensor keeps its dtype and is ordered by event
DataSource make_plane_source(py::object fn) {
  auto holder = std::make_shared<PyCallable>(std::move(fn));
  return [holder](const AllReduceInputRequest& req) -> AllReduceInput {
    std::optional<py::gil_scoped_acquire> g;
    {
      TraceScope span("worker", [] { return std::make_pair(std::string("gil"), std::string()); });
      g.emplace();
    }
    py::object r;
    {
      TraceScope span("worker", [] { return std::make_pair(std::string("py source"), std::string()); });
      r = holder->fn(req);
    }
    if (py::isinstance<AllReduceInput>(r)) return r.cast<AllReduceInput>();
    TraceScope span("worker", [] { return std::make_pair(std::string("import"), std::string()); });
    return AllReduceInput{typed_payload_from_py(r)};
  };
}

PlaneWorkerActor* plane_worker_of(const ActorRef& ref) {
  auto* l = dynamic_cast<LocalActorRef*>(ref.get());
  if (!l) throw py::value_error("not a local actor");
  auto c = l->cell();
  if (!c) throw py::value_error("actor is stopped");
  auto* w = dynamic_cast<PlaneWorkerActor*>(c->actor());
  if (!w) throw py::value_error("not a plane worker actor");
  return w;
}

WorkerActor* worker_of(const ActorRef& ref) {
  auto* l = dynamic_cast<LocalActorRef*>(ref.get());
  if (!l) throw py::value_error("not a local actor");
  auto c = l->cell();
  if (!c) throw py::value_error("actor is stopped");
  auto* w = dynamic_cast<WorkerActor*>(c->actor());
  if (!w) throw py::value_error("not a worker actor");
  return w;
}

MasterActor* master_of(const ActorRef& ref) {
  auto* l = dynamic_cast<LocalActorRef*>(ref.get());
  if (!l) throw py::value_error("not a local actor");
  auto c = l->cell();
  if (!c) throw py::value_error("actor is stopped");
  auto* m = dynamic_cast<MasterActor*>(c->actor());
  if (!m) throw py::value_error("not a master actor");
  return m;
}

py::dict worker_stats_dict(const WorkerStats& s) {
  py::dict d;
#define F(x) d[#x] = s.x
  F(scatter_in); F(reduce_in); F(start_in); F(scatter_out); F(reduce_out); F(complete_out);
  F(bytes_out); F(bytes_in); F(outdated_dropped); F(future_requeued); F(stashed);
  F(forced_completions); F(rounds_completed); F(reductions); F(duplicate_arrivals); F(malformed_dropped); F(stale_epoch_dropped);
#undef F
  return d;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native threshold allreduce: protocol, actor runtime, HIP data plane";

  // ---------------------------------------------------------------- actor refs
  py::class_<ActorRefBase, std::shared_ptr<ActorRefBase>>(m, "ActorRef")
      .def("tell", [](ActorRefBase& self, py::handle msg, ActorRef sender) {
            Message mm = message_from_py(msg);
            py::gil_scoped_release r;
            self.tell(std::move(mm), std::move(sender));
          }, py::arg("msg"), py::arg("sender") = nullptr)
      .def_property_readonly("path", &ActorRefBase::path)
      .def_property_readonly("uid", &ActorRefBase::uid)
      .def_property_readonly("is_remote", &ActorRefBase::is_remote)
      .def("__eq__", [](const ActorRefBase& a, py::object b) {
        if (b.is_none() || !py::isinstance<ActorRefBase>(b)) return false;
        return a.uid() == b.cast<ActorRefBase&>().uid() || a.path() == b.cast<ActorRefBase&>().path();
      })
      .def("__hash__", [](const ActorRefBase& a) { return std::hash<std::string>()(a.path()); })
      .def("__repr__", [](const ActorRefBase& a) { return "ActorRef(" + a.path() + ")"; });

  // ---------------------------------------------------------------- messages
  py::class_<InitWorkers>(m, "InitWorkers")
      .def(py::init([](std::map<int, ActorRef> workers, ActorRef master, int destId, float thReduce,
                       float thComplete, int maxLag, int dataSize, int maxChunkSize, int64_t epoch, int startRound) {
             return InitWorkers{std::move(workers), std::move(master), destId, thReduce, thComplete,
                                maxLag, dataSize, maxChunkSize, epoch, startRound};
           }),
           py::arg("workers"), py::arg("master"), py::arg("destId"), py::arg("thReduce"), py::arg("thComplete"),
           py::arg("maxLag"), py::arg("dataSize"), py::arg("maxChunkSize"), py::arg("epoch") = 0,
           py::arg("startRound") = 0)
      .def_readwrite("startRound", &InitWorkers::startRound)
      .def_readwrite("planes", &InitWorkers::planes)
      .def_readwrite("roundBase", &InitWorkers::roundBase)
      .def_readwrite("workers", &InitWorkers::workers)
      .def_readwrite("master", &InitWorkers::master)
      .def_readwrite("destId", &InitWorkers::destId)
      .def_readwrite("thReduce", &InitWorkers::thReduce)
      .def_readwrite("thComplete", &InitWorkers::thComplete)
      .def_readwrite("maxLag", &InitWorkers::maxLag)
      .def_readwrite("dataSize", &InitWorkers::dataSize)
      .def_readwrite("maxChunkSize", &InitWorkers::maxChunkSize)
      .def_readwrite("epoch", &InitWorkers::epoch)
      .def("__repr__", [](const InitWorkers& x) {
        std::ostringstream os;
        os << "InitWorkers(workers=" << x.workers.size() << ", destId=" << x.destId << ", thReduce=" << x.thReduce
           << ", thComplete=" << x.thComplete << ", maxLag=" << x.maxLag << ", dataSize=" << x.dataSize
           << ", maxChunkSize=" << x.maxChunkSize << ", epoch=" << x.epoch << ")";
        return os.str();
      });

  py::class_<StartAllreduce>(m, "StartAllreduce")
      .def(py::init([](int r, int64_t epoch) { return StartAllreduce{r, epoch}; }), py::arg("round"),
           py::arg("epoch") = 0)
      .def_readwrite("round", &StartAllreduce::round)
      .def_readwrite("epoch", &StartAllreduce::epoch)
      .def("__eq__", [](const StartAllreduce& a, py::object b) {
        if (!py::isinstance<StartAllreduce>(b)) return false;
        const auto& x = b.cast<const StartAllreduce&>();
        return a.round == x.round && a.epoch == x.epoch;
      })
      .def("__hash__", [](const StartAllreduce& a) { return a.round; })
      .def("__repr__", [](const StartAllreduce& a) { return "StartAllreduce(" + std::to_string(a.round) + ")"; });

  py::class_<ScatterBlock>(m, "ScatterBlock")
      .def(py::init([](py::object value, int srcId, int destId, int chunkId, int round, int64_t epoch) {
             return ScatterBlock{payload_from_py(value), srcId, destId, chunkId, round, epoch};
           }),
           py::arg("value"), py::arg("srcId"), py::arg("destId"), py::arg("chunkId"), py::arg("round"),
           py::arg("epoch") = 0)
      .def_readwrite("epoch", &ScatterBlock::epoch)
      .def_property("value", [](const ScatterBlock& s) { return payload_to_py(s.value); },
                    [](ScatterBlock& s, py::object v) { s.value = payload_from_py(v); })
      .def_property_readonly("on_device", [](const ScatterBlock& s) { return s.value && s.value->on_device(); })
      .def_readwrite("srcId", &ScatterBlock::srcId)
      .def_readwrite("destId", &ScatterBlock::destId)
      .def_readwrite("chunkId", &ScatterBlock::chunkId)
      .def_readwrite("round", &ScatterBlock::round)
      .def("__eq__", [](const ScatterBlock& a, py::object o) {
        if (!py::isinstance<ScatterBlock>(o)) return false;
        const auto& b = o.cast<const ScatterBlock&>();
        return a.srcId == b.srcId && a.destId == b.destId && a.chunkId == b.chunkId && a.round == b.round &&
               a.epoch == b.epoch && payload_eq(a.value, b.value);
      })
      .def("__repr__", [](const ScatterBlock& s) {
        std::ostringstream os;
        os << "ScatterBlock(" << vec_str(s.value) << ", srcId=" << s.srcId << ", destId=" << s.destId
           << ", chunkId=" << s.chunkId << ", round=" << s.round << ")";
        return os.str();
      });

  py::class_<ReduceBlock>(m, "ReduceBlock")
      .def(py::init([](py::object value, int srcId, int destId, int chunkId, int round, int count, int64_t epoch) {
             return ReduceBlock{payload_from_py(value), srcId, destId, chunkId, round, count, epoch};
           }),
           py::arg("value"), py::arg("srcId"), py::arg("destId"), py::arg("chunkId"), py::arg("round"),
           py::arg("count"), py::arg("epoch") = 0)
      .def_readwrite("epoch", &ReduceBlock::epoch)
      .def_property("value", [](const ReduceBlock& s) { return payload_to_py(s.value); },
                    [](ReduceBlock& s, py::object v) { s.value = payload_from_py(v); })
      .def_property_readonly("on_device", [](const ReduceBlock& s) { return s.value && s.value->on_device(); })
      .def_readwrite("srcId", &ReduceBlock::srcId)
      .def_readwrite("destId", &ReduceBlock::destId)
      .def_readwrite("chunkId", &ReduceBlock::chunkId)
      .def_readwrite("round", &ReduceBlock::round)
      .def_readwrite("count", &ReduceBlock::count)
      .def("__eq__", [](const ReduceBlock& a, py::object o) {
        if (!py::isinstance<ReduceBlock>(o)) return false;
        const auto& b = o.cast<const ReduceBlock&>();
        return a.srcId == b.srcId && a.destId == b.destId && a.chunkId == b.chunkId && a.round == b.round &&
               a.count == b.count && a.epoch == b.epoch && payload_eq(a.value, b.value);
      })
      .def("__repr__", [](const ReduceBlock& s) {
        std::ostringstream os;
        os << "ReduceBlock(" << vec_str(s.value) << ", srcId=" << s.srcId << ", destId=" << s.destId
           << ", chunkId=" << s.chunkId << ", round=" << s.round << ", count=" << s.count << ")";
        return os.str();
      });

  py::class_<CompleteAllreduce>(m, "CompleteAllreduce")
      .def(py::init([](int src, int r, int64_t epoch) { return CompleteAllreduce{src, r, epoch}; }), py::arg("srcId"),
           py::arg("round"), py::arg("epoch") = 0)
      .def_readwrite("srcId", &CompleteAllreduce::srcId)
      .def_readwrite("round", &CompleteAllreduce::round)
      .def_readwrite("epoch", &CompleteAllreduce::epoch)
      .def("__eq__", [](const CompleteAllreduce& a, py::object o) {
        if (!py::isinstance<CompleteAllreduce>(o)) return false;
        const auto& b = o.cast<const CompleteAllreduce&>();
        return a.srcId == b.srcId && a.round == b.round && a.epoch == b.epoch;
      })
      .def("__hash__", [](const CompleteAllreduce& a) { return a.srcId * 1000003 + a.round; })
      .def("__repr__", [](const CompleteAllreduce& c) {
        return "CompleteAllreduce(" + std::to_string(c.srcId) + ", " + std::to_string(c.round) + ")";
      });

  py::class_<MemberUp>(m, "MemberUp")
      .def(py::init([](ActorRef ref, std::string role, std::string address, std::string meta) {
             return MemberUp{std::move(ref), std::move(role), std::move(address), std::move(meta)};
           }),
           py::arg("ref"), py::arg("role") = "worker", py::arg("address") = "", py::arg("meta") = "")
      .def_readwrite("ref", &MemberUp::ref)
      .def_readwrite("role", &MemberUp::role)
      .def_readwrite("address", &MemberUp::address)
      .def_readwrite("meta", &MemberUp::meta)
      .def("__repr__", [](const MemberUp& u) { return "MemberUp(" + (u.ref ? u.ref->path() : "?") + ", " + u.role + ")"; });

  py::class_<Terminated>(m, "Terminated")
      .def(py::init([](ActorRef ref) { return Terminated{std::move(ref)}; }), py::arg("ref"))
      .def_readwrite("ref", &Terminated::ref)
      .def("__repr__", [](const Terminated& t) { return "Terminated(" + (t.ref ? t.ref->path() : "?") + ")"; });

  py::class_<AllreduceFinished>(m, "AllreduceFinished")
      .def(py::init([](int r) { return AllreduceFinished{r}; }), py::arg("rounds"))
      .def_readwrite("rounds", &AllreduceFinished::rounds)
      .def("__eq__", [](const AllreduceFinished& a, py::object o) {
        return py::isinstance<AllreduceFinished>(o) && a.rounds == o.cast<AllreduceFinished>().rounds;
      })
      .def("__repr__", [](const AllreduceFinished& f) { return "AllreduceFinished(" + std::to_string(f.rounds) + ")"; });

  py::class_<PoisonPill>(m, "PoisonPill").def(py::init<>());
  py::class_<TextMessage>(m, "TextMessage")
      .def(py::init([](std::string s) { return TextMessage{std::move(s)}; }))
      .def_readwrite("text", &TextMessage::text)
      .def("__eq__", [](const TextMessage& a, py::object o) {
        return py::isinstance<TextMessage>(o) && a.text == o.cast<TextMessage>().text;
      })
      .def("__repr__", [](const TextMessage& t) { return "TextMessage(" + t.text + ")"; });

  py::class_<RoundTimeout>(m, "RoundTimeout")
      .def(py::init([](int64_t epoch, int round) { return RoundTimeout{epoch, round}; }), py::arg("epoch"),
           py::arg("round"))
      .def_readwrite("epoch", &RoundTimeout::epoch)
      .def_readwrite("round", &RoundTimeout::round)
      .def("__repr__", [](const RoundTimeout& t) {
        return "RoundTimeout(epoch=" + std::to_string(t.epoch) + ", round=" + std::to_string(t.round) + ")";
      });
  py::class_<BridgeCommand>(m, "BridgeCommand")
      .def_readonly("round", &BridgeCommand::round)
      .def_readonly("client", &BridgeCommand::client)
      .def_property_readonly("kind", [](const BridgeCommand& b) {
        return b.kind == BridgeCommand::Start ? "StartAllreduce" : "Status";
      });
  m.def("parse_flat_json", [](const std::string& line) -> py::object {
    std::map<std::string, std::string> kv;
    if (!parse_flat_json(line, kv)) return py::none();
    return py::cast(kv);
  }, "The bridge's line parser (flat JSON object -> {key: raw value}); None when malformed");
  py::class_<PlaneRoundDone>(m, "PlaneRoundDone")
      .def_readonly("epoch", &PlaneRoundDone::epoch)
      .def_readonly("error", &PlaneRoundDone::error)
      .def_readonly("cold", &PlaneRoundDone::cold)
      .def_property_readonly("iteration", [](const PlaneRoundDone& d) { return d.output.iteration; });

  py::class_<AllReduceInputRequest>(m, "AllReduceInputRequest")
      .def(py::init([](int it) { return AllReduceInputRequest{it}; }), py::arg("iteration"))
      .def_readwrite("iteration", &AllReduceInputRequest::iteration)
      .def("__repr__", [](const AllReduceInputRequest& r) { return "AllReduceInputRequest(" + std::to_string(r.iteration) + ")"; });

  py::class_<AllReduceInput>(m, "AllReduceInput")
      .def(py::init([](py::object data) { return AllReduceInput{payload_from_py(data)}; }), py::arg("data"))
      .def_property("data", [](const AllReduceInput& s) { return payload_to_py(s.data); },
                    [](AllReduceInput& s, py::object v) { s.data = payload_from_py(v); })
      .def("__len__", [](const AllReduceInput& s) { return payload_size(s.data); });

  py::class_<AllReduceOutput>(m, "AllReduceOutput")
      .def(py::init([](py::object data, std::vector<int> count, int iteration) {
             return AllReduceOutput{payload_from_py(data), std::move(count), iteration};
           }),
           py::arg("data"), py::arg("count"), py::arg("iteration"))
      .def_property_readonly("data", [](const AllReduceOutput& s) { return payload_to_py(s.data); })
      .def_property_readonly("on_device", [](const AllReduceOutput& s) { return s.data && s.data->on_device(); })
      .def_readonly("count", &AllReduceOutput::count)
      .def_readonly("iteration", &AllReduceOutput::iteration)
      .def("__repr__", [](const AllReduceOutput& o) {
        return "AllReduceOutput(" + vec_str(o.data) + ", iteration=" + std::to_string(o.iteration) + ")";
      });

  py::class_<NativeSource>(m, "NativeSource",
                           "A dataSource that runs without Python (hip.tensor_source); pass it to plane_worker");
  py::class_<NativeSink>(m, "NativeSink", "A dataSink that runs without Python (last_output_sink)")
      .def("last", [](NativeSink& k) -> py::object {
        std::lock_guard<std::mutex> g(k.keep->mu);
        if (!k.keep->out) return py::none();
        return py::cast(*k.keep->out);
      }, "the newest AllReduceOutput (None before the first round)")
      .def_property_readonly("rounds", [](NativeSink& k) {
        std::lock_guard<std::mutex> g(k.keep->mu);
        return k.keep->rounds;
      })
      .def("stamps", [](NativeSink& k) {
        std::lock_guard<std::mutex> g(k.keep->mu);
        return k.keep->stamps;
      }, "record=True: [(iteration, time.perf_counter()-compatible seconds at the sink)] per round")
      .def("count_stats", [](NativeSink& k) {
        std::lock_guard<std::mutex> g(k.keep->mu);
        py::dict d;
        d["sum"] = k.keep->count_sum;
        d["n"] = k.keep->count_n;
        d["zero"] = k.keep->count_zero;
        return d;
      }, "record=True: totals over every round's per-chunk counts (sum, entries, zero entries)");
  m.def("last_output_sink", [](bool record) {
    auto keep = std::make_shared<LastOutput>();
    keep->record = record;
    return NativeSink{[keep](const AllReduceOutput& o) {
                        const double t =
                            std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
                        std::lock_guard<std::mutex> g(keep->mu);
                        keep->out = o;  // holds the round output's buffer until the next round
                        keep->rounds++;
                        if (keep->record) {
                          if (keep->stamps.size() < (size_t{1} << 22)) keep->stamps.emplace_back(o.iteration, t);
                          for (int c : o.count) {
                            keep->count_sum += static_cast<uint64_t>(c > 0 ? c : 0);
                            keep->count_zero += c == 0 ? 1 : 0;
                          }
                          keep->count_n += o.count.size();
                        }
                      },
                      keep};
  }, py::arg("record") = false,
        "dataSink keeping only the newest round output, without the GIL (plane workers); record: per-round "
        "sink stamps and count totals too");

  m.def("plane_geometry",
        [](int peers, int dataSize, int maxChunkSize, float thReduce, float thComplete,
           std::map<int, std::string> descriptors, int64_t flag_maxch, int64_t es) {
          PlaneConfig c;
          c.peers = peers;
          c.dataSize = dataSize;
          c.maxChunkSize = maxChunkSize;
          c.thReduce = thReduce;
          c.thComplete = thComplete;
          c.descriptors = std::move(descriptors);
          const PlaneGeometry g = plane_geometry(c, flag_maxch, es);
          py::dict d;
          d["block"] = g.block;
          d["chunk"] = g.chunk;
          d["nch"] = g.nch;
          d["nch_ref"] = g.nch_ref;
          d["coarse"] = g.coarse;
          d["colocation"] = g.colocation;
          d["grid"] = g.grid;
          return d;
        },
        py::arg("peers"), py::arg("dataSize"), py::arg("maxChunkSize"), py::arg("thReduce"), py::arg("thComplete"),
        py::arg("descriptors"), py::arg("flag_maxch") = 1 << 20, py::arg("es") = 4,
        "The kernel geometry every worker of a membership derives from InitWorkers (csrc/runtime/plane_geometry.h)");

  // ---------------------------------------------------------------- core helpers
  // bring-up aid (no debugger on the GPU boxes): a native SIGSEGV / SIGBUS prints the faulting
  // thread's native frames to stderr, then the previous handler (Python's faulthandler) runs
  m.def("install_native_backtrace", [] {
    static struct sigaction prev_segv, prev_bus;
    struct sigaction sa {};
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sa.sa_sigaction = [](int sig, siginfo_t* info, void* ctx) {
      void* frames[64];
      const int n = backtrace(frames, 64);
      const char head[] = "\n[native backtrace]\n";
      (void)!write(2, head, sizeof(head) - 1);
      backtrace_symbols_fd(frames, n, 2);
      struct sigaction& prev = sig == SIGSEGV ? prev_segv : prev_bus;
      if (prev.sa_flags & SA_SIGINFO) {
        if (prev.sa_sigaction) prev.sa_sigaction(sig, info, ctx);
      } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler) {
        prev.sa_handler(sig);
      }
      signal(sig, SIG_DFL);
      raise(sig);
    };
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &prev_segv);
    sigaction(SIGBUS, &sa, &prev_bus);
  });
  m.def("f32_threshold_count", &f32_threshold_count, py::arg("threshold"), py::arg("peers"));
  m.def("f32_threshold_chunks", &f32_threshold_chunks, py::arg("threshold"), py::arg("peers"), py::arg("numChunks"));
  m.def("f32_ceil_div", &f32_ceil_div);

  py::class_<BlockLayout>(m, "BlockLayout")
      .def(py::init<int, int, int>(), py::arg("dataSize"), py::arg("peers"), py::arg("maxChunkSize"))
      .def_readonly("start", &BlockLayout::start)
      .def_readonly("end", &BlockLayout::end)
      .def_readonly("step", &BlockLayout::step)
      .def("block_size", &BlockLayout::block_size)
      .def("num_chunks", &BlockLayout::num_chunks)
      .def("total_chunks", &BlockLayout::total_chunks)
      .def("uniform_chunks", &BlockLayout::uniform_chunks);

  py::class_<ArrivalCounters>(m, "ArrivalCounters")
      .def(py::init<int, int, int, float, int>(), py::arg("rows"), py::arg("peers"), py::arg("numChunks"),
           py::arg("threshold"), py::arg("minChunksOverride") = -1)
      .def("add", &ArrivalCounters::add)
      .def("count", &ArrivalCounters::count)
      .def("reach_threshold", &ArrivalCounters::reach_threshold)
      .def("reach_round_threshold", &ArrivalCounters::reach_round_threshold)
      .def("up", &ArrivalCounters::up)
      .def("phys", &ArrivalCounters::phys)
      .def_property_readonly("min_required", &ArrivalCounters::min_required)
      .def_property_readonly("min_chunks_required", &ArrivalCounters::min_chunks_required);

  // ---------------------------------------------------------------- logging
  py::module_ tr = m.def_submodule("trace", "Chrome-trace timeline + roctx ranges (csrc/core/trace.h)");
  tr.def("enable", [](bool on) { Tracer::get().enable(on); }, py::arg("on") = true);
  tr.def("enabled", [] { return Tracer::get().enabled(); });
  tr.def("set_roctx", [](bool on) { Tracer::get().set_roctx(on); });
  tr.def("dump_json", [] { return Tracer::get().dump_json(); });
  tr.def("size", [] { return Tracer::get().size(); });
  tr.def("clear", [] { Tracer::get().clear(); });
  tr.def("instant", [](const std::string& name, const std::string& args) { trace_instant("user", name, args); },
         py::arg("name"), py::arg("args") = "");

  m.def("set_log_level", [](const std::string& l) { Logger::get().set_level(Logger::parse(l)); });
  m.def("get_log_level", [] { return std::string(Logger::level_name(Logger::get().level())); });
  m.def("set_log_sink", [](py::object fn) {
    if (fn.is_none()) {
      Logger::get().set_sink(nullptr);
      return;
    }
    auto holder = std::make_shared<PyCallable>(std::move(fn));
    Logger::get().set_sink([holder](LogLevel l, const std::string& src, const std::string& msg) {
      py::gil_scoped_acquire g;
      try {
        holder->fn(std::string(Logger::level_name(l)), src, msg);
      } catch (py::error_already_set& e) {
        e.discard_as_unraisable("mxar log sink");
      }
    });
  });

  // ---------------------------------------------------------------- runtime
  py::class_<ProbeRef, ActorRefBase, std::shared_ptr<ProbeRef>>(m, "ProbeRef")
      .def("receive", [](ProbeRef& p, double timeout_s) -> py::object {
            std::optional<Envelope> e;
            {
              py::gil_scoped_release r;
              e = p.receive(std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)));
            }
            if (!e) return py::none();
            return py::make_tuple(message_to_py(e->msg), e->sender ? py::cast(e->sender) : py::none());
          }, py::arg("timeout") = 3.0)
      .def("pending", [](ProbeRef& p) { py::gil_scoped_release r; return p.pending(); })
      .def("clear", &ProbeRef::clear);

  py::class_<SystemStats>(m, "SystemStats")
      .def_readonly("delivered", &SystemStats::delivered)
      .def_readonly("dead_letters", &SystemStats::dead_letters)
      .def_readonly("actor_failures", &SystemStats::actor_failures);

  py::class_<ActorSystem, std::shared_ptr<ActorSystem>>(m, "ActorSystem")
      .def(py::init([](std::string name, bool deterministic, int threads, int throughput) {
             return std::make_shared<ActorSystem>(
                 std::move(name), deterministic ? ActorSystem::Mode::Deterministic : ActorSystem::Mode::Threaded,
                 threads, throughput);
           }),
           py::arg("name"), py::arg("deterministic") = false, py::arg("threads") = 0, py::arg("throughput") = 64)
      .def_property_readonly("name", &ActorSystem::name)
      .def_property_readonly("deterministic", &ActorSystem::deterministic)
      .def("worker", [](ActorSystem& s, py::object source, py::object sink, std::string name,
                        std::shared_ptr<DataPlane> plane) {
            auto a = std::make_unique<WorkerActor>(make_source(std::move(source)), make_sink(std::move(sink)), plane);
            return s.actor_of(std::move(a), std::move(name));
          }, py::arg("source"), py::arg("sink") = py::none(), py::arg("name") = "", py::arg("plane") = nullptr)
      .def("master", [](ActorSystem& s, int totalWorkers, float thAllreduce, float thReduce, float thComplete,
                        int maxLag, int dataSize, int maxRound, int maxChunkSize, bool liveBarrier,
                        py::object on_finished, std::string name, int startRound, py::object on_round,
                        int roundTimeoutMs, bool reinitOnLoss, bool resumeOnJoin, bool externalRounds,
                        int bridgePort, std::string bridgeHost, int initWorkers) {
            MasterParams p{totalWorkers, thAllreduce, thReduce, thComplete, maxLag, dataSize, maxRound,
                           maxChunkSize, liveBarrier, startRound, roundTimeoutMs, reinitOnLoss, resumeOnJoin,
                           externalRounds, initWorkers};
            MasterActor::RoundCallback rcb;
            if (!on_round.is_none()) {
              auto h = std::make_shared<PyCallable>(std::move(on_round));
              rcb = [h](int round, int64_t epoch) {
                py::gil_scoped_acquire g;
                h->fn(round, epoch);
              };
            }
            MasterActor::FinishedCallback cb;
            if (!on_finished.is_none()) {
              auto h = std::make_shared<PyCallable>(std::move(on_finished));
              cb = [h](int rounds) {
                py::gil_scoped_acquire g;
                h->fn(rounds);
              };
            }
            auto actor = std::make_unique<MasterActor>(p, cb, rcb);
            std::shared_ptr<ControlBridge> bridge;
            if (bridgePort >= 0) {
              bridge = ControlBridge::start(bridgeHost, bridgePort);
              actor->set_bridge(bridge);
            }
            ActorRef ref = s.actor_of(std::move(actor), std::move(name));
            if (bridge) bridge->attach(ref, ref->path());
            return ref;
          }, py::arg("totalWorkers"), py::arg("thAllreduce"), py::arg("thReduce"), py::arg("thComplete"),
          py::arg("maxLag"), py::arg("dataSize"), py::arg("maxRound"), py::arg("maxChunkSize"),
          py::arg("liveBarrier") = false, py::arg("on_finished") = py::none(), py::arg("name") = "master",
          py::arg("startRound") = 0, py::arg("on_round") = py::none(), py::arg("roundTimeoutMs") = 0,
          py::arg("reinitOnLoss") = false, py::arg("resumeOnJoin") = false, py::arg("externalRounds") = false,
          py::arg("bridgePort") = -1, py::arg("bridgeHost") = "127.0.0.1", py::arg("initWorkers") = 0,
          "bridgePort >= 0 starts a control bridge (csrc/runtime/control_bridge.h; 0 = any free port, see "
          "master_bridge_port); externalRounds makes its clients drive the rounds")
      .def("master_bridge_port", [](ActorSystem&, ActorRef ref) {
        auto* m = master_of(ref);
        return m->bridge() ? m->bridge()->port() : -1;
      })
      .def("plane_worker", [](ActorSystem& s, py::object source, py::object sink, std::shared_ptr<RoundPlane> plane,
                              std::string name) {
            DataSource src = py::isinstance<NativeSource>(source) ? source.cast<NativeSource&>().fn
                                                                  : make_plane_source(std::move(source));
            DataSink snk = py::isinstance<NativeSink>(sink) ? sink.cast<NativeSink&>().fn : make_sink(std::move(sink));
            auto a = std::make_unique<PlaneWorkerActor>(std::move(src), std::move(snk), std::move(plane));
            return s.actor_of(std::move(a), std::move(name));
          }, py::arg("source"), py::arg("sink") = py::none(), py::arg("plane"), py::arg("name") = "",
          "Round-granular worker (csrc/runtime/plane_worker.h): the reference protocol with one plane launch "
          "per round; announce plane.descriptor as the member's meta (MemberUp / ClusterConfig.meta)")
      .def("plane_worker_rounds", [](ActorSystem&, ActorRef ref) {
        // (round, maxRound, launched): plain words read without stopping the worker - a
        // sampling probe (the straggler bench's lag), unlike plane_worker_state's statistics
        auto* w = plane_worker_of(ref);
        return std::make_tuple(w->round(), w->max_round(), w->launched());
      }, "(round, maxRound, launched) of a plane worker, safe to sample while it runs")
      .def("plane_worker_state", [](ActorSystem&, ActorRef ref) {
        auto* w = plane_worker_of(ref);
        py::dict d;
        d["id"] = w->id();
        d["round"] = w->round();
        d["maxRound"] = w->max_round();
        d["launched"] = w->launched();
        d["epoch"] = w->epoch();
        d["initialized"] = w->initialized();
        const PlaneWorkerStats& s = w->stats();
        py::dict st;
#define F(x) st[#x] = s.x
        F(start_in); F(rounds_launched); F(cold_rounds); F(forced_completions); F(rounds_completed);
        F(complete_out); F(stale_dropped); F(stashed); F(plane_errors); F(inits); F(starts_coalesced);
#undef F
        d["stats"] = st;
        const RoundLatency lat = w->round_latency();
        py::dict l;
        l["count"] = lat.count;
        l["p50_ms"] = lat.p50_ms;
        l["p99_ms"] = lat.p99_ms;
        l["mean_ms"] = lat.mean_ms;
        l["max_ms"] = lat.max_ms;
        d["round_latency"] = l;
        return d;
      })
      .def("probe", &ActorSystem::make_probe, py::arg("name") = "")
      .def("lookup", &ActorSystem::lookup)
      .def("stop", &ActorSystem::stop)
      .def_property_readonly("dead_letters", &ActorSystem::dead_letters)
      .def("run_until_idle", [](ActorSystem& s, size_t maxm) {
            py::gil_scoped_release r;
            return s.run_until_idle(maxm);
          }, py::arg("max_messages") = SIZE_MAX)
      .def("advance_time", [](ActorSystem& s, double seconds) {
            py::gil_scoped_release r;
            s.advance_time(std::chrono::milliseconds(static_cast<int64_t>(seconds * 1000)));
          })
      .def("await_idle", [](ActorSystem& s, double timeout) {
            py::gil_scoped_release r;
            return s.await_idle(std::chrono::milliseconds(static_cast<int64_t>(timeout * 1000)));
          }, py::arg("timeout") = 10.0)
      .def("schedule_once", [](ActorSystem& s, double delay, ActorRef target, py::handle msg) {
            return s.schedule_once(std::chrono::milliseconds(static_cast<int64_t>(delay * 1000)), std::move(target),
                                   message_from_py(msg));
          })
      .def("cancel", &ActorSystem::cancel)
      .def("stats", &ActorSystem::stats)
      .def("shutdown", [](ActorSystem& s) {
        py::gil_scoped_release r;
        s.shutdown();
      })
      .def_property_readonly("terminated", &ActorSystem::terminated)
      .def("worker_state", [](ActorSystem&, ActorRef ref) {
        auto* w = worker_of(ref);
        const WorkerCore& c = w->core();
        py::dict d;
        d["id"] = c.id();
        d["round"] = c.round();
        d["maxRound"] = c.max_round();
        d["maxScattered"] = c.max_scattered();
        d["completed"] = std::vector<int>(c.completed().begin(), c.completed().end());
        d["numPeers"] = c.num_peers();
        d["myNumChunks"] = c.my_num_chunks();
        d["maxNumChunks"] = c.max_num_chunks();
        d["initialized"] = c.initialized();
        d["stats"] = worker_stats_dict(c.stats());
        const RoundLatency lat = c.round_latency();
        py::dict l;
        l["count"] = lat.count;
        l["p50_ms"] = lat.p50_ms;
        l["p99_ms"] = lat.p99_ms;
        l["mean_ms"] = lat.mean_ms;
        l["max_ms"] = lat.max_ms;
        d["round_latency"] = l;
        d["describe"] = c.describe();
        return d;
      })
      .def("master_round_stamps", [](ActorSystem&, ActorRef ref) { return master_of(ref)->round_stamps(); },
           "perf_counter()-compatible seconds at which each round reached the master's barrier")
      .def("master_state", [](ActorSystem&, ActorRef ref) {
        auto* ma = master_of(ref);
        const MasterCore& c = ma->core();
        py::dict d;
        d["round"] = c.round();
        d["numComplete"] = c.num_complete();
        d["epoch"] = c.epoch();
        d["finished"] = c.finished();
        d["numWorkers"] = c.workers().size();
        d["inits"] = c.stats().inits;
        d["rounds_started"] = c.stats().rounds_started;
        d["stale_completes"] = c.stats().stale_completes;
        d["round_timeouts"] = c.stats().round_timeouts;
        d["loss_reinits"] = c.stats().loss_reinits;
        d["join_reinits"] = c.stats().join_reinits;
        return d;
      });

  py::class_<FaultStats>(m, "FaultStats")
      .def_readonly("seen", &FaultStats::seen)
      .def_readonly("forwarded", &FaultStats::forwarded)
      .def_readonly("dropped", &FaultStats::dropped)
      .def_readonly("duplicated", &FaultStats::duplicated)
      .def_readonly("delayed", &FaultStats::delayed);
  py::class_<FaultyRef, ActorRefBase, std::shared_ptr<FaultyRef>>(m, "FaultyRef")
      .def("stats", &FaultyRef::stats)
      .def("set_enabled", &FaultyRef::set_enabled)
      .def_property_readonly("target", &FaultyRef::target);
  m.def(
      "faulty",
      [](std::shared_ptr<ActorSystem> sys, ActorRef target, double drop, double duplicate, int delay_ms,
         double delay_prob, std::vector<std::string> kinds, int round_lo, int round_hi, uint64_t seed) {
        FaultPolicy p;
        p.drop = drop;
        p.duplicate = duplicate;
        p.delay_ms = delay_ms;
        p.delay_prob = delay_prob;
        p.kinds = std::set<std::string>(kinds.begin(), kinds.end());
        p.round_lo = round_lo;
        p.round_hi = round_hi;
        p.seed = seed;
        return std::make_shared<FaultyRef>(sys.get(), std::move(target), std::move(p));
      },
      py::arg("system"), py::arg("target"), py::arg("drop") = 0.0, py::arg("duplicate") = 0.0,
      py::arg("delay_ms") = 0, py::arg("delay_prob") = 1.0, py::arg("kinds") = std::vector<std::string>{},
      py::arg("round_lo") = INT32_MIN, py::arg("round_hi") = INT32_MAX, py::arg("seed") = 1,
      "Fault-injecting ActorRef decorator (drop / duplicate / delay selected messages)");

  py::class_<DataPlane, std::shared_ptr<DataPlane>>(m, "DataPlane").def_property_readonly("name", &DataPlane::name);
  py::class_<RoundPlane, std::shared_ptr<RoundPlane>>(m, "RoundPlane")
      .def_property_readonly("name", &RoundPlane::name)
      .def_property_readonly("descriptor", &RoundPlane::descriptor)
      .def_property_readonly("chunks", &RoundPlane::chunks);
  py::class_<LoopbackRoundPlane, RoundPlane, std::shared_ptr<LoopbackRoundPlane>>(m, "LoopbackRoundPlane")
      .def_property_readonly("stats",
                             [](LoopbackRoundPlane& p) {
                               const LoopbackPlaneStats s = p.stats();
                               py::dict d;
                               d["launches"] = s.launches;
                               d["cold"] = s.cold;
                               d["forced_rounds"] = s.forced_rounds;
                               d["peer_forces"] = s.peer_forces;
                               d["completed"] = s.completed;
                               return d;
                             })
      .def("force", [](LoopbackRoundPlane& p, int round) {
        py::gil_scoped_release r;
        p.force(round);
      })
      .def("drain", [](LoopbackRoundPlane& p) {
        py::gil_scoped_release r;
        p.drain();
      });
  m.def("loopback_plane", &make_loopback_plane, py::arg("hub"),
        "RoundPlane in host memory (csrc/runtime/loopback_plane.h): the round engine's semantics for the "
        "workers of one process, no GPU; every worker of a job names the same hub");
  m.def("host_plane", [] { return std::static_pointer_cast<DataPlane>(HostPlane::instance()); });
  // A process watchdog that needs no GIL (bench.py's dp section): a Python Timer cannot run
  // while the main thread blocks inside a C call holding the GIL (e.g. a kernel launch into a
  // full hardware queue behind a spinning kernel). Returns cancel() -> True if it disarmed
  // the watchdog, False if it had already fired.
  m.def(
      "watchdog_arm",
      [](double seconds, int fd, std::string line, int code) {
        auto state = std::make_shared<std::atomic<int>>(0);  // 0 armed, 1 cancelled, 2 fired
        auto mu = std::make_shared<std::mutex>();
        auto cv = std::make_shared<std::condition_variable>();
        std::thread([state, mu, cv, seconds, fd, line, code] {
          {
            std::unique_lock<std::mutex> lk(*mu);
            cv->wait_for(lk, std::chrono::duration<double>(seconds), [&] { return state->load() != 0; });
          }
          int armed = 0;
          if (!state->compare_exchange_strong(armed, 2)) return;
          if (fd >= 0 && !line.empty()) {
            const char* p = line.data();
            size_t left = line.size();
            while (left > 0) {
              const ssize_t w = ::write(fd, p, left);
              if (w <= 0) break;
              p += w;
              left -= static_cast<size_t>(w);
            }
          }
          ::_exit(code);
        }).detach();
        return py::cpp_function([state, mu, cv] {
          int armed = 0;
          const bool won = state->compare_exchange_strong(armed, 1);
          {
            std::lock_guard<std::mutex> g(*mu);
          }
          cv->notify_all();
          return won;
        });
      },
      py::arg("seconds"), py::arg("fd"), py::arg("line"), py::arg("code") = 0);

  bind_cluster(m);
  bind_hip(m);
  bind_akka(m);
}
