// Python bindings of the Akka classic-remoting codec (csrc/cluster/akka_wire.h) and the
// master's akka.tcp endpoint (csrc/runtime/akka_endpoint.h). The codec functions exist so the
// tests can check every layer against independent encoders (google.protobuf, a Python
// ObjectOutputStream writer) and drive the endpoint as an Akka client would.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../cluster/akka_wire.h"
#include "../runtime/akka_endpoint.h"
#include "../runtime/allreduce_actors.h"

namespace py = pybind11;

namespace mxar {

namespace {

MasterActor* master_actor(const ActorRef& ref) {
  auto* l = dynamic_cast<LocalActorRef*>(ref.get());
  auto c = l ? l->cell() : nullptr;
  auto* m = c ? dynamic_cast<MasterActor*>(c->actor()) : nullptr;
  if (!m) throw py::value_error("not a running local master actor");
  return m;
}

py::bytes B(const std::string& s) { return py::bytes(s); }

akka::SerializedMsg msg_from(const py::dict& d) {
  akka::SerializedMsg m;
  m.bytes = d["message"].cast<std::string>();
  m.serializer = d["serializerId"].cast<int32_t>();
  if (d.contains("messageManifest") && !d["messageManifest"].is_none()) {
    m.has_manifest = true;
    m.manifest = d["messageManifest"].cast<std::string>();
  }
  return m;
}

py::dict msg_dict(const akka::SerializedMsg& m) {
  py::dict d;
  d["message"] = B(m.bytes);
  d["serializerId"] = m.serializer;
  d["messageManifest"] = m.has_manifest ? py::object(B(m.manifest)) : py::object(py::none());
  return d;
}

py::dict addr_dict(const akka::Address& a) {
  py::dict d;
  d["system"] = a.system;
  d["hostname"] = a.host;
  d["port"] = a.port;
  d["protocol"] = a.protocol;
  return d;
}

}  // namespace

void bind_akka(py::module_& root) {
  py::module_ m = root.def_submodule("akka", "Akka classic remoting wire codec and endpoint (csrc/cluster/akka_wire.h)");
  m.attr("MAX_FRAME") = akka::kMaxFrame;
  m.def("sha1", [](const std::string& b) { return B(akka::sha1(b)); });
  m.def("case_class_suid",
        [](const std::string& fqcn, const std::vector<std::pair<std::string, std::string>>& params) {
          std::vector<std::pair<std::string, char>> ps;
          for (auto& p : params) {
            if (p.second.size() != 1) throw py::value_error("parameter types are JVM primitive type codes");
            ps.emplace_back(p.first, p.second[0]);
          }
          return akka::default_suid(akka::scala_case_class_model(fqcn, ps));
        },
        py::arg("fqcn"), py::arg("params"),
        "default serialVersionUID of `final case class` fqcn(params) as scalac 2.12 compiles it");
  m.def("class_suid",
        [](const std::string& name, int mods, std::vector<std::string> interfaces,
           const std::vector<std::tuple<std::string, int, std::string>>& fields,
           const std::vector<std::tuple<int, std::string>>& ctors,
           const std::vector<std::tuple<std::string, int, std::string>>& methods, bool clinit) {
          akka::ClassModel c;
          c.name = name;
          c.mods = mods;
          c.interfaces = std::move(interfaces);
          for (auto& f : fields) c.fields.push_back({std::get<0>(f), std::get<1>(f), std::get<2>(f)});
          for (auto& k : ctors) c.ctors.push_back({"<init>", std::get<0>(k), std::get<1>(k)});
          for (auto& x : methods) c.methods.push_back({std::get<0>(x), std::get<1>(x), std::get<2>(x)});
          c.has_clinit = clinit;
          return akka::default_suid(c);
        },
        py::arg("name"), py::arg("mods"), py::arg("interfaces"), py::arg("fields"), py::arg("ctors"),
        py::arg("methods"), py::arg("clinit") = false, "java.io.ObjectStreamClass.computeDefaultSUID of a class model");
  m.def("java_serialize",
        [](const std::string& fqcn, int64_t suid, const std::vector<std::tuple<std::string, std::string, py::object>>& fs) {
          akka::JavaObject o;
          o.class_name = fqcn;
          o.suid = suid;
          for (auto& f : fs) {
            akka::JavaField jf;
            if (std::get<0>(f).size() != 1) throw py::value_error("field types are JVM primitive type codes");
            jf.type = std::get<0>(f)[0];
            jf.name = std::get<1>(f);
            if (jf.type == 'F' || jf.type == 'D') jf.d = std::get<2>(f).cast<double>();
            else jf.i = std::get<2>(f).cast<int64_t>();
            o.fields.push_back(jf);
          }
          return B(akka::java_serialize(o));
        });
  m.def("java_deserialize", [](const std::string& b) {
    akka::JavaObject o;
    std::string err;
    if (!akka::java_deserialize(b, o, &err)) throw py::value_error(err);
    py::list fs;
    for (auto& f : o.fields) {
      py::object v = (f.type == 'F' || f.type == 'D') ? py::object(py::float_(f.d)) : py::object(py::int_(f.i));
      fs.append(py::make_tuple(std::string(1, f.type), f.name, v));
    }
    return py::make_tuple(o.class_name, o.suid, fs);
  });
  m.def("encode_associate",
        [](const std::string& system, const std::string& host, uint32_t port, uint64_t uid, const std::string& cookie,
           const std::string& protocol) {
          akka::Address a;
          a.protocol = protocol;
          a.system = system;
          a.host = host;
          a.port = port;
          return B(akka::encode_associate(a, uid, cookie));
        },
        py::arg("system"), py::arg("host"), py::arg("port"), py::arg("uid"), py::arg("cookie") = "",
        py::arg("protocol") = "akka.tcp");
  m.def("encode_control", [](int c) { return B(akka::encode_control(c)); });
  m.def("encode_payload_pdu", [](const std::string& c) { return B(akka::encode_payload_pdu(c)); });
  m.def("decode_pdu", [](const std::string& b) {
    akka::Pdu p;
    if (!akka::decode_pdu(b, p)) throw py::value_error("malformed AkkaProtocolMessage");
    py::dict d;
    if (p.is_payload) {
      d["payload"] = B(p.payload);
      return d;
    }
    d["command"] = p.command;
    if (p.has_handshake) {
      d["origin"] = addr_dict(p.origin);
      d["uid"] = p.uid;
      d["cookie"] = p.cookie;
    }
    return d;
  });
  m.def("encode_container", [](py::dict d) {
    akka::Envelope e;
    if (d.contains("ack") && !d["ack"].is_none()) {
      e.has_ack = true;
      py::dict a = d["ack"];
      e.cumulative_ack = a["cumulativeAck"].cast<uint64_t>();
      if (a.contains("nacks")) e.nacks = a["nacks"].cast<std::vector<uint64_t>>();
    }
    if (d.contains("envelope") && !d["envelope"].is_none()) {
      py::dict v = d["envelope"];
      e.has_envelope = true;
      e.recipient = v["recipient"].cast<std::string>();
      e.msg = msg_from(v["message"]);
      if (v.contains("sender") && !v["sender"].is_none()) {
        e.has_sender = true;
        e.sender = v["sender"].cast<std::string>();
      }
      if (v.contains("seq") && !v["seq"].is_none()) {
        e.has_seq = true;
        e.seq = v["seq"].cast<uint64_t>();
      }
    }
    return B(akka::encode_container(e));
  });
  m.def("decode_container", [](const std::string& b) {
    akka::Envelope e;
    if (!akka::decode_container(b, e)) throw py::value_error("malformed AckAndEnvelopeContainer");
    py::dict d;
    if (e.has_ack) {
      py::dict a;
      a["cumulativeAck"] = e.cumulative_ack;
      a["nacks"] = e.nacks;
      d["ack"] = a;
    }
    if (e.has_envelope) {
      py::dict v;
      v["recipient"] = e.recipient;
      v["message"] = msg_dict(e.msg);
      v["sender"] = e.has_sender ? py::object(py::str(e.sender)) : py::object(py::none());
      v["seq"] = e.has_seq ? py::object(py::int_(e.seq)) : py::object(py::none());
      d["envelope"] = v;
    }
    return d;
  });
  m.def("encode_selection", [](py::dict inner, const std::vector<std::pair<int, std::string>>& pattern, bool wildcard) {
    std::vector<akka::Selection> ps;
    for (auto& p : pattern) ps.push_back({p.first, p.second});
    return B(akka::encode_selection(msg_from(inner), ps, wildcard));
  }, py::arg("inner"), py::arg("pattern"), py::arg("wildcard") = false);
  m.def("decode_selection", [](const std::string& b) {
    akka::SerializedMsg inner;
    std::vector<akka::Selection> ps;
    bool wc = false;
    if (!akka::decode_selection(b, inner, ps, wc)) throw py::value_error("malformed SelectionEnvelope");
    std::vector<std::pair<int, std::string>> pat;
    for (auto& p : ps) pat.emplace_back(p.type, p.matcher);
    return py::make_tuple(msg_dict(inner), pat, wc);
  });
  m.def("parse_actor_path", [](const std::string& p) -> py::object {
    akka::Address a;
    std::vector<std::string> el;
    if (!akka::parse_actor_path(p, a, el)) return py::none();
    return py::make_tuple(addr_dict(a), el);
  });

  using Stats = AkkaEndpoint::Stats;
  py::class_<AkkaEndpoint, std::shared_ptr<AkkaEndpoint>>(m, "Endpoint")
      .def_property_readonly("port", &AkkaEndpoint::port)
      .def_property_readonly("address", &AkkaEndpoint::address)
      .def_property_readonly("master_path", &AkkaEndpoint::master_path)
      .def_property_readonly("suid_start", &AkkaEndpoint::suid_start)
      .def_property_readonly("suid_complete", &AkkaEndpoint::suid_complete)
      .def("associations", &AkkaEndpoint::associations)
      .def("stats", [](const AkkaEndpoint& e) {
        const Stats s = e.stats();
        py::dict d;
        d["associations"] = s.associations;
        d["frames_in"] = s.frames_in;
        d["frames_out"] = s.frames_out;
        d["starts"] = s.starts;
        d["completes_sent"] = s.completes_sent;
        d["identifies"] = s.identifies;
        d["watcher_heartbeats"] = s.watcher_heartbeats;
        d["system_messages"] = s.system_messages;
        d["unsupported"] = s.unsupported;
        d["suid_mismatches"] = s.suid_mismatches;
        d["rejected"] = s.rejected;
        d["client_suid_start"] = s.client_suid_start;
        return d;
      })
      .def("stop", &AkkaEndpoint::stop, py::call_guard<py::gil_scoped_release>());

  // system.akka_endpoint(master, ...): serve the master's bridge as akka.tcp (the master must
  // have a control bridge: system.master(..., bridgePort=0))
  m.def("start_endpoint",
        [](ActorRef master, int port, const std::string& host, const std::string& system, const std::string& name,
           const std::string& package, int64_t suid_start, int64_t suid_complete, double heartbeat_s,
           const std::string& cookie) {
          auto* ma = master_actor(master);
          if (!ma->bridge()) throw py::value_error("the master has no control bridge (bridgePort >= 0)");
          AkkaEndpoint::Options o;
          o.host = host;
          o.port = port;
          o.system = system;
          o.master = name;
          o.package = package;
          o.suid_start = suid_start;
          o.suid_complete = suid_complete;
          o.heartbeat_s = heartbeat_s;
          o.cookie = cookie;
          return AkkaEndpoint::start(ma->bridge(), o);
        },
        py::arg("master"), py::arg("port") = 0, py::arg("host") = "127.0.0.1", py::arg("system") = "ClusterSystem",
        py::arg("name") = "master", py::arg("package") = "sample.cluster.allreduce", py::arg("suid_start") = 0,
        py::arg("suid_complete") = 0, py::arg("heartbeat_s") = 1.0, py::arg("cookie") = "");
}

}  // namespace mxar
