// Python bindings of the cluster layer (csrc/cluster): ClusterConfig, ClusterNode.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../cluster/cluster_node.h"

namespace py = pybind11;

namespace mxar {

static py::dict member_dict(const MemberInfo& m) {
  py::dict d;
  d["address"] = m.address;
  d["roles"] = m.roles;
  d["uid"] = m.uid;
  d["status"] = static_cast<int>(m.status);
  d["meta"] = m.meta;
  return d;
}

void bind_cluster(py::module_& m) {
  py::class_<ClusterConfig>(m, "ClusterConfig")
      .def(py::init<>())
      .def_readwrite("host", &ClusterConfig::host)
      .def_readwrite("port", &ClusterConfig::port)
      .def_readwrite("roles", &ClusterConfig::roles)
      .def_readwrite("seed_nodes", &ClusterConfig::seed_nodes)
      .def_readwrite("heartbeat_interval_s", &ClusterConfig::heartbeat_interval_s)
      .def_readwrite("acceptable_heartbeat_pause_s", &ClusterConfig::acceptable_heartbeat_pause_s)
      .def_readwrite("auto_down_unreachable_after_s", &ClusterConfig::auto_down_unreachable_after_s)
      .def_readwrite("connect_timeout_s", &ClusterConfig::connect_timeout_s)
      .def_readwrite("worker_path", &ClusterConfig::worker_path)
      .def_readwrite("meta", &ClusterConfig::meta);

  py::class_<ClusterStats>(m, "ClusterStats")
      .def_readonly("frames_out", &ClusterStats::frames_out)
      .def_readonly("frames_in", &ClusterStats::frames_in)
      .def_readonly("bytes_out", &ClusterStats::bytes_out)
      .def_readonly("bytes_in", &ClusterStats::bytes_in)
      .def_readonly("connects", &ClusterStats::connects)
      .def_readonly("connect_failures", &ClusterStats::connect_failures)
      .def_readonly("send_failures", &ClusterStats::send_failures)
      .def_readonly("undeliverable", &ClusterStats::undeliverable)
      .def_readonly("decode_errors", &ClusterStats::decode_errors)
      .def_readonly("members_up", &ClusterStats::members_up)
      .def_readonly("members_removed", &ClusterStats::members_removed)
      .def_readonly("heartbeats_in", &ClusterStats::heartbeats_in);

  py::class_<ClusterNode, std::shared_ptr<ClusterNode>>(m, "ClusterNode")
      .def_static(
          "start",
          [](std::shared_ptr<ActorSystem> sys, const ClusterConfig& cfg) {
            py::gil_scoped_release r;
            return ClusterNode::start(std::move(sys), cfg);
          },
          py::arg("system"), py::arg("config"))
      .def_property_readonly("address", &ClusterNode::address)
      .def_property_readonly("port", &ClusterNode::port)
      .def_property_readonly("joined", &ClusterNode::joined)
      .def("resolve", &ClusterNode::resolve, py::arg("path"))
      .def("subscribe", &ClusterNode::subscribe)
      .def("unsubscribe", &ClusterNode::unsubscribe)
      .def("members",
           [](ClusterNode& n) {
             py::list l;
             for (auto& x : n.members()) l.append(member_dict(x));
             return l;
           })
      .def("leader", &ClusterNode::leader)
      .def("is_unreachable", &ClusterNode::is_unreachable)
      .def("leave", [](ClusterNode& n) {
        py::gil_scoped_release r;
        n.leave();
      })
      .def("shutdown", [](ClusterNode& n) {
        py::gil_scoped_release r;
        n.shutdown();
      })
      .def("stats", &ClusterNode::stats);
  m.def("normalize_address", &normalize_address);
  m.def("make_address", &make_address);
}

}  // namespace mxar
