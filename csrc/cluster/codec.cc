#include "codec.h"

#include <type_traits>

namespace mxar {

static void put_payload(Writer& w, const Payload& p) {
  if (!p) {
    w.floats(nullptr, 0);
    return;
  }
  if (p->on_device()) {
    const std::vector<float> h = p->to_host();
    w.floats(h.data(), h.size());
  } else {
    w.floats(p->data(), p->size());
  }
}

void encode_message(Writer& w, const Message& m, const RefCodec& rc) {
  w.u8(static_cast<uint8_t>(m.index()));
  std::visit(
      [&](const auto& x) {
        using T = std::decay_t<decltype(x)>;
        if constexpr (std::is_same_v<T, InitWorkers>) {
          w.u32(static_cast<uint32_t>(x.workers.size()));
          for (auto& [id, ref] : x.workers) {
            w.i32(id);
            w.str(rc.encode_ref(ref));
          }
          w.str(rc.encode_ref(x.master));
          w.i32(x.destId);
          w.f32(x.thReduce);
          w.f32(x.thComplete);
          w.i32(x.maxLag);
          w.i32(x.dataSize);
          w.i32(x.maxChunkSize);
          w.i64(x.epoch);
          w.i32(x.startRound);
          w.u32(static_cast<uint32_t>(x.planes.size()));
          for (auto& [id, d] : x.planes) {
            w.i32(id);
            w.str(d);
          }
          w.u32(x.roundBase);
        } else if constexpr (std::is_same_v<T, StartAllreduce>) {
          w.i32(x.round);
          w.i64(x.epoch);
        } else if constexpr (std::is_same_v<T, ScatterBlock>) {
          put_payload(w, x.value);
          w.i32(x.srcId);
          w.i32(x.destId);
          w.i32(x.chunkId);
          w.i32(x.round);
          w.i64(x.epoch);
        } else if constexpr (std::is_same_v<T, ReduceBlock>) {
          put_payload(w, x.value);
          w.i32(x.srcId);
          w.i32(x.destId);
          w.i32(x.chunkId);
          w.i32(x.round);
          w.i32(x.count);
          w.i64(x.epoch);
        } else if constexpr (std::is_same_v<T, CompleteAllreduce>) {
          w.i32(x.srcId);
          w.i32(x.round);
          w.i64(x.epoch);
        } else if constexpr (std::is_same_v<T, MemberUp>) {
          w.str(rc.encode_ref(x.ref));
          w.str(x.role);
          w.str(x.address);
          w.str(x.meta);
        } else if constexpr (std::is_same_v<T, Terminated>) {
          w.str(rc.encode_ref(x.ref));
        } else if constexpr (std::is_same_v<T, AllreduceFinished>) {
          w.i32(x.rounds);
        } else if constexpr (std::is_same_v<T, PoisonPill>) {
        } else if constexpr (std::is_same_v<T, TextMessage>) {
          w.str(x.text);
        } else if constexpr (std::is_same_v<T, RoundTimeout>) {
          w.i64(x.epoch);
          w.i32(x.round);
        } else if constexpr (std::is_same_v<T, PlaneRoundDone>) {
          // process-local (a plane's completion to its own worker); never crosses a node
          throw CodecError("PlaneRoundDone is local to a node");
        } else if constexpr (std::is_same_v<T, BridgeCommand>) {
          throw CodecError("BridgeCommand is local to a node");  // bridge client -> its own master
        }
      },
      m);
}

Message decode_message(Reader& r, RefCodec& rc) {
  const uint8_t kind = r.u8();
  switch (kind) {
    case 0: {
      InitWorkers x;
      const uint32_t n = r.u32();
      for (uint32_t i = 0; i < n; ++i) {
        const int id = r.i32();
        x.workers[id] = rc.decode_ref(r.str());
      }
      x.master = rc.decode_ref(r.str());
      x.destId = r.i32();
      x.thReduce = r.f32();
      x.thComplete = r.f32();
      x.maxLag = r.i32();
      x.dataSize = r.i32();
      x.maxChunkSize = r.i32();
      x.epoch = r.i64();
      x.startRound = r.i32();
      const uint32_t np = r.u32();
      for (uint32_t i = 0; i < np; ++i) {
        const int id = r.i32();
        x.planes[id] = r.str();
      }
      x.roundBase = r.u32();
      return x;
    }
    case 1: {
      StartAllreduce x;
      x.round = r.i32();
      x.epoch = r.i64();
      return x;
    }
    case 2: {
      ScatterBlock x;
      x.value = make_host_payload(r.floats());
      x.srcId = r.i32();
      x.destId = r.i32();
      x.chunkId = r.i32();
      x.round = r.i32();
      x.epoch = r.i64();
      return x;
    }
    case 3: {
      ReduceBlock x;
      x.value = make_host_payload(r.floats());
      x.srcId = r.i32();
      x.destId = r.i32();
      x.chunkId = r.i32();
      x.round = r.i32();
      x.count = r.i32();
      x.epoch = r.i64();
      return x;
    }
    case 4: {
      CompleteAllreduce x;
      x.srcId = r.i32();
      x.round = r.i32();
      x.epoch = r.i64();
      return x;
    }
    case 5: {
      MemberUp x;
      x.ref = rc.decode_ref(r.str());
      x.role = r.str();
      x.address = r.str();
      x.meta = r.str();
      return x;
    }
    case 6:
      return Terminated{rc.decode_ref(r.str())};
    case 7:
      return AllreduceFinished{r.i32()};
    case 8:
      return PoisonPill{};
    case 9:
      return TextMessage{r.str()};
    case 10: {
      RoundTimeout x;
      x.epoch = r.i64();
      x.round = r.i32();
      return x;
    }
    default:
      throw CodecError("unknown message kind " + std::to_string(kind));
  }
}

void encode_member(Writer& w, const MemberInfo& m) {
  w.str(m.address);
  w.u32(static_cast<uint32_t>(m.roles.size()));
  for (auto& s : m.roles) w.str(s);
  w.u64(m.uid);
  w.u8(static_cast<uint8_t>(m.status));
  w.str(m.meta);
}

MemberInfo decode_member(Reader& r) {
  MemberInfo m;
  m.address = r.str();
  const uint32_t n = r.u32();
  for (uint32_t i = 0; i < n; ++i) m.roles.push_back(r.str());
  m.uid = r.u64();
  m.status = static_cast<MemberStatus>(r.u8());
  m.meta = r.str();
  return m;
}

std::pair<std::string, std::string> split_ref(const std::string& full) {
  const size_t scheme = full.find("://");
  if (scheme == std::string::npos) return {"", full};  // already a local path
  const size_t slash = full.find('/', scheme + 3);
  if (slash == std::string::npos) return {full, ""};
  return {full.substr(0, slash), full.substr(slash)};
}

std::pair<std::string, int> parse_address(const std::string& address) {
  const size_t at = address.find('@');
  const size_t colon = address.rfind(':');
  if (at == std::string::npos || colon == std::string::npos || colon < at)
    throw CodecError("malformed address: " + address);
  std::string host = address.substr(at + 1, colon - at - 1);
  const std::string port = address.substr(colon + 1);
  int p = 0;
  try {
    p = std::stoi(port);
  } catch (...) {
    throw CodecError("malformed port in address: " + address);
  }
  if (p <= 0 || p > 65535) throw CodecError("port out of range in address: " + address);
  return {host, p};
}

std::string make_address(const std::string& system, const std::string& host, int port) {
  return "mxar.tcp://" + system + "@" + host + ":" + std::to_string(port);
}

}  // namespace mxar
