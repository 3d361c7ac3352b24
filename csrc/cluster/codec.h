// Binary wire codec for the cluster transport (replaces Akka classic remoting's Java
// serialization of the reference's case classes).
//
// Frame on the wire: u32 little-endian length, then `length` bytes starting with a u8
// frame kind. Strings are u32 length + bytes; float payloads are u32 count + raw IEEE
// little-endian floats. Actor refs travel as full addresses
// "mxar.tcp://<System>@<host>:<port>/user/<name>" and are re-materialised on the
// receiving node (local lookup when the address is its own, a RemoteActorRef otherwise).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../core/protocol.h"

namespace mxar {

enum class FrameKind : uint8_t {
  Hello = 1,        // {address}
  Envelope = 2,     // {sender full path | "", target path, Message}
  Join = 3,         // {address, roles[], uid}
  Welcome = 4,      // {members[]}
  MemberEvent = 5,  // {event, member}
  Heartbeat = 6,    // {from address, seq}
  Leave = 7,        // {address}
  // same-host fast path (shm_ring.h): the connecting node offers a ring, the peer maps it and
  // acks over its own connection, the offerer sends ShmSwitch over TCP and the ring from then on
  ShmOffer = 8,     // {ring name}
  ShmAck = 9,       // {acker address, ring name, ok}
  ShmSwitch = 10,   // {}
};

enum class MemberStatus : uint8_t { Joining = 0, Up = 1, Leaving = 2, Down = 3, Removed = 4 };
enum class MemberEventKind : uint8_t { Up = 1, Removed = 2, Unreachable = 3, Reachable = 4 };

struct MemberInfo {
  std::string address;
  std::vector<std::string> roles;
  uint64_t uid = 0;
  MemberStatus status = MemberStatus::Up;
  std::string meta;  // ClusterConfig.meta of the member (e.g. a GPU worker's plane descriptor)
  bool has_role(const std::string& r) const {
    for (auto& x : roles)
      if (x == r) return true;
    return false;
  }
};

class CodecError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class Writer {
 public:
  void u8(uint8_t v) { buf_.push_back(v); }
  void u32(uint32_t v) { raw(&v, 4); }
  void i32(int32_t v) { raw(&v, 4); }
  void i64(int64_t v) { raw(&v, 8); }
  void u64(uint64_t v) { raw(&v, 8); }
  void f32(float v) { raw(&v, 4); }
  void str(const std::string& s) {
    u32(static_cast<uint32_t>(s.size()));
    raw(s.data(), s.size());
  }
  void floats(const float* p, size_t n) {
    u32(static_cast<uint32_t>(n));
    raw(p, n * sizeof(float));
  }
  void raw(const void* p, size_t n) {
    const auto* b = static_cast<const uint8_t*>(p);
    buf_.insert(buf_.end(), b, b + n);
  }
  std::vector<uint8_t>& bytes() { return buf_; }

 private:
  std::vector<uint8_t> buf_;
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  uint8_t u8() { return get<uint8_t>(); }
  uint32_t u32() { return get<uint32_t>(); }
  int32_t i32() { return get<int32_t>(); }
  int64_t i64() { return get<int64_t>(); }
  uint64_t u64() { return get<uint64_t>(); }
  float f32() { return get<float>(); }
  std::string str() {
    const uint32_t n = u32();
    need(n);
    std::string s(reinterpret_cast<const char*>(p_ + off_), n);
    off_ += n;
    return s;
  }
  std::vector<float> floats() {
    const uint32_t n = u32();
    need(static_cast<size_t>(n) * 4);
    std::vector<float> v(n);
    if (n) std::memcpy(v.data(), p_ + off_, static_cast<size_t>(n) * 4);
    off_ += static_cast<size_t>(n) * 4;
    return v;
  }
  bool done() const { return off_ == n_; }

 private:
  template <class T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p_ + off_, sizeof(T));
    off_ += sizeof(T);
    return v;
  }
  void need(size_t k) const {
    if (off_ + k > n_) throw CodecError("truncated frame");
  }
  const uint8_t* p_;
  size_t n_;
  size_t off_ = 0;
};

// Ref <-> string hooks supplied by the cluster node.
struct RefCodec {
  virtual ~RefCodec() = default;
  virtual std::string encode_ref(const ActorRef& r) const = 0;  // "" for null
  virtual ActorRef decode_ref(const std::string& s) = 0;          // nullptr for ""
};

void encode_message(Writer& w, const Message& m, const RefCodec& rc);
Message decode_message(Reader& r, RefCodec& rc);
void encode_member(Writer& w, const MemberInfo& m);
MemberInfo decode_member(Reader& r);

// "mxar.tcp://Sys@host:port/user/x" -> {"mxar.tcp://Sys@host:port", "/user/x"}
// (also accepts the reference's "akka.tcp://" scheme).
std::pair<std::string, std::string> split_ref(const std::string& full);
// "mxar.tcp://Sys@host:port" -> {host, port}; throws on malformed input.
std::pair<std::string, int> parse_address(const std::string& address);
std::string make_address(const std::string& system, const std::string& host, int port);

}  // namespace mxar
