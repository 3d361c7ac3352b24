// Akka classic remoting on the wire (akka-remote 2.5, the reference's build.sbt:3 akkaVersion
// 2.5.4, transport `akka.remote.netty.tcp` of its application.conf:5-9), for the control
// endpoint in csrc/runtime/akka_endpoint.h.
//
// Layers, outermost first:
//   TCP frame          u32 big-endian length + body (Netty LengthFieldPrepender(4)); the
//                      reference's transport caps a frame at 128000 bytes (kMaxFrame)
//   AkkaProtocolMessage { payload bytes = 1 | instruction AkkaControlMessage = 2 }
//                      ASSOCIATE (handshake: origin AddressData, uid, cookie), HEARTBEAT,
//                      DISASSOCIATE* -- both sides send ASSOCIATE once per connection
//   AckAndEnvelopeContainer { ack = 1, envelope = 2 }
//   RemoteEnvelope     { recipient ActorRefData = 1, message SerializedMessage = 2,
//                        sender ActorRefData = 4, seq fixed64 = 5 (system messages only) }
//   SerializedMessage  { message bytes = 1, serializerId int32 = 2, messageManifest = 3 }
// Serializers spoken: 1 java (the reference's case classes, AllreduceMessage.scala:7-20: no
// serializer binding, so Akka falls back to Java serialization), 6 message container
// (ActorSelection: SelectionEnvelope), 16 misc (Identify / ActorIdentity, the remote
// watcher's heartbeat and its response).
//
// Java serialization (java.io.ObjectOutputStream, stream version 5) is supported for flat
// classes of primitive fields - every reference message but InitWorkers (which carries a
// Map[Int, ActorRef] and is never sent to a client here). A receiver checks the class's
// serialVersionUID: the reference's case classes declare none, so the JVM computes the
// default one (java.io.ObjectStreamClass.computeDefaultSUID: SHA-1 over the class's name,
// modifiers, interfaces, fields, constructors and methods). `scala_case_class_model` lists
// the members scalac 2.12 emits for a final case class of primitive parameters and
// `default_suid` hashes them the JVM's way. No JVM exists in this image, so the SUIDs are
// parity-unpinned: the endpoint compares its model with the SUID a client's StartAllreduce
// carries and reports a mismatch, and `mxar.akka.suid.*` overrides it (docs/AKKA_WIRE.md).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace mxar {
namespace akka {

constexpr size_t kMaxFrame = 128000;  // akka.remote.netty.tcp.maximum-frame-size default

// ---- protobuf (proto2) wire primitives ---------------------------------------------------

class PbWriter {
 public:
  void varint(uint32_t field, uint64_t v);
  void fixed64(uint32_t field, uint64_t v);
  void bytes(uint32_t field, std::string_view b);
  const std::string& str() const { return buf_; }
  std::string take() { return std::move(buf_); }

 private:
  void raw_varint(uint64_t v);
  std::string buf_;
};

struct PbField {
  uint32_t num = 0;
  uint8_t wire = 0;       // 0 varint, 1 fixed64, 2 length-delimited, 5 fixed32
  uint64_t v = 0;         // varint / fixed value
  std::string_view data;  // length-delimited body (a view into the parsed buffer)
};

// One message level. False on a malformed buffer (truncated, bad wire type, groups).
bool pb_parse(std::string_view buf, std::vector<PbField>& out);

// ---- Akka addresses and PDUs -------------------------------------------------------------

struct Address {
  std::string protocol = "akka.tcp";
  std::string system;
  std::string host;
  uint32_t port = 0;
  std::string str() const;  // akka.tcp://System@host:port
};
// "akka.tcp://Sys@host:port/user/a#123" -> address and the path elements ("user", "a"),
// the "#uid" suffix dropped. False when the text is not an actor path with an address.
bool parse_actor_path(std::string_view path, Address& addr, std::vector<std::string>& elems);

enum Command : int { kAssociate = 1, kDisassociate = 2, kHeartbeat = 3, kShuttingDown = 4, kQuarantined = 5 };

struct Pdu {
  bool is_payload = false;
  std::string payload;  // is_payload: an AckAndEnvelopeContainer
  int command = 0;      // !is_payload
  bool has_handshake = false;
  Address origin;
  uint64_t uid = 0;
  std::string cookie;
};

std::string encode_associate(const Address& origin, uint64_t uid, const std::string& cookie = "");
std::string encode_control(int command);
std::string encode_payload_pdu(std::string_view container);
bool decode_pdu(std::string_view body, Pdu& out);

struct SerializedMsg {
  std::string bytes;
  int32_t serializer = 0;
  bool has_manifest = false;
  std::string manifest;
};

struct Envelope {
  bool has_ack = false;
  uint64_t cumulative_ack = 0;
  std::vector<uint64_t> nacks;
  bool has_envelope = false;
  std::string recipient;
  bool has_sender = false;
  std::string sender;
  bool has_seq = false;
  uint64_t seq = 0;
  SerializedMsg msg;
};

std::string encode_container(const Envelope& e);
bool decode_container(std::string_view body, Envelope& out);

// ActorSelection (serializer 6): the enclosed message and the pattern below the anchor.
struct Selection {
  int type = 1;  // 0 PARENT, 1 CHILD_NAME, 2 CHILD_PATTERN
  std::string matcher;
};
std::string encode_selection(const SerializedMsg& inner, const std::vector<Selection>& pattern, bool wildcard);
bool decode_selection(std::string_view body, SerializedMsg& inner, std::vector<Selection>& pattern, bool& wildcard);

// Serializer ids and misc-serializer manifests (akka-remote 2.5 reference.conf bindings).
constexpr int32_t kJavaSerializer = 1;
constexpr int32_t kContainerSerializer = 6;
constexpr int32_t kMiscSerializer = 16;
constexpr const char* kIdentifyManifest = "A";
constexpr const char* kActorIdentityManifest = "B";
constexpr const char* kWatcherHeartbeatManifest = "RH";
constexpr const char* kWatcherHeartbeatRspManifest = "RHR";

// Identify{messageId Payload = 1}: the raw Payload bytes (echoed verbatim in the reply).
bool decode_identify(std::string_view body, std::string& message_id_payload);
// ActorIdentity{correlationId Payload = 1, ref ActorRef{path = 1} = 2}; empty path = None.
std::string encode_actor_identity(std::string_view message_id_payload, const std::string& ref_path);
// RemoteWatcher.HeartbeatRsp{uid uint64 = 1} (the Int address uid, sign-extended).
std::string encode_heartbeat_rsp(int32_t address_uid);

// ---- Java serialization of flat case classes ---------------------------------------------

struct JavaField {
  char type = 'I';  // JVM type code: B C D F I J S Z
  std::string name;
  int64_t i = 0;    // integral types and Z / C
  double d = 0.0;   // F / D
};

struct JavaObject {
  std::string class_name;
  int64_t suid = 0;
  std::vector<JavaField> fields;  // any order; the stream uses ObjectStreamClass's
};

std::string java_serialize(const JavaObject& o);
// Reads one object of a class (and superclasses) with primitive fields only.
bool java_deserialize(std::string_view b, JavaObject& o, std::string* err = nullptr);

// ---- serialVersionUID ---------------------------------------------------------------------

struct ClassModel {
  struct Member {
    std::string name;
    int mods = 0;
    std::string desc;  // JVM descriptor with '/' separators
  };
  std::string name;  // binary name with dots
  int mods = 0;      // class access flags
  std::vector<std::string> interfaces;
  std::vector<Member> fields, ctors, methods;
  bool has_clinit = false;
};

// java.io.ObjectStreamClass.computeDefaultSUID over the model.
int64_t default_suid(const ClassModel& m);
// The members scalac 2.12 emits for `final case class Name(p1: T1, ...)` with primitive
// parameters (JVM type codes) and a synthetic companion: fields, constructor, accessors,
// copy / copy$default$k, the Product / Equals / Any overrides and the companion's static
// forwarders (apply, unapply, and andThen / compose for one parameter, tupled / curried for
// more).
ClassModel scala_case_class_model(const std::string& fqcn, const std::vector<std::pair<std::string, char>>& params);

std::string sha1(std::string_view data);  // 20 raw bytes

}  // namespace akka
}  // namespace mxar
