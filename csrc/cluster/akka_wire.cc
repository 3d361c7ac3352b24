#include "akka_wire.h"

#include <algorithm>
#include <cstring>

namespace mxar {
namespace akka {

// ---- protobuf ------------------------------------------------------------------------------

void PbWriter::raw_varint(uint64_t v) {
  while (v >= 0x80) {
    buf_.push_back(static_cast<char>((v & 0x7f) | 0x80));
    v >>= 7;
  }
  buf_.push_back(static_cast<char>(v));
}

void PbWriter::varint(uint32_t field, uint64_t v) {
  raw_varint(static_cast<uint64_t>(field) << 3 | 0);
  raw_varint(v);
}

void PbWriter::fixed64(uint32_t field, uint64_t v) {
  raw_varint(static_cast<uint64_t>(field) << 3 | 1);
  for (int i = 0; i < 8; ++i) buf_.push_back(static_cast<char>(v >> (8 * i)));
}

void PbWriter::bytes(uint32_t field, std::string_view b) {
  raw_varint(static_cast<uint64_t>(field) << 3 | 2);
  raw_varint(b.size());
  buf_.append(b.data(), b.size());
}

namespace {

bool read_varint(std::string_view b, size_t& i, uint64_t& v) {
  v = 0;
  for (int shift = 0; shift < 64; shift += 7) {
    if (i >= b.size()) return false;
    const uint8_t c = static_cast<uint8_t>(b[i++]);
    v |= static_cast<uint64_t>(c & 0x7f) << shift;
    if (!(c & 0x80)) return true;
  }
  return false;
}

const PbField* find(const std::vector<PbField>& fs, uint32_t num, uint8_t wire) {
  const PbField* last = nullptr;  // proto2: the last occurrence of a singular field wins
  for (auto& f : fs)
    if (f.num == num && f.wire == wire) last = &f;
  return last;
}

std::string sv(std::string_view v) { return std::string(v.data(), v.size()); }

}  // namespace

bool pb_parse(std::string_view b, std::vector<PbField>& out) {
  out.clear();
  size_t i = 0;
  while (i < b.size()) {
    uint64_t key;
    if (!read_varint(b, i, key)) return false;
    PbField f;
    f.num = static_cast<uint32_t>(key >> 3);
    f.wire = static_cast<uint8_t>(key & 7);
    if (f.num == 0) return false;
    switch (f.wire) {
      case 0:
        if (!read_varint(b, i, f.v)) return false;
        break;
      case 1:
        if (b.size() - i < 8) return false;
        for (int k = 0; k < 8; ++k) f.v |= static_cast<uint64_t>(static_cast<uint8_t>(b[i + k])) << (8 * k);
        i += 8;
        break;
      case 2: {
        uint64_t n;
        if (!read_varint(b, i, n) || n > b.size() - i) return false;
        f.data = b.substr(i, n);
        i += n;
        break;
      }
      case 5:
        if (b.size() - i < 4) return false;
        for (int k = 0; k < 4; ++k) f.v |= static_cast<uint64_t>(static_cast<uint8_t>(b[i + k])) << (8 * k);
        i += 4;
        break;
      default:
        return false;  // groups (3/4) never appear in these schemas
    }
    out.push_back(f);
  }
  return true;
}

// ---- addresses and PDUs ---------------------------------------------------------------------

std::string Address::str() const { return protocol + "://" + system + "@" + host + ":" + std::to_string(port); }

bool parse_actor_path(std::string_view p, Address& a, std::vector<std::string>& elems) {
  elems.clear();
  const size_t proto_end = p.find("://");
  if (proto_end == std::string_view::npos) return false;
  a.protocol = sv(p.substr(0, proto_end));
  std::string_view rest = p.substr(proto_end + 3);
  const size_t at = rest.find('@');
  const size_t slash = rest.find('/');
  if (at == std::string_view::npos || (slash != std::string_view::npos && slash < at)) return false;
  a.system = sv(rest.substr(0, at));
  std::string_view hp = rest.substr(at + 1, slash == std::string_view::npos ? std::string_view::npos : slash - at - 1);
  const size_t colon = hp.rfind(':');
  if (colon == std::string_view::npos) return false;
  a.host = sv(hp.substr(0, colon));
  uint64_t port = 0;
  for (char c : hp.substr(colon + 1)) {
    if (c < '0' || c > '9') return false;
    port = port * 10 + static_cast<uint64_t>(c - '0');
    if (port > 65535) return false;
  }
  a.port = static_cast<uint32_t>(port);
  if (slash == std::string_view::npos) return true;
  std::string_view path = rest.substr(slash);
  const size_t hash = path.find('#');
  if (hash != std::string_view::npos) path = path.substr(0, hash);
  size_t i = 0;
  while (i < path.size()) {
    while (i < path.size() && path[i] == '/') ++i;
    size_t j = i;
    while (j < path.size() && path[j] != '/') ++j;
    if (j > i) elems.push_back(sv(path.substr(i, j - i)));
    i = j;
  }
  return true;
}

namespace {

std::string encode_address(const Address& a) {
  PbWriter w;
  w.bytes(1, a.system);
  w.bytes(2, a.host);
  w.varint(3, a.port);
  w.bytes(4, a.protocol);
  return w.take();
}

bool decode_address(std::string_view b, Address& a) {
  std::vector<PbField> fs;
  if (!pb_parse(b, fs)) return false;
  auto sys = find(fs, 1, 2), host = find(fs, 2, 2), port = find(fs, 3, 0), proto = find(fs, 4, 2);
  if (!sys || !host || !port) return false;  // required fields
  a.system = sv(sys->data);
  a.host = sv(host->data);
  a.port = static_cast<uint32_t>(port->v);
  a.protocol = proto ? sv(proto->data) : std::string("akka.tcp");
  return true;
}

}  // namespace

std::string encode_associate(const Address& origin, uint64_t uid, const std::string& cookie) {
  PbWriter hs;
  hs.bytes(1, encode_address(origin));
  hs.fixed64(2, uid);
  if (!cookie.empty()) hs.bytes(3, cookie);
  PbWriter ctl;
  ctl.varint(1, kAssociate);
  ctl.bytes(2, hs.str());
  PbWriter pdu;
  pdu.bytes(2, ctl.str());
  return pdu.take();
}

std::string encode_control(int command) {
  PbWriter ctl;
  ctl.varint(1, static_cast<uint64_t>(command));
  PbWriter pdu;
  pdu.bytes(2, ctl.str());
  return pdu.take();
}

std::string encode_payload_pdu(std::string_view container) {
  PbWriter pdu;
  pdu.bytes(1, container);
  return pdu.take();
}

bool decode_pdu(std::string_view body, Pdu& out) {
  out = Pdu{};
  std::vector<PbField> fs;
  if (!pb_parse(body, fs)) return false;
  if (auto p = find(fs, 1, 2)) {
    out.is_payload = true;
    out.payload = sv(p->data);
    return true;
  }
  auto ins = find(fs, 2, 2);
  if (!ins) return false;
  std::vector<PbField> cf;
  if (!pb_parse(ins->data, cf)) return false;
  auto cmd = find(cf, 1, 0);
  if (!cmd) return false;
  out.command = static_cast<int>(cmd->v);
  if (auto hs = find(cf, 2, 2)) {
    std::vector<PbField> hf;
    if (!pb_parse(hs->data, hf)) return false;
    auto origin = find(hf, 1, 2), uid = find(hf, 2, 1), cookie = find(hf, 3, 2);
    if (!origin || !uid || !decode_address(origin->data, out.origin)) return false;
    out.has_handshake = true;
    out.uid = uid->v;
    if (cookie) out.cookie = sv(cookie->data);
  }
  return true;
}

namespace {

std::string encode_ref(const std::string& path) {
  PbWriter w;
  w.bytes(1, path);
  return w.take();
}

bool decode_ref(std::string_view b, std::string& path) {
  std::vector<PbField> fs;
  if (!pb_parse(b, fs)) return false;
  auto p = find(fs, 1, 2);
  if (!p) return false;
  path = sv(p->data);
  return true;
}

std::string encode_serialized(const SerializedMsg& m) {
  PbWriter w;
  w.bytes(1, m.bytes);
  w.varint(2, static_cast<uint64_t>(static_cast<int64_t>(m.serializer)));  // int32: sign-extended
  if (m.has_manifest) w.bytes(3, m.manifest);
  return w.take();
}

bool decode_serialized(std::string_view b, SerializedMsg& m) {
  std::vector<PbField> fs;
  if (!pb_parse(b, fs)) return false;
  auto msg = find(fs, 1, 2), ser = find(fs, 2, 0), man = find(fs, 3, 2);
  if (!msg || !ser) return false;
  m.bytes = sv(msg->data);
  m.serializer = static_cast<int32_t>(ser->v);
  m.has_manifest = man != nullptr;
  m.manifest = man ? sv(man->data) : std::string();
  return true;
}

}  // namespace

std::string encode_container(const Envelope& e) {
  PbWriter w;
  if (e.has_ack) {
    PbWriter ack;
    ack.fixed64(1, e.cumulative_ack);
    for (uint64_t n : e.nacks) ack.fixed64(2, n);
    w.bytes(1, ack.str());
  }
  if (e.has_envelope) {
    PbWriter env;
    env.bytes(1, encode_ref(e.recipient));
    env.bytes(2, encode_serialized(e.msg));
    if (e.has_sender) env.bytes(4, encode_ref(e.sender));
    if (e.has_seq) env.fixed64(5, e.seq);
    w.bytes(2, env.str());
  }
  return w.take();
}

bool decode_container(std::string_view body, Envelope& out) {
  out = Envelope{};
  std::vector<PbField> fs;
  if (!pb_parse(body, fs)) return false;
  if (auto a = find(fs, 1, 2)) {
    std::vector<PbField> af;
    if (!pb_parse(a->data, af)) return false;
    auto cum = find(af, 1, 1);
    if (!cum) return false;
    out.has_ack = true;
    out.cumulative_ack = cum->v;
    for (auto& f : af) {
      if (f.num != 2) continue;
      if (f.wire == 1) {
        out.nacks.push_back(f.v);
      } else if (f.wire == 2) {  // packed
        if (f.data.size() % 8) return false;
        for (size_t k = 0; k < f.data.size(); k += 8) {
          uint64_t v = 0;
          for (int j = 0; j < 8; ++j) v |= static_cast<uint64_t>(static_cast<uint8_t>(f.data[k + j])) << (8 * j);
          out.nacks.push_back(v);
        }
      }
    }
  }
  if (auto e = find(fs, 2, 2)) {
    std::vector<PbField> ef;
    if (!pb_parse(e->data, ef)) return false;
    auto rec = find(ef, 1, 2), msg = find(ef, 2, 2), snd = find(ef, 4, 2), seq = find(ef, 5, 1);
    if (!rec || !msg || !decode_ref(rec->data, out.recipient) || !decode_serialized(msg->data, out.msg)) return false;
    out.has_envelope = true;
    if (snd) {
      if (!decode_ref(snd->data, out.sender)) return false;
      out.has_sender = true;
    }
    if (seq) {
      out.has_seq = true;
      out.seq = seq->v;
    }
  }
  return true;
}

std::string encode_selection(const SerializedMsg& inner, const std::vector<Selection>& pattern, bool wildcard) {
  PbWriter w;
  w.bytes(1, inner.bytes);
  w.varint(2, static_cast<uint64_t>(static_cast<int64_t>(inner.serializer)));
  for (auto& s : pattern) {
    PbWriter p;
    p.varint(1, static_cast<uint64_t>(s.type));
    if (!s.matcher.empty()) p.bytes(2, s.matcher);
    w.bytes(3, p.str());
  }
  if (inner.has_manifest) w.bytes(4, inner.manifest);
  if (wildcard) w.varint(5, 1);
  return w.take();
}

bool decode_selection(std::string_view body, SerializedMsg& inner, std::vector<Selection>& pattern, bool& wildcard) {
  pattern.clear();
  std::vector<PbField> fs;
  if (!pb_parse(body, fs)) return false;
  auto msg = find(fs, 1, 2), ser = find(fs, 2, 0), man = find(fs, 4, 2), wc = find(fs, 5, 0);
  if (!msg || !ser) return false;
  inner.bytes = sv(msg->data);
  inner.serializer = static_cast<int32_t>(ser->v);
  inner.has_manifest = man != nullptr;
  inner.manifest = man ? sv(man->data) : std::string();
  wildcard = wc && wc->v != 0;
  for (auto& f : fs) {
    if (f.num != 3 || f.wire != 2) continue;
    std::vector<PbField> pf;
    if (!pb_parse(f.data, pf)) return false;
    auto t = find(pf, 1, 0), m = find(pf, 2, 2);
    if (!t) return false;
    Selection s;
    s.type = static_cast<int>(t->v);
    if (m) s.matcher = sv(m->data);
    pattern.push_back(std::move(s));
  }
  return true;
}

bool decode_identify(std::string_view body, std::string& payload) {
  std::vector<PbField> fs;
  if (!pb_parse(body, fs)) return false;
  auto p = find(fs, 1, 2);
  if (!p) return false;
  payload = sv(p->data);
  return true;
}

std::string encode_actor_identity(std::string_view message_id_payload, const std::string& ref_path) {
  PbWriter w;
  w.bytes(1, message_id_payload);
  if (!ref_path.empty()) w.bytes(2, encode_ref(ref_path));
  return w.take();
}

std::string encode_heartbeat_rsp(int32_t address_uid) {
  PbWriter w;
  w.varint(1, static_cast<uint64_t>(static_cast<int64_t>(address_uid)));
  return w.take();
}

// ---- Java serialization ----------------------------------------------------------------------

namespace {

constexpr uint8_t TC_NULL = 0x70, TC_CLASSDESC = 0x72, TC_OBJECT = 0x73, TC_STRING = 0x74,
                  TC_ENDBLOCKDATA = 0x78, TC_REFERENCE = 0x71;
constexpr uint8_t SC_WRITE_METHOD = 0x01, SC_SERIALIZABLE = 0x02, SC_EXTERNALIZABLE = 0x04;

int prim_size(char t) {
  switch (t) {
    case 'B': case 'Z': return 1;
    case 'C': case 'S': return 2;
    case 'I': case 'F': return 4;
    case 'J': case 'D': return 8;
    default: return -1;
  }
}

struct Out {
  std::string b;
  void u8(uint8_t v) { b.push_back(static_cast<char>(v)); }
  void be(uint64_t v, int n) {
    for (int k = n - 1; k >= 0; --k) b.push_back(static_cast<char>(v >> (8 * k)));
  }
  void utf(std::string_view s) {  // DataOutput.writeUTF (ASCII / pre-encoded modified UTF-8)
    be(s.size(), 2);
    b.append(s.data(), s.size());
  }
};

struct In {
  std::string_view b;
  size_t i = 0;
  bool ok = true;
  uint64_t be(int n) {
    if (b.size() - i < static_cast<size_t>(n)) {
      ok = false;
      return 0;
    }
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v = v << 8 | static_cast<uint8_t>(b[i + k]);
    i += static_cast<size_t>(n);
    return v;
  }
  uint8_t u8() { return static_cast<uint8_t>(be(1)); }
  std::string utf() {
    const size_t n = static_cast<size_t>(be(2));
    if (!ok || b.size() - i < n) {
      ok = false;
      return {};
    }
    std::string s = sv(b.substr(i, n));
    i += n;
    return s;
  }
};

bool fail(std::string* err, const std::string& why) {
  if (err) *err = why;
  return false;
}

void sort_fields(std::vector<JavaField>& fs) {  // ObjectStreamField.compareTo (all primitive here)
  std::sort(fs.begin(), fs.end(), [](const JavaField& a, const JavaField& b) { return a.name < b.name; });
}

}  // namespace

std::string java_serialize(const JavaObject& o) {
  std::vector<JavaField> fs = o.fields;
  sort_fields(fs);
  Out w;
  w.be(0xACED, 2);  // STREAM_MAGIC
  w.be(5, 2);       // STREAM_VERSION
  w.u8(TC_OBJECT);
  w.u8(TC_CLASSDESC);
  w.utf(o.class_name);
  w.be(static_cast<uint64_t>(o.suid), 8);
  w.u8(SC_SERIALIZABLE);
  w.be(fs.size(), 2);
  for (auto& f : fs) {
    w.u8(static_cast<uint8_t>(f.type));
    w.utf(f.name);
  }
  w.u8(TC_ENDBLOCKDATA);  // no class annotation
  w.u8(TC_NULL);          // superclass: java.lang.Object is not Serializable
  for (auto& f : fs) {
    switch (f.type) {
      case 'F': {
        float v = static_cast<float>(f.d);
        uint32_t u;
        std::memcpy(&u, &v, 4);
        w.be(u, 4);
        break;
      }
      case 'D': {
        uint64_t u;
        std::memcpy(&u, &f.d, 8);
        w.be(u, 8);
        break;
      }
      default:
        w.be(static_cast<uint64_t>(f.i), prim_size(f.type) > 0 ? prim_size(f.type) : 4);
    }
  }
  return w.b;
}

bool java_deserialize(std::string_view b, JavaObject& o, std::string* err) {
  o = JavaObject{};
  In r{b};
  if (r.be(2) != 0xACED || r.be(2) != 5) return fail(err, "not a Java serialization stream");
  if (r.u8() != TC_OBJECT) return fail(err, "stream does not start with an object");
  // class descriptors, most-derived first; the values are written least-derived first
  struct Desc {
    std::string name;
    int64_t suid;
    std::vector<JavaField> fields;
  };
  std::vector<Desc> chain;
  for (;;) {
    const uint8_t tc = r.u8();
    if (!r.ok) return fail(err, "truncated class descriptor");
    if (tc == TC_NULL) break;
    if (tc == TC_REFERENCE) return fail(err, "shared class descriptors are not supported");
    if (tc != TC_CLASSDESC) return fail(err, "unsupported class descriptor (proxy or unknown tag)");
    Desc d;
    d.name = r.utf();
    d.suid = static_cast<int64_t>(r.be(8));
    const uint8_t flags = r.u8();
    if (!(flags & SC_SERIALIZABLE) || (flags & (SC_EXTERNALIZABLE | SC_WRITE_METHOD)))
      return fail(err, d.name + ": only default-serialized classes are supported");
    const int n = static_cast<int>(r.be(2));
    for (int k = 0; k < n && r.ok; ++k) {
      JavaField f;
      f.type = static_cast<char>(r.u8());
      f.name = r.utf();
      if (prim_size(f.type) < 0) return fail(err, d.name + "." + f.name + ": object fields are not supported");
      d.fields.push_back(std::move(f));
    }
    if (r.u8() != TC_ENDBLOCKDATA) return fail(err, d.name + ": class annotations are not supported");
    if (!r.ok) return fail(err, "truncated class descriptor");
    chain.push_back(std::move(d));
  }
  if (chain.empty()) return fail(err, "no class descriptor");
  for (size_t c = chain.size(); c-- > 0;) {
    for (auto& f : chain[c].fields) {
      const uint64_t u = r.be(prim_size(f.type));
      switch (f.type) {
        case 'F': {
          uint32_t x = static_cast<uint32_t>(u);
          float v;
          std::memcpy(&v, &x, 4);
          f.d = v;
          break;
        }
        case 'D': std::memcpy(&f.d, &u, 8); break;
        case 'B': f.i = static_cast<int8_t>(u); break;
        case 'S': f.i = static_cast<int16_t>(u); break;
        case 'I': f.i = static_cast<int32_t>(u); break;
        default: f.i = static_cast<int64_t>(u);  // J, C, Z
      }
      o.fields.push_back(f);
    }
  }
  if (!r.ok) return fail(err, "truncated field values");
  o.class_name = chain.front().name;
  o.suid = chain.front().suid;
  return true;
}

// ---- SHA-1 and the default serialVersionUID ----------------------------------------------------

std::string sha1(std::string_view data) {
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  std::string m(data.data(), data.size());
  const uint64_t bits = static_cast<uint64_t>(data.size()) * 8;
  m.push_back(static_cast<char>(0x80));
  while (m.size() % 64 != 56) m.push_back('\0');
  for (int k = 7; k >= 0; --k) m.push_back(static_cast<char>(bits >> (8 * k)));
  auto rol = [](uint32_t x, int s) { return (x << s) | (x >> (32 - s)); };
  for (size_t off = 0; off < m.size(); off += 64) {
    uint32_t w[80];
    for (int t = 0; t < 16; ++t)
      w[t] = static_cast<uint32_t>(static_cast<uint8_t>(m[off + 4 * t])) << 24 |
             static_cast<uint32_t>(static_cast<uint8_t>(m[off + 4 * t + 1])) << 16 |
             static_cast<uint32_t>(static_cast<uint8_t>(m[off + 4 * t + 2])) << 8 |
             static_cast<uint32_t>(static_cast<uint8_t>(m[off + 4 * t + 3]));
    for (int t = 16; t < 80; ++t) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; ++t) {
      uint32_t f, k;
      if (t < 20) f = (b & c) | (~b & d), k = 0x5A827999u;
      else if (t < 40) f = b ^ c ^ d, k = 0x6ED9EBA1u;
      else if (t < 60) f = (b & c) | (b & d) | (c & d), k = 0x8F1BBCDCu;
      else f = b ^ c ^ d, k = 0xCA62C1D6u;
      const uint32_t x = rol(a, 5) + f + e + k + w[t];
      e = d;
      d = c;
      c = rol(b, 30);
      b = a;
      a = x;
    }
    h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e;
  }
  std::string out(20, '\0');
  for (int i = 0; i < 5; ++i)
    for (int k = 0; k < 4; ++k) out[4 * i + k] = static_cast<char>(h[i] >> (24 - 8 * k));
  return out;
}

namespace {
// java.lang.reflect.Modifier
constexpr int PUBLIC = 0x1, PRIVATE = 0x2, PROTECTED = 0x4, STATIC = 0x8, FINAL = 0x10, SYNCHRONIZED = 0x20,
              VOLATILE = 0x40, TRANSIENT = 0x80, NATIVE = 0x100, INTERFACE = 0x200, ABSTRACT = 0x400,
              STRICT = 0x800;

std::string dotted(std::string s) {
  std::replace(s.begin(), s.end(), '/', '.');
  return s;
}
}  // namespace

int64_t default_suid(const ClassModel& m) {
  Out d;
  d.utf(m.name);
  int cmods = m.mods & (PUBLIC | FINAL | INTERFACE | ABSTRACT);
  if (cmods & INTERFACE) cmods = m.methods.empty() ? (cmods & ~ABSTRACT) : (cmods | ABSTRACT);
  d.be(static_cast<uint32_t>(cmods), 4);
  std::vector<std::string> ifs = m.interfaces;
  std::sort(ifs.begin(), ifs.end());
  for (auto& s : ifs) d.utf(s);
  auto fields = m.fields;
  std::sort(fields.begin(), fields.end(), [](auto& a, auto& b) { return a.name < b.name; });
  for (auto& f : fields) {
    const int mods = f.mods & (PUBLIC | PRIVATE | PROTECTED | STATIC | FINAL | VOLATILE | TRANSIENT);
    if (!(mods & PRIVATE) || !(mods & (STATIC | TRANSIENT))) {
      d.utf(f.name);
      d.be(static_cast<uint32_t>(mods), 4);
      d.utf(f.desc);
    }
  }
  if (m.has_clinit) {
    d.utf("<clinit>");
    d.be(STATIC, 4);
    d.utf("()V");
  }
  constexpr int kMethodMask = PUBLIC | PRIVATE | PROTECTED | STATIC | FINAL | SYNCHRONIZED | NATIVE | ABSTRACT | STRICT;
  auto ctors = m.ctors;
  std::sort(ctors.begin(), ctors.end(), [](auto& a, auto& b) { return a.desc < b.desc; });
  for (auto& c : ctors) {
    const int mods = c.mods & kMethodMask;
    if (mods & PRIVATE) continue;
    d.utf("<init>");
    d.be(static_cast<uint32_t>(mods), 4);
    d.utf(dotted(c.desc));
  }
  auto methods = m.methods;
  std::sort(methods.begin(), methods.end(),
            [](auto& a, auto& b) { return a.name != b.name ? a.name < b.name : a.desc < b.desc; });
  for (auto& x : methods) {
    const int mods = x.mods & kMethodMask;
    if (mods & PRIVATE) continue;
    d.utf(x.name);
    d.be(static_cast<uint32_t>(mods), 4);
    d.utf(dotted(x.desc));
  }
  const std::string h = sha1(d.b);
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = v << 8 | static_cast<uint8_t>(h[static_cast<size_t>(i)]);
  return static_cast<int64_t>(v);
}

ClassModel scala_case_class_model(const std::string& fqcn, const std::vector<std::pair<std::string, char>>& params) {
  ClassModel m;
  m.name = fqcn;
  m.mods = PUBLIC | FINAL;
  m.interfaces = {"scala.Product", "scala.Serializable"};
  std::string internal = fqcn;
  std::replace(internal.begin(), internal.end(), '.', '/');
  const std::string self = "L" + internal + ";";
  std::string args;
  for (auto& p : params) args.push_back(p.second);
  for (auto& p : params) {
    m.fields.push_back({p.first, PRIVATE | FINAL, std::string(1, p.second)});
    m.methods.push_back({p.first, PUBLIC, "()" + std::string(1, p.second)});  // accessor
  }
  m.ctors.push_back({"<init>", PUBLIC, "(" + args + ")V"});
  m.methods.push_back({"copy", PUBLIC, "(" + args + ")" + self});
  for (size_t k = 0; k < params.size(); ++k)
    m.methods.push_back({"copy$default$" + std::to_string(k + 1), PUBLIC, "()" + std::string(1, params[k].second)});
  m.methods.push_back({"productPrefix", PUBLIC, "()Ljava/lang/String;"});
  m.methods.push_back({"productArity", PUBLIC, "()I"});
  m.methods.push_back({"productElement", PUBLIC, "(I)Ljava/lang/Object;"});
  m.methods.push_back({"productIterator", PUBLIC, "()Lscala/collection/Iterator;"});
  m.methods.push_back({"canEqual", PUBLIC, "(Ljava/lang/Object;)Z"});
  m.methods.push_back({"hashCode", PUBLIC, "()I"});
  m.methods.push_back({"toString", PUBLIC, "()Ljava/lang/String;"});
  m.methods.push_back({"equals", PUBLIC, "(Ljava/lang/Object;)Z"});
  // static forwarders of the synthetic companion (AbstractFunctionN[..., Name])
  m.methods.push_back({"apply", PUBLIC | STATIC, "(" + args + ")" + self});
  m.methods.push_back({"unapply", PUBLIC | STATIC, "(" + self + ")Lscala/Option;"});
  if (params.size() == 1) {
    m.methods.push_back({"andThen", PUBLIC | STATIC, "(Lscala/Function1;)Lscala/Function1;"});
    m.methods.push_back({"compose", PUBLIC | STATIC, "(Lscala/Function1;)Lscala/Function1;"});
  } else if (params.size() > 1) {
    m.methods.push_back({"tupled", PUBLIC | STATIC, "()Lscala/Function1;"});
    m.methods.push_back({"curried", PUBLIC | STATIC, "()Lscala/Function1;"});
  }
  return m;
}

}  // namespace akka
}  // namespace mxar
