#include "akka_endpoint.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <random>
#include <stdexcept>

#include "../core/log.h"

namespace mxar {

namespace {

constexpr size_t kMaxQueuedBytes = 4u << 20;
// Frames above the reference transport's 128000-byte cap are refused (a client never sends
// them: its own transport would drop them first).
constexpr size_t kMaxInFrame = akka::kMaxFrame + 4096;

bool read_full(int fd, char* p, size_t n) {
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

std::string frame(const std::string& pdu) {
  std::string f(4, '\0');
  const uint32_t n = static_cast<uint32_t>(pdu.size());
  for (int k = 0; k < 4; ++k) f[static_cast<size_t>(k)] = static_cast<char>(n >> (24 - 8 * k));
  return f + pdu;
}

// Value of "key": in a flat JSON event line (numbers / booleans only).
bool json_int(const std::string& line, const char* key, long& v) {
  const std::string k = std::string("\"") + key + "\":";
  const size_t i = line.find(k);
  if (i == std::string::npos) return false;
  char* end = nullptr;
  v = std::strtol(line.c_str() + i + k.size(), &end, 10);
  return end != line.c_str() + i + k.size();
}

bool has_type(const std::string& line, const char* type) {
  return line.find(std::string("\"type\":\"") + type + "\"") != std::string::npos;
}

std::string simple_name(const std::string& cls) {
  size_t i = cls.find_last_of(".$");
  return i == std::string::npos ? cls : cls.substr(i + 1);
}

std::string package_of(const std::string& cls) {
  size_t i = cls.rfind('.');
  return i == std::string::npos ? std::string() : cls.substr(0, i);
}

// ActorSelection's CHILD_PATTERN: '*' and '?' globs (akka.util.Helpers.makePattern).
bool glob(const char* p, const char* s) {
  if (!*p) return !*s;
  if (*p == '*') return glob(p + 1, s) || (*s && glob(p, s + 1));
  if (*s && (*p == '?' || *p == *s)) return glob(p + 1, s + 1);
  return false;
}

}  // namespace

std::shared_ptr<AkkaEndpoint> AkkaEndpoint::start(std::shared_ptr<ControlBridge> bridge, Options o) {
  if (!bridge) throw std::runtime_error("akka endpoint: needs a control bridge");
  std::shared_ptr<AkkaEndpoint> e(new AkkaEndpoint());
  e->opt_ = std::move(o);
  e->bridge_ = std::move(bridge);
  std::random_device rd;
  // the handshake uid (a Long); its low 32 bits are the Int address uid of HeartbeatRsp, kept
  // positive so either width reads the same number
  e->uid_ = (static_cast<uint64_t>(rd()) << 32 | rd()) & ~(uint64_t{1} << 31);
  e->suid_start_ = e->opt_.suid_start
                       ? e->opt_.suid_start
                       : akka::default_suid(akka::scala_case_class_model(e->opt_.package + ".StartAllreduce",
                                                                         {{"round", 'I'}}));
  e->suid_complete_ = e->opt_.suid_complete
                          ? e->opt_.suid_complete
                          : akka::default_suid(akka::scala_case_class_model(e->opt_.package + ".CompleteAllreduce",
                                                                            {{"srcId", 'I'}, {"round", 'I'}}));
  e->lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (e->lfd_ < 0) throw std::runtime_error("akka endpoint: socket failed");
  int one = 1;
  ::setsockopt(e->lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(e->opt_.port));
  if (::inet_pton(AF_INET, e->opt_.host.c_str(), &a.sin_addr) != 1)
    throw std::runtime_error("akka endpoint: bad host " + e->opt_.host);
  if (::bind(e->lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(e->lfd_, 16) != 0)
    throw std::runtime_error("akka endpoint: cannot listen on " + e->opt_.host + ":" + std::to_string(e->opt_.port) +
                             ": " + std::strerror(errno));
  socklen_t len = sizeof(a);
  ::getsockname(e->lfd_, reinterpret_cast<sockaddr*>(&a), &len);
  e->port_ = ntohs(a.sin_port);
  if (::pipe2(e->wake_, O_CLOEXEC) != 0) throw std::runtime_error("akka endpoint: pipe failed");
  std::weak_ptr<AkkaEndpoint> weak = e;
  e->bridge_->on_stop([weak] {
    if (auto s = weak.lock()) s->stop();
  });
  e->acceptor_ = std::thread([e] { e->accept_loop(e); });
  MXAR_LOG(INFO, "akka", "----akka.tcp endpoint " << e->address() << " serves " << e->master_path());
  return e;
}

AkkaEndpoint::~AkkaEndpoint() { stop(); }

std::string AkkaEndpoint::address() const {
  akka::Address a;
  a.system = opt_.system;
  a.host = opt_.host;
  a.port = static_cast<uint32_t>(port_);
  return a.str();
}

std::string AkkaEndpoint::master_path() const {
  return address() + "/user/" + opt_.master + "#" + std::to_string(static_cast<int32_t>(uid_));
}

AkkaEndpoint::Stats AkkaEndpoint::stats() const {
  Stats s;
  s.associations = n_assoc_.load();
  s.frames_in = n_in_.load();
  s.frames_out = n_out_.load();
  s.starts = n_start_.load();
  s.completes_sent = n_complete_.load();
  s.identifies = n_identify_.load();
  s.watcher_heartbeats = n_rh_.load();
  s.system_messages = n_sys_.load();
  s.unsupported = n_unsup_.load();
  s.suid_mismatches = n_suid_.load();
  s.rejected = n_rej_.load();
  s.client_suid_start = client_suid_.load();
  return s;
}

size_t AkkaEndpoint::associations() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (auto& a : assocs_) n += !a->dead.load();
  return n;
}

void AkkaEndpoint::warn_once(const std::string& key, const std::string& what) {
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& w : warned_)
      if (w == key) return;
    if (warned_.size() < 64) warned_.push_back(key);
  }
  MXAR_LOG(WARNING, "akka", what);
}

void AkkaEndpoint::Assoc::kill() {
  if (dead.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(wmu);
    out.clear();
    queued = 0;
  }
  wcv.notify_all();
  ::shutdown(fd, SHUT_RDWR);
}

AkkaEndpoint::Assoc::~Assoc() {
  if (reader.joinable()) reader.detach();
  if (writer.joinable()) writer.detach();
  if (fd >= 0) ::close(fd);
}

bool AkkaEndpoint::send_pdu(Assoc& a, const std::string& pdu) {
  if (a.dead.load()) return false;
  std::string f = frame(pdu);
  bool overflow = false;
  {
    std::lock_guard<std::mutex> g(a.wmu);
    if (a.queued + f.size() > kMaxQueuedBytes) {
      overflow = true;
    } else {
      a.queued += f.size();
      a.out.push_back(std::move(f));
    }
  }
  if (overflow) {
    MXAR_LOG(WARNING, "akka", "association " << a.remote.str() << " stopped reading: disassociating");
    a.kill();
    return false;
  }
  a.wcv.notify_one();
  return true;
}

void AkkaEndpoint::send_message(Assoc& a, const std::string& recipient, const akka::SerializedMsg& m) {
  akka::Envelope e;
  e.has_envelope = true;
  e.recipient = recipient;
  e.msg = m;
  e.has_sender = true;
  e.sender = master_path();
  send_pdu(a, akka::encode_payload_pdu(akka::encode_container(e)));
}

void AkkaEndpoint::write_loop(std::shared_ptr<AkkaEndpoint> self, std::shared_ptr<Assoc> a) {
  (void)self;
  const auto period = std::chrono::duration<double>(opt_.heartbeat_s);
  auto next_hb = std::chrono::steady_clock::now() + std::chrono::duration_cast<std::chrono::nanoseconds>(period);
  const std::string hb = frame(akka::encode_control(akka::kHeartbeat));
  std::string buf;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(a->wmu);
      // a system_clock deadline: pthread_cond_timedwait (a steady_clock wait_until becomes
      // pthread_cond_clockwait, which this toolchain's ThreadSanitizer does not intercept)
      const auto left = next_hb - std::chrono::steady_clock::now();
      a->wcv.wait_until(g, std::chrono::system_clock::now() + left,
                        [&] { return !a->out.empty() || a->dead.load(); });
      if (a->dead.load()) return;
      buf.clear();
      size_t frames = 0;
      while (!a->out.empty()) {
        buf += a->out.front();
        a->out.pop_front();
        ++frames;
      }
      a->queued = 0;
      a->inflight = true;
      n_out_ += frames;
    }
    const auto now = std::chrono::steady_clock::now();
    if (now >= next_hb) {  // transport failure detector (akka.remote.transport-failure-detector)
      if (a->open.load()) buf += hb;  // never ahead of our ASSOCIATE reply
      next_hb = now + std::chrono::duration_cast<std::chrono::nanoseconds>(period);
    }
    size_t off = 0;
    while (off < buf.size()) {
      ssize_t n = ::send(a->fd, buf.data() + off, buf.size() - off, MSG_NOSIGNAL);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        a->kill();
        return;
      }
      off += static_cast<size_t>(n);
    }
    a->inflight = false;
  }
}

void AkkaEndpoint::accept_loop(std::shared_ptr<AkkaEndpoint> self) {
  while (!stop_.load()) {
    pollfd p[2] = {{lfd_, POLLIN, 0}, {wake_[0], POLLIN, 0}};
    int r = ::poll(p, 2, 200);
    reap();
    if (r <= 0 || stop_.load()) continue;
    if (!(p[0].revents & POLLIN)) continue;
    int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    auto a = std::make_shared<Assoc>();
    a->fd = fd;
    {
      std::lock_guard<std::mutex> g(mu_);
      assocs_.push_back(a);
    }
    // both threads start here (stop() joins the writer: it must never be assigned later
    // by another thread)
    a->writer = std::thread([self, a] { self->write_loop(self, a); });
    a->reader = std::thread([self, a] { self->read_loop(self, a); });
  }
}

void AkkaEndpoint::read_loop(std::shared_ptr<AkkaEndpoint> self, std::shared_ptr<Assoc> a) {
  bool open = false;
  std::string body;
  while (!stop_.load() && !a->dead.load()) {
    char hdr[4];
    if (!read_full(a->fd, hdr, 4)) break;
    size_t n = 0;
    for (char c : hdr) n = n << 8 | static_cast<uint8_t>(c);
    if (n > kMaxInFrame) {
      MXAR_LOG(WARNING, "akka", "frame of " << n << " bytes refused (cap " << kMaxInFrame << "): disassociating");
      ++n_rej_;
      break;
    }
    body.resize(n);
    if (n && !read_full(a->fd, body.data(), n)) break;
    ++n_in_;
    akka::Pdu pdu;
    if (!akka::decode_pdu(body, pdu)) {
      MXAR_LOG(WARNING, "akka", "undecodable AkkaProtocolMessage: disassociating");
      ++n_rej_;
      break;
    }
    if (!open) {  // ProtocolStateActor WaitHandshake (inbound): the first PDU must be ASSOCIATE
      if (pdu.is_payload || pdu.command != akka::kAssociate || !pdu.has_handshake) {
        MXAR_LOG(WARNING, "akka", "association without a handshake: closing");
        ++n_rej_;
        break;
      }
      if (!opt_.cookie.empty() && pdu.cookie != opt_.cookie) {
        MXAR_LOG(WARNING, "akka", "association from " << pdu.origin.str() << " with a wrong cookie: closing");
        ++n_rej_;
        break;
      }
      a->remote = pdu.origin;
      a->remote_uid = pdu.uid;
      akka::Address me;
      me.system = opt_.system;
      me.host = opt_.host;
      me.port = static_cast<uint32_t>(port_);
      send_pdu(*a, akka::encode_associate(me, uid_, opt_.cookie));
      a->open = true;
      std::weak_ptr<AkkaEndpoint> we = self;
      std::weak_ptr<Assoc> wa = a;
      if (!stop_.load())  // (after stop() the bridge drops every tap anyway)
        a->tap = bridge_->add_tap([we, wa](const std::string& line) {
          auto e = we.lock();
          auto x = wa.lock();
          if (e && x) e->on_line(*x, line);
        });
      open = true;
      ++n_assoc_;
      MXAR_LOG(INFO, "akka", "----associated with " << a->remote.str() << " (uid " << a->remote_uid << ")");
      continue;
    }
    if (!pdu.is_payload) {
      if (pdu.command == akka::kHeartbeat || pdu.command == akka::kAssociate) continue;
      MXAR_LOG(INFO, "akka", "----" << a->remote.str() << " disassociated (command " << pdu.command << ")");
      break;
    }
    akka::Envelope env;
    if (!akka::decode_container(pdu.payload, env)) {
      MXAR_LOG(WARNING, "akka", "undecodable AckAndEnvelopeContainer from " << a->remote.str() << ": dropped");
      ++n_rej_;
      continue;
    }
    if (env.has_envelope) on_envelope(*a, env);
  }
  if (const uint64_t t = a->tap.exchange(0)) bridge_->remove_tap(t);
  a->kill();
}

void AkkaEndpoint::on_envelope(Assoc& a, const akka::Envelope& e) {
  if (e.has_seq) {
    // A system message (Watch / Unwatch / ...: reliable delivery). Acknowledge it so the
    // client's ReliableDeliverySupervisor does not resend it; the master has no Akka watchers
    // to notify (a client learns of a stopped endpoint from the transport).
    ++n_sys_;
    akka::Envelope ack;
    ack.has_ack = true;
    ack.cumulative_ack = e.seq;
    send_pdu(a, akka::encode_payload_pdu(akka::encode_container(ack)));
    return;
  }
  akka::Address addr;
  std::vector<std::string> elems;
  if (!akka::parse_actor_path(e.recipient, addr, elems)) {
    ++n_rej_;
    warn_once("path:" + e.recipient, "recipient is not an actor path: " + e.recipient);
    return;
  }
  if (addr.system != opt_.system || addr.port != static_cast<uint32_t>(port_)) {
    ++n_rej_;
    warn_once("addr:" + addr.str(), "message for " + addr.str() + " arrived at " + address() + ": dropped");
    return;
  }
  const std::string sender = e.has_sender ? e.sender : std::string();
  if (e.msg.serializer == akka::kContainerSerializer) {  // ActorSelectionMessage
    akka::SerializedMsg inner;
    std::vector<akka::Selection> pattern;
    bool wildcard = false;
    if (!akka::decode_selection(e.msg.bytes, inner, pattern, wildcard)) {
      ++n_rej_;
      warn_once("selection", "undecodable SelectionEnvelope: dropped");
      return;
    }
    for (auto& s : pattern) {
      if (s.type == 0) {
        if (!elems.empty()) elems.pop_back();
      } else if (s.type == 1) {
        elems.push_back(s.matcher);
      } else {  // a pattern selects whichever of our two path levels it matches
        const std::string cand = elems.empty() ? "user" : opt_.master;
        elems.push_back(glob(s.matcher.c_str(), cand.c_str()) ? cand : s.matcher);
      }
    }
    deliver(a, std::move(elems), inner, sender);
    return;
  }
  deliver(a, std::move(elems), e.msg, sender);
}

void AkkaEndpoint::deliver(Assoc& a, std::vector<std::string> elems, const akka::SerializedMsg& m,
                           const std::string& sender) {
  const bool is_master = elems.size() == 2 && elems[0] == "user" && elems[1] == opt_.master;
  if (m.serializer == akka::kMiscSerializer && m.manifest == akka::kIdentifyManifest) {
    ++n_identify_;
    std::string id;
    if (!akka::decode_identify(m.bytes, id) || sender.empty()) return;
    akka::SerializedMsg r;
    r.serializer = akka::kMiscSerializer;
    r.has_manifest = true;
    r.manifest = akka::kActorIdentityManifest;
    r.bytes = akka::encode_actor_identity(id, is_master ? master_path() : std::string());
    send_message(a, sender, r);
    return;
  }
  if (m.serializer == akka::kMiscSerializer && m.manifest == akka::kWatcherHeartbeatManifest) {
    ++n_rh_;
    if (sender.empty()) return;
    akka::SerializedMsg r;
    r.serializer = akka::kMiscSerializer;
    r.has_manifest = true;
    r.manifest = akka::kWatcherHeartbeatRspManifest;
    r.bytes = akka::encode_heartbeat_rsp(static_cast<int32_t>(uid_));
    send_message(a, sender, r);
    return;
  }
  if (m.serializer != akka::kJavaSerializer) {
    ++n_unsup_;
    warn_once("ser:" + std::to_string(m.serializer) + ":" + m.manifest,
              "unsupported message (serializer " + std::to_string(m.serializer) + ", manifest '" + m.manifest +
                  "'): dropped");
    return;
  }
  akka::JavaObject o;
  std::string err;
  if (!akka::java_deserialize(m.bytes, o, &err)) {
    ++n_unsup_;
    warn_once("java:" + err, "unsupported Java-serialized message (" + err + "): dropped");
    return;
  }
  if (simple_name(o.class_name) != "StartAllreduce" || o.fields.size() != 1 || o.fields[0].name != "round" ||
      o.fields[0].type != 'I') {
    ++n_unsup_;
    warn_once("cls:" + o.class_name, "unsupported message " + o.class_name + " (only StartAllreduce(round: Int)): dropped");
    return;
  }
  client_suid_ = o.suid;
  if (package_of(o.class_name) == opt_.package && o.suid != suid_start_) {
    // The client's classes disagree with the scalac model this endpoint hashed (or with the
    // override): CompleteAllreduce replies would fail its deserialization the same way.
    ++n_suid_;
    warn_once("suid", "the client's StartAllreduce has serialVersionUID " + std::to_string(o.suid) + ", this endpoint " +
                          "expects " + std::to_string(suid_start_) + ": set mxar.akka.suid.* from `serialver` (docs/AKKA_WIRE.md)");
  } else if (package_of(o.class_name) != opt_.package) {
    warn_once("pkg:" + o.class_name, "StartAllreduce of package " + package_of(o.class_name) + " (replies use " +
                                         opt_.package + ", mxar.akka.package)");
  }
  if (!sender.empty()) {
    std::lock_guard<std::mutex> g(a.smu);
    bool known = false;
    for (auto& s : a.subscribers) known |= s == sender;
    if (!known && a.subscribers.size() < 16) a.subscribers.push_back(sender);
  }
  ++n_start_;
  BridgeCommand cmd;
  cmd.kind = BridgeCommand::Start;
  cmd.round = static_cast<int>(o.fields[0].i);
  cmd.client = a.tap.load();
  if (cmd.round < 0 || !bridge_->submit(cmd)) warn_once("start", "StartAllreduce refused (negative round or no master)");
}

void AkkaEndpoint::on_line(Assoc& a, const std::string& line) {
  if (has_type(line, "CompleteAllreduce")) {
    long src = 0, round = 0;
    if (!json_int(line, "srcId", src) || !json_int(line, "round", round)) return;
    std::vector<std::string> subs;
    {
      std::lock_guard<std::mutex> g(a.smu);
      subs = a.subscribers;
    }
    if (subs.empty()) return;
    akka::JavaObject o;
    o.class_name = opt_.package + ".CompleteAllreduce";
    o.suid = suid_complete_;
    o.fields = {{'I', "srcId", src, 0.0}, {'I', "round", round, 0.0}};
    akka::SerializedMsg m;
    m.serializer = akka::kJavaSerializer;
    m.bytes = akka::java_serialize(o);
    for (auto& s : subs) {
      send_message(a, s, m);
      ++n_complete_;
    }
  } else if (has_type(line, "Error")) {
    MXAR_LOG(WARNING, "akka", "master refused a command from " << a.remote.str() << ": " << line);
  }
}

void AkkaEndpoint::reap() {
  std::vector<std::shared_ptr<Assoc>> dead;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = assocs_.begin(); it != assocs_.end();) {
      if ((*it)->dead.load()) {
        dead.push_back(*it);
        it = assocs_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& a : dead) {
    if (a->reader.joinable()) a->reader.detach();  // may sit in submit() (see ControlBridge::reap)
    if (a->writer.joinable()) a->writer.join();
  }
}

void AkkaEndpoint::stop() {
  if (stop_.exchange(true)) return;
  if (wake_[1] >= 0) {
    char x = 1;
    (void)!::write(wake_[1], &x, 1);
  }
  auto join = [](std::thread& t) {
    if (!t.joinable()) return;
    if (t.get_id() == std::this_thread::get_id()) t.detach();
    else t.join();
  };
  join(acceptor_);
  std::vector<std::shared_ptr<Assoc>> as;
  {
    std::lock_guard<std::mutex> g(mu_);
    as.swap(assocs_);
  }
  const std::string bye = akka::encode_control(akka::kShuttingDown);
  for (auto& a : as)  // best effort: tell every client we are going down (through its writer)
    if (const uint64_t t = a->tap.exchange(0)) {
      bridge_->remove_tap(t);
      if (a->open.load()) send_pdu(*a, bye);
    }
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
  for (auto& a : as)
    for (;;) {
      bool drained;
      {
        std::lock_guard<std::mutex> g(a->wmu);
        drained = a->out.empty() && !a->inflight.load();
      }
      if (drained || a->dead.load() || std::chrono::steady_clock::now() > until) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  for (auto& a : as) {
    a->kill();
    if (a->reader.joinable()) a->reader.detach();
    join(a->writer);
  }
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  for (int& f : wake_)
    if (f >= 0) ::close(f), f = -1;
}

}  // namespace mxar
