#include "cluster_node.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../core/log.h"
#include "../core/trace.h"

namespace mxar {

namespace {
using Clock = std::chrono::steady_clock;

std::chrono::milliseconds ms_of(double s) { return std::chrono::milliseconds(static_cast<int64_t>(s * 1000.0)); }

// One frame = u32 length + payload in ONE gather write: one syscall and (TCP_NODELAY) one
// segment per message instead of two - a protocol round is a chain of such messages.
bool write_frame(int fd, const void* p, uint32_t n) {
  uint32_t len = n;
  iovec iov[2] = {{&len, 4}, {const_cast<void*>(p), n}};
  int first = 0;
  size_t left = 4 + static_cast<size_t>(n);
  while (left > 0) {
    msghdr mh{};
    mh.msg_iov = iov + first;
    mh.msg_iovlen = static_cast<size_t>(2 - first);
    const ssize_t k = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    left -= static_cast<size_t>(k);
    size_t adv = static_cast<size_t>(k);
    while (first < 2 && adv >= iov[first].iov_len) {
      adv -= iov[first].iov_len;
      iov[first].iov_len = 0;
      ++first;
    }
    if (first < 2) {
      iov[first].iov_base = static_cast<char*>(iov[first].iov_base) + adv;
      iov[first].iov_len -= adv;
    }
  }
  return true;
}

// Buffered frame reader: one recv() takes every frame the peer has queued (a round's
// Scatter/Reduce burst arrives together), instead of two recv() calls per frame.
class FrameReader {
 public:
  // spin_us > 0: before blocking in recv(), poll the socket (non-blocking recv) for up to
  // spin_us after the previous frame - a protocol round's next Start / Complete arrives within
  // one round, and a blocked reader's wake-up costs several microseconds per hop
  explicit FrameReader(int fd, int spin_us = 0) : fd_(fd), buf_(64 << 10), spin_us_(spin_us) {}
  // From now on the frames come from this ring (the socket only tells when the peer is gone).
  void use_ring(ShmRing* r) { ring_ = r; }
  // Next frame's payload (valid until the next call); false at EOF / error / bad length.
  bool next(const uint8_t** p, uint32_t* n) {
    if (!fill(4)) return false;
    uint32_t len;
    std::memcpy(&len, buf_.data() + head_, 4);
    if (len == 0 || len > (1u << 30)) return false;
    if (!fill(4 + static_cast<size_t>(len))) return false;
    *p = buf_.data() + head_ + 4;
    *n = len;
    head_ += 4 + static_cast<size_t>(len);
    return true;
  }

 private:
  bool fill(size_t need) {
    while (tail_ - head_ < need) {
      if (head_ > 0 && (buf_.size() - head_ < need || head_ == tail_)) {  // compact
        std::memmove(buf_.data(), buf_.data() + head_, tail_ - head_);
        tail_ -= head_;
        head_ = 0;
      }
      if (buf_.size() < need) buf_.resize(need);
      if (ring_ != nullptr) {
        if (!fill_ring()) return false;
        continue;
      }
      ssize_t k = -1;
      if (spin_us_ > 0) {
        const auto until = last_ + std::chrono::microseconds(spin_us_);
        do {
          k = ::recv(fd_, buf_.data() + tail_, buf_.size() - tail_, MSG_DONTWAIT);
          if (k >= 0 || (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) break;
          for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
        } while (Clock::now() < until);
      }
      if (k < 0 && (spin_us_ <= 0 || errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR))
        k = ::recv(fd_, buf_.data() + tail_, buf_.size() - tail_, 0);
      last_ = Clock::now();
      if (k == 0) return false;
      if (k < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      tail_ += static_cast<size_t>(k);
    }
    return true;
  }
  // Ring mode: poll the ring for the spin budget after the last frame, then sleep on its futex
  // in 20 ms slices, checking between them whether the peer closed the socket.
  bool fill_ring() {
    const auto until = last_ + std::chrono::microseconds(spin_us_);
    for (;;) {
      const size_t k = ring_->read(buf_.data() + tail_, buf_.size() - tail_);
      if (k > 0) {
        tail_ += k;
        last_ = Clock::now();
        return true;
      }
      if (Clock::now() < until) {
        for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
        continue;
      }
      if (ring_->wait(20)) continue;
      pollfd pfd{fd_, POLLIN | POLLRDHUP, 0};
      if (::poll(&pfd, 1, 0) != 0) {  // the peer closed (nothing else travels on the socket now)
        if (pfd.revents & (POLLHUP | POLLRDHUP | POLLERR | POLLNVAL)) return !ring_->empty() ? true : false;
        char c;
        if (::recv(fd_, &c, 1, MSG_DONTWAIT | MSG_PEEK) == 0) return false;
      }
    }
  }
  int fd_;
  std::vector<uint8_t> buf_;
  size_t head_ = 0, tail_ = 0;
  int spin_us_ = 0;
  Clock::time_point last_ = Clock::now();
  ShmRing* ring_ = nullptr;
};

// Same-host fast path (shm_ring.h): on unless MXAR_SHM=0; ring bytes per connection.
bool shm_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("MXAR_SHM");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}
constexpr size_t kShmRingBytes = size_t{1} << 20;

int tcp_spin_us() {
  static const int v = [] {
    const char* e = std::getenv("MXAR_TCP_SPIN_US");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return v;
}

int connect_with_timeout(const std::string& host, int port, double timeout_s) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  const int fd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    freeaddrinfo(res);
    return -1;
  }
  const int flags = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, flags | O_NONBLOCK);
  int rc = ::connect(fd, res->ai_addr, res->ai_addrlen);
  freeaddrinfo(res);
  if (rc < 0 && errno != EINPROGRESS) {
    ::close(fd);
    return -1;
  }
  if (rc < 0) {
    pollfd pfd{fd, POLLOUT, 0};
    rc = ::poll(&pfd, 1, static_cast<int>(timeout_s * 1000));
    int err = 0;
    socklen_t len = sizeof(err);
    if (rc <= 0 || getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len) < 0 || err != 0) {
      ::close(fd);
      return -1;
    }
  }
  fcntl(fd, F_SETFL, flags);
  const int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}
}  // namespace

std::string normalize_address(const std::string& in) {
  static const std::string akka = "akka.tcp://";
  std::string a = in.compare(0, akka.size(), akka) == 0 ? "mxar.tcp://" + in.substr(akka.size()) : in;
  while (!a.empty() && a.back() == '/') a.pop_back();
  return a;
}

// ------------------------------------------------------------------ RemoteActorRef
void RemoteActorRef::tell(Message msg, ActorRef sender) {
  if (auto n = node_.lock()) n->send(address_, path_, msg, sender);
}

// ------------------------------------------------------------------ lifecycle
ClusterNode::ClusterNode(std::shared_ptr<ActorSystem> sys, ClusterConfig cfg) : sys_(sys), cfg_(std::move(cfg)) {
  std::random_device rd;
  uid_ = (static_cast<uint64_t>(rd()) << 32) ^ rd();
  for (auto& s : cfg_.seed_nodes) s = normalize_address(s);
}

std::shared_ptr<ClusterNode> ClusterNode::start(std::shared_ptr<ActorSystem> sys, ClusterConfig cfg) {
  if (!sys) throw std::invalid_argument("ClusterNode: null actor system");
  if (sys->deterministic()) throw std::invalid_argument("ClusterNode needs a threaded ActorSystem");
  std::shared_ptr<ClusterNode> n(new ClusterNode(sys, std::move(cfg)));
  n->listen();
  n->address_ = make_address(sys->name(), n->cfg_.host, n->port_);
  std::weak_ptr<ClusterNode> weak = n;
  sys->set_remote_watch_hook([weak](const ActorRef& target, const ActorRef& watcher, bool on) {
    if (auto c = weak.lock()) c->watch_remote(target, watcher, on);
  });
  const bool first_seed = n->cfg_.seed_nodes.empty() || n->cfg_.seed_nodes.front() == n->address_;
  if (first_seed) {  // the first seed joins itself and starts the cluster
    MemberInfo me{n->address_, n->cfg_.roles, n->uid_, MemberStatus::Up, n->cfg_.meta};
    {
      std::lock_guard<std::mutex> g(n->mem_mu_);
      n->members_[n->address_] = me;
      n->last_seen_[n->address_] = Clock::now();
    }
    n->joined_ = true;
    n->on_member_up(me);
  }
  n->accept_thread_ = std::thread([raw = n.get()] { raw->accept_loop(); });
  n->ticker_thread_ = std::thread([raw = n.get()] { raw->ticker_loop(); });
  MXAR_LOG(INFO, "cluster", "node " << n->address_ << " started (roles:" << n->cfg_.roles.size()
                                    << ", seeds:" << n->cfg_.seed_nodes.size() << ")");
  return n;
}

ClusterNode::~ClusterNode() { shutdown(); }

void ClusterNode::listen() {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) throw std::runtime_error("cluster: socket() failed");
  const int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(cfg_.port));
  if (inet_pton(AF_INET, cfg_.host.c_str(), &addr.sin_addr) != 1) addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0) {
    const std::string e = std::strerror(errno);
    ::close(listen_fd_);
    listen_fd_ = -1;
    throw std::runtime_error("cluster: cannot bind " + cfg_.host + ":" + std::to_string(cfg_.port) + ": " + e);
  }
  if (::listen(listen_fd_, 64) < 0) throw std::runtime_error("cluster: listen() failed");
  socklen_t len = sizeof(addr);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
}

void ClusterNode::leave() {
  if (stopping_.load() || leaving_.exchange(true)) return;
  Writer w;
  w.u8(static_cast<uint8_t>(FrameKind::Leave));
  w.str(address_);
  if (!joined_.load()) {
    // a seed may already list this node while its Welcome is still in flight: every seed that
    // admitted it removes it, the others ignore the frame (unknown member)
    for (auto& s : cfg_.seed_nodes)
      if (s != address_) send_frame(s, w.bytes());
    return;
  }
  const std::string lead = leader();
  if (!lead.empty() && lead != address_) {
    send_frame(lead, w.bytes());
  } else {
    MemberInfo me{address_, cfg_.roles, uid_, MemberStatus::Removed, cfg_.meta};
    broadcast(frame_member_event(MemberEventKind::Removed, me), address_);
  }
  joined_ = false;
}

void ClusterNode::shutdown() {
  if (stopping_.exchange(true)) return;
  // the accept loop polls with a short timeout and sees `stopping_`; only after it has
  // exited is the listening socket closed (it reads listen_fd_)
  if (accept_thread_.joinable()) accept_thread_.join();
  if (ticker_thread_.joinable()) ticker_thread_.join();
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
    listen_fd_ = -1;
  }
  {
    std::lock_guard<std::mutex> g(readers_mu_);
    for (int fd : reader_fds_)
      if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  }
  std::vector<std::thread> rs;
  {
    std::lock_guard<std::mutex> g(readers_mu_);
    rs.swap(readers_);
  }
  for (auto& t : rs)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> g(conn_mu_);
  for (auto& [a, c] : conns_) {
    std::lock_guard<std::mutex> gc(c->mu);
    if (c->fd >= 0) ::close(c->fd);
    c->fd = -1;
  }
  conns_.clear();
  if (auto sys = sys_.lock()) sys->set_remote_watch_hook(nullptr);
}

// ------------------------------------------------------------------ transport
void ClusterNode::accept_loop() {
  while (!stopping_.load()) {
    pollfd pfd{listen_fd_, POLLIN, 0};
    const int rc = ::poll(&pfd, 1, 200);
    if (rc <= 0 || stopping_.load()) continue;
    const int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(readers_mu_);
    reader_fds_.push_back(fd);
    readers_.emplace_back([this, fd] { reader_loop(fd); });
  }
}

void ClusterNode::reader_loop(int fd) {
  FrameReader in(fd, tcp_spin_us());
  std::string peer;                  // the connecting node (its Hello)
  std::unique_ptr<ShmRing> offered;  // its ring, mapped at ShmOffer, read from ShmSwitch on
  while (!stopping_.load()) {
    const uint8_t* data = nullptr;
    uint32_t len = 0;
    if (!in.next(&data, &len)) break;
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      ++stats_.frames_in;
      stats_.bytes_in += len + 4;
    }
    try {
      const auto kind = static_cast<FrameKind>(data[0]);
      if (kind == FrameKind::Hello || kind == FrameKind::ShmOffer || kind == FrameKind::ShmSwitch) {
        Reader r(data, len);
        (void)r.u8();
        if (kind == FrameKind::Hello) {
          peer = r.str();
        } else if (kind == FrameKind::ShmOffer) {
          const std::string name = r.str();
          offered = shm_enabled() ? ShmRing::open(name) : nullptr;
          Writer ack;  // over OUR connection to the offerer: it switches only on a good ack
          ack.u8(static_cast<uint8_t>(FrameKind::ShmAck));
          ack.str(address_);
          ack.str(name);
          ack.u8(offered ? 1 : 0);
          if (peer.empty() || !send_frame(peer, ack.bytes())) offered.reset();
        } else if (offered) {  // ShmSwitch: every later frame of this peer is in the ring
          in.use_ring(offered.get());
          std::lock_guard<std::mutex> g(stats_mu_);
          ++stats_.shm_links_in;
        }
        continue;
      }
      handle_frame(data, len);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(stats_mu_);
      ++stats_.decode_errors;
      MXAR_LOG(WARNING, "cluster", "dropping malformed frame: " << e.what());
    }
  }
  std::lock_guard<std::mutex> g(readers_mu_);
  for (int& f : reader_fds_)
    if (f == fd) f = -1;  // shutdown() must not touch a recycled descriptor
  ::close(fd);
}

bool ClusterNode::send_frame(const std::string& address, const std::vector<uint8_t>& payload) {
  if (stopping_.load()) return false;
  std::shared_ptr<OutConn> c;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    auto& slot = conns_[address];
    if (!slot) slot = std::make_shared<OutConn>();
    c = slot;
  }
  std::lock_guard<std::mutex> g(c->mu);
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (c->fd < 0) {
      std::pair<std::string, int> hp;
      try {
        hp = parse_address(address);
      } catch (const std::exception&) {
        return false;
      }
      c->fd = connect_with_timeout(hp.first, hp.second, cfg_.connect_timeout_s);
      if (c->fd < 0) {
        std::lock_guard<std::mutex> gs(stats_mu_);
        ++stats_.connect_failures;
        return false;
      }
      Writer hello;
      hello.u8(static_cast<uint8_t>(FrameKind::Hello));
      hello.str(address_);
      if (!write_frame(c->fd, hello.bytes().data(), static_cast<uint32_t>(hello.bytes().size()))) {
        ::close(c->fd);
        c->fd = -1;
        continue;
      }
      {
        std::lock_guard<std::mutex> gs(stats_mu_);
        ++stats_.connects;
      }
      c->ring.reset();
      c->ring_live = false;
      c->ring_tried = false;
    }
    if (!c->ring_tried && shm_enabled() && same_host(address)) {
      // offer a ring; frames keep going over TCP until the peer's ShmAck (on_shm_ack)
      c->ring_tried = true;
      c->ring = ShmRing::create(kShmRingBytes);
      if (c->ring) {
        Writer offer;
        offer.u8(static_cast<uint8_t>(FrameKind::ShmOffer));
        offer.str(c->ring->name());
        if (!write_frame(c->fd, offer.bytes().data(), static_cast<uint32_t>(offer.bytes().size()))) c->ring.reset();
      }
    }
    const uint32_t len = static_cast<uint32_t>(payload.size());
    if (c->ring_live) {
      const uint32_t l = len;
      if (c->ring->write(&l, 4, &stopping_) && c->ring->write(payload.data(), len, &stopping_)) {
        std::lock_guard<std::mutex> gs(stats_mu_);
        ++stats_.frames_out;
        stats_.bytes_out += len + 4;
        return true;
      }
      return false;
    }
    if (write_frame(c->fd, payload.data(), len)) {
      std::lock_guard<std::mutex> gs(stats_mu_);
      ++stats_.frames_out;
      stats_.bytes_out += len + 4;
      return true;
    }
    ::close(c->fd);
    c->fd = -1;
  }
  std::lock_guard<std::mutex> gs(stats_mu_);
  ++stats_.send_failures;
  return false;
}

void ClusterNode::close_connection(const std::string& address) {
  std::shared_ptr<OutConn> c;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    auto it = conns_.find(address);
    if (it == conns_.end()) return;
    c = it->second;
    conns_.erase(it);
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (c->fd >= 0) ::close(c->fd);
  c->fd = -1;
  c->ring.reset();
  c->ring_live = false;
}

bool ClusterNode::same_host(const std::string& address) const {
  try {
    const std::string h = parse_address(address).first;
    return h == "127.0.0.1" || h == "localhost" || h == cfg_.host;
  } catch (const std::exception&) {
    return false;
  }
}

void ClusterNode::on_shm_ack(const std::string& from, const std::string& name, bool ok) {
  std::shared_ptr<OutConn> c;
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    auto it = conns_.find(from);
    if (it == conns_.end()) return;
    c = it->second;
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (!c->ring || c->ring->name() != name || c->ring_live || c->fd < 0) return;
  if (!ok) {  // the peer could not map it: stay on TCP
    c->ring.reset();
    return;
  }
  Writer sw;  // the last frame on the socket: the peer's reader switches to the ring behind it
  sw.u8(static_cast<uint8_t>(FrameKind::ShmSwitch));
  if (!write_frame(c->fd, sw.bytes().data(), static_cast<uint32_t>(sw.bytes().size()))) {
    c->ring.reset();
    return;
  }
  c->ring_live = true;
  std::lock_guard<std::mutex> gs(stats_mu_);
  ++stats_.shm_links_out;
}

void ClusterNode::broadcast(const std::vector<uint8_t>& payload, const std::string& except) {
  std::vector<std::string> targets;
  {
    std::lock_guard<std::mutex> g(mem_mu_);
    for (auto& [a, m] : members_)
      if (a != address_ && a != except) targets.push_back(a);
  }
  for (auto& a : targets) send_frame(a, payload);
}

void ClusterNode::send(const std::string& address, const std::string& path, const Message& m, const ActorRef& sender) {
  if (address == address_) {
    deliver_local(path, m, sender);
    return;
  }
  Writer w;
  w.u8(static_cast<uint8_t>(FrameKind::Envelope));
  w.str(encode_ref(sender));
  w.str(path);
  encode_message(w, m, *this);
  if (!send_frame(address, w.bytes())) {
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      ++stats_.undeliverable;
    }
    if (auto sys = sys_.lock()) sys->note_dead_letter(m, sender);
  }
}

void ClusterNode::deliver_local(const std::string& path, Message m, const ActorRef& sender) {
  auto sys = sys_.lock();
  if (!sys) return;
  ActorRef target = sys->lookup(path);
  if (!target) {
    {
      std::lock_guard<std::mutex> g(stats_mu_);
      ++stats_.undeliverable;
    }
    sys->dead_letters()->tell(std::move(m), sender);
    return;
  }
  target->tell(std::move(m), sender);
}

// ------------------------------------------------------------------ refs
std::string ClusterNode::encode_ref(const ActorRef& r) const {
  if (!r) return "";
  if (r->is_remote()) return r->path();
  return address_ + r->path();
}

ActorRef ClusterNode::decode_ref(const std::string& s) {
  if (s.empty()) return nullptr;
  return resolve(s);
}

ActorRef ClusterNode::resolve(const std::string& full_in) {
  const std::string full = normalize_address(full_in);
  auto [addr, path] = split_ref(full);
  if (addr.empty() || addr == address_) {
    if (auto sys = sys_.lock())
      if (ActorRef local = sys->lookup(path)) return local;
    addr = address_;
  }
  const std::string key = addr + path;
  std::lock_guard<std::mutex> g(ref_mu_);
  auto it = ref_cache_.find(key);
  if (it != ref_cache_.end()) return it->second;
  ActorRef r = std::make_shared<RemoteActorRef>(weak_from_this(), addr, path);
  ref_cache_[key] = r;
  return r;
}

// ------------------------------------------------------------------ membership
std::vector<uint8_t> ClusterNode::frame_member_event(MemberEventKind k, const MemberInfo& m) {
  Writer w;
  w.u8(static_cast<uint8_t>(FrameKind::MemberEvent));
  w.u8(static_cast<uint8_t>(k));
  encode_member(w, m);
  return std::move(w.bytes());
}

MemberUp ClusterNode::member_up_event(const MemberInfo& m) {
  MemberUp up;
  up.role = m.roles.empty() ? "" : m.roles.front();
  up.address = m.address;
  up.meta = m.meta;
  up.ref = resolve(m.address + (m.has_role("worker") ? cfg_.worker_path : std::string("/user")));
  return up;
}

void ClusterNode::on_member_up(const MemberInfo& m) {
  std::vector<ActorRef> subs;
  {
    std::lock_guard<std::mutex> g(mem_mu_);
    subs.assign(subscribers_.begin(), subscribers_.end());
  }
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    ++stats_.members_up;
  }
  MXAR_LOG(INFO, "cluster", "Member is Up: " << m.address);
  trace_instant("cluster", "MemberUp " + m.address);
  for (auto& s : subs) s->tell(member_up_event(m), nullptr);
}

void ClusterNode::on_member_removed(const std::string& address) {
  std::vector<std::pair<ActorRef, ActorRef>> fire;
  bool known = false;
  {
    std::lock_guard<std::mutex> g(mem_mu_);
    known = members_.erase(address) > 0;
    last_seen_.erase(address);
    unreachable_since_.erase(address);
    auto it = watches_.find(address);
    if (it != watches_.end()) {
      fire.swap(it->second);
      watches_.erase(it);
    }
  }
  if (known) {
    std::lock_guard<std::mutex> g(stats_mu_);
    ++stats_.members_removed;
  }
  MXAR_LOG(INFO, "cluster", "Member removed: " << address);
  trace_instant("cluster", "MemberRemoved " + address);
  close_connection(address);
  for (auto& [target, watcher] : fire) watcher->tell(Terminated{target}, target);
  if (address == address_) joined_ = false;
}

void ClusterNode::watch_remote(const ActorRef& target, const ActorRef& watcher, bool on) {
  auto* rr = dynamic_cast<RemoteActorRef*>(target.get());
  if (!rr) return;
  bool gone = false;
  {
    std::lock_guard<std::mutex> g(mem_mu_);
    auto& v = watches_[rr->address()];
    if (on) {
      gone = joined_.load() && !members_.count(rr->address()) && rr->address() != address_;
      if (!gone) v.emplace_back(target, watcher);
    } else {
      for (auto it = v.begin(); it != v.end();)
        it = (it->first == target && it->second == watcher) ? v.erase(it) : std::next(it);
    }
  }
  if (gone) watcher->tell(Terminated{target}, target);  // watching a node already gone
}

void ClusterNode::subscribe(const ActorRef& subscriber) {
  std::vector<MemberInfo> current;
  {
    std::lock_guard<std::mutex> g(mem_mu_);
    subscribers_.insert(subscriber);
    for (auto& [a, m] : members_) current.push_back(m);
  }
  for (auto& m : current) subscriber->tell(member_up_event(m), nullptr);  // InitialStateAsEvents
}

void ClusterNode::unsubscribe(const ActorRef& subscriber) {
  std::lock_guard<std::mutex> g(mem_mu_);
  subscribers_.erase(subscriber);
}

std::vector<MemberInfo> ClusterNode::members() {
  std::lock_guard<std::mutex> g(mem_mu_);
  std::vector<MemberInfo> v;
  for (auto& [a, m] : members_) v.push_back(m);
  return v;
}

std::string ClusterNode::leader() {
  std::lock_guard<std::mutex> g(mem_mu_);
  for (auto& [a, m] : members_)  // std::map: ascending address order
    if (!unreachable_since_.count(a)) return a;
  return "";
}

bool ClusterNode::is_unreachable(const std::string& address) {
  std::lock_guard<std::mutex> g(mem_mu_);
  return unreachable_since_.count(normalize_address(address)) > 0;
}

ClusterStats ClusterNode::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

void ClusterNode::handle_frame(const uint8_t* p, size_t n) {
  Reader r(p, n);
  const auto kind = static_cast<FrameKind>(r.u8());
  switch (kind) {
    case FrameKind::Hello:
      (void)r.str();
      break;
    case FrameKind::ShmAck: {
      const std::string from = r.str();
      const std::string name = r.str();
      on_shm_ack(from, name, r.u8() != 0);
      break;
    }
    case FrameKind::Envelope: {
      const std::string sender = r.str();
      const std::string path = r.str();
      Message m = decode_message(r, *this);
      deliver_local(path, std::move(m), decode_ref(sender));
      break;
    }
    case FrameKind::Join: {
      MemberInfo m = decode_member(r);
      m.status = MemberStatus::Up;
      if (!joined_.load()) break;  // only members admit joiners; the joiner retries
      bool restarted = false, fresh = false;
      std::vector<MemberInfo> all;
      {
        std::lock_guard<std::mutex> g(mem_mu_);
        auto it = members_.find(m.address);
        if (it != members_.end() && it->second.uid != m.uid) restarted = true;
        fresh = it == members_.end() || restarted;
      }
      if (restarted) {  // same address, new incarnation: the old one is gone
        broadcast(frame_member_event(MemberEventKind::Removed, m), m.address);
        on_member_removed(m.address);
      }
      {
        std::lock_guard<std::mutex> g(mem_mu_);
        members_[m.address] = m;
        last_seen_[m.address] = Clock::now();
        unreachable_since_.erase(m.address);
        for (auto& [a, x] : members_) all.push_back(x);
      }
      Writer w;
      w.u8(static_cast<uint8_t>(FrameKind::Welcome));
      w.u32(static_cast<uint32_t>(all.size()));
      for (auto& x : all) encode_member(w, x);
      send_frame(m.address, w.bytes());
      if (fresh) {
        broadcast(frame_member_event(MemberEventKind::Up, m), m.address);
        on_member_up(m);
      }
      break;
    }
    case FrameKind::Welcome: {
      if (leaving_.load()) break;  // admitted after leave(): the Leave sent to the seeds undoes it
      const uint32_t cnt = r.u32();
      std::vector<MemberInfo> fresh;
      {
        std::lock_guard<std::mutex> g(mem_mu_);
        for (uint32_t i = 0; i < cnt; ++i) {
          MemberInfo m = decode_member(r);
          if (!members_.count(m.address)) fresh.push_back(m);
          members_[m.address] = m;
          last_seen_[m.address] = Clock::now();
        }
      }
      joined_ = true;
      for (auto& m : fresh) on_member_up(m);
      break;
    }
    case FrameKind::MemberEvent: {
      const auto ev = static_cast<MemberEventKind>(r.u8());
      MemberInfo m = decode_member(r);
      if (ev == MemberEventKind::Up) {
        bool fresh = false;
        {
          std::lock_guard<std::mutex> g(mem_mu_);
          fresh = !members_.count(m.address);
          members_[m.address] = m;
          last_seen_[m.address] = Clock::now();
        }
        if (fresh) on_member_up(m);
      } else if (ev == MemberEventKind::Removed) {
        on_member_removed(m.address);
      }
      break;
    }
    case FrameKind::Heartbeat: {
      const std::string from = r.str();
      (void)r.u64();
      std::lock_guard<std::mutex> g(mem_mu_);
      if (members_.count(from)) last_seen_[from] = Clock::now();
      std::lock_guard<std::mutex> gs(stats_mu_);
      ++stats_.heartbeats_in;
      break;
    }
    case FrameKind::Leave: {
      const std::string who = r.str();
      MemberInfo m;
      {
        std::lock_guard<std::mutex> g(mem_mu_);
        auto it = members_.find(who);
        if (it == members_.end()) break;
        m = it->second;
      }
      m.status = MemberStatus::Removed;
      broadcast(frame_member_event(MemberEventKind::Removed, m), who);
      on_member_removed(who);
      break;
    }
    default:
      throw CodecError("unknown frame kind");
  }
}

void ClusterNode::ticker_loop() {
  const auto period = ms_of(cfg_.heartbeat_interval_s);
  while (!stopping_.load()) {
    // sleep in small slices so shutdown is prompt
    const auto until = Clock::now() + period;
    while (!stopping_.load() && Clock::now() < until) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    if (stopping_.load()) break;
    if (!joined_.load()) {
      if (leaving_.load()) continue;
      Writer w;
      w.u8(static_cast<uint8_t>(FrameKind::Join));
      encode_member(w, MemberInfo{address_, cfg_.roles, uid_, MemberStatus::Joining, cfg_.meta});
      for (auto& s : cfg_.seed_nodes)
        if (s != address_) send_frame(s, w.bytes());
      continue;
    }
    Writer hb;
    hb.u8(static_cast<uint8_t>(FrameKind::Heartbeat));
    hb.str(address_);
    hb.u64(++hb_seq_);
    broadcast(hb.bytes());
    // failure detector
    const auto now = Clock::now();
    std::vector<std::string> to_down, newly_unreachable, back;
    std::string lead;
    {
      std::lock_guard<std::mutex> g(mem_mu_);
      last_seen_[address_] = now;
      for (auto& [a, m] : members_) {
        if (a == address_) continue;
        const auto silent = now - last_seen_[a];
        if (silent > ms_of(cfg_.acceptable_heartbeat_pause_s)) {
          if (!unreachable_since_.count(a)) {
            unreachable_since_[a] = now;
            newly_unreachable.push_back(a);
          }
        } else if (unreachable_since_.erase(a)) {
          back.push_back(a);
        }
      }
      for (auto& [a, m] : members_)
        if (!unreachable_since_.count(a)) {
          lead = a;
          break;
        }
      if (lead == address_ && cfg_.auto_down_unreachable_after_s >= 0)
        for (auto& [a, since] : unreachable_since_)
          if (now - since > ms_of(cfg_.auto_down_unreachable_after_s)) to_down.push_back(a);
    }
    for (auto& a : newly_unreachable) MXAR_LOG(WARNING, "cluster", "Marking node as UNREACHABLE: " << a);
    for (auto& a : back) MXAR_LOG(INFO, "cluster", "Marking node as REACHABLE: " << a);
    for (auto& a : to_down) {
      MXAR_LOG(INFO, "cluster", "Leader is auto-downing unreachable node " << a);
      MemberInfo m;
      m.address = a;
      m.status = MemberStatus::Down;
      broadcast(frame_member_event(MemberEventKind::Removed, m), a);
      on_member_removed(a);
    }
  }
}

}  // namespace mxar
