#include "control_bridge.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

#include "../core/log.h"

namespace mxar {

namespace {

size_t skip_ws(const std::string& s, size_t i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\r' || s[i] == '\n')) ++i;
  return i;
}

// Parses a JSON string starting at s[i] == '"'; returns the index after the closing quote.
size_t parse_string(const std::string& s, size_t i, std::string& out) {
  if (i >= s.size() || s[i] != '"') return std::string::npos;
  out.clear();
  for (++i; i < s.size(); ++i) {
    char c = s[i];
    if (c == '"') return i + 1;
    if (c != '\\') {
      out.push_back(c);
      continue;
    }
    if (++i >= s.size()) return std::string::npos;
    switch (s[i]) {
      case '"': out.push_back('"'); break;
      case '\\': out.push_back('\\'); break;
      case '/': out.push_back('/'); break;
      case 'n': out.push_back('\n'); break;
      case 't': out.push_back('\t'); break;
      case 'r': out.push_back('\r'); break;
      case 'b': out.push_back('\b'); break;
      case 'f': out.push_back('\f'); break;
      case 'u': {  // control messages are ASCII; keep BMP code points < 0x80, else '?'
        if (i + 4 >= s.size()) return std::string::npos;
        unsigned v = 0;
        for (int k = 1; k <= 4; ++k) {
          char h = s[i + k];
          v <<= 4;
          if (h >= '0' && h <= '9') v |= h - '0';
          else if (h >= 'a' && h <= 'f') v |= h - 'a' + 10;
          else if (h >= 'A' && h <= 'F') v |= h - 'A' + 10;
          else return std::string::npos;
        }
        out.push_back(v < 0x80 ? static_cast<char>(v) : '?');
        i += 4;
        break;
      }
      default: return std::string::npos;
    }
  }
  return std::string::npos;
}

}  // namespace

bool parse_flat_json(const std::string& s, std::map<std::string, std::string>& out) {
  out.clear();
  size_t i = skip_ws(s, 0);
  if (i >= s.size() || s[i] != '{') return false;
  i = skip_ws(s, i + 1);
  if (i < s.size() && s[i] == '}') return skip_ws(s, i + 1) == s.size();
  for (;;) {
    std::string key, val;
    i = parse_string(s, i, key);
    if (i == std::string::npos) return false;
    i = skip_ws(s, i);
    if (i >= s.size() || s[i] != ':') return false;
    i = skip_ws(s, i + 1);
    if (i >= s.size()) return false;
    if (s[i] == '"') {
      i = parse_string(s, i, val);
      if (i == std::string::npos) return false;
    } else {  // number / true / false / null, verbatim
      size_t j = i;
      while (j < s.size() && s[j] != ',' && s[j] != '}' && s[j] != ' ' && s[j] != '\t') ++j;
      val = s.substr(i, j - i);
      if (val.empty() || val[0] == '{' || val[0] == '[') return false;  // flat objects only
      i = j;
    }
    out[key] = val;
    i = skip_ws(s, i);
    if (i >= s.size()) return false;
    if (s[i] == '}') return skip_ws(s, i + 1) == s.size();
    if (s[i] != ',') return false;
    i = skip_ws(s, i + 1);
  }
}

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(c);
    } else if (static_cast<unsigned char>(c) < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o.push_back(c);
    }
  }
  return o;
}

std::shared_ptr<ControlBridge> ControlBridge::start(const std::string& host, int port) {
  std::shared_ptr<ControlBridge> b(new ControlBridge());
  b->lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (b->lfd_ < 0) throw std::runtime_error("bridge: socket failed");
  int one = 1;
  ::setsockopt(b->lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (::inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw std::runtime_error("bridge: bad host " + host);
  if (::bind(b->lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(b->lfd_, 16) != 0)
    throw std::runtime_error("bridge: cannot listen on " + host + ":" + std::to_string(port) + ": " +
                             std::strerror(errno));
  socklen_t len = sizeof(a);
  ::getsockname(b->lfd_, reinterpret_cast<sockaddr*>(&a), &len);
  b->port_ = ntohs(a.sin_port);
  if (::pipe2(b->wake_, O_CLOEXEC) != 0) throw std::runtime_error("bridge: pipe failed");
  b->acceptor_ = std::thread([b] { b->accept_loop(b); });
  MXAR_LOG(INFO, "bridge", "----control bridge listening on " << host << ":" << b->port_);
  return b;
}

ControlBridge::~ControlBridge() { stop(); }

void ControlBridge::attach(ActorRef master, std::string master_path) {
  std::lock_guard<std::mutex> g(mu_);
  master_ = std::move(master);
  master_path_ = std::move(master_path);
}

void ControlBridge::set_init_line(std::string line) {
  std::lock_guard<std::mutex> g(mu_);
  init_line_ = std::move(line);
}

size_t ControlBridge::clients() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (auto& c : clients_) n += !c->dead.load();
  return n;
}

void ControlBridge::Client::kill() {
  if (dead.exchange(true)) return;
  {
    std::lock_guard<std::mutex> g(wmu);
    out.clear();
    queued = 0;
  }
  wcv.notify_all();
  ::shutdown(fd, SHUT_RDWR);  // the reader sees EOF, a blocked send returns
}

bool ControlBridge::write_line(Client& c, const std::string& line) {
  if (c.dead.load()) return false;
  bool overflow = false;
  {
    std::lock_guard<std::mutex> g(c.wmu);
    if (c.queued + line.size() + 1 > max_queued_.load()) {
      overflow = true;
    } else {
      c.out.push_back(line + "\n");
      c.queued += line.size() + 1;
    }
  }
  if (overflow) {
    MXAR_LOG(WARNING, "bridge", "client " << c.id << " stopped reading (" << max_queued_.load()
                                           << " bytes of events queued): disconnecting it");
    c.kill();
    return false;
  }
  c.wcv.notify_one();
  return true;
}

void ControlBridge::write_loop(std::shared_ptr<ControlBridge> self, std::shared_ptr<Client> c) {
  (void)self;  // keeps the bridge alive while this thread runs
  std::string buf;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(c->wmu);
      c->wcv.wait(g, [&] { return !c->out.empty() || c->dead.load(); });
      if (c->dead.load()) return;
      buf.clear();
      while (!c->out.empty()) {  // coalesce: one send for everything queued
        buf += c->out.front();
        c->out.pop_front();
      }
      c->queued = 0;
    }
    size_t off = 0;
    while (off < buf.size()) {
      ssize_t n = ::send(c->fd, buf.data() + off, buf.size() - off, MSG_NOSIGNAL);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        c->kill();
        return;
      }
      off += static_cast<size_t>(n);
    }
  }
}

void ControlBridge::publish(const std::string& line) {
  std::vector<std::shared_ptr<Client>> cs;
  std::vector<Tap> ts;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs = clients_;
    for (auto& t : taps_) ts.push_back(t.second);
  }
  for (auto& c : cs) write_line(*c, line);
  for (auto& t : ts) t(line);
}

void ControlBridge::reply(uint64_t client, const std::string& line) {
  std::shared_ptr<Client> c;
  Tap tap;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& x : clients_)
      if (x->id == client) c = x;
    for (auto& t : taps_)
      if (t.first == client) tap = t.second;
  }
  if (c) write_line(*c, line);
  if (tap) tap(line);
}

uint64_t ControlBridge::add_tap(Tap tap) {
  std::lock_guard<std::mutex> g(mu_);
  const uint64_t id = next_id_++;  // shares the client id space: replies find it by id
  taps_.emplace_back(id, std::move(tap));
  return id;
}

void ControlBridge::remove_tap(uint64_t id) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = taps_.begin(); it != taps_.end(); ++it)
    if (it->first == id) {
      taps_.erase(it);
      return;
    }
}

bool ControlBridge::submit(const BridgeCommand& cmd) {
  ActorRef m;
  {
    std::lock_guard<std::mutex> g(mu_);
    m = master_;
  }
  if (!m) return false;
  m->tell(Message(cmd), nullptr);
  return true;
}

void ControlBridge::on_stop(std::function<void()> hook) {
  std::lock_guard<std::mutex> g(mu_);
  stop_hooks_.push_back(std::move(hook));
}

void ControlBridge::reap() {  // join readers of clients that went away (mu_ not held)
  std::vector<std::shared_ptr<Client>> dead;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = clients_.begin(); it != clients_.end();) {
      if ((*it)->dead.load()) {
        dead.push_back(*it);
        it = clients_.erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& c : dead) {  // the fd closes with the last reference
    // A reader may still be inside tell() to the master (which can block while the actor
    // system shuts down): it is never joined, only detached - it holds references to the
    // bridge and its client, so it finishes safely on its own.
    if (c->reader.joinable()) c->reader.detach();
    if (c->writer.joinable()) c->writer.join();
  }
}

ControlBridge::Client::~Client() {
  // only reachable with a joinable thread from that thread itself at shutdown
  if (reader.joinable()) reader.detach();
  if (writer.joinable()) writer.detach();
  if (fd >= 0) ::close(fd);
}

void ControlBridge::accept_loop(std::shared_ptr<ControlBridge> self) {
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
    auto c = std::make_shared<Client>();
    c->fd = fd;
    std::string init;
    {
      std::lock_guard<std::mutex> g(mu_);
      c->id = next_id_++;
      clients_.push_back(c);
      init = init_line_;
    }
    write_line(*c, "{\"type\":\"Hello\",\"protocol\":\"mxar-bridge/1\",\"client\":" + std::to_string(c->id) +
                       ",\"master\":\"" + json_escape(master_path_) + "\"}");
    if (!init.empty()) write_line(*c, init);
    c->writer = std::thread([self, c] { self->write_loop(self, c); });
    c->reader = std::thread([self, c] { self->read_loop(self, c); });
  }
}

void ControlBridge::read_loop(std::shared_ptr<ControlBridge> self, std::shared_ptr<Client> c) {
  (void)self;  // keeps the bridge alive while this thread runs (tell() may drop the master)
  std::string buf;
  char tmp[4096];
  while (!stop_.load() && !c->dead.load()) {
    ssize_t n = ::recv(c->fd, tmp, sizeof(tmp), 0);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) break;
    buf.append(tmp, static_cast<size_t>(n));
    if (buf.size() > (1u << 20)) break;  // a control line is short; refuse a runaway peer
    size_t nl;
    while ((nl = buf.find('\n')) != std::string::npos) {
      std::string line = buf.substr(0, nl);
      buf.erase(0, nl + 1);
      if (line.find_first_not_of(" \t\r") == std::string::npos) continue;
      std::map<std::string, std::string> kv;
      if (!parse_flat_json(line, kv) || !kv.count("type")) {
        write_line(*c, "{\"type\":\"Error\",\"cmd\":\"?\",\"reason\":\"malformed line (want one flat JSON object "
                       "with a \\\"type\\\")\"}");
        continue;
      }
      const std::string& type = kv["type"];
      BridgeCommand cmd;
      cmd.client = c->id;
      if (type == "StartAllreduce") {
        cmd.kind = BridgeCommand::Start;
        char* end = nullptr;
        const std::string& rs = kv["round"];
        long v = std::strtol(rs.c_str(), &end, 10);
        if (rs.empty() || *end != '\0' || v < 0 || v > (1L << 30)) {
          write_line(*c, "{\"type\":\"Error\",\"cmd\":\"StartAllreduce\",\"reason\":\"round must be a "
                         "non-negative integer\"}");
          continue;
        }
        cmd.round = static_cast<int>(v);
      } else if (type == "Status") {
        cmd.kind = BridgeCommand::Status;
      } else {
        write_line(*c, "{\"type\":\"Error\",\"cmd\":\"" + json_escape(type) + "\",\"reason\":\"unknown command\"}");
        continue;
      }
      ActorRef m;
      {
        std::lock_guard<std::mutex> g(mu_);
        m = master_;
      }
      if (!m) {
        write_line(*c, "{\"type\":\"Error\",\"cmd\":\"" + json_escape(type) + "\",\"reason\":\"no master\"}");
        continue;
      }
      m->tell(Message(cmd), nullptr);
    }
  }
  c->kill();
}

void ControlBridge::stop() {
  if (stop_.exchange(true)) return;
  std::vector<std::function<void()>> hooks;
  {
    std::lock_guard<std::mutex> g(mu_);
    hooks.swap(stop_hooks_);
  }
  for (auto& h : hooks) h();
  if (wake_[1] >= 0) {
    char x = 1;
    (void)!::write(wake_[1], &x, 1);
  }
  // stop() can run on one of our own threads: a reader's tell() briefly owns the master's
  // cell, and if the system dropped it meanwhile ~MasterActor stops the bridge there (the
  // reader's own reference keeps the object alive until that thread returns).
  auto join = [](std::thread& t) {
    if (!t.joinable()) return;
    if (t.get_id() == std::this_thread::get_id()) t.detach();
    else t.join();
  };
  join(acceptor_);
  std::vector<std::shared_ptr<Client>> cs;
  {
    std::lock_guard<std::mutex> g(mu_);
    cs.swap(clients_);
    taps_.clear();
    master_ = nullptr;
  }
  for (auto& c : cs) {
    c->kill();
    // readers are detached, not joined: one may be blocked in tell() on the very system
    // whose shutdown is running this stop() (see reap)
    if (c->reader.joinable()) c->reader.detach();
    join(c->writer);
  }
  if (lfd_ >= 0) ::close(lfd_);
  for (int& f : wake_)
    if (f >= 0) ::close(f), f = -1;
  lfd_ = -1;
}

}  // namespace mxar
