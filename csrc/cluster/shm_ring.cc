#include "shm_ring.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <ctime>
#include <random>
#include <thread>

namespace mxar {

namespace {
constexpr size_t kHeaderBytes = 4096;

long futex(std::atomic<uint32_t>* w, int op, uint32_t v, const timespec* ts) {
  return ::syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, v, ts, nullptr, 0);
}
}  // namespace

std::unique_ptr<ShmRing> ShmRing::create(size_t capacity) {
  if (capacity < 4096 || (capacity & (capacity - 1))) return nullptr;
  std::random_device rd;
  const std::string name = "/mxar-" + std::to_string(::getpid()) + "-" + std::to_string(rd()) + std::to_string(rd());
  const int fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR | O_CLOEXEC, 0600);
  if (fd < 0) return nullptr;
  const size_t bytes = kHeaderBytes + capacity;
  if (::ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
    ::close(fd);
    ::shm_unlink(name.c_str());
    return nullptr;
  }
  void* m = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) {
    ::shm_unlink(name.c_str());
    return nullptr;
  }
  std::unique_ptr<ShmRing> r(new ShmRing());
  r->name_ = name;
  r->cap_ = capacity;
  r->map_bytes_ = bytes;
  r->map_ = m;
  r->h_ = new (m) Header();
  r->h_->tail.store(0);
  r->h_->head.store(0);
  r->h_->seq.store(0);
  r->h_->sleeping.store(0);
  r->data_ = static_cast<uint8_t*>(m) + kHeaderBytes;
  r->owner_ = true;
  return r;
}

std::unique_ptr<ShmRing> ShmRing::open(const std::string& name) {
  if (name.rfind("/mxar-", 0) != 0 || name.find('/', 1) != std::string::npos) return nullptr;
  const int fd = ::shm_open(name.c_str(), O_RDWR | O_CLOEXEC, 0600);
  if (fd < 0) return nullptr;
  struct stat st {};
  if (::fstat(fd, &st) != 0 || st.st_size <= static_cast<off_t>(kHeaderBytes)) {
    ::close(fd);
    return nullptr;
  }
  const size_t bytes = static_cast<size_t>(st.st_size);
  const size_t cap = bytes - kHeaderBytes;
  if (cap & (cap - 1)) {
    ::close(fd);
    return nullptr;
  }
  void* m = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return nullptr;
  ::shm_unlink(name.c_str());  // both sides hold a mapping: the name is no longer needed
  std::unique_ptr<ShmRing> r(new ShmRing());
  r->name_ = name;
  r->cap_ = cap;
  r->map_bytes_ = bytes;
  r->map_ = m;
  r->h_ = static_cast<Header*>(m);
  r->data_ = static_cast<uint8_t*>(m) + kHeaderBytes;
  return r;
}

ShmRing::~ShmRing() {
  if (map_) ::munmap(map_, map_bytes_);
  if (owner_) ::shm_unlink(name_.c_str());  // in case the peer never opened it (ENOENT otherwise)
}

bool ShmRing::write(const void* p, size_t n, const std::atomic<bool>* abandon) {
  const uint8_t* src = static_cast<const uint8_t*>(p);
  uint64_t tail = h_->tail.load(std::memory_order_relaxed);
  int idle = 0;
  while (n > 0) {
    const uint64_t head = h_->head.load(std::memory_order_acquire);
    const size_t room = cap_ - static_cast<size_t>(tail - head);
    if (room == 0) {  // full: the reader is behind (wake it if it sleeps on the data so far)
      if (abandon && abandon->load(std::memory_order_relaxed)) return false;
      if (idle == 0 && h_->sleeping.load(std::memory_order_seq_cst)) {
        h_->seq.fetch_add(1, std::memory_order_seq_cst);
        futex(&h_->seq, FUTEX_WAKE, 1, nullptr);
      }
      if (++idle < 256) {
        __builtin_ia32_pause();
      } else {
        std::this_thread::yield();
      }
      continue;
    }
    idle = 0;
    const size_t at = static_cast<size_t>(tail & (cap_ - 1));
    const size_t k = std::min({n, room, cap_ - at});
    std::memcpy(data_ + at, src, k);
    src += k;
    n -= k;
    tail += k;
    h_->tail.store(tail, std::memory_order_release);
  }
  // wake a sleeping reader (seq_cst pairs with the reader's sleeping store + tail re-check)
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (h_->sleeping.load(std::memory_order_relaxed)) {
    h_->seq.fetch_add(1, std::memory_order_seq_cst);
    futex(&h_->seq, FUTEX_WAKE, 1, nullptr);
  }
  return true;
}

size_t ShmRing::read(void* p, size_t n) {
  const uint64_t head = h_->head.load(std::memory_order_relaxed);
  const uint64_t tail = h_->tail.load(std::memory_order_acquire);
  size_t avail = static_cast<size_t>(tail - head);
  if (avail == 0) return 0;
  uint8_t* dst = static_cast<uint8_t*>(p);
  size_t got = 0;
  avail = std::min(avail, n);
  while (got < avail) {
    const size_t at = static_cast<size_t>((head + got) & (cap_ - 1));
    const size_t k = std::min(avail - got, cap_ - at);
    std::memcpy(dst + got, data_ + at, k);
    got += k;
  }
  h_->head.store(head + got, std::memory_order_release);
  return got;
}

bool ShmRing::empty() const {
  return h_->tail.load(std::memory_order_acquire) == h_->head.load(std::memory_order_relaxed);
}

bool ShmRing::wait(int timeout_ms) {
  const uint32_t s = h_->seq.load(std::memory_order_seq_cst);
  h_->sleeping.store(1, std::memory_order_seq_cst);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (!empty()) {
    h_->sleeping.store(0, std::memory_order_relaxed);
    return true;
  }
  timespec ts{timeout_ms / 1000, static_cast<long>(timeout_ms % 1000) * 1000000L};
  futex(&h_->seq, FUTEX_WAIT, s, &ts);
  h_->sleeping.store(0, std::memory_order_relaxed);
  return !empty();
}

}  // namespace mxar
