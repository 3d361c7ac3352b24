// Shared-memory byte stream between two processes of one host: the cluster transport's fast
// path for co-located members (ClusterNode, same-host peers - the reference deployment runs
// the master and its workers as processes on one machine, AllreduceMaster.scala:116-120).
// A TCP hop costs two syscalls and a wake-up per frame; here a frame is a memcpy into a
// single-producer / single-consumer ring plus one release store, and a polling reader sees
// it a fraction of a microsecond later. The ring carries the same length-prefixed frames as
// the socket, as a byte stream (a frame larger than the ring is written in pieces).
//
// Wake-up: the reader polls (the transport's spin budget, MXAR_TCP_SPIN_US), then sleeps on a
// futex in the shared page; the writer wakes it only when it announced that it sleeps.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace mxar {

class ShmRing {
 public:
  // Creator side: a fresh POSIX shm object of `capacity` bytes (a power of two) named
  // "/mxar-<pid>-<random>"; nullptr on failure.
  static std::unique_ptr<ShmRing> create(size_t capacity);
  // Peer side: maps the named object and unlinks the name (the mapping keeps it alive).
  static std::unique_ptr<ShmRing> open(const std::string& name);
  ~ShmRing();
  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;

  const std::string& name() const { return name_; }
  size_t capacity() const { return cap_; }

  // Writer: appends n bytes, waiting (spin, then yield) while the ring is full; false when
  // `abandon` becomes true meanwhile (the connection is closing).
  bool write(const void* p, size_t n, const std::atomic<bool>* abandon = nullptr);
  // Reader: copies up to n available bytes; 0 when nothing is there.
  size_t read(void* p, size_t n);
  // Reader: waits up to timeout_ms for data (futex; the writer wakes it). True if data.
  bool wait(int timeout_ms);
  bool empty() const;

 private:
  struct Header {
    alignas(64) std::atomic<uint64_t> tail;   // bytes written (writer)
    alignas(64) std::atomic<uint64_t> head;   // bytes consumed (reader)
    alignas(64) std::atomic<uint32_t> seq;    // futex word: bumped by the writer
    std::atomic<uint32_t> sleeping;           // the reader sleeps on seq
  };
  ShmRing() = default;
  std::string name_;
  size_t cap_ = 0;
  size_t map_bytes_ = 0;
  void* map_ = nullptr;
  Header* h_ = nullptr;
  uint8_t* data_ = nullptr;
  bool owner_ = false;
};

}  // namespace mxar
