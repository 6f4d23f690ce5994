#include "shm_ring.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace rfqrt {

namespace {

// Spin for a few microseconds (a step's metadata is usually ready within the
// window), then back off to short sleeps so an idle worker does not burn a core.
template <typename Pred>
bool wait_until(Pred ready, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (int i = 0; i < 2000; ++i)
    if (ready()) return true;
  while (true) {
    if (ready()) return true;
    if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_s) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

}  // namespace

ShmRing::ShmRing(const std::string& name, int64_t capacity, int n_readers, bool create,
                 int reader_id)
    : name_(name), capacity_(capacity), n_readers_(n_readers), owner_(create),
      reader_id_(reader_id) {
  if (n_readers < 0 || n_readers > kMaxReaders) throw std::invalid_argument("shm ring: readers");
  if (!create && (reader_id < 0 || reader_id >= n_readers))
    throw std::invalid_argument("shm ring: reader id");
  map_bytes_ = sizeof(Header) + (size_t)capacity;
  const std::string path = "/" + name;
  int fd = create ? shm_open(path.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600)
                  : shm_open(path.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open failed for " + path);
  if (create && ftruncate(fd, (off_t)map_bytes_) != 0) {
    close(fd);
    shm_unlink(path.c_str());
    throw std::runtime_error("ftruncate failed for " + path);
  }
  void* p = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("mmap failed for " + path);
  hdr_ = reinterpret_cast<Header*>(p);
  data_ = reinterpret_cast<uint8_t*>(p) + sizeof(Header);
  if (create) {
    hdr_->seq.store(0);
    hdr_->len.store(0);
    for (auto& a : hdr_->ack) a.store(0);
    hdr_->n_readers = n_readers;
  } else {
    last_seen_ = hdr_->seq.load(std::memory_order_acquire);
  }
}

ShmRing::~ShmRing() {
  if (hdr_) munmap(hdr_, map_bytes_);
  if (owner_) shm_unlink(("/" + name_).c_str());
}

bool ShmRing::publish(const void* data, int64_t n, double timeout_s) {
  if (n > capacity_) throw std::length_error("shm ring: message exceeds capacity");
  const uint64_t cur = hdr_->seq.load(std::memory_order_relaxed);
  const bool acked = wait_until([&] {
    for (int r = 0; r < n_readers_; ++r)
      if (hdr_->ack[r].load(std::memory_order_acquire) < cur) return false;
    return true;
  }, timeout_s);
  if (!acked) return false;
  std::memcpy(data_, data, (size_t)n);
  hdr_->len.store(n, std::memory_order_relaxed);
  hdr_->seq.store(cur + 1, std::memory_order_release);
  return true;
}

bool ShmRing::receive(std::vector<uint8_t>& out, double timeout_s) {
  const bool ready = wait_until(
      [&] { return hdr_->seq.load(std::memory_order_acquire) > last_seen_; }, timeout_s);
  if (!ready) return false;
  const uint64_t s = hdr_->seq.load(std::memory_order_acquire);
  const int64_t n = hdr_->len.load(std::memory_order_relaxed);
  out.resize((size_t)n);
  std::memcpy(out.data(), data_, (size_t)n);
  last_seen_ = s;
  hdr_->ack[reader_id_].store(s, std::memory_order_release);
  return true;
}

}  // namespace rfqrt
