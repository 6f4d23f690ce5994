// Host shared-memory broadcast channel for the TP control plane (SURVEY.md §2.5 C4,
// §5.8): TP rank 0 owns the scheduler and publishes each packed step (header +
// payload, a few KB) to the worker ranks of its node through one POSIX shared
// memory segment instead of a device collective.  Workers copy the step out and
// upload it to their own GPU; no RCCL call, no device->host round trip.
//
// Single writer, N readers, one slot: the writer waits until every reader has
// acknowledged the previous message before overwriting it (steps are strictly
// sequential anyway).  Sequence numbers are 64-bit atomics in the segment;
// waits spin briefly and then sleep, and give up after a timeout so a dead peer
// surfaces as an error instead of a hang.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace rfqrt {

class ShmRing {
 public:
  static constexpr int kMaxReaders = 16;

  // create=true: writer (owner, unlinks on destruction); false: reader `reader_id`.
  ShmRing(const std::string& name, int64_t capacity, int n_readers, bool create,
          int reader_id = -1);
  ~ShmRing();
  ShmRing(const ShmRing&) = delete;
  ShmRing& operator=(const ShmRing&) = delete;

  // Writer: returns false on timeout (a reader stopped acknowledging).
  bool publish(const void* data, int64_t n, double timeout_s);
  // Reader: copies the next message into `out`; false on timeout.
  bool receive(std::vector<uint8_t>& out, double timeout_s);

  int64_t capacity() const { return capacity_; }
  const std::string& name() const { return name_; }

 private:
  struct Header {
    std::atomic<uint64_t> seq;
    std::atomic<int64_t> len;
    std::atomic<uint64_t> ack[kMaxReaders];
    int32_t n_readers;
    int32_t pad[15];
  };
  std::string name_;
  int64_t capacity_;
  int n_readers_;
  bool owner_;
  int reader_id_;
  uint64_t last_seen_ = 0;
  size_t map_bytes_ = 0;
  Header* hdr_ = nullptr;
  uint8_t* data_ = nullptr;
};

}  // namespace rfqrt
