// Paged KV-cache block manager with a content-addressed prefix cache.
//
// The reference prompt is ~465 tokens of identical system message + template
// followed by the document.  Full 32-token blocks are identified
// by a chained 64-bit hash of their token ids (hash of block i covers blocks
// 0..i), so any request whose prompt starts with the same blocks reuses their KV
// pages: refcounted sharing, and blocks whose refcount drops to zero stay
// cached (LRU) until the allocator needs them.
#pragma once
#include <cstdint>
#include <list>
#include <unordered_map>
#include <vector>

namespace rfqrt {

class BlockManager {
 public:
  BlockManager(int32_t num_blocks, int32_t block_size);

  int32_t num_blocks() const { return num_blocks_; }
  int32_t block_size() const { return block_size_; }
  int32_t num_free() const { return (int32_t)free_.size() + (int32_t)lru_.size(); }
  int32_t num_cached() const { return (int32_t)hash_to_block_.size(); }

  // Allocate n fresh blocks (refcount 1); evicts LRU cached blocks when needed.
  // Returns false (allocating nothing) if fewer than n blocks are available.
  bool allocate(int32_t n, std::vector<int32_t>& out);
  void release(const int32_t* blocks, int32_t n);
  // Longest cached prefix of `hashes`: appends the blocks (refcount +1) to out.
  int32_t match_prefix(const uint64_t* hashes, int32_t n, std::vector<int32_t>& out);
  // Publish a completely filled block under `hash` (no-op if the hash is present).
  void register_block(int32_t block, uint64_t hash);
  int32_t refcount(int32_t block) const { return refcnt_[block]; }

  static uint64_t hash_block(uint64_t parent, const int32_t* tokens, int32_t n);

  uint64_t hits = 0, queries = 0, evictions = 0;

 private:
  void lru_remove(int32_t b);
  int32_t num_blocks_, block_size_;
  std::vector<int32_t> refcnt_;
  std::vector<int32_t> free_;
  std::vector<uint64_t> block_hash_;
  std::vector<uint8_t> has_hash_;
  std::unordered_map<uint64_t, int32_t> hash_to_block_;
  std::list<int32_t> lru_;
  std::vector<std::list<int32_t>::iterator> lru_pos_;
  std::vector<uint8_t> in_lru_;
};

}  // namespace rfqrt
