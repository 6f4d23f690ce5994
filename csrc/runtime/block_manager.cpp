#include "block_manager.h"

namespace rfqrt {

BlockManager::BlockManager(int32_t num_blocks, int32_t block_size)
    : num_blocks_(num_blocks), block_size_(block_size), refcnt_(num_blocks, 0),
      block_hash_(num_blocks, 0), has_hash_(num_blocks, 0), lru_pos_(num_blocks),
      in_lru_(num_blocks, 0) {
  free_.reserve(num_blocks);
  for (int32_t b = num_blocks - 1; b >= 0; --b) free_.push_back(b);  // pop order 0,1,2,...
}

void BlockManager::lru_remove(int32_t b) {
  if (in_lru_[b]) {
    lru_.erase(lru_pos_[b]);
    in_lru_[b] = 0;
  }
}

bool BlockManager::allocate(int32_t n, std::vector<int32_t>& out) {
  if (n > num_free()) return false;
  for (int32_t i = 0; i < n; ++i) {
    int32_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {  // evict the least recently released cached block
      b = lru_.front();
      lru_.pop_front();
      in_lru_[b] = 0;
      if (has_hash_[b]) {
        auto it = hash_to_block_.find(block_hash_[b]);
        if (it != hash_to_block_.end() && it->second == b) hash_to_block_.erase(it);
        has_hash_[b] = 0;
      }
      ++evictions;
    }
    refcnt_[b] = 1;
    out.push_back(b);
  }
  return true;
}

void BlockManager::release(const int32_t* blocks, int32_t n) {
  for (int32_t i = 0; i < n; ++i) {
    const int32_t b = blocks[i];
    if (b < 0 || b >= num_blocks_ || refcnt_[b] <= 0) continue;
    if (--refcnt_[b] == 0) {
      if (has_hash_[b]) {
        lru_.push_back(b);
        lru_pos_[b] = std::prev(lru_.end());
        in_lru_[b] = 1;
      } else {
        free_.push_back(b);
      }
    }
  }
}

int32_t BlockManager::match_prefix(const uint64_t* hashes, int32_t n, std::vector<int32_t>& out) {
  int32_t m = 0;
  ++queries;
  for (; m < n; ++m) {
    auto it = hash_to_block_.find(hashes[m]);
    if (it == hash_to_block_.end()) break;
    const int32_t b = it->second;
    lru_remove(b);
    ++refcnt_[b];
    out.push_back(b);
  }
  if (m > 0) ++hits;
  return m;
}

void BlockManager::register_block(int32_t block, uint64_t hash) {
  if (block < 0 || block >= num_blocks_ || has_hash_[block]) return;
  if (hash_to_block_.count(hash)) return;
  hash_to_block_[hash] = block;
  block_hash_[block] = hash;
  has_hash_[block] = 1;
}

uint64_t BlockManager::hash_block(uint64_t parent, const int32_t* tokens, int32_t n) {
  uint64_t h = parent ^ 0x9E3779B97F4A7C15ULL;
  for (int32_t i = 0; i < n; ++i) {
    h ^= (uint64_t)(uint32_t)tokens[i] + 0x9E3779B97F4A7C15ULL + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ULL;
    h ^= h >> 31;
  }
  return h ? h : 1;
}

}  // namespace rfqrt
