#include "engine_core.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace rfqrt {

namespace {

int64_t seed64(int64_t req_seed, int64_t pos) {
  uint64_t x = (uint64_t)req_seed * 0x9E3779B97F4A7C15ull + (uint64_t)pos * 0xBF58476D1CE4E5B9ull +
               0x94D049BB133111EBull;
  x ^= x >> 31;
  return (int64_t)x;
}

inline int32_t f2i(float f) {
  int32_t i;
  std::memcpy(&i, &f, 4);
  return i;
}

}  // namespace

EngineCore::EngineCore(const CoreConfig& cfg, std::shared_ptr<const Grammar> grammar)
    : cfg_(cfg), max_batched_tokens0_(cfg.max_batched_tokens), grammar_(std::move(grammar)),
      bm_(cfg.num_blocks, cfg.block_size) {}

// ------------------------------------------------------------------ requests
int32_t EngineCore::add(const int32_t* prompt, int32_t n, const SeqParams& p, double t_arrival) {
  int32_t id;
  if (!free_ids_.empty()) {
    id = free_ids_.back();
    free_ids_.pop_back();
  } else {
    id = (int32_t)seqs_.size();
    seqs_.emplace_back();
  }
  Seq& s = seqs_[id];
  s = Seq();
  s.live = true;
  s.tokens.assign(prompt, prompt + n);
  s.prompt_len = n;
  s.p = p;
  if (s.p.max_tokens > cfg_.max_model_len - n) s.p.max_tokens = std::max(1, cfg_.max_model_len - n);
  s.t_arrival = t_arrival;
  if (p.grammar && grammar_) {
    std::vector<int32_t> forced;
    s.gs = grammar_->initial(forced, p.min_items, p.profile, s.p.max_tokens);
    s.has_gs = true;
    s.tokens.insert(s.tokens.end(), forced.begin(), forced.end());
    s.num_forced += (int32_t)forced.size();
    s.mask_idx = grammar_->mask(s.gs);
  }
  waiting_.push_back(id);
  return id;
}

void EngineCore::release(int32_t id) {
  if (id < 0 || id >= (int32_t)seqs_.size() || !seqs_[id].live) return;
  Seq& s = seqs_[id];
  if (s.status != S_FINISHED) throw std::runtime_error("release of an unfinished sequence");
  s = Seq();
  free_ids_.push_back(id);
}

std::vector<int32_t> EngineCore::abort_all(FinishReason why, double now) {
  std::vector<int32_t> out;
  std::vector<int32_t> all(running_.begin(), running_.end());
  all.insert(all.end(), waiting_.begin(), waiting_.end());
  for (int32_t id : all) finish(id, why, now, out);
  running_.clear();
  waiting_.clear();
  decode_.clear();
  extend_.clear();
  rows_.clear();
  return out;
}

bool EngineCore::abort(int32_t id, FinishReason why, double now) {
  if (id < 0 || id >= (int32_t)seqs_.size() || !seqs_[id].live) return false;
  if (seqs_[id].status == S_FINISHED) return false;
  auto w = std::find(waiting_.begin(), waiting_.end(), id);
  if (w != waiting_.end()) waiting_.erase(w);
  auto r = std::find(running_.begin(), running_.end(), id);
  if (r != running_.end()) running_.erase(r);
  std::vector<int32_t> sink;
  finish(id, why, now, sink);
  return true;
}

// ---------------------------------------------------------------- KV blocks
int32_t EngineCore::blocks_needed(const Seq& s, int32_t upto) const {
  const int32_t need = (upto + cfg_.block_size - 1) / cfg_.block_size;
  return std::max(0, need - (int32_t)s.blocks.size());
}

bool EngineCore::grow(Seq& s, int32_t upto) {
  const int32_t n = blocks_needed(s, upto);
  if (n == 0) return true;
  scratch_.clear();
  if (!bm_.allocate(n, scratch_)) return false;
  s.blocks.insert(s.blocks.end(), scratch_.begin(), scratch_.end());
  return true;
}

void EngineCore::admit(Seq& s) {
  const int32_t bs = cfg_.block_size;
  if (!cfg_.prefix_cache || s.prompt_len <= bs) return;
  const int32_t nfull = s.prompt_len / bs;
  s.block_hashes.resize(nfull);
  uint64_t h = 0;
  for (int32_t i = 0; i < nfull; ++i) {
    h = BlockManager::hash_block(h, s.tokens.data() + (int64_t)i * bs, bs);
    s.block_hashes[i] = h;
  }
  // keep >= 1 prompt token to compute so the first sampled token has logits
  const int32_t usable = (s.prompt_len - 1) / bs;
  std::vector<int32_t> hit;
  bm_.match_prefix(s.block_hashes.data(), usable, hit);
  if (!hit.empty()) {
    s.blocks = hit;
    s.num_cached = (int32_t)hit.size() * bs;
    s.num_registered = (int32_t)hit.size();
    s.prefix_hit = s.num_cached;
  }
}

void EngineCore::publish(Seq& s) {
  if (!cfg_.prefix_cache || s.block_hashes.empty()) return;
  int32_t full = std::min(s.num_cached, s.prompt_len) / cfg_.block_size;
  full = std::min(full, (int32_t)s.block_hashes.size());
  for (int32_t i = s.num_registered; i < full; ++i) bm_.register_block(s.blocks[i], s.block_hashes[i]);
  s.num_registered = std::max(s.num_registered, full);
}

void EngineCore::preempt(int32_t id) {
  Seq& s = seqs_[id];
  if (!s.blocks.empty()) bm_.release(s.blocks.data(), (int32_t)s.blocks.size());
  s.blocks.clear();
  s.num_cached = 0;
  s.num_registered = 0;
  s.status = S_WAITING;
  auto it = std::find(running_.begin(), running_.end(), id);
  if (it != running_.end()) running_.erase(it);
  waiting_.push_front(id);
  ++num_preempted;
}

int32_t EngineCore::preempt_victim(int32_t exclude) const {
  auto it = std::find(running_.begin(), running_.end(), exclude);
  const size_t start = it == running_.end() ? 0 : (size_t)(it - running_.begin()) + 1;
  for (size_t k = running_.size(); k > start; --k) {
    const int32_t v = running_[k - 1];
    const Seq& s = seqs_[v];
    if (s.status == S_RUNNING && !s.blocks.empty()) return v;
  }
  return -1;
}

void EngineCore::finish(int32_t id, FinishReason why, double now, std::vector<int32_t>& out) {
  Seq& s = seqs_[id];
  if (s.status == S_FINISHED) return;
  s.status = S_FINISHED;
  s.finish = why;
  s.t_finish = now;
  if (!s.blocks.empty()) bm_.release(s.blocks.data(), (int32_t)s.blocks.size());
  s.blocks.clear();
  out.push_back(id);
}

// ----------------------------------------------------------------- schedule
void EngineCore::schedule(double now) {
  decode_.clear();
  extend_.clear();
  int32_t budget = cfg_.max_batched_tokens;
  std::vector<int32_t> keep;
  keep.reserve(running_.size());
  const std::vector<int32_t> snapshot = running_;
  for (int32_t id : snapshot) {
    Seq& s = seqs_[id];
    if (s.status != S_RUNNING) continue;                 // preempted earlier in this loop
    if (s.pending() <= 0) {
      keep.push_back(id);
      continue;
    }
    int32_t q;
    if (s.pending() == 1 && !s.in_prefill()) q = 1;
    else if (s.in_prefill() || cfg_.jump_forward) q = std::min(s.pending(), std::max(1, budget));
    else q = 1;
    if (q > 1 && budget <= 1) {                           // out of budget: next step
      keep.push_back(id);
      continue;
    }
    while (!grow(s, s.num_cached + q)) {
      const int32_t v = preempt_victim(id);
      if (v < 0) break;
      preempt(v);
      auto it = std::find(keep.begin(), keep.end(), v);
      if (it != keep.end()) keep.erase(it);
    }
    if (blocks_needed(s, s.num_cached + q)) {
      preempt(id);
      continue;
    }
    keep.push_back(id);
    if (q == 1 && !s.in_prefill()) decode_.push_back(id);
    else extend_.push_back({id, q});
    budget -= q;
  }
  running_.clear();
  for (int32_t id : keep)
    if (seqs_[id].status == S_RUNNING) running_.push_back(id);
  // admission
  while (!waiting_.empty() && budget > 0 && (int32_t)running_.size() < cfg_.max_num_seqs) {
    const int32_t id = waiting_.front();
    Seq& s = seqs_[id];
    if (s.blocks.empty()) admit(s);
    const int32_t q = std::min(s.pending(), budget);
    if (!grow(s, s.num_cached + q)) break;
    waiting_.pop_front();
    s.status = S_RUNNING;
    if (!s.t_first_sched) s.t_first_sched = now;
    running_.push_back(id);
    extend_.push_back({id, q});
    budget -= q;
  }
  // Nothing runnable although the whole pool is free: the head request cannot fit
  // even alone.  Retire it (truncated if it had generated tokens) instead of
  // spinning on it forever.
  if (decode_.empty() && extend_.empty() && running_.empty() && !waiting_.empty()) {
    const int32_t id = waiting_.front();
    waiting_.pop_front();
    finish(id, seqs_[id].generated() > seqs_[id].num_forced ? F_LENGTH : F_ABORT, now, finished_);
  }
}

std::vector<int32_t> EngineCore::drain_finished() {
  std::vector<int32_t> out;
  out.swap(finished_);
  return out;
}

int32_t EngineCore::decode_splits(int32_t na, int32_t max_ctx, bool graph) const {
  if (na == 0 || !cfg_.is_cuda) return 1;
  const int64_t wg = (int64_t)na * cfg_.hkv;
  int32_t s = 1;
  while (wg * s < 1024 && s < 16) s *= 2;
  if (!graph) s = std::max(1, std::min(s, (max_ctx + 255) / 256));
  return s;
}

int32_t EngineCore::pin_prefix(const int32_t* tokens, int32_t n) {
  const int32_t bs = cfg_.block_size, nfull = n / bs;
  std::vector<uint64_t> hashes(nfull);
  uint64_t h = 0;
  for (int32_t i = 0; i < nfull; ++i) {
    h = BlockManager::hash_block(h, tokens + (int64_t)i * bs, bs);
    hashes[i] = h;
  }
  std::vector<int32_t> got;
  bm_.match_prefix(hashes.data(), nfull, got);   // +1 reference each, never released
  pinned_.insert(pinned_.end(), got.begin(), got.end());
  return (int32_t)got.size();
}

void EngineCore::set_graph_keys(const std::vector<std::pair<int32_t, int32_t>>& keys) {
  graph_keys_ = keys;
  std::sort(graph_keys_.begin(), graph_keys_.end());
  nb_buckets_.clear();
  for (auto& k : graph_keys_)
    if (nb_buckets_.empty() || nb_buckets_.back() != k.first) nb_buckets_.push_back(k.first);
}

// Smallest captured (sequence bucket, token bucket) that holds na sequences and t
// tokens.  Normally only the first sequence bucket >= na is tried: past it the
// padding would cost more than eager launches save.  In the latency regime (a
// bucket of at most kLatencyBucket sequences) a step whose jump-forward extends
// outgrow that bucket's token multiples (t > 8 na) moves up to the next buckets:
// padded rows of a replayed graph cost far less than ~500 eager launches.
constexpr int32_t kLatencyBucket = 16;

bool EngineCore::graph_key(int32_t na, int32_t t, int32_t& nb, int32_t& tb) const {
  for (int32_t b : nb_buckets_) {
    if (b < na) continue;
    for (int32_t m : cfg_.token_mults) {
      const std::pair<int32_t, int32_t> k{b, b * m};
      if (b * m >= t && std::binary_search(graph_keys_.begin(), graph_keys_.end(), k)) {
        nb = b;
        tb = b * m;
        return true;
      }
    }
    if (b > kLatencyBucket) return false;
  }
  return false;
}

int64_t EngineCore::payload_bound() const {
  const int64_t N = std::max(cfg_.max_num_seqs, nb_buckets_.empty() ? 1 : nb_buckets_.back());
  int64_t T = (int64_t)cfg_.max_batched_tokens + N;
  for (auto& k : graph_keys_) T = std::max<int64_t>(T, k.second);
  const int64_t maxb = (cfg_.max_model_len + cfg_.block_size - 1) / cfg_.block_size;
  const int64_t WA = T * cfg_.group / 16 + N + 1, WB = T / 32 + N + 1;
  return 2 * N + 3 * T + 2 * N * maxb + 6 * N + 2 * WA + 2 * WB + 3 * N + 64;
}

// --------------------------------------------------------------------- pack
int64_t EngineCore::schedule_and_pack(int32_t* header, int32_t* payload, int64_t capacity,
                                      double now) {
  schedule(now);
  std::fill(header, header + HEADER, 0);
  rows_.clear();
  if (decode_.empty() && extend_.empty()) return 0;
  const int32_t bs = cfg_.block_size, G = cfg_.group;
  // sections: A = decode rows + short extends, B = prefill chunks
  std::vector<Row> A, B;
  A.reserve(decode_.size() + extend_.size());
  for (int32_t id : decode_) A.push_back({id, 1});
  for (auto& r : extend_) (r.q <= cfg_.ext_max ? A : B).push_back(r);
  int32_t TA = 0, TB = 0, WA = 0, WB = 0, maxb = 1, max_ctx = 0;
  const int32_t NTL = std::max(1, cfg_.decode_tiles);
  auto items = [&](int32_t q) { return ((q * G + 15) / 16 + NTL - 1) / NTL; };
  for (auto& r : A) {
    TA += r.q;
    WA += items(r.q);
    maxb = std::max(maxb, (int32_t)seqs_[r.id].blocks.size());
    max_ctx = std::max(max_ctx, seqs_[r.id].num_cached + r.q);
  }
  int32_t S = (int32_t)A.size();
  for (auto& r : B) {
    TB += r.q;
    WB += (r.q + cfg_.prefill_qblk - 1) / cfg_.prefill_qblk;
    maxb = std::max(maxb, (int32_t)seqs_[r.id].blocks.size());
    const Seq& s = seqs_[r.id];
    S += (s.num_cached + r.q == (int32_t)s.tokens.size());
  }
  const int32_t T = TA + TB, NA = (int32_t)A.size(), NB = (int32_t)B.size();
  int32_t gnb = 0, gtb = 0;
  const bool graph = cfg_.is_cuda && cfg_.use_graphs && NB == 0 && graph_key(NA, T, gnb, gtb);
  // padded (graph) or exact sizes
  int32_t Th = T, TAh = TA, NAh = NA, WAh = WA, Sh = S, splits;
  if (graph) {
    maxb = (cfg_.max_model_len + bs - 1) / bs;
    Th = TAh = WAh = gtb;
    NAh = Sh = gnb;
    splits = decode_splits(gnb, 0, true);
  } else {
    splits = decode_splits(NA, max_ctx, false);
  }
  const int64_t need = 2 * (int64_t)Sh + 3 * (int64_t)Th + (int64_t)NAh * maxb + 3 * NAh + 2 * WAh +
                       (int64_t)NB * maxb + 3 * NB + 2 * WB + 3 * Sh;
  if (need > capacity) throw std::runtime_error("step payload exceeds the staging buffer");

  int64_t* seeds = reinterpret_cast<int64_t*>(payload);     // payload is 8-byte aligned
  int32_t* ids = payload + 2 * Sh;
  int32_t* pos = ids + Th;
  int32_t* slots = pos + Th;
  int32_t* a_bt = slots + Th;
  int32_t* a_qs = a_bt + (int64_t)NAh * maxb;
  int32_t* a_ql = a_qs + NAh;
  int32_t* a_kvl = a_ql + NAh;
  int32_t* a_ws = a_kvl + NAh;
  int32_t* a_wct = a_ws + WAh;
  int32_t* b_bt = a_wct + WAh;
  int32_t* b_qs = b_bt + (int64_t)NB * maxb;
  int32_t* b_ql = b_qs + NB;
  int32_t* b_kvl = b_ql + NB;
  int32_t* b_ws = b_kvl + NB;
  int32_t* b_wq = b_ws + WB;
  int32_t* lidx = b_wq + WB;
  int32_t* midx = lidx + Sh;
  int32_t* temps = midx + Sh;

  int32_t t = 0, w = 0, k = 0;
  for (int32_t j = 0; j < NA; ++j) {
    const Row& r = A[j];
    const Seq& s = seqs_[r.id];
    const int32_t p0 = s.num_cached;
    for (int32_t i = 0; i < r.q; ++i) {
      const int32_t p = p0 + i;
      ids[t + i] = s.tokens[p];
      pos[t + i] = p;
      slots[t + i] = s.blocks[p / bs] * bs + p % bs;
    }
    int32_t* bt = a_bt + (int64_t)j * maxb;
    const int32_t nb = (int32_t)s.blocks.size();
    std::copy(s.blocks.begin(), s.blocks.end(), bt);
    std::fill(bt + nb, bt + maxb, cfg_.scratch_block);
    a_qs[j] = t;
    a_ql[j] = r.q;
    a_kvl[j] = p0 + r.q;
    const int32_t nct = items(r.q);
    for (int32_t c = 0; c < nct; ++c, ++w) {
      a_ws[w] = j;
      a_wct[w] = c;
    }
    lidx[k] = t + r.q - 1;
    rows_.push_back({r.id, p0 + r.q == (int32_t)s.tokens.size()});
    ++k;
    t += r.q;
  }
  w = 0;
  for (int32_t j = 0; j < NB; ++j) {
    const Row& r = B[j];
    const Seq& s = seqs_[r.id];
    const int32_t p0 = s.num_cached;
    for (int32_t i = 0; i < r.q; ++i) {
      const int32_t p = p0 + i;
      ids[t + i] = s.tokens[p];
      pos[t + i] = p;
      slots[t + i] = s.blocks[p / bs] * bs + p % bs;
    }
    int32_t* bt = b_bt + (int64_t)j * maxb;
    const int32_t nb = (int32_t)s.blocks.size();
    std::copy(s.blocks.begin(), s.blocks.end(), bt);
    std::fill(bt + nb, bt + maxb, cfg_.scratch_block);
    b_qs[j] = t - TA;
    b_ql[j] = r.q;
    b_kvl[j] = p0 + r.q;
    const int32_t nqb = (r.q + cfg_.prefill_qblk - 1) / cfg_.prefill_qblk;
    for (int32_t c = 0; c < nqb; ++c, ++w) {
      b_ws[w] = j;
      b_wq[w] = c;
    }
    if (p0 + r.q == (int32_t)s.tokens.size()) {
      lidx[k] = t + r.q - 1;
      rows_.push_back({r.id, true});
      ++k;
    }
    t += r.q;
  }
  for (int32_t i = 0; i < k; ++i) {
    const Seq& s = seqs_[rows_[i].first];
    midx[i] = s.p.grammar && s.has_gs ? s.mask_idx : -1;
    temps[i] = f2i(s.p.temperature);
    seeds[i] = seed64(s.p.seed, (int64_t)s.tokens.size());
  }
  if (graph) {   // pad to the captured bucket: padding rows touch only the scratch page
    for (int32_t i = T; i < Th; ++i) { ids[i] = 0; pos[i] = 0; slots[i] = -1; }
    for (int32_t j = NA; j < NAh; ++j) {
      std::fill(a_bt + (int64_t)j * maxb, a_bt + (int64_t)(j + 1) * maxb, cfg_.scratch_block);
      a_qs[j] = 0; a_ql[j] = 0; a_kvl[j] = 1;
    }
    for (int32_t i = WA; i < WAh; ++i) { a_ws[i] = -1; a_wct[i] = 0; }
    for (int32_t i = k; i < Sh; ++i) { lidx[i] = 0; midx[i] = -1; temps[i] = 0; seeds[i] = 0; }
    header[H_GNB] = gnb;
    header[H_GTB] = gtb;
  }
  header[H_T] = Th; header[H_TA] = TAh; header[H_NA] = NAh; header[H_WA] = WAh;
  header[H_NB] = NB; header[H_WB] = WB; header[H_S] = Sh; header[H_MAXB] = maxb;
  header[H_SPLITS] = splits; header[H_PAYLOAD] = (int32_t)need; header[H_TILES] = NTL;
  ++num_steps;
  return need;
}

// --------------------------------------------------------------------- post
std::vector<int32_t> EngineCore::post(const int32_t* sampled, int32_t n, double now) {
  std::vector<int32_t> done;
  done.swap(finished_);
  for (int32_t id : decode_) seqs_[id].num_cached += 1;
  for (auto& r : extend_) {
    Seq& s = seqs_[r.id];
    s.num_cached += r.q;
    publish(s);
    if (!s.t_prefill_done && !s.in_prefill()) s.t_prefill_done = now;
  }
  if (n < (int32_t)rows_.size()) throw std::runtime_error("post: fewer sampled ids than rows");
  std::vector<int32_t> forced;
  for (size_t i = 0; i < rows_.size(); ++i) {
    if (!rows_[i].second) continue;
    const int32_t id = rows_[i].first;
    Seq& s = seqs_[id];
    const int32_t tok = sampled[i];
    s.tokens.push_back(tok);
    s.num_sampled += 1;
    if (!s.t_first_token) s.t_first_token = now;
    if (s.has_gs) {
      forced.clear();
      const bool ok = grammar_->advance(s.gs, tok, forced, s.p.max_tokens - s.generated());
      s.tokens.insert(s.tokens.end(), forced.begin(), forced.end());
      s.num_forced += (int32_t)forced.size();
      s.mask_idx = grammar_->mask(s.gs);
      if (!ok) finish(id, F_GRAMMAR_ERROR, now, done);
      else if (s.mask_idx < 0) finish(id, F_STOP, now, done);
      else if (s.generated() >= s.p.max_tokens) finish(id, F_LENGTH, now, done);
    } else {
      if (std::find(cfg_.eos_ids.begin(), cfg_.eos_ids.end(), tok) != cfg_.eos_ids.end())
        finish(id, F_STOP, now, done);
      else if (s.generated() >= s.p.max_tokens)
        finish(id, F_LENGTH, now, done);
    }
  }
  if (!done.empty()) {
    running_.erase(std::remove_if(running_.begin(), running_.end(),
                                  [&](int32_t id) { return seqs_[id].status == S_FINISHED; }),
                   running_.end());
  }
  decode_.clear();
  extend_.clear();
  rows_.clear();
  return done;
}

}  // namespace rfqrt
