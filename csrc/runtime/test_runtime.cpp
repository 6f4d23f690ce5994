// Sanitizer harness for the host runtime (race / memory-error
// detection).  Built with -fsanitize=address,undefined (host only — GPU ASan is
// unavailable on this pool) by tests/engine/test_runtime_sanitized.py:
//
//   test_runtime <grammar.bin> [walks] [seed]
//
//  1. BlockManager fuzz: random allocate / release / register / match_prefix
//     against a shadow model of refcounts, checking every invariant.
//  2. Grammar random walks: from initial(min_items, profile, budget), repeatedly
//     pick a random token allowed by the current mask row and advance — every
//     pick must be accepted and every walk must finish inside its token budget
//     (random budgets 200..1200 exercise the close-out).
// Prints "OK ..." and exits 0 on success; any violation aborts.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "block_manager.h"
#include "engine_core.h"
#include "grammar.h"

using namespace rfqrt;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                       \
    }                                                                     \
  } while (0)

// ---------------------------------------------------------------- blob reader
// record := name[32] kind(u8: 'i' int32, 'b' uint8, 'u' uint32) pad[7] count(i64) data
struct Blob {
  std::map<std::string, std::vector<uint8_t>> raw;
  std::map<std::string, char> kind;
  template <typename T>
  std::vector<T> get(const char* k) const {
    auto it = raw.find(k);
    CHECK(it != raw.end());
    std::vector<T> v(it->second.size() / sizeof(T));
    if (!v.empty()) std::memcpy(v.data(), it->second.data(), v.size() * sizeof(T));
    return v;
  }
};

static Blob read_blob(const char* path) {
  Blob b;
  FILE* f = std::fopen(path, "rb");
  CHECK(f);
  char name[33] = {0};
  while (std::fread(name, 1, 32, f) == 32) {
    uint8_t hdr[8];
    int64_t n;
    CHECK(std::fread(hdr, 1, 8, f) == 8);
    CHECK(std::fread(&n, 8, 1, f) == 1);
    size_t es = hdr[0] == 'b' ? 1 : 4;
    std::vector<uint8_t> d(n * es);
    CHECK(std::fread(d.data(), 1, d.size(), f) == d.size());
    b.raw[name] = std::move(d);
    b.kind[name] = (char)hdr[0];
  }
  std::fclose(f);
  return b;
}

static Grammar build(const Blob& b) {
  Grammar g;
  auto ops = b.get<int32_t>("ops");
  for (size_t i = 0; i + 6 <= ops.size(); i += 6)
    g.ops.push_back(Op{ops[i], ops[i + 1], ops[i + 2], ops[i + 3], ops[i + 4], ops[i + 5]});
  g.lit_off = b.get<int32_t>("lit_off");
  g.lit_tok = b.get<int32_t>("lit_tok");
  g.lit1_off = b.get<int32_t>("lit1_off");
  g.lit1_tok = b.get<int32_t>("lit1_tok");
  g.lit_first = b.get<int32_t>("lit_first");
  g.choice_off = b.get<int32_t>("choice_off");
  auto a = b.get<int32_t>("alts");
  for (size_t i = 0; i + 6 <= a.size(); i += 6)
    g.alts.push_back(Alt{a[i], a[i + 1], a[i + 2], a[i + 3], a[i + 4], a[i + 5]});
  g.alt_rest = b.get<int32_t>("alt_rest");
  g.choice_masks = b.get<int32_t>("choice_masks");
  g.max_items = b.get<int32_t>("max_items");
  g.honors_min = b.get<int32_t>("honors_min");
  g.caps = b.get<int32_t>("caps");
  g.num_masks = b.get<int32_t>("num_masks");
  g.num_caps = b.get<int32_t>("num_caps");
  g.fin = b.get<int32_t>("fin");
  g.fin1 = b.get<int32_t>("fin1");
  g.close_alt = b.get<int32_t>("close_alt");
  g.null_ids = b.get<int32_t>("null_ids");
  g.tok_class = b.get<uint8_t>("tok_class");
  g.tok_chars = b.get<uint8_t>("tok_chars");
  g.tok_digits = b.get<uint8_t>("tok_digits");
  g.tok_utf = b.get<uint8_t>("tok_utf");
  auto sm = b.get<int32_t>("str_masks");
  CHECK(sm.size() == STR_SUBS);
  for (int i = 0; i < STR_SUBS; ++i) g.str_masks[i] = sm[i];
  auto sc = b.get<int32_t>("scalars");
  CHECK(sc.size() >= 8);
  g.quote = sc[0]; g.zero = sc[1]; g.dot = sc[2]; g.backslash = sc[3]; g.slack = sc[4];
  g.start_pc = sc[5]; g.ncap = sc[6]; g.cont = sc[7];
  CHECK(g.fin.size() == g.ops.size() * NPROF);
  return g;
}

// ------------------------------------------------------------ block manager
static void fuzz_block_manager(uint32_t seed) {
  std::mt19937 rng(seed);
  const int32_t NB = 64;
  BlockManager bm(NB, 32);
  std::vector<std::vector<int32_t>> owners;        // live allocations
  std::vector<uint64_t> published;
  std::vector<int32_t> shadow(NB, 0);
  for (int it = 0; it < 20000; ++it) {
    int op = rng() % 4;
    if (op == 0) {
      int32_t n = 1 + rng() % 6;
      std::vector<int32_t> got;
      if (bm.allocate(n, got)) {
        CHECK((int32_t)got.size() == n);
        for (int32_t x : got) {
          CHECK(x >= 0 && x < NB);
          CHECK(shadow[x] == 0);
          shadow[x] = 1;
          CHECK(bm.refcount(x) == 1);
        }
        owners.push_back(got);
      }
    } else if (op == 1 && !owners.empty()) {
      size_t k = rng() % owners.size();
      auto v = owners[k];
      owners.erase(owners.begin() + k);
      for (int32_t x : v) --shadow[x];
      bm.release(v.data(), (int32_t)v.size());
    } else if (op == 2 && !owners.empty()) {
      auto& v = owners[rng() % owners.size()];
      int32_t blk = v[rng() % v.size()];
      int32_t toks[32];
      for (int j = 0; j < 32; ++j) toks[j] = (int32_t)(rng() % 1000);
      uint64_t h = BlockManager::hash_block(rng() % 4, toks, 32);
      bm.register_block(blk, h);
      published.push_back(h);
    } else if (op == 3 && !published.empty()) {
      uint64_t h = published[rng() % published.size()];
      std::vector<int32_t> got;
      int32_t m = bm.match_prefix(&h, 1, got);
      CHECK(m == (int32_t)got.size() && m <= 1);
      for (int32_t x : got) ++shadow[x];
      if (m) owners.push_back(got);
    }
    int32_t live = 0;
    for (int32_t x = 0; x < NB; ++x) {
      CHECK(bm.refcount(x) == shadow[x]);
      live += shadow[x] > 0;
    }
    CHECK(bm.num_free() == NB - live);
  }
  for (auto& v : owners) bm.release(v.data(), (int32_t)v.size());
  CHECK(bm.num_free() == NB);
}

// ----------------------------------------------------------- grammar walks
static int grammar_walks(const Grammar& g, const std::vector<uint32_t>& masks, int32_t words,
                         int walks, uint32_t seed) {
  std::mt19937 rng(seed);
  int64_t total = 0;
  int32_t longest = 0;
  for (int w = 0; w < walks; ++w) {
    std::vector<int32_t> forced;
    int32_t minv = (int32_t)(rng() % 9);
    const int32_t prof = (int32_t)(rng() % 2);
    // random budgets exercise the close-out; every walk must end inside its budget
    const int32_t budget = 200 + (int32_t)(rng() % 1001);
    State st = g.initial(forced, minv, prof, budget);
    int32_t n = (int32_t)forced.size();
    for (int steps = 0;; ++steps) {
      CHECK(steps < 4000);
      int32_t m = g.mask(st);
      if (m < 0) break;
      CHECK((size_t)(m + 1) * words <= masks.size());
      const uint32_t* row = masks.data() + (size_t)m * words;
      std::vector<int32_t> allowed;
      for (int32_t wd = 0; wd < words; ++wd)
        for (uint32_t bits = row[wd]; bits; bits &= bits - 1)
          allowed.push_back(wd * 32 + __builtin_ctz(bits));
      CHECK(!allowed.empty());
      int32_t tok = allowed[rng() % allowed.size()];
      forced.clear();
      CHECK(g.advance(st, tok, forced, budget - n - 1));
      n += 1 + (int32_t)forced.size();
      CHECK(n <= budget);
    }
    CHECK(g.done(st));
    total += n;
    longest = n > longest ? n : longest;
  }
  std::printf("grammar walks=%d mean_tokens=%.1f max_tokens=%d\n", walks,
              (double)total / walks, longest);
  return longest;
}

// ------------------------------------------------------------ engine core
// Continuous batching with grammar-masked random tokens over a small KV pool
// (forces chunked prefill, prefix sharing and preemption), checking the packed
// layout's invariants every step and that every request retires with a valid
// reason and all blocks return to the pool.
static void fuzz_engine_core(std::shared_ptr<const Grammar> g, const std::vector<uint32_t>& masks,
                             int32_t words, uint32_t seed) {
  std::mt19937 rng(seed);
  CoreConfig cfg;
  cfg.num_blocks = 48;
  cfg.scratch_block = 48;
  cfg.max_num_seqs = 6;
  cfg.max_batched_tokens = 256;
  cfg.max_model_len = 2048;
  cfg.group = 4;
  cfg.hkv = 2;
  cfg.is_cuda = true;
  EngineCore core(cfg, g);
  std::vector<std::pair<int32_t, int32_t>> keys;
  for (int nb : {1, 2, 4, 8})
    for (int m : {1, 2, 3, 4, 6, 8}) keys.push_back({nb, nb * m});
  core.set_graph_keys(keys);
  std::vector<int32_t> header(HEADER), payload(core.payload_bound() + 2);
  int32_t* pay = payload.data() + ((reinterpret_cast<uintptr_t>(payload.data()) & 7) ? 1 : 0);
  const int nreq = 24;
  std::vector<int32_t> shared(300);
  for (auto& t : shared) t = (int32_t)(rng() % 1000);
  for (int i = 0; i < nreq; ++i) {
    std::vector<int32_t> prompt(shared.begin(), shared.begin() + 200 + rng() % 100);
    for (int j = 0; j < (int)(rng() % 200); ++j) prompt.push_back((int32_t)(rng() % 1000));
    SeqParams p;
    p.seed = i;
    p.min_items = (int32_t)(rng() % 4);
    p.profile = (int32_t)(rng() % 2);
    p.max_tokens = 200 + (int32_t)(rng() % 1001);
    core.add(prompt.data(), (int32_t)prompt.size(), p, 0.0);
  }
  int finished = 0, steps = 0;
  while (core.has_work()) {
    CHECK(++steps < 200000);
    const int64_t n = core.schedule_and_pack(header.data(), pay, (int64_t)payload.size() - 1, 0.0);
    std::vector<int32_t> done;
    if (n == 0) {
      done = core.drain_finished();
    } else {
      const int32_t T = header[H_T], NA = header[H_NA], S = header[H_S], maxb = header[H_MAXB];
      CHECK(header[H_PAYLOAD] == n && T > 0 && S >= 0 && maxb > 0);
      // midx sits 2 words before the end of the payload's last three arrays
      const int32_t* midx = pay + n - 2 * S;
      const int32_t* slots = pay + 2 * S + 2 * T;
      for (int32_t i = 0; i < T; ++i) CHECK(slots[i] >= -1 && slots[i] < 49 * 32);
      (void)NA;
      std::vector<int32_t> toks(S);
      for (int32_t k = 0; k < S; ++k) {
        const int32_t m = midx[k];
        if (m < 0) { toks[k] = 0; continue; }
        const uint32_t* row = masks.data() + (size_t)m * words;
        std::vector<int32_t> allowed;
        for (int32_t wd = 0; wd < words; ++wd)
          for (uint32_t bits = row[wd]; bits; bits &= bits - 1)
            allowed.push_back(wd * 32 + __builtin_ctz(bits));
        CHECK(!allowed.empty());
        toks[k] = allowed[rng() % allowed.size()];
      }
      done = core.post(toks.data(), S, 0.0);
    }
    for (int32_t id : done) {
      const Seq& s = core.seq(id);
      CHECK(s.status == S_FINISHED);
      CHECK(s.finish == F_STOP);                     // the close-out always fits the budget
      CHECK(s.generated() <= s.p.max_tokens);
      core.release(id);
      ++finished;
    }
  }
  CHECK(finished == nreq);
  CHECK(core.num_preempted > 0);                     // the small pool must have forced it
  CHECK(core.bm().num_free() == cfg.num_blocks);
  std::printf("engine core fuzz ok: steps=%d preempted=%lld prefix_hits=%llu\n", steps,
              (long long)core.num_preempted, (unsigned long long)core.bm().hits);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s grammar.bin [walks] [seed]\n", argv[0]);
    return 2;
  }
  int walks = argc > 2 ? std::atoi(argv[2]) : 200;
  uint32_t seed = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 1;
  fuzz_block_manager(seed);
  std::printf("block manager fuzz ok\n");
  Blob b = read_blob(argv[1]);
  auto g = std::make_shared<Grammar>(build(b));
  auto masks = b.get<uint32_t>("mask_rows");
  int32_t words = b.get<int32_t>("mask_words")[0];
  int32_t budget = b.get<int32_t>("max_tokens")[0];
  int32_t longest = grammar_walks(*g, masks, words, walks, seed);
  CHECK(longest <= budget);
  fuzz_engine_core(g, masks, words, seed);
  std::printf("OK\n");
  return 0;
}
