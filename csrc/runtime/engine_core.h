// Native engine core: per-sequence state, continuous-batching scheduler, step
// packer and sampled-token post-processing — everything the engine does on the
// host between two GPU steps.
//
// At ~1000 sequences in flight the Python scheduler/packer/post-processor cost
// ~6 ms per step (≈11 % of a 55 ms throughput step, during which the GPU
// idles).  Here the same work is a few tight C++ loops over contiguous state:
//
//   schedule()     decode rows (q = 1), jump-forward / prefill extends (q > 1)
//                  under the token budget; FCFS admission with prefix-cache
//                  matching; recompute-style preemption when KV runs out.
//   pack()         writes the step's metadata straight into the caller's pinned
//                  staging buffer in the layout replisense_rfq_amd/engine/runner.py
//                  documents (_layout), padded to a captured hipGraph bucket
//                  when one fits.
//   post()         consumes the sampled ids: grammar automaton advance +
//                  jump-forward tokens, prefix-cache publication, stop / length /
//                  grammar-error retirement, KV release.
//
// The Python engine keeps request intake, the device side and result delivery.
#pragma once
#include <cstdint>
#include <algorithm>
#include <deque>
#include <memory>
#include <utility>
#include <vector>

#include "block_manager.h"
#include "grammar.h"

namespace rfqrt {

enum SeqStatus : int8_t { S_WAITING = 0, S_RUNNING = 1, S_FINISHED = 2 };
enum FinishReason : int8_t {
  F_NONE = 0, F_STOP = 1, F_LENGTH = 2, F_GRAMMAR_ERROR = 3, F_ABORT = 4, F_ENGINE_ERROR = 5,
  F_TIMEOUT = 6
};

struct SeqParams {
  float temperature = 0.1f;
  int32_t max_tokens = 1200;
  int64_t seed = 0;
  bool grammar = true;
  int32_t min_items = 0;
  int32_t profile = 0;                   // grammar profile (grammar.h Profile)
};

struct Seq {
  bool live = false;
  std::vector<int32_t> tokens;           // prompt + generated (sampled and forced)
  int32_t prompt_len = 0;
  int32_t num_cached = 0;                // tokens whose KV is written
  int32_t num_registered = 0;            // prompt blocks published to the prefix cache
  int32_t prefix_hit = 0;
  std::vector<int32_t> blocks;
  std::vector<uint64_t> block_hashes;
  SeqParams p;
  bool has_gs = false;
  State gs{};
  int32_t mask_idx = -1;
  int32_t num_sampled = 0, num_forced = 0;
  SeqStatus status = S_WAITING;
  FinishReason finish = F_NONE;
  double t_arrival = 0, t_first_sched = 0, t_prefill_done = 0, t_first_token = 0, t_finish = 0;

  int32_t pending() const { return (int32_t)tokens.size() - num_cached; }
  bool in_prefill() const { return num_cached < prompt_len; }
  int32_t generated() const { return (int32_t)tokens.size() - prompt_len; }
};

struct CoreConfig {
  int32_t block_size = 32;
  int32_t num_blocks = 0;                // allocatable blocks (scratch page excluded)
  int32_t scratch_block = 0;
  int32_t max_num_seqs = 256;
  int32_t max_batched_tokens = 16384;
  int32_t max_model_len = 8192;
  int32_t ext_max = 32;                  // extends up to this many tokens go to section A
  int32_t group = 4;                     // q heads per kv head (decode work-item tiling)
  int32_t hkv = 8;                       // local kv heads (decode split heuristic)
  int32_t decode_tiles = 1;              // 16-column tiles per decode attention work item
  int32_t prefill_qblk = 32;             // queries per prefill attention work item (32 | 64)
  bool jump_forward = true;
  bool prefix_cache = true;
  bool is_cuda = true;
  bool use_graphs = true;
  std::vector<int32_t> token_mults{1, 2, 3, 4, 6, 8};
  std::vector<int32_t> eos_ids;
};

// header slots (must match runner.py)
enum : int {
  H_T = 0, H_TA, H_NA, H_WA, H_NB, H_WB, H_S, H_MAXB, H_GNB, H_GTB, H_SPLITS, H_PAYLOAD, H_STOP,
  H_TILES, HEADER = 16
};

class EngineCore {
 public:
  EngineCore(const CoreConfig& cfg, std::shared_ptr<const Grammar> grammar);

  // --- requests
  int32_t add(const int32_t* prompt, int32_t n, const SeqParams& p, double t_arrival);
  void release(int32_t id);              // forget a finished sequence's record
  std::vector<int32_t> abort_all(FinishReason why, double now);
  // Retire one queued/running sequence between steps (releases its blocks).
  // Returns false if it already finished.
  bool abort(int32_t id, FinishReason why, double now);

  // --- one step
  // Schedules the next step and packs it.  Returns the payload length (int32
  // words; 0 = nothing to run).  `payload` must hold payload_bound() words.
  int64_t schedule_and_pack(int32_t* header, int32_t* payload, int64_t capacity, double now);
  int64_t payload_bound() const;
  // Consume the sampled id of every logits row of the last packed step; returns
  // the ids of sequences that finished.
  std::vector<int32_t> post(const int32_t* sampled, int32_t n, double now);
  // Sequences retired outside post() (a request that cannot fit in the whole KV
  // pool even alone); returned and cleared.
  std::vector<int32_t> drain_finished();

  void set_graph_keys(const std::vector<std::pair<int32_t, int32_t>>& keys);
  // Lower the per-step token budget (prefill chunk) at run time; never above the
  // construction value, so payload_bound() stays an upper bound of every step.
  void set_max_batched_tokens(int32_t n) {
    cfg_.max_batched_tokens = std::max(1, std::min(n, max_batched_tokens0_));
  }
  // (nb, tb) of the captured graph a step of na sequences / t tokens would replay,
  // or (-1, -1) for an eager step (exposed for tests)
  std::pair<int32_t, int32_t> find_graph_key(int32_t na, int32_t t) const {
    int32_t nb = -1, tb = -1;
    if (!graph_key(na, t, nb, tb)) nb = tb = -1;
    return {nb, tb};
  }
  // Pin the cached full blocks of `tokens` (a prompt prefix whose KV is already
  // published, e.g. by a warm-up prefill): they hold a reference for the engine's
  // lifetime, so the shared prompt template is never evicted.  Returns the number
  // of blocks pinned.
  int32_t pin_prefix(const int32_t* tokens, int32_t n);
  int32_t num_pinned() const { return (int32_t)pinned_.size(); }

  // --- inspection
  const Seq& seq(int32_t id) const { return seqs_[id]; }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  int32_t num_running() const { return (int32_t)running_.size(); }
  int32_t num_waiting() const { return (int32_t)waiting_.size(); }
  int64_t num_preempted = 0;
  int64_t num_steps = 0;
  BlockManager& bm() { return bm_; }
  const CoreConfig& cfg() const { return cfg_; }

 private:
  struct Row { int32_t id; int32_t q; };
  bool grow(Seq& s, int32_t upto);
  int32_t blocks_needed(const Seq& s, int32_t upto) const;
  void admit(Seq& s);
  void publish(Seq& s);
  void preempt(int32_t id);
  int32_t preempt_victim(int32_t exclude) const;
  void finish(int32_t id, FinishReason why, double now, std::vector<int32_t>& out);
  void schedule(double now);
  int32_t decode_splits(int32_t na, int32_t max_ctx, bool graph) const;
  bool graph_key(int32_t na, int32_t t, int32_t& nb, int32_t& tb) const;

  CoreConfig cfg_;
  int32_t max_batched_tokens0_;
  std::shared_ptr<const Grammar> grammar_;
  BlockManager bm_;
  std::vector<Seq> seqs_;
  std::vector<int32_t> free_ids_;
  std::deque<int32_t> waiting_;
  std::vector<int32_t> running_;
  std::vector<int32_t> nb_buckets_;
  std::vector<std::pair<int32_t, int32_t>> graph_keys_;   // sorted
  // the last scheduled step
  std::vector<int32_t> decode_;
  std::vector<Row> extend_;
  std::vector<std::pair<int32_t, bool>> rows_;             // (seq, samples) per logits row
  std::vector<int32_t> scratch_;
  std::vector<int32_t> finished_;
  std::vector<int32_t> pinned_;
};

}  // namespace rfqrt
