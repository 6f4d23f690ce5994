// Token-level executor for the compiled RFQ JSON grammar
// (replisense_rfq_amd/engine/grammar/compiler.py builds the program; the Python
// twin engine/grammar/fsm.py is the test oracle).  Runs on the scheduler's hot
// path once per decode step for the whole batch: consume each sequence's sampled
// token, advance its automaton, emit the forced (jump-forward) tokens and the
// vocabulary-mask row the GPU sampler must apply next.  When the request's token
// budget runs low the automaton emits the deterministic close-out (cheapest
// alternatives) so the output is complete JSON within max_tokens.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rfqrt {

enum Opcode : int32_t { OP_LIT = 0, OP_CHOICE = 1, OP_STR = 2, OP_NUM = 3, OP_END = 4, OP_JMP = 5 };
enum NumKind : int32_t { NUM_INT = 0, NUM_DEC = 1 };
enum NumFlags : int32_t { NUM_NULLABLE = 1, NUM_STR_OK = 2, NUM_UNIT = 4 };
enum CntOp : int32_t { CNT_NONE = 0, CNT_SET1 = 1, CNT_INC = 2, CNT_RESET = 3 };
enum AltFlags : int32_t { ALT_CONTINUE = 1, ALT_CLOSE = 2, ALT_LENIENT = 4 };
enum TokClass : uint8_t { TC_STR = 1, TC_DIGITS = 2, TC_ZERO_LEAD = 4, TC_STR_OPEN = 8, TC_ESC = 16 };
enum Profile : int32_t { PROFILE_REFERENCE = 0, PROFILE_SYNTHETIC = 1, NPROF = 2 };
constexpr int32_t NUM_PHASES = 6;
constexpr int32_t STR_SUBS = 5;   // 0 plain, 1 after a lone backslash, 1+p owing p UTF-8 bytes
constexpr int32_t UNBOUNDED = 1 << 30;
constexpr int32_t NO_BUDGET = 1 << 30;

struct Op { int32_t code, a, b, c, d, e; };
struct Alt { int32_t first, rest_off, rest_len, target, cnt, flags; };

// minv: the request's minimum line-item count (schema hint for choices that honor it)
// prof: decoding profile (PROFILE_REFERENCE admits everything the reference emits)
struct State { int32_t pc, sub, cnt, rem, minv, prof; };

class Grammar {
 public:
  std::vector<Op> ops;
  std::vector<int32_t> lit_off, lit_tok, lit1_off, lit1_tok, lit_first;  // CSR literals
  std::vector<int32_t> choice_off;                             // CSR into alts
  std::vector<Alt> alts;
  std::vector<int32_t> alt_rest;                               // rest tokens of alternatives
  std::vector<int32_t> choice_masks;                           // [n_choices][8]
  std::vector<int32_t> max_items, honors_min;                  // per choice
  std::vector<int32_t> caps;                                   // [NPROF][ncap]
  int32_t ncap = 0;
  std::vector<int32_t> num_masks;                              // [n_nums][NPROF][NUM_PHASES]
  std::vector<int32_t> num_caps;                               // [n_nums][NPROF][2] digit caps
  std::vector<int32_t> fin, fin1;                              // [n_ops][NPROF]
  std::vector<int32_t> close_alt;                              // [n_choices][NPROF]
  std::vector<int32_t> null_ids;
  std::vector<uint8_t> tok_class, tok_chars, tok_digits;
  std::vector<uint8_t> tok_utf;                                // lead | owed << 2 | allcont << 4
  int32_t str_masks[STR_SUBS] = {0, 0, 0, 0, 0};
  int32_t quote = -1, zero = -1, dot = -1, backslash = -1, cont = -1;
  int32_t slack = 0, start_pc = 0;

  State initial(std::vector<int32_t>& forced, int32_t min_items = 0, int32_t profile = 0,
                int32_t budget = NO_BUDGET) const;
  // Consume a sampled token.  `budget` = tokens the request may still append after
  // it.  Returns false if the token is illegal (state and `forced` unchanged).
  bool advance(State& st, int32_t token, std::vector<int32_t>& forced,
               int32_t budget = NO_BUDGET) const;
  int32_t mask(const State& st) const;  // -1 when finished
  bool done(const State& st) const { return ops[st.pc].code == OP_END; }
  int32_t close_cost(const State& st) const;

 private:
  State enter(int32_t pc, const State& from, int32_t sub = 0) const;
  State enter_cnt(int32_t pc, const State& from, int32_t cnt) const;
  void settle(State& st, std::vector<int32_t>& forced) const;
  void maybe_close(State& st, std::vector<int32_t>& forced, int32_t budget, size_t mark) const;
  int combo(int32_t ci, const State& st) const;
  int enabled(int32_t ci, const State& st, const Alt** out) const;
  void take(const Alt& a, State& st, std::vector<int32_t>& forced, bool sampled) const;
  bool num(const Op& op, State& st, int32_t token, std::vector<int32_t>& forced) const;
  bool str(State& s, int32_t token) const;
  void close_str(State& st, std::vector<int32_t>& forced) const;
  bool end_number(int32_t succ, int32_t token, State& st, std::vector<int32_t>& forced) const;
  int32_t succ(int32_t pc) const { return pc + 1 + ((ops[pc].c & NUM_STR_OK) ? 1 : 0); }
  bool tok_has(int32_t token, uint8_t bit) const {
    return token >= 0 && token < (int32_t)tok_class.size() && (tok_class[token] & bit);
  }
  int32_t chars(int32_t token) const { return tok_chars[token] > 0 ? tok_chars[token] : 1; }
};

}  // namespace rfqrt
