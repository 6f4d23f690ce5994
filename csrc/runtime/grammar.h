// Token-level executor for the compiled RFQ JSON grammar
// (replisense_rfq_amd/engine/grammar/compiler.py builds the program; the Python
// twin engine/grammar/fsm.py is the test oracle).  Runs on the scheduler's hot
// path once per decode step for the whole batch: consume each sequence's sampled
// token, advance its automaton, emit the forced (jump-forward) tokens and the
// vocabulary-mask row the GPU sampler must apply next.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rfqrt {

enum Opcode : int32_t { OP_LIT = 0, OP_CHOICE = 1, OP_STR = 2, OP_NUM = 3, OP_END = 4 };
enum NumKind : int32_t { NUM_INT = 0, NUM_DEC = 1, NUM_FRAC = 2 };
enum CntOp : int32_t { CNT_NONE = 0, CNT_SET1 = 1, CNT_INC = 2 };

struct Op { int32_t code, a, b, c, d; };
struct Alt { int32_t first, rest_off, rest_len, target, cnt, is_continue, is_close; };

// minv: the request's minimum line-item count (schema hint for choices that honor it)
struct State { int32_t pc, sub, cnt, rem, minv; };

class Grammar {
 public:
  std::vector<Op> ops;
  std::vector<int32_t> lit_off, lit_tok, lit1_off, lit1_tok;   // CSR literals (+skip-first)
  std::vector<int32_t> choice_off;                             // CSR into alts
  std::vector<Alt> alts;
  std::vector<int32_t> alt_rest;                               // rest tokens of alternatives
  std::vector<int32_t> choice_mask, choice_mask_close, max_items, honors_min;
  std::vector<int32_t> num_masks;                              // [3 kinds][5 phases][3 end][2 null]
  std::vector<int32_t> null_rest;
  std::vector<uint8_t> tok_class, tok_chars, tok_digits;
  int32_t str_mask = 0, quote = -1, zero = -1, dot = -1, null_first = -1;
  int32_t end_tok[3] = {-1, -1, -1};
  int32_t start_pc = 0;

  State initial(std::vector<int32_t>& forced, int32_t min_items = 0) const;
  // Consume a sampled token.  Returns false if the token is illegal (state unchanged).
  bool advance(State& st, int32_t token, std::vector<int32_t>& forced) const;
  int32_t mask(const State& st) const;  // -1 when finished
  bool done(const State& st) const { return ops[st.pc].code == OP_END; }

 private:
  State enter(int32_t pc, int32_t cnt, int32_t minv, int32_t sub = 0) const;
  void settle(State& st, std::vector<int32_t>& forced) const;
  int enabled(int32_t ci, int32_t cnt, int32_t minv, const Alt** out) const;
  void take(const Alt& a, State& st, std::vector<int32_t>& forced, bool sampled) const;
  bool num(const Op& op, State& st, int32_t token, std::vector<int32_t>& forced) const;
};

}  // namespace rfqrt
