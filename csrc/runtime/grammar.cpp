#include "grammar.h"

namespace rfqrt {

State Grammar::enter(int32_t pc, int32_t cnt, int32_t minv, int32_t sub) const {
  const Op& op = ops[pc];
  if (op.code == OP_STR) return State{pc, 0, cnt, op.a, minv};
  return State{pc, sub, cnt, 0, minv};
}

int Grammar::enabled(int32_t ci, int32_t cnt, int32_t minv, const Alt** out) const {
  int n = 0;
  const int32_t lim = max_items[ci];
  const bool at_max = lim > 0 && cnt >= lim;
  const bool below_min = !at_max && honors_min[ci] && cnt < minv;
  for (int32_t i = choice_off[ci]; i < choice_off[ci + 1]; ++i) {
    const Alt& a = alts[i];
    if (at_max && a.is_continue) continue;
    if (below_min && a.is_close) continue;
    out[n++] = &a;
  }
  return n;
}

void Grammar::take(const Alt& a, State& st, std::vector<int32_t>& forced, bool sampled) const {
  if (!sampled) forced.push_back(a.first);
  forced.insert(forced.end(), alt_rest.begin() + a.rest_off,
                alt_rest.begin() + a.rest_off + a.rest_len);
  int32_t cnt = st.cnt;
  if (a.cnt == CNT_SET1) cnt = 1;
  else if (a.cnt == CNT_INC) cnt += 1;
  st = enter(a.target, cnt, st.minv);
}

void Grammar::settle(State& st, std::vector<int32_t>& forced) const {
  const Alt* en[16];
  for (;;) {
    const Op& op = ops[st.pc];
    switch (op.code) {
      case OP_LIT: {
        const auto& off = st.sub ? lit1_off : lit_off;
        const auto& tok = st.sub ? lit1_tok : lit_tok;
        forced.insert(forced.end(), tok.begin() + off[op.a], tok.begin() + off[op.a + 1]);
        st = enter(st.pc + 1, st.cnt, st.minv);
        break;
      }
      case OP_CHOICE: {
        if (enabled(op.a, st.cnt, st.minv, en) != 1) return;
        take(*en[0], st, forced, false);
        break;
      }
      case OP_STR:
        if (st.rem > 0) return;
        forced.push_back(quote);
        st = enter(st.pc + 1, st.cnt, st.minv);
        break;
      case OP_NUM:
        if (st.sub == 5 || (st.sub == 4 && op.a != NUM_DEC)) {
          st = enter(st.pc + 1, st.cnt, st.minv);
          break;
        }
        return;
      default:
        return;
    }
  }
}

State Grammar::initial(std::vector<int32_t>& forced, int32_t min_items) const {
  State st = enter(start_pc, 0, min_items);
  settle(st, forced);
  return st;
}

int32_t Grammar::mask(const State& st) const {
  const Op& op = ops[st.pc];
  switch (op.code) {
    case OP_CHOICE: return choice_mask[op.a];
    case OP_STR: return str_mask;
    case OP_NUM: {
      const int e = op.c & 15, nl = (op.c >> 4) & 1;
      return num_masks[((op.a * 5 + st.sub) * 3 + e) * 2 + nl];
    }
    default: return -1;
  }
}

bool Grammar::num(const Op& op, State& st, int32_t token, std::vector<int32_t>& forced) const {
  const int32_t kind = op.a, maxd = op.b, e = op.c & 15, nullable = (op.c >> 4) & 1, maxfrac = op.d;
  const bool is_dig = token >= 0 && token < (int32_t)tok_class.size() && (tok_class[token] & 2);
  const int32_t nd = is_dig ? tok_digits[token] : 0;
  const int32_t ph = st.sub;
  if (ph == 0) {
    if (nullable && token == null_first) {
      forced.insert(forced.end(), null_rest.begin(), null_rest.end());
      st = enter(st.pc + 1, st.cnt, st.minv);
      return true;
    }
    if (!is_dig) return false;
    if (kind == NUM_FRAC) {
      st.sub = nd >= maxd ? 5 : 3;
      st.rem = nd;
      return true;
    }
    if (token == zero) { st.sub = 4; st.rem = 1; return true; }
    st.sub = nd >= maxd ? 4 : 1;
    st.rem = nd;
    return true;
  }
  if ((ph == 1 || ph == 3 || ph == 4) && token == end_tok[e]) {
    st = enter(st.pc + 1, st.cnt, st.minv, 1);
    return true;
  }
  if (kind == NUM_DEC && (ph == 1 || ph == 4) && token == dot) {
    st.sub = 2; st.rem = 0;
    return true;
  }
  if (!is_dig || ph == 4) return false;
  if (ph == 1) {
    st.rem += nd;
    if (st.rem >= maxd) st.sub = 4;
  } else if (ph == 2) {
    st.sub = nd >= maxfrac ? 5 : 3;
    st.rem = nd;
  } else if (ph == 3) {
    st.rem += nd;
    if (st.rem >= (kind == NUM_DEC ? maxfrac : maxd)) st.sub = 5;
  }
  return true;
}

bool Grammar::advance(State& st, int32_t token, std::vector<int32_t>& forced) const {
  State s = st;
  const Op& op = ops[s.pc];
  const size_t mark = forced.size();
  bool ok = false;
  switch (op.code) {
    case OP_CHOICE: {
      const Alt* en[16];
      const int n = enabled(op.a, s.cnt, s.minv, en);
      for (int i = 0; i < n; ++i)
        if (en[i]->first == token) { take(*en[i], s, forced, true); ok = true; break; }
      break;
    }
    case OP_STR:
      if (token == quote) { s = enter(s.pc + 1, s.cnt, s.minv); ok = true; }
      else if (token >= 0 && token < (int32_t)tok_class.size() && (tok_class[token] & 1)) {
        s.rem -= tok_chars[token] > 0 ? tok_chars[token] : 1;
        ok = true;
      }
      break;
    case OP_NUM:
      ok = num(op, s, token, forced);
      break;
    default:
      break;
  }
  if (!ok) { forced.resize(mark); return false; }
  settle(s, forced);
  st = s;
  return true;
}

}  // namespace rfqrt
