#include "grammar.h"

namespace rfqrt {

State Grammar::enter(int32_t pc, const State& from, int32_t sub) const {
  State s = enter_cnt(pc, from, from.cnt);
  if (ops[pc].code != OP_STR) s.sub = sub;
  return s;
}

State Grammar::enter_cnt(int32_t pc, const State& from, int32_t cnt) const {
  const Op& op = ops[pc];
  if (op.code == OP_STR) {
    const int32_t cap = caps[from.prof * ncap + op.a];
    return State{pc, 0, cnt, cap > 0 ? cap : UNBOUNDED, from.minv, from.prof};
  }
  return State{pc, 0, cnt, 0, from.minv, from.prof};
}

int Grammar::combo(int32_t ci, const State& st) const {
  const bool synth = st.prof == PROFILE_SYNTHETIC;
  int c = synth ? 1 : 0;
  int32_t lim = synth ? max_items[ci] : 0;
  // SYNTHETIC + item hint: exactly the document's item count (a trained extractor emits
  // one object per part; a random-init model would otherwise flip a coin at every ',')
  if (lim > 0 && honors_min[ci] && st.minv > 0 && st.minv < lim) lim = st.minv;
  if (lim > 0 && st.cnt >= lim) c |= 2;
  else if (honors_min[ci] && st.cnt < st.minv) c |= 4;
  return c;
}

int Grammar::enabled(int32_t ci, const State& st, const Alt** out) const {
  const int c = combo(ci, st);
  int n = 0;
  for (int32_t i = choice_off[ci]; i < choice_off[ci + 1]; ++i) {
    const Alt& a = alts[i];
    if ((c & 1) && (a.flags & ALT_LENIENT)) continue;
    if ((c & 2) && (a.flags & ALT_CONTINUE)) continue;
    if ((c & 4) && (a.flags & ALT_CLOSE)) continue;
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
  else if (a.cnt == CNT_RESET) cnt = 0;
  st = enter_cnt(a.target, st, cnt);
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
        st = enter(st.pc + 1, st);
        break;
      }
      case OP_JMP:
        st = enter(op.a, st);
        break;
      case OP_CHOICE: {
        if (enabled(op.a, st, en) != 1) return;
        take(*en[0], st, forced, false);
        break;
      }
      case OP_STR:
        if (st.rem > 0) return;
        close_str(st, forced);
        break;
      case OP_NUM:
        if (st.sub == 5 || (st.sub == 4 && op.a != NUM_DEC && ops[succ(st.pc)].code == OP_LIT)) {
          st = enter(succ(st.pc), st);
          break;
        }
        if (st.sub == 0 && (op.c & NUM_UNIT) && st.prof == PROFILE_SYNTHETIC) {
          forced.push_back(zero);               // "0." then fraction digits
          forced.push_back(dot);
          st.sub = 2;
          st.rem = 0;
          break;
        }
        return;
      default:
        return;
    }
  }
}

void Grammar::close_str(State& st, std::vector<int32_t>& forced) const {
  if (st.sub == 1) forced.push_back(backslash);
  for (int32_t i = 1; i < st.sub; ++i) forced.push_back(cont);
  forced.push_back(quote);
  st = enter(st.pc + 1, st);
}

bool Grammar::str(State& s, int32_t token) const {
  if (token < 0 || token >= (int32_t)tok_class.size()) return false;
  const uint8_t c = tok_class[token], u = tok_utf[token];
  const int32_t lead = u & 3, owed = (u >> 2) & 3, allc = (u >> 4) & 1;
  int32_t nsub;
  if (s.sub == 0 && token == quote) {
    s = enter(s.pc + 1, s);
    return true;
  }
  if (s.sub == 1) {
    if (!(c & TC_ESC)) return false;
    nsub = owed ? 1 + owed : 0;
  } else {
    const int32_t p = s.sub > 1 ? s.sub - 1 : 0;
    if (allc && lead >= 1 && lead <= p) nsub = p > lead ? 1 + (p - lead) : 0;
    else if (lead == p && !allc && (c & TC_STR)) nsub = owed ? 1 + owed : 0;
    else if (lead == p && !allc && (c & TC_STR_OPEN)) nsub = 1;
    else return false;
  }
  s.sub = nsub;
  s.rem -= chars(token);
  return true;
}

int32_t Grammar::close_cost(const State& st) const {
  const Op& op = ops[st.pc];
  switch (op.code) {
    case OP_LIT: return (st.sub ? fin1 : fin)[st.pc * NPROF + st.prof];
    case OP_STR:  // quote; after a backslash '\\' first; owing p bytes p continuation tokens
      return (st.sub == 0 ? 1 : (st.sub > 2 ? st.sub : 2)) + fin[(st.pc + 1) * NPROF + st.prof];
    case OP_NUM: {
      const int32_t f = fin[succ(st.pc) * NPROF + st.prof];
      if (st.sub == 0) return ((op.c & NUM_NULLABLE) ? (int32_t)null_ids.size() : 1) + f;
      return f + (st.sub == 2 ? 1 : 0);
    }
    case OP_END: return 0;
    default: return fin[st.pc * NPROF + st.prof];
  }
}

void Grammar::maybe_close(State& st, std::vector<int32_t>& forced, int32_t budget,
                          size_t mark) const {
  const int64_t left = (int64_t)budget - (int64_t)(forced.size() - mark);
  if (left >= (int64_t)close_cost(st) + slack) return;
  for (;;) {
    const Op& op = ops[st.pc];
    switch (op.code) {
      case OP_END:
        return;
      case OP_LIT: {
        const auto& off = st.sub ? lit1_off : lit_off;
        const auto& tok = st.sub ? lit1_tok : lit_tok;
        forced.insert(forced.end(), tok.begin() + off[op.a], tok.begin() + off[op.a + 1]);
        st = enter(st.pc + 1, st);
        break;
      }
      case OP_JMP:
        st = enter(op.a, st);
        break;
      case OP_CHOICE:
        take(alts[choice_off[op.a] + close_alt[op.a * NPROF + st.prof]], st, forced, false);
        break;
      case OP_STR:
        close_str(st, forced);
        break;
      default: {  // OP_NUM
        if (st.sub == 0) {
          if (op.c & NUM_NULLABLE) forced.insert(forced.end(), null_ids.begin(), null_ids.end());
          else forced.push_back(zero);
        } else if (st.sub == 2) {
          forced.push_back(zero);
        }
        st = enter(succ(st.pc), st);
        break;
      }
    }
  }
}

State Grammar::initial(std::vector<int32_t>& forced, int32_t min_items, int32_t profile,
                       int32_t budget) const {
  State from{0, 0, 0, 0, min_items, profile == PROFILE_SYNTHETIC ? PROFILE_SYNTHETIC
                                                                 : PROFILE_REFERENCE};
  State st = enter(start_pc, from);
  const size_t mark = forced.size();
  settle(st, forced);
  maybe_close(st, forced, budget, mark);
  return st;
}

int32_t Grammar::mask(const State& st) const {
  const Op& op = ops[st.pc];
  switch (op.code) {
    case OP_CHOICE: return choice_masks[op.a * 8 + combo(op.a, st)];
    case OP_STR: return str_masks[st.sub];
    case OP_NUM: return num_masks[(op.e * NPROF + st.prof) * NUM_PHASES + st.sub];
    default: return -1;
  }
}

bool Grammar::end_number(int32_t s, int32_t token, State& st, std::vector<int32_t>& forced) const {
  const Op& nxt = ops[s];
  if (nxt.code == OP_LIT) {
    if (token != lit_first[nxt.a]) return false;
    st = enter(s, st, 1);
    return true;
  }
  State c = enter(s, st);
  const Alt* en[16];
  const int n = enabled(nxt.a, c, en);
  for (int i = 0; i < n; ++i)
    if (en[i]->first == token) {
      st = c;
      take(*en[i], st, forced, true);
      return true;
    }
  return false;
}

bool Grammar::num(const Op& op, State& st, int32_t token, std::vector<int32_t>& forced) const {
  const int32_t kind = op.a;
  const int32_t* cap = &num_caps[(op.e * NPROF + st.prof) * 2];
  const int32_t maxd = cap[0], maxfrac = cap[1];
  const bool is_dig = tok_has(token, TC_DIGITS);
  const int32_t nd = is_dig ? tok_digits[token] : 0;
  const int32_t ph = st.sub;
  const int32_t s = succ(st.pc);
  if (ph == 0) {
    if ((op.c & NUM_NULLABLE) && !null_ids.empty() && token == null_ids[0]) {
      forced.insert(forced.end(), null_ids.begin() + 1, null_ids.end());
      st = enter(s, st);
      return true;
    }
    if ((op.c & NUM_STR_OK) && st.prof != PROFILE_SYNTHETIC && token == quote) {
      st = enter(st.pc + 1, st);
      return true;
    }
    if (!is_dig) return false;
    if (token == zero) { st.sub = 4; st.rem = 1; return true; }
    if (tok_has(token, TC_ZERO_LEAD)) return false;
    st.sub = nd >= maxd ? 4 : 1;
    st.rem = nd;
    return true;
  }
  if ((ph == 1 || ph == 3 || ph == 4) && end_number(s, token, st, forced)) return true;
  if (kind == NUM_DEC && (ph == 1 || ph == 4) && token == dot) {
    st.sub = 2; st.rem = 0;
    return true;
  }
  if (!is_dig || ph == 4 || ph == 5) return false;
  if (ph == 1) {
    st.rem += nd;
    if (st.rem >= maxd) st.sub = 4;
  } else if (ph == 2) {
    st.sub = nd >= maxfrac ? 5 : 3;
    st.rem = nd;
  } else if (ph == 3) {
    st.rem += nd;
    if (st.rem >= maxfrac) st.sub = 5;
  }
  return true;
}

bool Grammar::advance(State& st, int32_t token, std::vector<int32_t>& forced, int32_t budget) const {
  State s = st;
  const Op& op = ops[s.pc];
  const size_t mark = forced.size();
  bool ok = false;
  switch (op.code) {
    case OP_CHOICE: {
      const Alt* en[16];
      const int n = enabled(op.a, s, en);
      for (int i = 0; i < n; ++i)
        if (en[i]->first == token) { take(*en[i], s, forced, true); ok = true; break; }
      break;
    }
    case OP_STR:
      ok = str(s, token);
      break;
    case OP_NUM:
      ok = num(op, s, token, forced);
      break;
    default:
      break;
  }
  if (!ok) { forced.resize(mark); return false; }
  settle(s, forced);
  maybe_close(s, forced, budget, mark);
  st = s;
  return true;
}

}  // namespace rfqrt
