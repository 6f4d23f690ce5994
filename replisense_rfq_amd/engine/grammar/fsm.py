"""Token-level executor of a compiled RFQ grammar (pure-Python twin of
csrc/runtime/grammar.cpp; the C++ executor is what the engine's step loop runs --
this one is its test oracle and the fallback when the runtime .so is absent).

State = (pc, sub, cnt, rem, minv, prof):
  LIT    sub=1 -> the literal's first char was already produced (by a NUM end token)
  STR    rem = characters still allowed (UNBOUNDED without a cap); sub 0 plain,
         1 after a lone backslash, 1+p while p UTF-8 continuation bytes are owed
  NUM    sub = phase (0 first, 1 int digits, 2 after '.', 3 frac digits, 4 end/dot
         only, 5 forced end), rem = digits used in the current part
  CHOICE cnt = array item counter; minv = the request's minimum line-item count
  prof   0 REFERENCE / 1 SYNTHETIC (compiler.py)

``budget`` (initial / advance) = tokens the request may still append after the
sampled token; when it falls below ``close_cost(state) + slack`` the automaton
emits the deterministic close-out, so the JSON always completes inside it.
"""
from __future__ import annotations

from .compiler import (CNT_INC, CNT_RESET, CNT_SET1, NUM_DEC, NUM_NULLABLE, NUM_STR_OK, NUM_UNIT,
                       OP_CHOICE,
                       OP_END, OP_JMP, OP_LIT, OP_NUM, OP_STR, PROFILE_SYNTHETIC, TC_DIGITS,
                       TC_ESC, TC_STR, TC_STR_OPEN, UNBOUNDED, CompiledGrammar)

DONE = -1
NO_BUDGET = 1 << 30


class GrammarError(ValueError):
    pass


class PyGrammarFSM:
    def __init__(self, g: CompiledGrammar):
        self.g = g
        self.quote = g.quote
        self.zero = g.zero_token

    # ------------------------------------------------------------------ entry
    def _enter(self, pc: int, st, sub: int = 0, cnt: int | None = None):
        g = self.g
        op = g.ops[pc]
        cnt = st[2] if cnt is None else cnt
        if op.code == OP_STR:
            cap = int(g.caps[st[5], op.a])
            return [pc, 0, cnt, cap if cap > 0 else UNBOUNDED, st[4], st[5]]
        return [pc, sub, cnt, 0, st[4], st[5]]

    def initial(self, min_items: int = 0, profile: int = 0, budget: int = NO_BUDGET):
        st = self._enter(self.g.start_pc, [0, 0, 0, 0, min_items, profile])
        forced: list[int] = []
        self._settle(st, forced)
        self._maybe_close(st, forced, budget)
        return tuple(st), forced

    def _succ(self, pc: int) -> int:
        return pc + 1 + (1 if self.g.ops[pc].c & NUM_STR_OK else 0)

    # ----------------------------------------------------------------- settle
    def _settle(self, st, forced):
        g = self.g
        while True:
            pc = st[0]
            op = g.ops[pc]
            if op.code == OP_LIT:
                forced.extend(g.literals_skip1[op.a] if st[1] else g.literals[op.a])
                st[:] = self._enter(pc + 1, st)
            elif op.code == OP_JMP:
                st[:] = self._enter(op.a, st)
            elif op.code == OP_CHOICE:
                alts = self._enabled(op.a, st)
                if len(alts) != 1:
                    return
                self._take(alts[0], st, forced)
            elif op.code == OP_STR:
                if st[3] > 0:
                    return
                self._close_str(st, forced)
            elif op.code == OP_NUM:
                if st[1] == 5 or (st[1] == 4 and op.a != NUM_DEC and
                                  g.ops[self._succ(pc)].code == OP_LIT):
                    st[:] = self._enter(self._succ(pc), st)      # only the end token is legal
                elif st[1] == 0 and op.c & NUM_UNIT and st[5] == PROFILE_SYNTHETIC:
                    forced.extend([self.zero, g.dot_token])       # "0." then fraction digits
                    st[1], st[3] = 2, 0
                else:
                    return
            else:
                return

    def _flags(self, ci: int, st) -> int:
        g = self.g
        prof, cnt, minv = st[5], st[2], st[4]
        combo = 1 if prof == PROFILE_SYNTHETIC else 0
        lim = g.max_items[ci] if prof == PROFILE_SYNTHETIC else 0
        if lim and g.honors_min[ci] and 0 < minv < lim:
            lim = minv          # SYNTHETIC + item hint: exactly the document's item count
        at_max = lim > 0 and cnt >= lim
        if at_max:
            combo |= 2
        elif g.honors_min[ci] and cnt < minv:
            combo |= 4
        return combo

    def _enabled(self, ci: int, st):
        combo = self._flags(ci, st)
        return [a for a in self.g.choices[ci]
                if not ((combo & 1 and a.lenient) or (combo & 2 and a.is_continue)
                        or (combo & 4 and a.is_close))]

    def _take(self, alt, st, forced, sampled=False):
        if not sampled:
            forced.append(alt.first)
        forced.extend(alt.rest)
        cnt = st[2]
        if alt.cnt == CNT_SET1:
            cnt = 1
        elif alt.cnt == CNT_INC:
            cnt += 1
        elif alt.cnt == CNT_RESET:
            cnt = 0
        st[:] = self._enter(alt.target, st, cnt=cnt)

    # ---------------------------------------------------------------- close-out
    def close_cost(self, state) -> int:
        """Tokens the close-out emits from `state` (compiler.py fin tables)."""
        g = self.g
        pc, sub, prof = state[0], state[1], state[5]
        op = g.ops[pc]
        if op.code == OP_LIT:
            return int((g.fin1 if sub else g.fin)[pc, prof])
        if op.code == OP_STR:
            # quote, after a backslash + '\\', owing p bytes + p continuation tokens
            return (1 if sub == 0 else max(2, sub)) + int(g.fin[pc + 1, prof])
        if op.code == OP_NUM:
            f = int(g.fin[self._succ(pc), prof])
            if sub == 0:
                return (len(g.null_ids) if op.c & NUM_NULLABLE else 1) + f
            return f + (1 if sub == 2 else 0)
        if op.code == OP_END:
            return 0
        return int(g.fin[pc, prof])

    def _maybe_close(self, st, forced, budget: int):
        if budget - len(forced) >= self.close_cost(st) + self.g.slack:
            return
        g = self.g
        while True:
            pc = st[0]
            op = g.ops[pc]
            if op.code == OP_END:
                return
            if op.code in (OP_LIT, OP_JMP):
                self._settle_one(st, forced)
            elif op.code == OP_CHOICE:
                alt = g.choices[op.a][int(g.close_alt[op.a, st[5]])]
                self._take(alt, st, forced)
            elif op.code == OP_STR:
                self._close_str(st, forced)
            else:  # NUM
                ph = st[1]
                if ph == 0:
                    if op.c & NUM_NULLABLE:
                        forced.extend(g.null_ids)
                    else:
                        forced.append(self.zero)
                elif ph == 2:
                    forced.append(self.zero)
                st[:] = self._enter(self._succ(pc), st)

    def _close_str(self, st, forced):
        """Finish a string: complete a pending escape / split character, close quote."""
        g = self.g
        sub = st[1]
        if sub == 1:
            forced.append(g.backslash)
        elif sub > 1:
            forced.extend([g.cont_token] * (sub - 1))
        forced.append(self.quote)
        st[:] = self._enter(st[0] + 1, st)

    def _settle_one(self, st, forced):
        g = self.g
        op = g.ops[st[0]]
        if op.code == OP_LIT:
            forced.extend(g.literals_skip1[op.a] if st[1] else g.literals[op.a])
            st[:] = self._enter(st[0] + 1, st)
        else:
            st[:] = self._enter(op.a, st)

    # ------------------------------------------------------------------ query
    def mask(self, state) -> int:
        g = self.g
        pc, sub = state[0], state[1]
        op = g.ops[pc]
        if op.code == OP_CHOICE:
            return int(g.choice_masks[op.a, self._flags(op.a, state)])
        if op.code == OP_STR:
            return g.str_masks[sub]
        if op.code == OP_NUM:
            return int(g.num_masks[op.e, state[5], sub])
        return DONE

    def done(self, state) -> bool:
        return self.g.ops[state[0]].code == OP_END

    # ---------------------------------------------------------------- advance
    def advance(self, state, token: int, budget: int = NO_BUDGET):
        """Consume one *sampled* token; returns (new_state, forced_tokens).
        `budget`: tokens the request may still append after `token`."""
        g = self.g
        st = list(state)
        forced: list[int] = []
        op = g.ops[st[0]]
        if op.code == OP_CHOICE:
            for a in self._enabled(op.a, st):
                if a.first == token:
                    self._take(a, st, forced, sampled=True)
                    break
            else:
                raise GrammarError(f"token {token} not allowed at choice pc={st[0]}")
        elif op.code == OP_STR:
            self._str(st, token)
        elif op.code == OP_NUM:
            self._num(op, st, token, forced)
        else:
            raise GrammarError("advance() on a finished grammar")
        self._settle(st, forced)
        self._maybe_close(st, forced, budget)
        return tuple(st), forced

    def _str(self, st, token):
        g = self.g
        c = int(g.tok_class[token])
        u = int(g.tok_utf[token])
        lead, owed, allc = u & 3, (u >> 2) & 3, (u >> 4) & 1
        sub = st[1]
        if sub == 0 and token == self.quote:
            st[:] = self._enter(st[0] + 1, st)
            return
        if sub == 1:
            if not c & TC_ESC:
                raise GrammarError(f"token {token} cannot follow a backslash")
            nsub = 1 + owed if owed else 0
        else:
            p = sub - 1 if sub > 1 else 0
            if allc and 1 <= lead <= p:
                nsub = 1 + (p - lead) if p > lead else 0
            elif lead == p and not allc and c & TC_STR:
                nsub = 1 + owed if owed else 0
            elif lead == p and not allc and c & TC_STR_OPEN:
                nsub = 1
            else:
                raise GrammarError(f"token {token} not allowed in a string (sub {sub})")
        st[1] = nsub
        st[3] -= max(1, int(g.tok_chars[token]))

    def _num(self, op, st, token, forced):
        g = self.g
        kind = op.a
        maxd, maxfrac = (int(x) for x in g.num_caps[op.e, st[5]])
        is_dig = bool(g.tok_class[token] & TC_DIGITS)
        nd = int(g.tok_digits[token])
        ph = st[1]
        pc = st[0]
        succ = self._succ(pc)
        if ph == 0:
            if op.c & NUM_NULLABLE and token == g.null_ids[0]:
                forced.extend(g.null_ids[1:])
                st[:] = self._enter(succ, st)
                return
            if op.c & NUM_STR_OK and st[5] != PROFILE_SYNTHETIC and token == self.quote:
                st[:] = self._enter(pc + 1, st)
                return
            if not is_dig:
                raise GrammarError("expected digits")
            if token == self.zero:
                st[1], st[3] = 4, 1
                return
            if g.tok_class[token] & 4:               # leading zero on a multi-digit token
                raise GrammarError("leading zero")
            st[1], st[3] = 1, nd
            if nd >= maxd:
                st[1] = 4
            return
        if ph in (1, 3, 4) and self._end(succ, token, st, forced):
            return
        if kind == NUM_DEC and ph in (1, 4) and token == g.dot_token:
            st[1], st[3] = 2, 0
            return
        if not is_dig or ph in (4, 5):
            raise GrammarError(f"token {token} not allowed in number phase {ph}")
        if ph == 1:
            st[3] += nd
            if st[3] >= maxd:
                st[1] = 4
        elif ph == 2:
            st[1], st[3] = 3, nd
            if nd >= maxfrac:
                st[1] = 5
        elif ph == 3:
            st[3] += nd
            if st[3] >= maxfrac:
                st[1] = 5

    def _end(self, succ, token, st, forced) -> bool:
        """A number's end token = the first token of its successor."""
        g = self.g
        nxt = g.ops[succ]
        if nxt.code == OP_LIT:
            if token != g.lit_first[nxt.a]:
                return False
            st[:] = self._enter(succ, st, sub=1)
            return True
        c = self._enter(succ, st)
        for a in self._enabled(nxt.a, c):
            if a.first == token:
                st[:] = c
                self._take(a, st, forced, sampled=True)
                return True
        return False


def run_tokens(fsm: PyGrammarFSM, choose, min_items: int = 0, profile: int = 0,
               max_tokens: int = 1200) -> list[int]:
    """Drive the automaton to completion; `choose(mask_row, state) -> token` picks
    free tokens.  Honours the token budget like the engine does."""
    st, out = fsm.initial(min_items, profile, max_tokens)
    while not fsm.done(st):
        t = choose(fsm.mask(st), st)
        out.append(t)
        st, forced = fsm.advance(st, t, max_tokens - len(out))
        out.extend(forced)
    return out
