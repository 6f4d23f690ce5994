"""Token-level executor of a compiled RFQ grammar (pure-Python twin of
csrc/runtime/grammar.cpp; the C++ executor is what the engine's step loop runs —
this one is its test oracle and the fallback when the runtime .so is absent).

State = (pc, sub, cnt, rem, minv):
  LIT    sub=1 -> the literal's first char was already produced (by a NUM end token)
  STR    rem = characters still allowed
  NUM    sub = phase (0 first, 1 int digits, 2 after '.', 3 frac digits, 4 end/dot only,
         5 forced end), rem = digits used in the current part
  CHOICE cnt = array item counter; minv = the request's minimum line-item count
         (schema hint: the close alternative is disabled while cnt < minv)
"""
from __future__ import annotations

from .compiler import (CNT_INC, CNT_SET1, NUM_DEC, NUM_FRAC, OP_CHOICE, OP_END, OP_LIT,
                       OP_NUM, OP_STR, TC_DIGITS, CompiledGrammar)

DONE = -1


class GrammarError(ValueError):
    pass


class PyGrammarFSM:
    def __init__(self, g: CompiledGrammar):
        self.g = g
        # the opening quote of strings is the single-token alternative shared by every
        # string choice; find it from the STR-bearing choices
        self.quote = self._find_quote()
        self.zero = g.meta["zero_token"]

    def _find_quote(self) -> int:
        g = self.g
        for pc, op in enumerate(g.ops):
            if op.code == OP_CHOICE:
                for a in g.choices[op.a]:
                    if a.target < len(g.ops) and g.ops[a.target].code == OP_STR and not a.rest:
                        return a.first
        raise GrammarError("grammar has no string choice")

    # ------------------------------------------------------------------ entry
    def _enter(self, pc: int, cnt: int, sub: int = 0, minv: int = 0):
        op = self.g.ops[pc]
        if op.code == OP_STR:
            return [pc, 0, cnt, op.a, minv]
        return [pc, sub, cnt, 0, minv]

    def initial(self, min_items: int = 0):
        st = self._enter(self.g.start_pc, 0, minv=min_items)
        forced: list[int] = []
        self._settle(st, forced)
        return tuple(st), forced

    # ----------------------------------------------------------------- settle
    def _settle(self, st, forced):
        g = self.g
        while True:
            pc = st[0]
            op = g.ops[pc]
            if op.code == OP_LIT:
                forced.extend(g.literals_skip1[op.a] if st[1] else g.literals[op.a])
                st[:] = self._enter(pc + 1, st[2], minv=st[4])
            elif op.code == OP_CHOICE:
                alts = self._enabled(op.a, st[2], st[4])
                if len(alts) != 1:
                    return
                self._take(alts[0], st, forced)
            elif op.code == OP_STR:
                if st[3] > 0:
                    return
                forced.append(self.quote)
                st[:] = self._enter(pc + 1, st[2], minv=st[4])
            elif op.code == OP_NUM:
                if st[1] == 5:
                    st[:] = self._enter(pc + 1, st[2], minv=st[4])
                elif st[1] == 4 and op.a != NUM_DEC:
                    st[:] = self._enter(pc + 1, st[2], minv=st[4])      # only the end token is legal
                else:
                    return
            else:
                return

    def _enabled(self, ci: int, cnt: int, minv: int = 0):
        g = self.g
        alts = g.choices[ci]
        lim = g.max_items[ci]
        if lim and cnt >= lim:
            return [a for a in alts if not a.is_continue]
        if g.honors_min[ci] and cnt < minv:
            return [a for a in alts if not a.is_close]
        return alts

    def _take(self, alt, st, forced, sampled=False):
        if not sampled:
            forced.append(alt.first)
        forced.extend(alt.rest)
        cnt = st[2]
        if alt.cnt == CNT_SET1:
            cnt = 1
        elif alt.cnt == CNT_INC:
            cnt += 1
        st[:] = self._enter(alt.target, cnt, minv=st[4])

    # ------------------------------------------------------------------ query
    def mask(self, state) -> int:
        g = self.g
        pc, sub, cnt, rem, minv = state
        op = g.ops[pc]
        if op.code == OP_CHOICE:
            return g.choice_mask[op.a]
        if op.code == OP_STR:
            return g.str_mask
        if op.code == OP_NUM:
            return g.num_masks[(op.a, sub, op.c & 15, (op.c >> 4) & 1)]
        return DONE

    def done(self, state) -> bool:
        return self.g.ops[state[0]].code == OP_END

    # ---------------------------------------------------------------- advance
    def advance(self, state, token: int):
        """Consume one *sampled* token; returns (new_state, forced_tokens)."""
        g = self.g
        st = list(state)
        forced: list[int] = []
        op = g.ops[st[0]]
        if op.code == OP_CHOICE:
            for a in self._enabled(op.a, st[2], st[4]):
                if a.first == token:
                    self._take(a, st, forced, sampled=True)
                    break
            else:
                raise GrammarError(f"token {token} not allowed at choice pc={st[0]}")
        elif op.code == OP_STR:
            if token == self.quote:
                st[:] = self._enter(st[0] + 1, st[2], minv=st[4])
            else:
                if not (g.tok_class[token] & 1):
                    raise GrammarError(f"token {token} not string-safe")
                st[3] -= max(1, int(g.tok_chars[token]))
        elif op.code == OP_NUM:
            self._num(op, st, token, forced)
        else:
            raise GrammarError("advance() on a finished grammar")
        self._settle(st, forced)
        return tuple(st), forced

    def _num(self, op, st, token, forced):
        g = self.g
        kind, maxd, end_idx, nullable, maxfrac = op.a, op.b, op.c & 15, (op.c >> 4) & 1, op.d
        end_tok = g.end_tokens[end_idx]
        is_dig = bool(g.tok_class[token] & TC_DIGITS)
        nd = int(g.tok_digits[token])
        ph = st[1]
        pc = st[0]

        def finish_skip1():
            st[:] = self._enter(pc + 1, st[2], sub=1, minv=st[4])

        if ph == 0:
            if nullable and token == g.null_first:
                forced.extend(g.null_rest)
                st[:] = self._enter(pc + 1, st[2], minv=st[4])
                return
            if not is_dig:
                raise GrammarError("expected digits")
            if kind == NUM_FRAC:
                st[1], st[3] = 3, nd
                if nd >= maxd:
                    st[1] = 5
                return
            if token == self.zero:
                st[1], st[3] = 4, 1
                return
            st[1], st[3] = 1, nd
            if nd >= maxd:
                st[1] = 4
            return
        if ph in (1, 3, 4) and token == end_tok:
            finish_skip1()
            return
        if kind == NUM_DEC and ph in (1, 4) and token == g.dot_token:
            st[1], st[3] = 2, 0
            return
        if not is_dig or ph == 4:
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
            lim = maxfrac if kind == NUM_DEC else maxd
            if st[3] >= lim:
                st[1] = 5


def run_tokens(fsm: PyGrammarFSM, choose, min_items: int = 0) -> list[int]:
    """Drive the automaton to completion; `choose(mask_row) -> token` picks free tokens."""
    st, out = fsm.initial(min_items)
    while not fsm.done(st):
        t = choose(fsm.mask(st), st)
        out.append(t)
        st, forced = fsm.advance(st, t)
        out.extend(forced)
    return out
