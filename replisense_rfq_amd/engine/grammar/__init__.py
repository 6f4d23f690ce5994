"""JSON-schema-constrained decoding for the RFQ response schema.

``RFQGrammar`` bundles the compiled program, the GPU mask table and an executor:
the native C++ automaton (csrc/runtime/grammar.cpp) when the runtime module is
built, else the Python twin (:mod:`.fsm`).  Both expose::

    initial(min_items=0) -> (state, forced_tokens)
    advance(state, token) -> (state, forced_tokens)
    batch_advance(states[n,5], tokens[n]) -> (mask_idx[n], forced_off[n+1], forced, ok[n])

State = (pc, sub, cnt, rem, min_items).
"""
from __future__ import annotations

import functools

import numpy as np

from .compiler import (Limits, NUM_DEC, NUM_FRAC, NUM_INT, CompiledGrammar, compile_rfq_grammar,
                       mask_table_int32)
from .fsm import DONE, GrammarError, PyGrammarFSM

__all__ = ["RFQGrammar", "get_grammar", "Limits", "GrammarError", "DONE"]


def pack_native(g: CompiledGrammar, quote: int) -> dict:
    """Flatten a CompiledGrammar into the arrays the C++ executor consumes."""
    def csr(lists):
        off = np.zeros(len(lists) + 1, np.int32)
        for i, l in enumerate(lists):
            off[i + 1] = off[i] + len(l)
        tok = np.array([t for l in lists for t in l], np.int32) if off[-1] else np.zeros(0, np.int32)
        return off, tok

    lit_off, lit_tok = csr(g.literals)
    lit1_off, lit1_tok = csr(g.literals_skip1)
    choice_off = np.zeros(len(g.choices) + 1, np.int32)
    alts, rest = [], []
    for ci, al in enumerate(g.choices):
        choice_off[ci + 1] = choice_off[ci] + len(al)
        for a in al:
            alts += [a.first, len(rest), len(a.rest), a.target, a.cnt, int(a.is_continue),
                     int(a.is_close)]
            rest += a.rest
    num = np.full(3 * 5 * 3 * 2, -1, np.int32)
    for (kind, phase, e, nl), row in g.num_masks.items():
        num[((kind * 5 + phase) * 3 + e) * 2 + nl] = row
    return dict(
        ops=np.array([[o.code, o.a, o.b, o.c, o.d] for o in g.ops], np.int32).reshape(-1),
        lit_off=lit_off, lit_tok=lit_tok, lit1_off=lit1_off, lit1_tok=lit1_tok,
        choice_off=choice_off, alts=np.array(alts, np.int32), alt_rest=np.array(rest, np.int32),
        choice_mask=np.array(g.choice_mask, np.int32),
        choice_mask_close=np.array(g.choice_mask_close, np.int32),
        max_items=np.array(g.max_items, np.int32), honors_min=np.array(g.honors_min, np.int32),
        num_masks=num,
        null_rest=np.array(g.null_rest, np.int32), tok_class=g.tok_class, tok_chars=g.tok_chars,
        tok_digits=g.tok_digits,
        scalars=np.array([g.str_mask, quote, g.meta["zero_token"], g.dot_token, g.null_first,
                          *g.end_tokens, g.start_pc], np.int32),
    )


class RFQGrammar:
    def __init__(self, tokenizer, limits: Limits | None = None, native: bool | None = None):
        self.compiled = compile_rfq_grammar(tokenizer, limits)
        self.py = PyGrammarFSM(self.compiled)
        self.native = None
        if native is not False:
            try:
                from ... import runtime

                self.native = runtime.load().Grammar(pack_native(self.compiled, self.py.quote))
            except Exception:
                if native:
                    raise
        self.vocab_size = self.compiled.vocab_size
        self.mask_words = self.compiled.mask_rows.shape[1]

    @property
    def exec(self):
        return self.native if self.native is not None else self.py

    def mask_table(self) -> np.ndarray:
        return mask_table_int32(self.compiled)

    def initial(self, min_items: int = 0):
        st, forced = self.exec.initial(min_items)
        return tuple(st), list(forced)

    def advance(self, state, token: int):
        if self.native is not None:
            try:
                st, forced = self.native.advance(tuple(state), int(token))
            except ValueError as e:
                raise GrammarError(str(e)) from None
            return tuple(st), list(forced)
        return self.py.advance(state, token)

    def mask(self, state) -> int:
        return self.exec.mask(tuple(state))

    def done(self, state) -> bool:
        return self.py.done(state)

    def batch_advance(self, states: np.ndarray, tokens: np.ndarray):
        if self.native is not None:
            return self.native.batch_advance(states, np.ascontiguousarray(tokens, np.int32))
        n = len(tokens)
        masks = np.empty(n, np.int32)
        offs = np.zeros(n + 1, np.int32)
        ok = np.ones(n, bool)
        forced_all: list[int] = []
        for i in range(n):
            offs[i] = len(forced_all)
            try:
                st, forced = self.py.advance(tuple(states[i]), int(tokens[i]))
                states[i] = st
                forced_all += forced
            except GrammarError:
                ok[i] = False
            masks[i] = self.py.mask(tuple(states[i]))
        offs[n] = len(forced_all)
        return masks, offs, np.array(forced_all, np.int32), ok


@functools.lru_cache(maxsize=4)
def get_grammar(flavor: str = "llama3", tokenizer=None) -> RFQGrammar:
    from ..tokenizer import get_tokenizer

    return RFQGrammar(tokenizer if tokenizer is not None else get_tokenizer(flavor))
