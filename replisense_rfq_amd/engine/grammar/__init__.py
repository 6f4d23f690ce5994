"""JSON-schema-constrained decoding for the RFQ response schema.

``RFQGrammar`` bundles the compiled program, the GPU mask table and an executor:
the native C++ automaton (csrc/runtime/grammar.cpp) when the runtime module is
built, else the Python twin (:mod:`.fsm`).  Both expose::

    initial(min_items=0, profile=0, budget=NO_BUDGET) -> (state, forced_tokens)
    advance(state, token, budget=NO_BUDGET) -> (state, forced_tokens)
    batch_advance(states[n,6], tokens[n], budgets[n]) -> (mask_idx[n], forced_off[n+1],
                                                          forced, ok[n])

State = (pc, sub, cnt, rem, min_items, profile); profiles and the token-budget
close-out are described in :mod:`.compiler`.
"""
from __future__ import annotations

import functools

import numpy as np

from .compiler import (PROFILE_REFERENCE, PROFILE_SYNTHETIC, CompiledGrammar, Limits,
                       compile_rfq_grammar, mask_table_int32)
from .fsm import DONE, NO_BUDGET, GrammarError, PyGrammarFSM

__all__ = ["RFQGrammar", "get_grammar", "Limits", "GrammarError", "DONE", "NO_BUDGET",
           "PROFILE_REFERENCE", "PROFILE_SYNTHETIC"]


def pack_native(g: CompiledGrammar, quote: int | None = None) -> dict:
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
            alts += [a.first, len(rest), len(a.rest), a.target, a.cnt, a.flags]
            rest += a.rest
    return dict(
        ops=np.array([[o.code, o.a, o.b, o.c, o.d, o.e] for o in g.ops], np.int32).reshape(-1),
        lit_off=lit_off, lit_tok=lit_tok, lit1_off=lit1_off, lit1_tok=lit1_tok,
        lit_first=np.array(g.lit_first, np.int32),
        choice_off=choice_off, alts=np.array(alts, np.int32), alt_rest=np.array(rest, np.int32),
        choice_masks=np.ascontiguousarray(g.choice_masks, np.int32).reshape(-1),
        max_items=np.array(g.max_items, np.int32), honors_min=np.array(g.honors_min, np.int32),
        caps=np.ascontiguousarray(g.caps, np.int32).reshape(-1),
        num_masks=np.ascontiguousarray(g.num_masks, np.int32).reshape(-1),
        num_caps=np.ascontiguousarray(g.num_caps, np.int32).reshape(-1),
        fin=np.ascontiguousarray(g.fin, np.int32).reshape(-1),
        fin1=np.ascontiguousarray(g.fin1, np.int32).reshape(-1),
        close_alt=np.ascontiguousarray(g.close_alt, np.int32).reshape(-1),
        null_ids=np.array(g.null_ids, np.int32), tok_class=g.tok_class, tok_chars=g.tok_chars,
        tok_digits=g.tok_digits, tok_utf=g.tok_utf,
        str_masks=np.array(g.str_masks, np.int32),
        scalars=np.array([g.quote, g.zero_token, g.dot_token, g.backslash, g.slack, g.start_pc,
                          g.caps.shape[1], g.cont_token], np.int32),
    )


class RFQGrammar:
    def __init__(self, tokenizer, limits: Limits | None = None, native: bool | None = None):
        self.compiled = compile_rfq_grammar(tokenizer, limits)
        self.py = PyGrammarFSM(self.compiled)
        self.native = None
        if native is not False:
            try:
                from ... import runtime

                self.native = runtime.load().Grammar(pack_native(self.compiled))
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

    def initial(self, min_items: int = 0, profile: int = PROFILE_REFERENCE,
                budget: int = NO_BUDGET):
        st, forced = self.exec.initial(min_items, profile, budget)
        return tuple(st), list(forced)

    def advance(self, state, token: int, budget: int = NO_BUDGET):
        if self.native is not None:
            try:
                st, forced = self.native.advance(tuple(state), int(token), int(budget))
            except ValueError as e:
                raise GrammarError(str(e)) from None
            return tuple(st), list(forced)
        return self.py.advance(state, token, budget)

    def mask(self, state) -> int:
        return self.exec.mask(tuple(state))

    def done(self, state) -> bool:
        return self.py.done(state)

    def batch_advance(self, states: np.ndarray, tokens: np.ndarray, budgets=None):
        n = len(tokens)
        budgets = (np.full(n, NO_BUDGET, np.int32) if budgets is None
                   else np.ascontiguousarray(budgets, np.int32))
        if self.native is not None:
            return self.native.batch_advance(states, np.ascontiguousarray(tokens, np.int32),
                                             budgets)
        masks = np.empty(n, np.int32)
        offs = np.zeros(n + 1, np.int32)
        ok = np.ones(n, bool)
        forced_all: list[int] = []
        for i in range(n):
            offs[i] = len(forced_all)
            try:
                st, forced = self.py.advance(tuple(states[i]), int(tokens[i]), int(budgets[i]))
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
