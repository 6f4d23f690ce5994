"""Drive the grammar automaton along a given JSON text.

``grammar_tokens(grammar, tok, text)`` finds the token sequence the constrained
decoder would have to produce to emit ``text`` exactly: at every sampling state it
tries the tokens that are both allowed by the state's mask row and a prefix of the
remaining text (longest first, backtracking on a dead end); forced (jump-forward)
tokens must spell the text themselves.  Raises ``GrammarError`` if the automaton
cannot produce the text, so "the grammar admits every completion the reference's
model returned" (cache_rows.json) is a checked property, not a claim.
"""
from __future__ import annotations

import numpy as np

from .fsm import GrammarError

MAX_TOKEN_BYTES = 48


class _Vocab:
    def __init__(self, tok):
        self.raw = tok.token_bytes_table()
        self.by_bytes: dict[bytes, list[int]] = {}
        for i, b in enumerate(self.raw):
            if b:
                self.by_bytes.setdefault(bytes(b), []).append(i)


_VOCABS: dict[int, _Vocab] = {}


def _vocab(tok) -> _Vocab:
    v = _VOCABS.get(id(tok))
    if v is None:
        v = _VOCABS[id(tok)] = _Vocab(tok)
    return v


def _allowed(mask_rows: np.ndarray, row: int, token: int) -> bool:
    return bool((int(mask_rows[row, token >> 5]) >> (token & 31)) & 1)


def grammar_tokens(executor, tok, text: str, mask_rows: np.ndarray, *, min_items: int = 0,
                   profile: int = 0, budget: int = 1 << 30, max_steps: int = 20000,
                   sampled: list | None = None) -> list[int]:
    """Token ids (sampled + forced) that make `executor` emit `text`.

    ``sampled``: if a list is given it receives one bool per returned id -- True where
    the decoder samples the token (one engine step), False where the grammar forces it
    (jump-forward) -- so ``sum(sampled)`` is the serial step count of that completion.

    `executor`: an object with ``initial(min_items, profile, budget)``,
    ``advance(state, token, budget)`` and ``mask(state)`` (the native automaton or
    the Python twin); `mask_rows`: the grammar's uint32 mask table."""
    voc = _vocab(tok)
    target = text.encode("utf-8")

    def spell(ids, pos):
        for t in ids:
            b = voc.raw[t] or b""
            if target[pos:pos + len(b)] != b:
                return -1
            pos += len(b)
        return pos

    st, forced = executor.initial(min_items, profile, budget)
    out = list(forced)
    flags = [False] * len(out)
    pos = spell(forced, 0)
    if pos < 0:
        raise GrammarError("the grammar's opening literal does not match the text")
    # DFS stack of (state, pos, out length, remaining candidates)
    stack = []
    steps = 0

    def candidates(state, p):
        row = executor.mask(state)
        if row < 0:
            return []
        c = []
        for n in range(min(MAX_TOKEN_BYTES, len(target) - p), 0, -1):
            for t in voc.by_bytes.get(target[p:p + n], ()):
                if _allowed(mask_rows, row, t):
                    c.append(t)
        return c

    cands = candidates(st, pos)
    while True:
        if executor.mask(st) < 0:
            if pos == len(target):
                if sampled is not None:
                    sampled[:] = flags
                return out
            cands = []                      # finished early: backtrack
        advanced = False
        while cands:
            t = cands.pop(0)
            steps += 1
            if steps > max_steps:
                raise GrammarError("search budget exhausted")
            try:
                nst, f = executor.advance(st, t, budget - len(out) - 1)
            except (GrammarError, ValueError):
                continue
            b = voc.raw[t]
            npos = spell(f, pos + len(b))
            if npos < 0:
                continue
            stack.append((st, pos, len(out), cands))
            out = out + [t] + list(f)
            flags = flags + [True] + [False] * len(f)
            st, pos = nst, npos
            cands = candidates(st, pos)
            advanced = True
            break
        if advanced:
            continue
        if not stack:
            raise GrammarError(f"text not admitted by the grammar at byte {pos}: "
                               f"{target[max(0, pos - 40):pos + 40]!r}")
        st, pos, n, cands = stack.pop()
        out = out[:n]
        flags = flags[:n]
