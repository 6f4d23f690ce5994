"""Grammar automaton: every path accepted by the automaton is valid RFQ JSON, the
C++ executor matches the Python twin token for token, masks match the executor."""
import json
import random

import numpy as np
import pytest

from replisense_rfq_amd.engine.grammar import RFQGrammar, get_grammar
from replisense_rfq_amd.engine.tokenizer import get_tokenizer
from replisense_rfq_amd.service.schema import RFQResponse


@pytest.fixture(scope="module")
def tok():
    return get_tokenizer("llama3")


@pytest.fixture(scope="module")
def grammar():
    return get_grammar("llama3")


def _allowed(g: RFQGrammar, row: int) -> np.ndarray:
    words = g.compiled.mask_rows[row]
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: g.vocab_size]
    return np.nonzero(bits)[0]


def _walk(g, seed, executor="native", max_steps=3000):
    rng = random.Random(seed)
    if executor == "native":
        st, out = g.initial()
        adv, msk = g.advance, g.mask
    else:
        st, out = g.py.initial()
        adv, msk = g.py.advance, g.py.mask
    steps = 0
    while True:
        m = msk(st)
        if m < 0:
            break
        allowed = _allowed(g, m)
        # bias toward closing quotes/short values half the time to explore all paths
        t = int(rng.choice(allowed))
        st, forced = adv(st, t)
        out = list(out) + [t] + list(forced)
        steps += 1
        assert steps < max_steps
    return out, steps


@pytest.mark.parametrize("seed", range(12))
def test_random_paths_are_valid_rfq_json(tok, grammar, seed):
    ids, steps = _walk(grammar, seed)
    text = tok.decode(ids)
    obj = json.loads(text)
    RFQResponse(**obj)   # validated path, never the fallback
    assert list(obj)[:3] == ["title", "client_name", "client_email"]
    assert len(ids) <= 1200


def test_native_matches_python(grammar):
    if grammar.native is None:
        pytest.skip("native runtime not built")
    for seed in range(6):
        a, _ = _walk(grammar, seed, "native")
        b, _ = _walk(grammar, seed, "python")
        assert a == b


def test_batch_advance_matches_single(grammar):
    rng = random.Random(5)
    n = 16
    states, toks = [], []
    for i in range(n):
        st, _ = grammar.initial()
        m = grammar.mask(st)
        states.append(st)
        toks.append(int(rng.choice(_allowed(grammar, m))))
    S = np.array(states, np.int32)
    masks, offs, forced, ok = grammar.batch_advance(S, np.array(toks, np.int32))
    assert ok.all()
    for i in range(n):
        st, f = grammar.advance(states[i], toks[i])
        assert tuple(S[i]) == tuple(st)
        assert list(forced[offs[i]:offs[i + 1]]) == list(f)
        assert masks[i] == grammar.mask(st)


def test_illegal_token_rejected(grammar, tok):
    st, _ = grammar.initial()
    bad = tok.encode("}")[0]
    S = np.array([st], np.int32)
    _, _, _, ok = grammar.batch_advance(S, np.array([bad], np.int32))
    assert not ok[0]


def test_worst_case_length_bound(grammar, tok):
    """Always choosing the longest continuation still terminates within 1200 tokens."""
    st, out = grammar.initial()
    chars = grammar.compiled.tok_chars.astype(np.int64)
    closers = {tok.encode("]")[0], tok.encode('"')[0], tok.encode("null")[0]}
    while grammar.mask(st) >= 0:
        allowed = _allowed(grammar, grammar.mask(st))
        # prefer continue alternatives and 1-char tokens (maximum token count)
        cost = np.where(chars[allowed] > 0, chars[allowed], 99) + \
            np.isin(allowed, list(closers)) * 1000
        pick = int(allowed[int(np.argmin(cost))])
        st, forced = grammar.advance(st, pick)
        out += [int(pick)] + forced
    assert len(out) <= 1200, len(out)
    json.loads(tok.decode(out))
