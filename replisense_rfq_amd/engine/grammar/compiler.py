"""RFQ JSON-schema grammar -> token-level automaton program + vocabulary bitmasks.

The reference asks the LLM for "valid JSON only" (rfq_agent.py:103,114) with the
RFQResponse field list (rfq_agent.py:20-59, prompt :75-105) and recovers JSON from
free text afterwards (rfq_agent.py:208-236).  The on-node engine instead makes
invalid output impossible: decoding is constrained by an automaton compiled from
the schema, so every completion parses and validates (the *validated* path of
rfq_agent.py:185-206, never the fallback).

Program model (executed per token by csrc/runtime/grammar.cpp, with a pure-Python
twin in :mod:`.fsm` used as its test oracle):

  LIT  i                   forced literal text (jump-forward: its canonical tokens
                           are appended without sampling)
  CHOICE c                 one sampled token picks an alternative; each alternative
                           = (first token, forced rest, target pc, counter op)
  STR  maxlen              string body after the opening quote: any string-safe
                           token (no '"', '\\', control chars, valid UTF-8) or the
                           closing '"'; forced close once maxlen chars are used
  NUM  kind,maxd,end,null  integer / decimal / fraction digits with an explicit end
                           token (the first char of the following literal)
  END                      accept

Per-state vocabulary masks are rows of a [n_masks, ceil(V/32)] u32 table uploaded
once to the GPU; the sampler kernel applies row ``mask_idx[b]`` per sequence.
Length bounds on every free-form value make any random-weight model terminate
well inside max_tokens=1200 (rfq_agent.py:67).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np

# opcodes
OP_LIT, OP_CHOICE, OP_STR, OP_NUM, OP_END = 0, 1, 2, 3, 4
# NUM kinds
NUM_INT, NUM_DEC, NUM_FRAC = 0, 1, 2
# counter ops on a CHOICE alternative
CNT_NONE, CNT_SET1, CNT_INC = 0, 1, 2
# token class bits
TC_STR = 1        # string-safe content
TC_DIGITS = 2     # all ASCII digits
TC_ZERO_LEAD = 4  # digits starting with '0'


@dataclass
class Alt:
    first: int
    rest: list[int]
    target: int
    cnt: int = CNT_NONE
    is_continue: bool = False    # disabled once the array counter hits max
    is_close: bool = False       # disabled while the counter is below the request's min_items


@dataclass
class Op:
    code: int
    a: int = 0
    b: int = 0
    c: int = 0
    d: int = 0


@dataclass
class Limits:
    title: int = 36
    field: int = 20
    description: int = 44
    part_number: int = 16
    item_description: int = 28
    currency: int = 6
    max_items: int = 8
    max_docs: int = 2
    doc: int = 20
    max_missing: int = 3
    missing: int = 16
    qty_digits: int = 6
    price_int_digits: int = 6
    price_frac_digits: int = 2
    conf_digits: int = 2


TOP_FIELDS = ["title", "client_name", "client_email", "client_contact", "client_phone", "rfq_to",
              "delivery_location", "delivery_deadline", "response_due_date", "description"]


@dataclass
class CompiledGrammar:
    ops: list[Op]
    literals: list[list[int]]          # canonical token ids per literal
    literals_skip1: list[list[int]]    # same literal minus its first char
    literal_text: list[str]
    choices: list[list[Alt]]
    choice_mask: list[int]             # mask row per choice (all alternatives)
    choice_mask_close: list[int]       # mask row with continue-alternatives removed (-1: n/a)
    max_items: list[int]               # per choice: counter limit (0 = no limit)
    honors_min: list[int]              # per choice: 1 if the request's min_items applies
    str_mask: int
    num_masks: dict                    # (kind, phase, end_char_idx, null) -> row
    end_tokens: list[int]              # token id of ',', '}', ']'
    null_first: int
    null_rest: list[int]
    mask_rows: np.ndarray              # [n_masks, W] uint32
    tok_class: np.ndarray              # [V] uint8
    tok_chars: np.ndarray              # [V] uint8 (decoded char length, capped 255)
    tok_digits: np.ndarray             # [V] uint8 (digit count for digit tokens)
    vocab_size: int
    start_pc: int = 0
    dot_token: int = -1
    meta: dict = field(default_factory=dict)

    @property
    def n_masks(self) -> int:
        return self.mask_rows.shape[0]


# ---------------------------------------------------------------- vocabulary

def token_table(tok) -> tuple[np.ndarray, np.ndarray, np.ndarray, list[bytes]]:
    """Classify every token id by its decoded bytes."""
    V = tok.vocab_size
    raw = tok.token_bytes_table()
    cls = np.zeros(V, np.uint8)
    nch = np.zeros(V, np.uint8)
    ndig = np.zeros(V, np.uint8)
    for i, b in enumerate(raw):
        if b is None or len(b) == 0:
            continue
        try:
            s = b.decode("utf-8")
        except UnicodeDecodeError:
            continue
        nch[i] = min(255, len(s))
        if all(c not in '"\\' and ord(c) >= 0x20 and ord(c) != 0x7F for c in s):
            cls[i] |= TC_STR
        if s.isascii() and s.isdigit():
            cls[i] |= TC_DIGITS
            ndig[i] = min(255, len(s))
            if s[0] == "0":
                cls[i] |= TC_ZERO_LEAD
    return cls, nch, ndig, raw


class _MaskBuilder:
    def __init__(self, V: int):
        self.V = V
        self.W = (V + 31) // 32
        self.rows: list[np.ndarray] = []
        self.index: dict[bytes, int] = {}

    def add(self, allowed: np.ndarray) -> int:
        bits = np.zeros(self.W * 32, np.uint8)
        bits[: self.V] = allowed.astype(np.uint8)
        row = np.packbits(bits, bitorder="little").view("<u4").astype(np.uint32)
        key = row.tobytes()
        if key in self.index:
            return self.index[key]
        self.rows.append(row)
        self.index[key] = len(self.rows) - 1
        return self.index[key]

    def ids(self, ids) -> int:
        a = np.zeros(self.V, bool)
        a[list(ids)] = True
        return self.add(a)

    def table(self) -> np.ndarray:
        return np.stack(self.rows)


# ------------------------------------------------------------------ compiler

class _Prog:
    def __init__(self, tok):
        self.tok = tok
        self.ops: list[Op] = []
        self.literals: list[list[int]] = []
        self.literals_skip1: list[list[int]] = []
        self.literal_text: list[str] = []
        self.choices: list[list[Alt]] = []
        self.choice_limits: list[int] = []
        self.choice_min: list[int] = []

    def enc(self, s: str) -> list[int]:
        return self.tok.encode(s)

    def single(self, s: str) -> int:
        ids = self.enc(s)
        if len(ids) != 1:
            raise ValueError(f"grammar needs {s!r} to be a single token, got {ids}")
        return ids[0]

    def pc(self) -> int:
        return len(self.ops)

    def lit(self, text: str):
        # merge with a directly preceding literal
        if self.ops and self.ops[-1].code == OP_LIT and getattr(self, "_last_lit_open", False):
            i = self.ops[-1].a
            text = self.literal_text[i] + text
            self.literal_text[i] = text
            self.literals[i] = self.enc(text)
            self.literals_skip1[i] = self.enc(text[1:]) if len(text) > 1 else []
            return
        self.literal_text.append(text)
        self.literals.append(self.enc(text))
        self.literals_skip1.append(self.enc(text[1:]) if len(text) > 1 else [])
        self.ops.append(Op(OP_LIT, len(self.literals) - 1))
        self._last_lit_open = True

    def _seal(self):
        self._last_lit_open = False

    def choice(self, alts: list[Alt], limit: int = 0, honors_min: bool = False) -> int:
        self._seal()
        self.choices.append(alts)
        self.choice_limits.append(limit)
        self.choice_min.append(int(honors_min))
        self.ops.append(Op(OP_CHOICE, len(self.choices) - 1))
        return self.pc() - 1

    def op(self, code, a=0, b=0, c=0, d=0) -> int:
        self._seal()
        self.ops.append(Op(code, a, b, c, d))
        return self.pc() - 1


def compile_rfq_grammar(tok, limits: Limits | None = None) -> CompiledGrammar:
    """Compile the RFQResponse schema (field order = rfq_agent.py:41-59) for `tok`."""
    L = limits or Limits()
    P = _Prog(tok)
    quote = P.single('"')
    comma, rbrace, rbrack = P.single(","), P.single("}"), P.single("]")
    lbrace = P.single("{")
    dot = P.single(".")
    null_ids = P.enc("null")
    true_ids, false_ids = P.enc("true"), P.enc("false")
    END_IDX = {",": 0, "}": 1, "]": 2}

    def str_or_null(maxlen: int):
        # CHOICE(null | '"') ; STR ; (continues at next op)
        p = P.choice([])            # patched below
        P.op(OP_STR, maxlen)
        nxt = P.pc()
        P.choices[P.ops[p].a][:] = [Alt(null_ids[0], null_ids[1:], nxt), Alt(quote, [], p + 1)]

    def number(kind: int, maxd: int, end: str, nullable: bool, maxfrac: int = 0):
        P.op(OP_NUM, kind, maxd, END_IDX[end] | (int(nullable) << 4), maxfrac)

    # ---- top level -------------------------------------------------------
    first = True
    for f in TOP_FIELDS:
        P.lit(("{" if first else ", ") + f'"{f}": ')
        first = False
        mx = L.title if f == "title" else (L.description if f == "description" else L.field)
        str_or_null(mx)

    # ---- line_items: [ {part_number, description, quantity, target_price, currency}, ... ]
    P.lit(', "line_items": [')
    open_pc = P.choice([], honors_min=True)
    body = P.pc()
    P.lit('"part_number": ')
    str_or_null(L.part_number)
    P.lit(', "description": ')
    str_or_null(L.item_description)
    P.lit(', "quantity": ')
    number(NUM_INT, L.qty_digits, ",", True)
    P.lit(', "target_price": ')
    number(NUM_DEC, L.price_int_digits, ",", True, L.price_frac_digits)
    P.lit(', "currency": ')
    str_or_null(L.currency)
    P.lit("}")
    next_pc = P.choice([], limit=L.max_items, honors_min=True)
    after_items = P.pc()
    P.choices[P.ops[open_pc].a][:] = [
        Alt(rbrack, [], after_items, is_close=True),
        Alt(lbrace, [], body, CNT_SET1, is_continue=True)]
    P.choices[P.ops[next_pc].a][:] = [
        Alt(rbrack, [], after_items, is_close=True),
        Alt(comma, P.enc(" {"), body, CNT_INC, is_continue=True)]

    def str_array(maxn: int, maxlen: int, after_text: str):
        o = P.choice([])
        sbody = P.op(OP_STR, maxlen)
        n = P.choice([], limit=maxn)
        aft = P.pc()
        P.choices[P.ops[o].a][:] = [Alt(rbrack, [], aft),
                                    Alt(quote, [], sbody, CNT_SET1, is_continue=True)]
        P.choices[P.ops[n].a][:] = [Alt(rbrack, [], aft),
                                    Alt(comma, P.enc(' "'), sbody, CNT_INC, is_continue=True)]
        P.lit(after_text)

    P.lit(', "requested_documents": [')
    str_array(L.max_docs, L.doc, ', "confidence_score": 0.')
    number(NUM_FRAC, L.conf_digits, ",", False)
    P.lit(', "missing_fields": [')
    str_array(L.max_missing, L.missing, ', "requires_review": ')
    P.choice([Alt(true_ids[0], true_ids[1:], P.pc() + 1), Alt(false_ids[0], false_ids[1:], P.pc() + 1)])
    P.lit("}")
    P.op(OP_END)

    # ---- masks -------------------------------------------------------------
    cls, nch, ndig, _ = token_table(tok)
    V = tok.vocab_size
    mb = _MaskBuilder(V)
    mb.ids([0])  # row 0: placeholder (never used for sampling)
    str_allowed = (cls & TC_STR) != 0
    str_allowed_q = str_allowed.copy()
    str_allowed_q[quote] = True
    str_mask = mb.add(str_allowed_q)
    digits = (cls & TC_DIGITS) != 0
    nz_digits = digits & ((cls & TC_ZERO_LEAD) == 0)
    zero_tok = P.single("0")
    end_tokens = [comma, rbrace, rbrack]
    num_masks = {}
    for kind in (NUM_INT, NUM_DEC, NUM_FRAC):
        for e in range(3):
            for nullable in (0, 1):
                # phase 0: first token
                a = (digits.copy() if kind == NUM_FRAC else nz_digits.copy())
                if kind != NUM_FRAC:
                    a[zero_tok] = True
                if nullable:
                    a[null_ids[0]] = True
                num_masks[(kind, 0, e, nullable)] = mb.add(a)
                # phase 1: more digits or end (DEC: also '.')
                a = digits.copy()
                a[end_tokens[e]] = True
                if kind == NUM_DEC:
                    a[dot] = True
                num_masks[(kind, 1, e, nullable)] = mb.add(a)
                # phase 2 (DEC after '.'): fraction digits, at least one
                num_masks[(kind, 2, e, nullable)] = mb.add(digits.copy())
                # phase 3 (DEC fraction continuing): digits or end
                a = digits.copy()
                a[end_tokens[e]] = True
                num_masks[(kind, 3, e, nullable)] = mb.add(a)
                # end only (integer part "0" or digit budget exhausted): end or '.'
                a = np.zeros(V, bool)
                a[end_tokens[e]] = True
                if kind == NUM_DEC:
                    a[dot] = True
                num_masks[(kind, 4, e, nullable)] = mb.add(a)
    choice_mask, choice_mask_close = [], []
    for alts in P.choices:
        if len({a.first for a in alts}) != len(alts):
            raise ValueError("ambiguous grammar choice (shared first token)")
        choice_mask.append(mb.ids([a.first for a in alts]))
        close = [a.first for a in alts if not a.is_continue]
        choice_mask_close.append(mb.ids(close) if close and len(close) < len(alts) else -1)
    g = CompiledGrammar(
        ops=P.ops, literals=P.literals, literals_skip1=P.literals_skip1,
        literal_text=P.literal_text, choices=P.choices, choice_mask=choice_mask,
        choice_mask_close=choice_mask_close, max_items=P.choice_limits,
        honors_min=P.choice_min, str_mask=str_mask,
        num_masks=num_masks, end_tokens=end_tokens, null_first=null_ids[0],
        null_rest=null_ids[1:], mask_rows=mb.table(), tok_class=cls, tok_chars=nch,
        tok_digits=ndig, vocab_size=V, dot_token=dot,
        meta={"limits": L.__dict__, "zero_token": zero_tok})
    return g


def mask_table_int32(g: CompiledGrammar) -> np.ndarray:
    """The mask table as int32 (bit-identical) for torch upload."""
    return g.mask_rows.view(np.int32)


def describe(g: CompiledGrammar) -> str:
    return json.dumps({"ops": len(g.ops), "literals": len(g.literals), "choices": len(g.choices),
                       "masks": g.n_masks, "vocab": g.vocab_size})
