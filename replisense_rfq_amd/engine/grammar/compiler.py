"""RFQ JSON-schema grammar -> token-level automaton program + vocabulary bitmasks.

The reference asks the LLM for "valid JSON only" (rfq_agent.py:103,114) with the
RFQResponse field list (rfq_agent.py:20-59, prompt :75-105) and recovers JSON from
free text afterwards (rfq_agent.py:208-236).  The on-node engine constrains
decoding with an automaton compiled from the schema instead, so every completion
is well-formed JSON with the schema's keys in the schema's order.

What the automaton admits is set by what the reference's model actually emits
(all 14 recorded completions, ``tests/assets/golden/cache_rows.json``, re-serialised
with ``json.dumps``, are accepted token for token -- tests/engine/test_grammar.py):

* strings of any length with JSON escapes (``\\"``, ``\\\\``, ``\\n``, ...);
* any number of ``line_items``; ``currency`` optional (rows 1-10 omit it);
* ``quantity`` / ``target_price`` as a number, ``null`` or a string (rows 4, 11-14:
  ``"2,000"``, ``"20.00"`` -- the LineItem validators strip the commas);
* ``requested_documents`` / ``missing_fields`` as a list or ``null`` (rows 6, 7, 10);
* a top-level string field as a list of strings (row 3's ``delivery_deadline``).

The only length bound is the request's token budget (``max_tokens`` 1200,
rfq_agent.py:67): ``fin[pc]`` is the exact number of tokens the deterministic
*close-out* (cheapest alternatives, close strings/arrays, numbers end) needs from a
state, ``K`` bounds how much one more sampled token can add to it, and once the
remaining budget drops below ``close_cost(state) + K`` the executor force-emits the
close-out.  A constrained completion therefore always ends as parseable JSON
inside the budget, where the reference would return a truncated reply.

Profiles (per request, ``SamplingParams.profile``):

  0  REFERENCE  everything above (the service default).
  1  SYNTHETIC  bench-only decoding hints for random-init weights, which have no
                notion of when a value is complete: the schema-deviating
                ("lenient") alternatives are disabled, strings get character caps
                and arrays item caps (``Limits``), so outputs validate and have the
                reference's length distribution (utils/synth.py:decode_hints).

Program model (executed per token by csrc/runtime/grammar.cpp, with a pure-Python
twin in :mod:`.fsm` used as its test oracle):

  LIT    a=literal           forced text (jump-forward: canonical tokens appended
                             without sampling)
  CHOICE a=choice            one sampled token picks an alternative = (first token,
                             forced rest, target pc, counter op, flags)
  STR    a=cap class         string body after the opening quote; sub=1 after a lone
                             backslash (an escape character must follow), sub=1+p
                             while p UTF-8 continuation bytes of a character split
                             across byte-level tokens are still owed
  NUM    a=kind b=max int digits c=flags(1 nullable, 2 string ok, 4 unit) d=max
         frac digits e=num index
                             integer/decimal with its end token = the first token of
                             the successor (pc+1, or pc+2 past the string op when
                             the number may also be a string); digit caps per
                             profile in ``num_caps``; a unit number (confidence)
                             starts with a forced "0." under the SYNTHETIC profile
  JMP    a=target
  END                        accept
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np

# opcodes
OP_LIT, OP_CHOICE, OP_STR, OP_NUM, OP_END, OP_JMP = 0, 1, 2, 3, 4, 5
# NUM kinds
NUM_INT, NUM_DEC = 0, 1
NUM_NULLABLE, NUM_STR_OK, NUM_UNIT = 1, 2, 4   # NUM_UNIT: SYNTHETIC profile forces '0.'
# counter ops on a CHOICE alternative
CNT_NONE, CNT_SET1, CNT_INC, CNT_RESET = 0, 1, 2, 3
# alternative flags
ALT_CONTINUE, ALT_CLOSE, ALT_LENIENT = 1, 2, 4
# token class bits
TC_STR = 1        # complete string fragment (no '"', no control chars, escapes complete)
TC_DIGITS = 2     # all ASCII digits
TC_ZERO_LEAD = 4  # digits starting with '0'
TC_STR_OPEN = 8   # string fragment ending in a lone backslash
TC_ESC = 16       # starts with an escape character, the rest a complete fragment
STR_SUBS = 5      # STR sub-states: 0 plain, 1 after a lone backslash, 2..4 owing 1..3 bytes
# profiles
PROFILE_REFERENCE, PROFILE_SYNTHETIC = 0, 1
NPROF = 2
UNBOUNDED = 1 << 30            # STR rem when the profile has no cap
NUM_PHASES = 6

# STR cap classes
(CAP_TITLE, CAP_FIELD, CAP_DESCRIPTION, CAP_PART, CAP_ITEM_DESC, CAP_CURRENCY, CAP_DOC,
 CAP_MISSING, CAP_NUMSTR, CAP_ARRAY_STR) = range(10)
NCAP = 10


@dataclass
class Alt:
    first: int
    rest: list[int]
    target: int
    cnt: int = CNT_NONE
    flags: int = 0

    @property
    def is_continue(self) -> bool:
        return bool(self.flags & ALT_CONTINUE)

    @property
    def is_close(self) -> bool:
        return bool(self.flags & ALT_CLOSE)

    @property
    def lenient(self) -> bool:
        return bool(self.flags & ALT_LENIENT)


@dataclass
class Op:
    code: int
    a: int = 0
    b: int = 0
    c: int = 0
    d: int = 0
    e: int = 0


@dataclass
class Limits:
    """Caps of the SYNTHETIC profile (0 = none).  The REFERENCE profile has none.

    Calibrated to the reference's decode shape: the 14
    recorded completions (cache_rows.json, rows 1-14) replayed through this grammar and
    tokenizer take p50 160 sampled steps (one engine step each) and p50 341.5 completion
    tokens.  The caps are measured against the ENGINE itself -- the 8B bench's own
    documents decoded by the random-init Llama-3-8B under Gumbel sampling at T = 0.1 on
    one MI355X (profiles/r6_decode_shape.md, tests/assets/decode_shape_calibration.json):
    a uniform random walk over the same grammar under-reads the engine's sampled steps by
    ~20 % (163.5 vs 200 at the r5 caps), because a random-init model's picks follow its
    context, not a uniform draw.  With the r5 caps x 0.72 below the engine decodes p50
    ~158 sampled steps and ~345 completion tokens per document.  The item array takes
    exactly the document's part count (min_items) up to ``max_items`` = 3 (the recorded
    p50 is 3.5; the bench reports how many documents' hints exceed the cap:
    per_doc.items_hint_truncated_share)."""
    title: int = 104
    field: int = 58
    description: int = 127
    part_number: int = 46
    item_description: int = 81
    currency: int = 6
    max_items: int = 3
    max_docs: int = 2
    doc: int = 58
    max_missing: int = 5
    missing: int = 46

    @classmethod
    def from_env(cls) -> "Limits":
        """Defaults, with the bench calibration knobs RFQ_SYNTH_CAP_SCALE (multiplies the
        string caps) and RFQ_SYNTH_MAX_ITEMS (the line-item cap) when set."""
        import os

        lim = cls()
        scale = float(os.environ.get("RFQ_SYNTH_CAP_SCALE", "1") or 1)
        if scale != 1.0:
            for f in ("title", "field", "description", "part_number", "item_description", "doc",
                      "missing"):
                setattr(lim, f, max(8, int(round(getattr(lim, f) * scale))))
        items = os.environ.get("RFQ_SYNTH_MAX_ITEMS")
        if items:
            lim.max_items = int(items)
        return lim

    def caps(self) -> list[int]:
        c = [0] * NCAP
        c[CAP_TITLE], c[CAP_FIELD], c[CAP_DESCRIPTION] = self.title, self.field, self.description
        c[CAP_PART], c[CAP_ITEM_DESC], c[CAP_CURRENCY] = (self.part_number, self.item_description,
                                                          self.currency)
        c[CAP_DOC], c[CAP_MISSING] = self.doc, self.missing
        c[CAP_NUMSTR], c[CAP_ARRAY_STR] = 12, self.field
        return c


TOP_FIELDS = ["title", "client_name", "client_email", "client_contact", "client_phone", "rfq_to",
              "delivery_location", "delivery_deadline", "response_due_date", "description"]
# (int digits, frac digits) per profile: REFERENCE generous, SYNTHETIC = the reference's
# observed shapes (cache_rows.json: quantities <= 4 digits, prices "31.50", confidence 0.xx)
QTY_CAPS, PRICE_CAPS, CONF_CAPS = ((12, 0), (6, 0)), ((12, 6), (6, 2)), ((1, 4), (1, 2))


@dataclass
class CompiledGrammar:
    ops: list[Op]
    literals: list[list[int]]          # canonical token ids per literal
    literals_skip1: list[list[int]]    # same literal minus its first char
    lit_first: list[int]               # single token of each literal's first char
    literal_text: list[str]
    choices: list[list[Alt]]
    choice_masks: np.ndarray           # [n_choices, 8] mask row per disabled-set combo (-1 none)
    max_items: list[int]               # per choice: SYNTHETIC-profile counter limit (0 = none)
    honors_min: list[int]              # per choice: 1 if the request's min_items applies
    caps: np.ndarray                   # [NPROF, NCAP] STR character caps (0 = none)
    str_masks: tuple                   # STR mask row per sub-state (STR_SUBS)
    num_masks: np.ndarray              # [n_nums, NPROF, NUM_PHASES] mask rows (-1 n/a)
    num_caps: np.ndarray               # [n_nums, NPROF, 2] (max int digits, max frac digits)
    fin: np.ndarray                    # [n_ops, NPROF] close-out tokens from a fresh entry
    fin1: np.ndarray                   # [n_ops, NPROF] same for a LIT entered skip-first
    close_alt: np.ndarray              # [n_choices, NPROF] alternative the close-out takes
    slack: int                         # K: bound on one token's growth of the close-out
    null_ids: list[int]
    backslash: int
    zero_token: int
    dot_token: int
    quote: int
    mask_rows: np.ndarray              # [n_masks, W] uint32
    tok_class: np.ndarray              # [V] uint8
    tok_chars: np.ndarray              # [V] uint8 (decoded char length, capped 255)
    tok_digits: np.ndarray             # [V] uint8 (digit count for digit tokens)
    tok_utf: np.ndarray                # [V] uint8 UTF-8 framing (token_table)
    cont_token: int                    # a lone continuation byte (close-out of a split char)
    vocab_size: int
    start_pc: int = 0
    meta: dict = field(default_factory=dict)

    @property
    def n_masks(self) -> int:
        return self.mask_rows.shape[0]


# ---------------------------------------------------------------- vocabulary

def _fragment(s: str):
    """'ok' if `s` can appear verbatim inside a JSON string, 'open' if it can but
    ends with a lone backslash, else None.  ``\\u`` escapes are not admitted."""
    i, n = 0, len(s)
    while i < n:
        c = s[i]
        if c == '"' or ord(c) < 0x20 or ord(c) == 0x7F:
            return None
        if c == "\\":
            if i + 1 == n:
                return "open"
            if s[i + 1] not in '"\\/bfnrt':
                return None
            i += 2
            continue
        i += 1
    return "ok"


def _utf8_split(b: bytes):
    """Split a byte-level token into (leading continuation bytes c, owed bytes m of
    a trailing partial character, all-continuation flag, decoded middle) or None
    when no valid UTF-8 stream can contain it."""
    c = 0
    while c < len(b) and 0x80 <= b[c] < 0xC0:
        c += 1
    if c > 3:
        return None
    allc = c == len(b)
    rest, m = b[c:], 0
    for k in range(1, min(4, len(rest)) + 1):
        x = rest[-k]
        if x < 0x80:
            break
        if x >= 0xC0:
            need = 2 if x < 0xE0 else 3 if x < 0xF0 else 4 if x < 0xF8 else 0
            if need == 0:
                return None
            if need > k:
                m, rest = need - k, rest[:-k]
            break
    try:
        s = rest.decode("utf-8")
    except UnicodeDecodeError:
        return None
    return c, m, allc, s


def token_table(tok) -> tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, list[bytes]]:
    """Classify every token id by its bytes: class bits, decoded char count, digit
    count and UTF-8 framing (c | m << 2 | all-continuation << 4)."""
    V = tok.vocab_size
    raw = tok.token_bytes_table()
    cls = np.zeros(V, np.uint8)
    nch = np.zeros(V, np.uint8)
    ndig = np.zeros(V, np.uint8)
    utf = np.zeros(V, np.uint8)
    for i, b in enumerate(raw):
        if b is None or len(b) == 0:
            continue
        sp = _utf8_split(bytes(b))
        if sp is None:
            continue
        c, m, allc, s = sp
        utf[i] = c | (m << 2) | (int(allc) << 4)
        nch[i] = min(255, len(s) + (1 if m else 0))
        f = _fragment(s)
        if f == "ok":
            cls[i] |= TC_STR
        elif f == "open" and m == 0:
            cls[i] |= TC_STR_OPEN
        if c == 0 and s and s[0] in '"\\/bfnrt' and _fragment(s[1:]) == "ok":
            cls[i] |= TC_ESC
        if c == 0 and m == 0 and s.isascii() and s.isdigit():
            cls[i] |= TC_DIGITS
            ndig[i] = min(255, len(s))
            if s[0] == "0":
                cls[i] |= TC_ZERO_LEAD
    return cls, nch, ndig, utf, raw


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
        self.lit_first: list[int] = []
        self.literal_text: list[str] = []
        self.choices: list[list[Alt]] = []
        self.choice_limits: list[int] = []
        self.choice_min: list[int] = []
        self.n_nums = 0
        self.num_caps: list = []
        self._open_lit = False

    def enc(self, s: str) -> list[int]:
        return self.tok.encode(s)

    def single(self, s: str) -> int:
        ids = self.enc(s)
        if len(ids) != 1:
            raise ValueError(f"grammar needs {s!r} to be a single token, got {ids}")
        return ids[0]

    def maybe_single(self, s: str) -> int | None:
        ids = self.enc(s)
        return ids[0] if len(ids) == 1 else None

    def pc(self) -> int:
        return len(self.ops)

    def lit(self, text: str):
        if self._open_lit:                       # merge with the directly preceding literal
            i = self.ops[-1].a
            text = self.literal_text[i] + text
            self.literal_text[i] = text
            self.literals[i] = self.enc(text)
            self.literals_skip1[i] = self.enc(text[1:]) if len(text) > 1 else []
            return
        self.literal_text.append(text)
        self.literals.append(self.enc(text))
        self.literals_skip1.append(self.enc(text[1:]) if len(text) > 1 else [])
        self.lit_first.append(self.single(text[0]))
        self.ops.append(Op(OP_LIT, len(self.literals) - 1))
        self._open_lit = True

    def choice(self, limit: int = 0, honors_min: bool = False) -> int:
        """Emit a CHOICE whose alternatives are filled in later (`set_alts`)."""
        self._open_lit = False
        self.choices.append([])
        self.choice_limits.append(limit)
        self.choice_min.append(int(honors_min))
        self.ops.append(Op(OP_CHOICE, len(self.choices) - 1))
        return self.pc() - 1

    def set_alts(self, pc: int, alts: list[Alt]):
        self.choices[self.ops[pc].a][:] = [a for a in alts if a.first is not None]

    def op(self, code, a=0, b=0, c=0, d=0, e=0) -> int:
        self._open_lit = False
        self.ops.append(Op(code, a, b, c, d, e))
        return self.pc() - 1

    def num(self, kind: int, flags: int, caps) -> int:
        pc = self.op(OP_NUM, kind, caps[0][0], flags, caps[0][1], self.n_nums)
        self.num_caps.append(caps)
        self.n_nums += 1
        return pc


def compile_rfq_grammar(tok, limits: Limits | None = None) -> CompiledGrammar:
    """Compile the RFQResponse schema (field order = rfq_agent.py:41-59) for `tok`."""
    L = limits or Limits.from_env()
    P = _Prog(tok)
    quote = P.single('"')
    comma, rbrack, lbrace, lbrack = P.single(","), P.single("]"), P.single("{"), P.single("[")
    null_ids = P.enc("null")
    true_ids, false_ids = P.enc("true"), P.enc("false")
    # merged-token alternatives a real tokenizer prefers ('["', '[]', '[{'); absent ones drop out
    lbrack_q, empty_arr, lbrack_b = P.maybe_single('["'), P.maybe_single("[]"), P.maybe_single("[{")
    comma_q, comma_b = P.enc(' "'), P.enc(" {")
    NULL = lambda tgt, flags=0, cnt=CNT_NONE: Alt(null_ids[0], null_ids[1:], tgt, cnt, flags)

    def str_or_null(cap: int):
        """CHOICE(null | '"' STR) -> continues at the op after the STR."""
        c = P.choice()
        s = P.op(OP_STR, cap)
        P.set_alts(c, [NULL(s + 1), Alt(quote, [], s)])

    def str_array_body(cap: int, limit: int, after: int | None, patch: list):
        """[ "...", ... ] body: returns (open choice pc, element STR pc, next choice pc).
        `after` is the pc the closed array continues at (patched later when None)."""
        o = P.choice()
        s = P.op(OP_STR, cap)
        n = P.choice(limit=limit)
        patch.append((o, n, s))
        return o, s, n

    def close_arrays(patch, after):
        for o, n, s in patch:
            P.set_alts(o, [Alt(rbrack, [], after, CNT_RESET, ALT_CLOSE),
                           Alt(quote, [], s, CNT_SET1, ALT_CONTINUE)])
            P.set_alts(n, [Alt(rbrack, [], after, CNT_RESET, ALT_CLOSE),
                           Alt(comma, comma_q, s, CNT_INC, ALT_CONTINUE)])

    # ---- top level: 10 string fields (null | string | lenient: list of strings) --
    for i, f in enumerate(TOP_FIELDS):
        P.lit(("{" if i == 0 else ", ") + f'"{f}": ')
        cap = CAP_TITLE if f == "title" else (CAP_DESCRIPTION if f == "description" else CAP_FIELD)
        c = P.choice()
        patch: list = []
        o, s_arr, _ = str_array_body(CAP_ARRAY_STR, 0, None, patch)
        s = P.op(OP_STR, cap)
        after = P.pc()
        close_arrays(patch, after)
        P.set_alts(c, [NULL(after), Alt(quote, [], s),
                       Alt(lbrack, [], o, CNT_RESET, ALT_LENIENT),
                       Alt(lbrack_q, [], s_arr, CNT_SET1, ALT_LENIENT),
                       Alt(empty_arr, [], after, CNT_RESET, ALT_LENIENT)])

    # ---- line_items: [ {part_number, description, quantity, target_price[, currency]}, ... ]
    P.lit(', "line_items": ')
    entry = P.choice(honors_min=True)
    open_pc = P.choice(honors_min=True)
    body = P.pc()
    P.lit('"part_number": ')
    str_or_null(CAP_PART)
    P.lit(', "description": ')
    str_or_null(CAP_ITEM_DESC)
    P.lit(', "quantity": ')
    P.num(NUM_INT, NUM_NULLABLE | NUM_STR_OK, QTY_CAPS)
    P.op(OP_STR, CAP_NUMSTR)
    P.lit(', "target_price": ')
    P.num(NUM_DEC, NUM_NULLABLE | NUM_STR_OK, PRICE_CAPS)
    P.op(OP_STR, CAP_NUMSTR)
    cur_choice = P.choice()
    cur = P.pc()
    str_or_null(CAP_CURRENCY)
    P.lit("}")
    next_pc = P.choice(limit=L.max_items, honors_min=True)
    after_items = P.pc()
    P.set_alts(cur_choice, [Alt(comma, P.enc(' "currency": '), cur),
                            Alt(P.single("}"), [], next_pc, CNT_NONE, ALT_LENIENT)])
    P.set_alts(entry, [Alt(lbrack, [], open_pc),
                       Alt(empty_arr, [], after_items, CNT_RESET, ALT_CLOSE),
                       Alt(lbrack_b, [], body, CNT_SET1, ALT_CONTINUE),
                       NULL(after_items, ALT_CLOSE | ALT_LENIENT, CNT_RESET)])
    P.set_alts(open_pc, [Alt(rbrack, [], after_items, CNT_RESET, ALT_CLOSE),
                         Alt(lbrace, [], body, CNT_SET1, ALT_CONTINUE)])
    P.set_alts(next_pc, [Alt(rbrack, [], after_items, CNT_RESET, ALT_CLOSE),
                         Alt(comma, comma_b, body, CNT_INC, ALT_CONTINUE)])

    # ---- list fields: list of strings (lenient: null) ---------------------------
    def str_list(limit: int, cap: int, after_text: str):
        c = P.choice()
        patch: list = []
        o, s, _ = str_array_body(cap, limit, None, patch)
        after = P.pc()
        close_arrays(patch, after)
        P.set_alts(c, [Alt(lbrack, [], o), Alt(empty_arr, [], after, CNT_RESET),
                       Alt(lbrack_q, [], s, CNT_SET1),
                       NULL(after, ALT_LENIENT, CNT_RESET)])
        P.lit(after_text)

    P.lit(', "requested_documents": ')
    str_list(L.max_docs, CAP_DOC, ', "confidence_score": ')
    P.num(NUM_DEC, NUM_UNIT, CONF_CAPS)
    P.lit(', "missing_fields": ')
    str_list(L.max_missing, CAP_MISSING, ', "requires_review": ')
    rr = P.choice()
    P.set_alts(rr, [Alt(true_ids[0], true_ids[1:], rr + 1), Alt(false_ids[0], false_ids[1:], rr + 1)])
    P.lit("}")
    P.op(OP_END)

    ops = P.ops
    caps = np.zeros((NPROF, NCAP), np.int32)
    caps[PROFILE_SYNTHETIC] = L.caps()

    # ---- masks -------------------------------------------------------------
    cls, nch, ndig, utf, raw = token_table(tok)
    V = tok.vocab_size
    mb = _MaskBuilder(V)
    mb.ids([0])                                   # row 0: placeholder
    frag = (cls & (TC_STR | TC_STR_OPEN)) != 0
    lead_c, allc = utf & 3, (utf >> 4) & 1
    str_sub0 = frag & (lead_c == 0) & (allc == 0)
    str_sub0[quote] = True
    str_masks = [mb.add(str_sub0), mb.add((cls & TC_ESC) != 0)]
    for p in (1, 2, 3):
        str_masks.append(mb.add(((allc == 1) & (lead_c >= 1) & (lead_c <= p)) |
                                (frag & (allc == 0) & (lead_c == p))))
    cont = [i for i, b in enumerate(raw) if b == b"\x80"]
    if not cont:
        raise ValueError("tokenizer has no single continuation-byte token")
    digits = (cls & TC_DIGITS) != 0
    nz_digits = digits & ((cls & TC_ZERO_LEAD) == 0)
    zero_tok, dot_tok = P.single("0"), P.single(".")

    def allowed_alts(ci: int, prof: int) -> list[Alt]:
        return [a for a in P.choices[ci] if not (prof == PROFILE_SYNTHETIC and a.lenient)]

    def successor_firsts(pc: int, prof: int) -> list[int]:
        succ = pc + 1 + (1 if ops[pc].c & NUM_STR_OK else 0)
        o = ops[succ]
        if o.code == OP_LIT:
            return [P.lit_first[o.a]]
        if o.code == OP_CHOICE:
            return [a.first for a in allowed_alts(o.a, prof)]
        raise ValueError(f"NUM at pc={pc} must be followed by a literal or a choice")

    num_masks = np.full((P.n_nums, NPROF, NUM_PHASES), -1, np.int32)
    for pc, o in enumerate(ops):
        if o.code != OP_NUM:
            continue
        for prof in range(NPROF):
            ends = successor_firsts(pc, prof)
            a = nz_digits.copy()
            a[zero_tok] = True
            if o.c & NUM_NULLABLE:
                a[null_ids[0]] = True
            if o.c & NUM_STR_OK and prof == PROFILE_REFERENCE:
                a[quote] = True
            row = num_masks[o.e, prof]
            row[0] = mb.add(a)
            a = digits.copy()
            a[ends] = True
            if o.a == NUM_DEC:
                a[dot_tok] = True
            row[1] = mb.add(a)
            row[2] = mb.add(digits.copy())
            a = digits.copy()
            a[ends] = True
            row[3] = mb.add(a)
            a = np.zeros(V, bool)
            a[ends] = True
            if o.a == NUM_DEC:
                a[dot_tok] = True
            row[4] = mb.add(a)

    choice_masks = np.full((len(P.choices), 8), -1, np.int32)
    for ci, alts in enumerate(P.choices):
        if len({a.first for a in alts}) != len(alts):
            raise ValueError("ambiguous grammar choice (shared first token)")
        for combo in range(8):
            en = [a for a in alts if not ((combo & 1 and a.lenient) or (combo & 2 and a.is_continue)
                                          or (combo & 4 and a.is_close))]
            if en:
                choice_masks[ci, combo] = mb.ids([a.first for a in en])

    # ---- close-out costs ----------------------------------------------------
    g = CompiledGrammar(
        ops=ops, literals=P.literals, literals_skip1=P.literals_skip1, lit_first=P.lit_first,
        literal_text=P.literal_text, choices=P.choices, choice_masks=choice_masks,
        max_items=P.choice_limits, honors_min=P.choice_min, caps=caps, str_masks=tuple(str_masks),
        num_masks=num_masks, num_caps=np.array(P.num_caps, np.int32).reshape(-1, NPROF, 2),
        fin=np.zeros((len(ops), NPROF), np.int32),
        fin1=np.zeros((len(ops), NPROF), np.int32),
        close_alt=np.zeros((len(P.choices), NPROF), np.int32), slack=0,
        null_ids=null_ids, backslash=P.single("\\"), zero_token=zero_tok, dot_token=dot_tok,
        quote=quote, mask_rows=mb.table(), tok_class=cls, tok_chars=nch, tok_digits=ndig,
        tok_utf=utf, cont_token=cont[0], vocab_size=V, meta={"limits": L.__dict__})
    _close_tables(g)
    return g


def _close_tables(g: CompiledGrammar) -> None:
    """fin / fin1 / close_alt by fixpoint over the program (cycles go through array
    continue alternatives, never the cheapest), then K = the largest growth of the
    close-out cost one sampled token can cause (+ margin for forced continuations)."""
    ops, n = g.ops, len(g.ops)
    INF = 1 << 28
    for prof in range(NPROF):
        fin = [INF] * n
        fin1 = [INF] * n
        for _ in range(4 * n):
            changed = False
            for pc in range(n - 1, -1, -1):
                o = ops[pc]
                if o.code == OP_END:
                    v = v1 = 0
                elif o.code == OP_LIT:
                    v = len(g.literals[o.a]) + fin[pc + 1]
                    v1 = len(g.literals_skip1[o.a]) + fin[pc + 1]
                elif o.code == OP_JMP:
                    v = v1 = fin[o.a]
                elif o.code == OP_STR:
                    v = v1 = 1 + fin[pc + 1]
                elif o.code == OP_NUM:
                    succ = pc + 1 + (1 if o.c & NUM_STR_OK else 0)
                    v = v1 = (len(g.null_ids) if o.c & NUM_NULLABLE else 1) + fin[succ]
                else:  # CHOICE
                    best, bi = INF, 0
                    for i, a in enumerate(g.choices[o.a]):
                        if prof == PROFILE_SYNTHETIC and a.lenient:
                            continue
                        c = 1 + len(a.rest) + fin[a.target]
                        if c < best:
                            best, bi = c, i
                    v = v1 = best
                    g.close_alt[o.a, prof] = bi
                if v < fin[pc] or v1 < fin1[pc]:
                    fin[pc], fin1[pc] = min(fin[pc], v), min(fin1[pc], v1)
                    changed = True
            if not changed:
                break
        if max(fin) >= INF:
            raise ValueError("grammar has a state with no close-out path")
        g.fin[:, prof] = fin
        g.fin1[:, prof] = fin1
    grow = 0
    for ci, alts in enumerate(g.choices):
        for prof in range(NPROF):
            base = 1 + len(alts[g.close_alt[ci, prof]].rest) + \
                int(g.fin[alts[g.close_alt[ci, prof]].target, prof])
            for a in alts:
                grow = max(grow, 1 + len(a.rest) + int(g.fin[a.target, prof]) - base)
    lit_max = max(len(x) for x in g.literals)
    # one forced array continuation (min_items) can follow a sampled token's own growth
    g.slack = int(2 * grow + lit_max + 8)


def mask_table_int32(g: CompiledGrammar) -> np.ndarray:
    """The mask table as int32 (bit-identical) for torch upload."""
    return g.mask_rows.view(np.int32)


def describe(g: CompiledGrammar) -> str:
    return json.dumps({"ops": len(g.ops), "literals": len(g.literals), "choices": len(g.choices),
                       "masks": g.n_masks, "vocab": g.vocab_size, "slack": g.slack,
                       "max_close": int(g.fin.max())})
