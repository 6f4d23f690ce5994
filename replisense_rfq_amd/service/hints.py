"""Cheap document statistics used as decoding hints.

``estimate_line_items`` counts the distinct part-number-like tokens a document
mentions (mixed letters+digits such as ``62GB-56T-16-8S``, ``ACX-4015-03``,
``D38999/20WB35PN``).  It is a *bench-only* hint: with random-init weights the
benchmark passes it to the grammar as ``min_items`` so a constrained decode emits
one ``line_items`` object per requested part -- what a trained extraction model
does and what the reference's recorded completions show (cache.db rows 11-14: 4,
4, 3 and 23 items).  Under the SYNTHETIC profile the item count is then exact
(min_items = max), capped at the profile's item limit.  The service path applies it only with ``RFQ_DECODE_HINTS=1``
(load tests on random weights).  Emails and phone numbers are excluded; the count
is clamped to the SYNTHETIC profile's item limit.
"""
from __future__ import annotations

import re

_PN = re.compile(r"(?<![\w@.])(?=[A-Za-z0-9/.-]*\d)(?=[A-Za-z0-9/.-]*[A-Za-z])"
                 r"[A-Za-z0-9][A-Za-z0-9/.-]{3,}[A-Za-z0-9](?![\w@])")
_SKIP = re.compile(r"@|https?://|www\.")
_NOT_PN = re.compile(r"^(\d+([.,/]\d+)?/?[a-z]{1,5}|\d+(st|nd|rd|th)|\d+(pcs|pc|mm|m|kg|ft|v|a|w|va|ohm|days?)|"
                     r"rfq-?\d+|iso\d*|v\d+(\.\d+)*|\d{1,2}-[a-z]{3}-\d{2,4}|[a-z]{3}-\d{4}|"
                     r"\d+(\.\d+)?[kmg]|m\d{1,2}|cat\d+[a-z]?|nema\d+|ip\d{2}|usb-?c|din\d+|"
                     r"\d+x\d+(mm)?|rs-?\d+|pg\d+)$", re.I)


def decode_hints_for(document: str, enabled: bool) -> dict:
    """SamplingParams keywords of the bench-only decoding hints (``RFQ_DECODE_HINTS``):
    the grammar's SYNTHETIC profile and ``min_items`` from the document.  Empty when
    disabled -- the service decodes with the REFERENCE profile and no item floor."""
    if not enabled:
        return {}
    from ..engine.grammar import PROFILE_SYNTHETIC

    return {"min_items": estimate_line_items(document), "profile": PROFILE_SYNTHETIC}


def synthetic_item_limit() -> int:
    """The SYNTHETIC profile's line-item cap (engine/grammar/compiler.py Limits)."""
    from ..engine.grammar import Limits

    return Limits.from_env().max_items


def estimate_line_items(text: str, limit: int = 8) -> int:
    seen = []
    for line in text.splitlines():
        if _SKIP.search(line):
            continue
        for m in _PN.finditer(line):
            tok = m.group(0).strip(".-/")
            if _NOT_PN.match(tok) or tok.replace("-", "").replace("/", "").isdigit():
                continue
            if tok.lower() not in seen:
                seen.append(tok.lower())
            break                      # one part per line
    return min(limit, len(seen))
