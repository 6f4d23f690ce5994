"""Extraction prompt — byte-identical to the reference so prompts (and token counts)
match the recorded workload.

Reference: app/rfq_agent.py:75-105 (template), :114 (system message), :147-151
(8,000-char truncation and the triple-quoted user message).  The strings below are
verified against the user/system messages recorded in .cache/42/cache.db rows
11-13 by tests/extract/test_prompt_golden.py.
"""
from __future__ import annotations

SYSTEM_MESSAGE = ("You are an expert at extracting structured RFQ data from raw text. "
                  "Return valid JSON only with no additional text or explanations.")

_FIELDS = [
    ("title", "Document title or subject"),
    ("client_name", "Client/company name"),
    ("client_email", "Contact email address"),
    ("client_contact", "Contact person name"),
    ("client_phone", "Phone number"),
    ("rfq_to", "Who the RFQ is addressed to"),
    ("delivery_location", "Where items should be delivered"),
    ("delivery_deadline", "When delivery is needed"),
    ("response_due_date", "When response is due"),
    ("description", "Brief description of requirements"),
    ("line_items", "Array of objects with part_number, description, quantity, target_price "
                   "(numeric value only), currency (currency symbol or word as found in text)"),
    ("requested_documents", "Array of required document types"),
    ("confidence_score", "Float 0.0-1.0 indicating extraction confidence"),
    ("missing_fields", "Array of field names that couldn't be extracted"),
    ("requires_review", "Boolean indicating if human review is needed"),
]

_EXAMPLES = [
    ('"$100"', '"100"', '"$"'),
    ('"50 euros"', '"50"', '"euros"'),
    ('"75 GBP"', '"75"', '"GBP"'),
    ('"₹500"', '"500"', '"₹"'),
]


def _build_template() -> str:
    out = ["Extract the following fields from the RFQ text below and return ONLY valid JSON:",
           "Required fields:"]
    out += [f"- {k}: {v}" for k, v in _FIELDS]
    out += ["", "IMPORTANT: For line_items, separate price and currency:",
            '- target_price: Extract only the numeric value (e.g., "100", "50.75", "1000")',
            "- currency: Extract currency as found in text - can be symbol ($, €, £, ₹) or word "
            "(dollars, euros, pounds, rupees) or code (USD, EUR, GBP, INR)",
            "- Examples:"]
    for i, (src, price, cur) in enumerate(_EXAMPLES):
        pad = "  " if i == 1 else ""   # the reference line carries two trailing spaces
        out.append(f"  * {src} → target_price: {price}, currency: {cur}{pad}")
    out.append('  * "25" (no currency) → target_price: "25", currency: null')
    out += ["", "Return only valid JSON. Do not include any explanatory text.",
            "Text to analyze:", ""]
    return "\n".join(out)


EXTRACTION_PROMPT_TEMPLATE = _build_template()

MAX_INPUT_CHARS = 8000
TRUNCATION_SUFFIX = "... [truncated]"


def truncate(raw_text: str) -> str:
    """rfq_agent.py:147-149 — cap the document at 8,000 chars."""
    if len(raw_text) > MAX_INPUT_CHARS:
        return raw_text[:MAX_INPUT_CHARS] + TRUNCATION_SUFFIX
    return raw_text


# Every user message starts with this (~84 % of its characters): the tokenizer
# encodes it once (Tokenizer.register_prefix) instead of per request.
USER_MESSAGE_PREFIX = f'{EXTRACTION_PROMPT_TEMPLATE}\n"""\n'


def register_prompt_prefix(tokenizer) -> None:
    tokenizer.register_prefix(USER_MESSAGE_PREFIX)


def build_user_message(raw_text: str) -> str:
    """rfq_agent.py:151 — template + triple-quoted (already truncated) document."""
    return f'{EXTRACTION_PROMPT_TEMPLATE}\n"""\n{raw_text}\n"""'


def build_messages(raw_text: str) -> list[dict]:
    return [{"role": "system", "content": SYSTEM_MESSAGE},
            {"role": "user", "content": build_user_message(truncate(raw_text))}]


def shared_prefix_ids(tokenizer) -> list[int]:
    """Token ids every extraction prompt starts with (system message + chat
    template + EXTRACTION_PROMPT_TEMPLATE up to the document): the longest common
    prefix of two prompts that differ only in their document."""
    a = tokenizer.chat_ids(build_messages("A"))
    b = tokenizer.chat_ids(build_messages("Z"))
    n = 0
    while n < min(len(a), len(b)) and a[n] == b[n]:
        n += 1
    return a[:n]
