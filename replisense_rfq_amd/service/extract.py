"""Extraction service — the reference's RFQFieldGenerator (app/rfq_agent.py:107-273)
re-built on the on-node engine.

Contract kept from the reference:
  * ``generate_async(raw_text, source_file="email-body")`` / ``generate(...)`` return
    the RFQResponse dict (field order rfq_agent.py:41-59) with
    ``source_file``/``success``/``message`` overwritten (rfq_agent.py:197-201);
  * empty text -> error dict (rfq_agent.py:142-144); text > 8,000 chars truncated
    (rfq_agent.py:147-149); prompt bytes identical (rfq_agent.py:151,114);
  * JSON recovery: direct parse -> greedy ``{...}`` -> strip ```json fences
    (rfq_agent.py:208-236);
  * schema violations -> fallback dict with raw values, ``requires_review=True``,
    confidence >= 0.3 (rfq_agent.py:249-267);
  * any exception inside generation -> error dict, HTTP 200 (rfq_agent.py:178-182);
  * retry: 3 attempts, exponential backoff 4-10 s, re-raise (rfq_agent.py:121-125) —
    implemented without tenacity (not available offline).

What changed: no GROQ_API_KEY, no thread per request — the async path awaits the
engine's future directly; a ``Backend`` protocol selects the on-node engine, a
deterministic mock (BASELINE config 1), or a replay of the reference's recorded
completions (.cache/42/cache.db rows, via tests/assets/golden/cache_rows.json).
"""
from __future__ import annotations

import asyncio
import functools
import json
import logging
import re
import time
from typing import Any, Protocol

from pydantic import ValidationError

from ..utils.dotenv import load_dotenv
from .prompt import SYSTEM_MESSAGE, build_user_message, register_prompt_prefix, truncate

load_dotenv()                              # rfq_agent.py:13
from .schema import RFQResponse

log = logging.getLogger("replisense_rfq_amd.service.extract")


class Backend(Protocol):
    def complete(self, messages: list[dict]) -> str: ...

    async def acomplete(self, messages: list[dict]) -> str: ...


# --------------------------------------------------------------- retry policy
def async_retry(attempts: int = 3, multiplier: float = 1.0, wait_min: float = 4.0,
                wait_max: float = 10.0, sleep=asyncio.sleep):
    """tenacity's stop_after_attempt(3) + wait_exponential(1, 4, 10), reraise=True."""
    def deco(fn):
        @functools.wraps(fn)
        async def wrapper(*a, **kw):
            for i in range(attempts):
                try:
                    return await fn(*a, **kw)
                except Exception:
                    if i == attempts - 1:
                        raise
                    await sleep(min(wait_max, max(wait_min, multiplier * (2 ** (i + 1)))))
        return wrapper
    return deco


# ------------------------------------------------------------ post-processing
def extract_json_from_string(response_str: str) -> dict:
    """rfq_agent.py:208-236 — three recovery strategies."""
    try:
        return json.loads(response_str)
    except json.JSONDecodeError:
        pass
    m = re.search(r"\{.*\}", response_str, re.DOTALL)
    if m:
        try:
            return json.loads(m.group())
        except json.JSONDecodeError:
            pass
    cleaned = response_str.strip()
    if cleaned.startswith("```json"):
        cleaned = cleaned[7:]
    if cleaned.endswith("```"):
        cleaned = cleaned[:-3]
    try:
        return json.loads(cleaned.strip())
    except json.JSONDecodeError as e:
        raise ValueError(f"Unable to parse JSON from LLM response: {str(e)}")


def create_error_response(error_message: str) -> dict[str, Any]:
    """rfq_agent.py:238-247 (note: no `message` key)."""
    return {"success": False, "error": error_message, "confidence_score": 0.0,
            "requires_review": True, "missing_fields": ["all"], "source_file": "unknown"}


def create_fallback_response(raw_reply: dict, source_file: str, validation_error: str) -> dict:
    """rfq_agent.py:249-267: copy known keys WITHOUT validation, flag for review."""
    fb = RFQResponse()
    for name, value in raw_reply.items():
        if name in RFQResponse.model_fields:
            try:
                setattr(fb, name, value)
            except Exception:
                continue
    fb.source_file = source_file
    fb.success = True
    fb.message = f"RFQ processed with validation warnings: {validation_error}"
    fb.requires_review = True
    try:
        fb.confidence_score = max(0.3, fb.confidence_score)
    except TypeError:
        fb.confidence_score = 0.3
    return fb.model_dump(warnings=False)


def parse_and_validate_response(reply: Any, source_file: str) -> dict[str, Any]:
    """rfq_agent.py:185-206."""
    if isinstance(reply, str):
        reply = extract_json_from_string(reply)
    if not isinstance(reply, dict):
        raise ValueError("LLM did not return a valid dictionary structure")
    try:
        v = RFQResponse(**reply)
        v.source_file = source_file
        v.success = True
        v.message = f"RFQ processed from {source_file}"
        return v.model_dump()
    except ValidationError as e:
        log.warning("Validation failed, using fallback: %s", e)
        return create_fallback_response(reply, source_file, str(e))


def build_messages(raw_text: str) -> list[dict]:
    return [{"role": "system", "content": SYSTEM_MESSAGE},
            {"role": "user", "content": build_user_message(truncate(raw_text))}]


# The reference's LLM client raises openai.APITimeoutError("Request timed out.") when
# its 30 s timeout (rfq_agent.py:69) expires, and _generate_sync puts str(e) into the
# error dict (rfq_agent.py:178-182).  Here the engine's deadline surfaces as
# asyncio.TimeoutError / TimeoutError, whose str() is empty: map it to the client's
# message so data.error is never blank.
TIMEOUT_MESSAGE = "Request timed out."


def error_text(e: BaseException) -> str:
    """str(e) as the reference reports it, never empty."""
    import asyncio

    if isinstance(e, (TimeoutError, asyncio.TimeoutError)):
        return str(e) or TIMEOUT_MESSAGE
    return str(e) or type(e).__name__


# ------------------------------------------------------------------- service
class ExtractService:
    """Drop-in for RFQFieldGenerator with a pluggable inference backend."""

    def __init__(self, backend: Backend):
        self.backend = backend
        self.last_latency_s: float | None = None
        log.info("RFQ Field Generator initialized successfully")

    @property
    def healthy(self) -> bool:
        """False when the engine behind the backend is stalled or has no live replica."""
        b = self.backend
        while hasattr(b, "inner"):           # unwrap CachedBackend
            if not getattr(b, "healthy", True):
                return False
            b = b.inner
        return bool(getattr(b, "healthy", True))

    def _prepare(self, raw_text: str):
        if not raw_text or not raw_text.strip():
            log.warning("Empty raw text provided")
            return None
        if len(raw_text) > 8000:
            log.warning("Text truncated to 8000 characters for processing")
        return build_messages(raw_text)

    def _finish(self, reply: Any, source_file: str, t0: float) -> dict:
        self.last_latency_s = time.perf_counter() - t0
        log.info("LLM response received in %.2fs", self.last_latency_s)
        out = parse_and_validate_response(reply, source_file)
        log.info("Successfully parsed RFQ fields with confidence: %s",
                 out.get("confidence_score", 0.0))
        return out

    def _generate_sync(self, raw_text: str, source_file: str) -> dict:
        msgs = self._prepare(raw_text)
        if msgs is None:
            return create_error_response("Empty or invalid input text")
        try:
            t0 = time.perf_counter()
            reply = self.backend.complete(msgs)
            return self._finish(reply, source_file, t0)
        except Exception as e:
            log.error("Exception during generation: %s", e)
            return create_error_response(error_text(e))

    def generate(self, raw_text: str, source_file: str = "email-body") -> dict:
        return self._generate_sync(raw_text, source_file)

    @async_retry()
    async def generate_async(self, raw_text: str, source_file: str = "email-body") -> dict:
        msgs = self._prepare(raw_text)
        if msgs is None:
            return create_error_response("Empty or invalid input text")
        try:
            t0 = time.perf_counter()
            reply = await self.backend.acomplete(msgs)
            return self._finish(reply, source_file, t0)
        except Exception as e:
            log.error("Exception during generation: %s", e)
            return create_error_response(error_text(e))


# ------------------------------------------------------------------ backends
class MockBackend:
    """Deterministic canned completion (BASELINE config 1: CPU plumbing, no GPU)."""

    def __init__(self, reply: str | None = None):
        self.reply = reply or json.dumps({
            "title": "Request for Quotation", "client_name": None, "client_email": None,
            "client_contact": None, "client_phone": None, "rfq_to": None,
            "delivery_location": None, "delivery_deadline": None, "response_due_date": None,
            "description": None, "line_items": [], "requested_documents": [],
            "confidence_score": 0.5, "missing_fields": [], "requires_review": True})
        self.calls: list[list[dict]] = []

    def complete(self, messages):
        self.calls.append(messages)
        return self.reply

    async def acomplete(self, messages):
        return self.complete(messages)


class ReplayBackend:
    """Serves the reference's recorded Groq completions for byte-identical prompts
    (the de-facto record/replay fixture of the reference)."""

    def __init__(self, rows: list[dict], fallback: Backend | None = None):
        self.table = {(r["system"], r["user"]): r["completion"] for r in rows
                      if r.get("system") and r.get("user")}
        self.fallback = fallback

    def complete(self, messages):
        key = (messages[0]["content"], messages[1]["content"])
        if key in self.table:
            return self.table[key]
        if self.fallback is None:
            raise KeyError("no recorded completion for this prompt")
        return self.fallback.complete(messages)

    async def acomplete(self, messages):
        key = (messages[0]["content"], messages[1]["content"])
        if key in self.table or self.fallback is None:
            return self.complete(messages)
        return await self.fallback.acomplete(messages)


def document_of(messages: list[dict]) -> str:
    """The (truncated) document embedded in the user message (rfq_agent.py:151)."""
    u = messages[-1]["content"]
    i = u.find('\n"""\n')
    return u[i + 5:-4] if i >= 0 and u.endswith('\n"""') else u


class EngineBackend:
    """On-node engine backend: chat template -> tokens -> AsyncEngine -> text.

    Requests decode with the grammar's REFERENCE profile (everything the
    reference's model emits, bounded only by max_tokens).  ``RFQ_DECODE_HINTS=1``
    switches to the bench-only hints of service/hints.py (random-init weights).
    """

    def __init__(self, engine, async_engine=None, timeout_s: float | None = None):
        self.engine = engine
        self.tokenizer = engine.tokenizer
        register_prompt_prefix(self.tokenizer)
        self.async_engine = async_engine
        self.timeout_s = timeout_s if timeout_s is not None else engine.cfg.request_timeout_s
        self.spans: list[dict] = []

    @property
    def healthy(self) -> bool:
        return self.async_engine is None or self.async_engine.healthy

    def _text(self, seq) -> str:
        if seq.finish_reason in ("engine_error", "grammar_error"):
            raise RuntimeError(f"generation failed: {seq.finish_reason}")
        if self.engine.cfg.trace:
            self.spans.append(seq.span())
        return self.tokenizer.decode(seq.output_ids)

    def _params(self, messages):
        from .hints import decode_hints_for

        return self.engine.default_params(
            **decode_hints_for(document_of(messages), self.engine.cfg.decode_hints))

    def complete(self, messages):
        ids = self.tokenizer.chat_ids(messages)
        seq, = self.engine.generate([ids], self._params(messages))
        return self._text(seq)

    async def acomplete(self, messages):
        if self.async_engine is None:
            return self.complete(messages)
        ids = self.tokenizer.chat_ids(messages)
        seq = await self.async_engine.generate(ids, self._params(messages),
                                               timeout=self.timeout_s)
        return self._text(seq)


# --------------------------------------------------------- reference aliases
RFQFieldGenerator = ExtractService          # rfq_agent.py:107 name, same contract


def default_service() -> ExtractService:
    """The service the API builds (backend from RFQ_BACKEND, see api/main.py)."""
    from ..api.main import build_generator

    return build_generator()


async def generate_rfq_fields_async(raw_text: str, source_file: str = "email-body") -> dict:
    """rfq_agent.py:270-273 convenience: a fresh generator per call."""
    return await default_service().generate_async(raw_text, source_file)
