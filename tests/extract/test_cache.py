"""Exact-request response cache (the reference's ag2 diskcache, cache_seed 42)
and the rfq_agent.py module-level convenience API."""
import asyncio

from replisense_rfq_amd.service.cache import CachedBackend, ResponseCache, request_key
from replisense_rfq_amd.service.extract import (ExtractService, MockBackend, RFQFieldGenerator,
                                                generate_rfq_fields_async)
from replisense_rfq_amd.service.prompt import build_messages


def test_cache_key_covers_request_fields():
    m = build_messages("RFQ for 10 bolts")
    k = request_key(m, "llama3-8b", 0.1, 1200)
    assert k == request_key(m, "llama3-8b", 0.1, 1200)
    assert k != request_key(m, "llama3-8b", 0.2, 1200)
    assert k != request_key(build_messages("RFQ for 11 bolts"), "llama3-8b", 0.1, 1200)


def test_cached_backend_hits_and_sqlite_persistence(tmp_path):
    path = str(tmp_path / "cache.sqlite")
    inner = MockBackend()
    svc = ExtractService(CachedBackend(inner, ResponseCache(path), "m", 0.1, 1200))
    a = svc.generate("Please quote 5 x PN-100 valves", "email-body")
    b = asyncio.run(svc.generate_async("Please quote 5 x PN-100 valves", "email-body"))
    assert len(inner.calls) == 1
    assert {k: v for k, v in a.items() if k != "source_file"} == \
        {k: v for k, v in b.items() if k != "source_file"}
    # a new process-level cache over the same file serves the stored completion
    inner2 = MockBackend()
    svc2 = ExtractService(CachedBackend(inner2, ResponseCache(path), "m", 0.1, 1200))
    svc2.generate("Please quote 5 x PN-100 valves", "email-body")
    assert len(inner2.calls) == 0


def test_lru_bound():
    c = ResponseCache(None, max_entries=2)
    for i in range(3):
        c.put(str(i), "v")
    assert c.get("0") is None and c.get("2") == "v"


def test_module_level_convenience(monkeypatch):
    monkeypatch.setenv("RFQ_BACKEND", "mock")
    assert RFQFieldGenerator is ExtractService
    out = asyncio.run(generate_rfq_fields_async("Need 4 x ABC-123 pumps", "email-body"))
    assert out["source_file"] == "email-body" and "confidence_score" in out
