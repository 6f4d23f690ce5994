"""Engine logic on CPU (torch-oracle ops): block manager + prefix cache, scheduler
chunking / preemption, end-to-end constrained generation, determinism, async
front-end, runner packing."""
import asyncio
import json

import numpy as np
import pytest

from replisense_rfq_amd import runtime
from replisense_rfq_amd.engine.engine import AsyncEngine, LLMEngine
from replisense_rfq_amd.engine.runner import EXT_MAX
from replisense_rfq_amd.service.extract import EngineBackend, ExtractService
from replisense_rfq_amd.service.prompt import build_messages
from replisense_rfq_amd.service.schema import RFQResponse
from replisense_rfq_amd.utils import synth
from replisense_rfq_amd.utils.config import EngineConfig


@pytest.fixture(scope="module")
def engine():
    return LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4,
                                  max_batched_tokens=2048))


def _prompts(eng, n, base=0):
    return [eng.tokenizer.chat_ids(build_messages(synth.make_rfq(base + i).text)) for i in range(n)]


def test_block_manager_refcounts_and_lru():
    bm = runtime.load().BlockManager(8, 32)
    a = bm.allocate(3)
    assert a == [0, 1, 2] and bm.num_free == 5
    toks = np.arange(96, dtype=np.int32)
    h = bm.hash_blocks(toks, 32, 0)
    assert len(h) == 3 and len(set(h)) == 3
    for b, hh in zip(a, h):
        bm.register_block(b, hh)
    bm.release(a)                       # cached, evictable
    assert bm.num_free == 8 and bm.num_cached == 3
    hit = bm.match_prefix(h[:2])
    assert hit == [0, 1] and bm.refcount(0) == 1
    assert bm.allocate(7) is None       # only 6 available (2 pinned)
    got = bm.allocate(6)                # evicts cached block 2 (LRU)
    assert 2 in got and bm.evictions == 1
    # hash chain: same tokens, different prefix -> different hash
    h2 = bm.hash_blocks(toks[32:64], 32, 0)
    assert h2[0] != h[1]


def test_generation_valid_and_prefix_cache(engine):
    seqs = engine.generate(_prompts(engine, 3))
    for s in seqs:
        assert s.finish_reason == "stop"
        RFQResponse(**json.loads(engine.decode_text(s)))
        assert s.num_forced > s.num_sampled          # jump-forward did most of the work
    seqs2 = engine.generate(_prompts(engine, 2, base=50))
    assert all(s.prefix_hit_tokens >= 384 for s in seqs2)
    assert engine.kv.stats()["prefix_hits"] >= 2


def test_determinism_same_seed(engine):
    p = _prompts(engine, 1, base=7)
    a = engine.generate(p, seeds=[123])[0].output_ids
    b = engine.generate(p, seeds=[123])[0].output_ids
    assert a == b


def test_batching_invariance(engine):
    """A request's output does not depend on what it is batched with."""
    p = _prompts(engine, 3, base=20)
    solo = engine.generate([p[0]], seeds=[9])[0].output_ids
    batched = engine.generate(p, seeds=[9, 10, 11])[0].output_ids
    assert solo == batched


def test_min_items_hint(engine):
    p = _prompts(engine, 1, base=30)
    s, = engine.generate(p, engine.default_params(min_items=3))
    assert len(json.loads(engine.decode_text(s))["line_items"]) >= 3


def test_chunked_prefill_and_preemption():
    cfg = EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4, max_batched_tokens=96,
                       max_kv_blocks=60, prefix_cache=False)
    eng = LLMEngine(cfg)
    seqs = eng.generate(_prompts(eng, 4, base=40))
    for s in seqs:
        assert s.finish_reason == "stop", s.finish_reason
        RFQResponse(**json.loads(eng.decode_text(s)))
    assert eng.num_steps > 4 * (550 // 96)             # prompts were chunked
    assert eng.scheduler.num_preempted > 0              # 60 blocks cannot hold 4 sequences


def test_runner_sections(engine):
    """Decode rows and short extends go to the paged-decode section, long chunks to prefill."""
    from replisense_rfq_amd.engine.runner import H_NA, H_NB, H_TA
    from replisense_rfq_amd.engine.scheduler import StepPlan
    from replisense_rfq_amd.engine.sequence import SamplingParams, Sequence

    kv = engine.kv
    mk = lambda n, cached: Sequence(list(range(1, n + 1)), SamplingParams())  # noqa: E731
    a, b, c = mk(40, 39), mk(50, 45), mk(300, 0)
    a.num_cached, b.num_cached = 39, 45
    for s in (a, b, c):
        kv.grow(s, len(s.tokens))
    pk = engine.runner.pack(StepPlan(decode=[a], extend=[(b, 5), (c, 300)]))
    h = pk.header
    assert (h[H_NA], h[H_TA], h[H_NB]) == (2, 6, 1)
    assert 5 <= EXT_MAX < 300
    for s in (a, b, c):
        kv.free(s)


def test_async_engine_and_extract_service(engine):
    aeng = AsyncEngine(engine)
    svc = ExtractService(EngineBackend(engine, aeng))

    async def go():
        docs = [synth.make_rfq(60 + i).text for i in range(3)]
        return await asyncio.gather(*(svc.generate_async(d, "mail") for d in docs))

    try:
        outs = asyncio.run(go())
    finally:
        aeng.shutdown()
    for o in outs:
        assert o["success"] is True and o["message"] == "RFQ processed from mail"
