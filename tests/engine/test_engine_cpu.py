"""Engine logic on CPU (torch-oracle ops): block manager + prefix cache, scheduler
chunking / preemption, end-to-end constrained generation, determinism, async
front-end, runner packing."""
import asyncio
import json
import time

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
                                  max_batched_tokens=2048, decode_hints=True))


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
                       max_kv_blocks=60, prefix_cache=False, decode_hints=True)
    eng = LLMEngine(cfg)
    seqs = eng.generate(_prompts(eng, 4, base=40))
    for s in seqs:
        assert s.finish_reason == "stop", s.finish_reason
        RFQResponse(**json.loads(eng.decode_text(s)))
    assert eng.num_steps > 4 * (550 // 96)             # prompts were chunked
    assert eng.stats()["preempted"] > 0                 # 60 blocks cannot hold 4 sequences
    assert eng.stats()["free"] == 59 and not eng.has_work()


def _core(**kw):
    conf = dict(block_size=32, num_blocks=64, scratch_block=64, max_num_seqs=8,
                max_batched_tokens=512, max_model_len=2048, ext_max=EXT_MAX, group=4, hkv=1,
                jump_forward=True, prefix_cache=True, is_cuda=False, use_graphs=False,
                eos_ids=[7])
    conf.update(kw)
    return runtime.load().EngineCore(conf, None)


def _views(header, payload):
    import torch

    from replisense_rfq_amd.engine.runner import ModelRunner

    return {k: v.numpy() for k, v in ModelRunner._views(torch.from_numpy(payload), header).items()}


def test_core_sections_and_layout():
    """Prefill chunks go to section B, decode rows and short extends to section A;
    the packed arrays follow runner._layout."""
    from replisense_rfq_amd.engine.runner import (H_NA, H_NB, H_PAYLOAD, H_S, H_T, H_TA,
                                                  HEADER, _seed64)

    core = _core()
    h = np.zeros(HEADER, np.int32)
    buf = np.zeros(core.payload_bound(), np.int32)
    a = core.add(np.arange(100, 400, dtype=np.int32), 0.5, 50, 11, False, 0, 0, 0.0)
    b = core.add(np.arange(1, 11, dtype=np.int32), 0.5, 50, 12, False, 0, 0, 0.0)
    n = core.schedule_and_pack(h, buf, 0.0)
    assert n == h[H_PAYLOAD] > 0
    assert (h[H_T], h[H_TA], h[H_NA], h[H_NB], h[H_S]) == (310, 10, 1, 1, 2)
    v = _views(h, buf[:n])
    assert list(v["ids"][:10]) == list(range(1, 11))          # short prompt: section A
    assert v["ids"][10] == 100 and v["pos"][309] == 299        # long prompt: section B
    assert list(v["lidx"]) == [9, 309]
    assert v["seeds"][0] == _seed64(12, 10) and v["seeds"][1] == _seed64(11, 300)
    assert abs(v["temps"][0] - 0.5) < 1e-7
    assert list(v["midx"]) == [-1, -1]
    # slots: contiguous pages starting at the blocks the core handed out
    assert v["slots"][0] == v["a_bt"][0, 0] * 32
    done = core.post(np.array([5, 6], np.int32), 1.0)
    assert done == []
    n = core.schedule_and_pack(h, buf, 1.0)                    # both decode now
    assert (h[H_T], h[H_NA], h[H_NB]) == (2, 2, 0)
    v = _views(h, buf[:n])
    assert sorted(v["ids"].tolist()) == [5, 6] and sorted(v["a_kvl"].tolist()) == [11, 301]
    done = core.post(np.array([7, 7], np.int32), 2.0)          # eos for both
    assert sorted(done) == sorted([a, b])
    assert core.info(a)["finish"] == 1 and core.tokens(a)[-2:].tolist() == [6, 7]
    assert core.tokens(b)[-2:].tolist() == [5, 7]
    assert not core.has_work
    for i in done:
        core.release(i)


def test_core_prefix_cache_and_preemption():
    core = _core(num_blocks=24, max_batched_tokens=4096)
    h = np.zeros(16, np.int32)
    buf = np.zeros(core.payload_bound(), np.int32)
    prompt = np.arange(1, 300, dtype=np.int32)
    a = core.add(prompt, 0.1, 600, 1, False, 0, 0, 0.0)
    core.schedule_and_pack(h, buf, 0.0)
    core.post(np.array([9], np.int32), 0.0)
    b = core.add(prompt, 0.1, 600, 2, False, 0, 0, 0.0)          # shares 9 full prompt blocks
    core.schedule_and_pack(h, buf, 0.0)
    core.post(np.array([9, 9], np.int32), 0.0)
    assert core.info(b)["prefix_hit"] == 9 * 32 and core.prefix_hits >= 1
    # run until the pool (24 blocks) forces a preemption
    steps = 0
    while core.has_work and steps < 2000:
        n = core.schedule_and_pack(h, buf, 0.0)
        done = core.post(np.full(h[6], 9, np.int32), 0.0) if n else core.drain_finished()
        for i in done:
            assert core.info(i)["finish"] == 2                 # length (pool-bound)
            core.release(i)
        steps += 1
    assert core.num_preempted > 0 and not core.has_work
    assert core.num_free_blocks == 24


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


def test_reference_profile_closes_inside_budget(engine):
    """The service default (REFERENCE profile, no hints): random weights never close
    a string by themselves, so the token-budget close-out must end every output as
    parseable JSON within max_tokens -- finish 'stop', never 'length'."""
    from replisense_rfq_amd.engine.grammar import PROFILE_REFERENCE
    from replisense_rfq_amd.service.extract import parse_and_validate_response

    p = _prompts(engine, 2, base=50)
    seqs = engine.generate(p, engine.default_params(profile=PROFILE_REFERENCE, max_tokens=300))
    for s in seqs:
        assert s.finish_reason == "stop" and len(s.output_ids) <= 300
        text = engine.decode_text(s)
        json.loads(text)
        assert parse_and_validate_response(text, "direct_text_input")["success"] is True


def test_shared_prefix_warm_and_pinned(engine):
    """the shared system + template prefix is prefilled at
    start-up and its blocks pinned; the first request already hits it."""
    from replisense_rfq_amd.service.prompt import shared_prefix_ids

    n = len(shared_prefix_ids(engine.tokenizer))
    assert engine.pinned_blocks == n // engine.kv.block_size > 0
    hits0 = engine.core.prefix_hits
    s, = engine.generate(_prompts(engine, 1, base=90))
    assert s.prefix_hit_tokens >= engine.pinned_blocks * engine.kv.block_size
    assert engine.core.prefix_hits > hits0
    assert engine.stats()["pinned_blocks"] == engine.pinned_blocks


def test_graph_key_latency_fallthrough():
    """Graph selection (engine_core.cpp graph_key): the first sequence bucket >= na
    with a token multiple >= t; in the latency regime (buckets <= 16) a step whose
    jump-forward extends outgrow that bucket moves up to the next bucket's padded
    graph instead of running eagerly; larger buckets never pad across buckets."""
    from replisense_rfq_amd.engine.runner import TOKEN_MULTS

    core = _core(token_mults=list(TOKEN_MULTS))
    buckets = (1, 2, 4, 8, 16, 32, 64)
    core.set_graph_keys(sorted((b, b * m) for b in buckets for m in TOKEN_MULTS))
    assert core.graph_key(1, 1) == (1, 1)
    assert core.graph_key(1, 7) == (1, 8)
    assert core.graph_key(1, 9) == (2, 12)        # was eager
    assert core.graph_key(1, 30) == (4, 32)
    assert core.graph_key(3, 20) == (4, 24)
    assert core.graph_key(3, 40) == (8, 48)
    assert core.graph_key(16, 200) == (32, 256)   # bucket 16 still falls through
    assert core.graph_key(17, 300) == (-1, -1)    # bucket 32: eager, no cross-bucket pad
    assert core.graph_key(64, 512) == (64, 512)
    assert core.graph_key(65, 65) == (-1, -1)     # beyond the captured buckets


def test_async_engine_admits_during_step_defers_aborts(engine):
    """AsyncEngine drains its inbox from runner.busy_hook while a step runs on the
    device: adds are applied there, aborts (which free KV blocks of sequences that may
    be in the running step) wait for the loop top, in order."""
    from replisense_rfq_amd.engine.engine import _Request

    aeng = AsyncEngine.__new__(AsyncEngine)          # no loop thread: drive _drain by hand
    aeng.engine = engine
    aeng._inbox = __import__("queue").Queue()
    aeng._held = []
    got = []
    req, req2 = _Request(), _Request()
    p = _prompts(engine, 2, base=70)
    aeng._inbox.put(("add", p[0], engine.default_params(max_tokens=8), got.append, req))
    aeng._inbox.put(("abort", req))
    aeng._inbox.put(("add", p[1], engine.default_params(max_tokens=8), got.append, req2))
    aeng._drain(in_step=True)
    assert req.seq is not None and req2.seq is not None     # both adds applied in-step
    assert [m[0] for m in aeng._held] == ["abort"]           # the abort was deferred
    aeng._drain()                                            # loop top: abort applied
    assert aeng._held == [] and req.seq.finish_reason == "timeout"
    assert got and got[0] is req.seq
    while engine.has_work():
        engine.step()
    assert req2.seq.finish_reason not in (None, "timeout")        # ran to its own end


def test_async_engine_hook_installed_and_removed(engine):
    aeng = AsyncEngine(engine)
    try:
        deadline = time.time() + 10
        while engine.runner.busy_hook is None and time.time() < deadline:
            time.sleep(0.01)
        assert engine.runner.busy_hook == aeng._in_step
        seq = asyncio.run(aeng.generate(_prompts(engine, 1, base=80)[0],
                                        engine.default_params(max_tokens=8)))
        assert seq.finish_reason not in (None, "timeout", "engine_error")
    finally:
        aeng.shutdown()
    assert engine.runner.busy_hook is None


def test_busy_hook_failure_raised_after_step_drains(engine):
    """A busy_hook that raises does not cut the step short: the runner reads the
    step's tokens back (no kernel left in flight) and then re-raises the hook's error;
    the next step runs normally."""
    calls = []

    def bad_hook():
        calls.append(engine.runner.stats["steps"])
        raise ValueError("hook failed")

    p = _prompts(engine, 1, base=90)
    seq = engine.add_request(p[0], engine.default_params(max_tokens=8), None)
    engine.runner.busy_hook = bad_hook
    try:
        with pytest.raises(ValueError, match="hook failed"):
            while engine.has_work():
                engine.step()
    finally:
        engine.runner.busy_hook = None
    assert calls and engine.runner.stats["wait_s"] >= 0.0
    engine.abort_request(seq, "test")
    while engine.has_work():
        engine.step()


def test_async_engine_survives_add_failing_in_step_and_at_loop_top(engine):
    """an add that raises inside the step hook is held and replayed
    at the loop top; when the replay raises too, only that request fails (its caller
    gets an engine_error Sequence) and the engine thread keeps serving the others."""
    aeng = AsyncEngine(engine)
    orig = engine.add_request
    bad = _prompts(engine, 1, base=110)[0]

    def flaky_add(prompt, params=None, callback=None):
        if list(prompt) == list(bad):
            raise RuntimeError("injected add failure")
        return orig(prompt, params, callback)

    engine.add_request = flaky_add
    try:
        async def run():
            good = _prompts(engine, 2, base=120)
            t1 = asyncio.ensure_future(aeng.generate(good[0], engine.default_params(max_tokens=8)))
            await asyncio.sleep(0.05)              # a step is (likely) running: in-step path
            tb = asyncio.ensure_future(aeng.generate(bad, engine.default_params(max_tokens=8),
                                                     timeout=30))
            t2 = asyncio.ensure_future(aeng.generate(good[1], engine.default_params(max_tokens=8),
                                                     timeout=30))
            return await asyncio.gather(t1, tb, t2)

        s1, sb, s2 = asyncio.run(run())
        assert sb.finish_reason == "engine_error"
        assert s1.finish_reason not in (None, "engine_error")
        assert s2.finish_reason not in (None, "engine_error")
        assert aeng.healthy and aeng._thread.is_alive()
        # a direct loop-top replay of a failing add also fails only that request
        from replisense_rfq_amd.engine.engine import _Request

        got, req = [], _Request()
        aeng._apply_or_fail(("add", bad, engine.default_params(max_tokens=8), got.append, req))
        assert got and got[0].finish_reason == "engine_error" and req.seq is got[0]
    finally:
        engine.add_request = orig
        aeng.shutdown()


def test_serve_loop_behind_attached_router_keeps_engine(engine):
    """The bench's two-process HTTP layout on one engine: serve_loop (engine side of the
    request queues) + a DPRouter attached to those queues (API side) serve requests
    through the extraction service; a None message ends the loop without shutting the
    engine down, which then still generates directly."""
    import queue
    import threading

    from replisense_rfq_amd.engine.router import DPRouter, serve_loop

    inq, outq = queue.Queue(), queue.Queue()
    th = threading.Thread(target=serve_loop, args=(engine, inq, outq),
                          kwargs={"shutdown_engine": False}, daemon=True)
    th.start()
    router = DPRouter(engine.cfg, 1, queues=(inq, outq))
    svc = ExtractService(router.backend())

    async def go():
        docs = [synth.make_rfq(90 + i).text for i in range(3)]
        return await asyncio.gather(*(svc.generate_async(d, "mail") for d in docs))

    try:
        outs = asyncio.run(go())
        assert router.stats()["completed"] == 3 and router.stats()["outstanding"] == 0
    finally:
        router._stop = True
        inq.put(None)
        th.join(timeout=30)
    assert not th.is_alive()
    for o in outs:
        assert o["success"] is True and o["message"] == "RFQ processed from mail"
    assert engine.runner.busy_hook is None
    seqs = engine.generate(_prompts(engine, 1, base=95))
    assert seqs[0].finish_reason in ("stop", "length", "grammar_done", "eos")
