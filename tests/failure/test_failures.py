"""Failure detection and recovery paths, driven by the
RFQ_FAULT injector on the CPU engine: a step that raises fails exactly the
in-flight requests and frees their KV blocks; a stalled step trips the
watchdog (/health -> unhealthy); a crashed DP replica fails its requests and is
restarted."""
import asyncio
import json

import pytest

from replisense_rfq_amd.engine.engine import AsyncEngine, LLMEngine
from replisense_rfq_amd.service.extract import EngineBackend, ExtractService
from replisense_rfq_amd.service.prompt import build_messages
from replisense_rfq_amd.service.schema import RFQResponse
from replisense_rfq_amd.utils import synth
from replisense_rfq_amd.utils.config import EngineConfig
from replisense_rfq_amd.utils.faults import FaultInjector


def _cfg(**kw):
    base = dict(model="tiny-llama", device="cpu", max_num_seqs=4, max_batched_tokens=2048,
                decode_hints=True)
    base.update(kw)
    return EngineConfig(**base)


def _prompt(eng, i):
    return eng.tokenizer.chat_ids(build_messages(synth.make_rfq(i).text))


def test_fault_spec_parsing():
    f = FaultInjector("step_raise:3, step_sleep:1:20,replica_exit:5")
    assert f.active and f.replica_exit_after() == 5
    f.on_step(0)
    with pytest.raises(RuntimeError):
        f.on_step(3)
    f.on_step(3)                          # one-shot
    assert not FaultInjector("").active


def test_step_fault_fails_inflight_and_frees_kv():
    eng = LLMEngine(_cfg())
    free0 = eng.kv.stats()["free"]
    eng.faults = FaultInjector("step_raise:2")
    aeng = AsyncEngine(eng)

    async def run():
        return await asyncio.gather(*[aeng.generate(_prompt(eng, i), timeout=120)
                                      for i in range(2)])

    seqs = asyncio.run(run())
    assert all(s.finish_reason == "engine_error" for s in seqs)
    assert aeng.error is not None
    assert eng.kv.stats()["free"] == free0 and not eng.has_work()
    # the engine keeps serving after the failure
    s, = asyncio.run(asyncio.wait_for(aeng.generate(_prompt(eng, 7)), 120)),
    assert s.finish_reason == "stop"
    RFQResponse(**json.loads(eng.decode_text(s)))
    # ExtractService maps an engine_error to the reference's retry-then-500 path
    svc = ExtractService(EngineBackend(eng, aeng))
    assert svc.healthy
    aeng.shutdown()


def test_nonfinite_logits_fail_the_step():
    """RFQ_CHECK_FINITE: a NaN in the lm_head makes the step's logits
    non-finite; the runner's device-side count fails exactly that step's requests
    (engine_error), and the engine serves again once the weights are repaired."""
    eng = LLMEngine(_cfg(check_finite=True))
    assert eng.runner.check_finite
    lm = eng.model.w["lm_head"]
    saved = lm[5].clone()
    lm[5, 3] = float("nan")
    aeng = AsyncEngine(eng)
    s = asyncio.run(asyncio.wait_for(aeng.generate(_prompt(eng, 1), timeout=120), 120))
    assert s.finish_reason == "engine_error"
    assert "non-finite logits" in str(aeng.error)
    lm[5].copy_(saved)
    s = asyncio.run(asyncio.wait_for(aeng.generate(_prompt(eng, 2)), 120))
    assert s.finish_reason == "stop"
    aeng.shutdown()


def test_watchdog_marks_stalled_engine_unhealthy():
    eng = LLMEngine(_cfg(step_timeout_s=0.2))
    # the next step (start-up prefix warm-up steps already counted)
    eng.faults = FaultInjector(f"step_sleep:{eng.num_steps}:1500")
    aeng = AsyncEngine(eng)
    s = asyncio.run(asyncio.wait_for(aeng.generate(_prompt(eng, 3)), 120))
    assert s.finish_reason == "stop"
    assert aeng.stalled and not aeng.healthy
    assert not ExtractService(EngineBackend(eng, aeng)).healthy
    aeng.shutdown()


@pytest.mark.slow
def test_router_replica_crash_is_restarted(monkeypatch):
    from replisense_rfq_amd.engine.router import DPRouter

    monkeypatch.setenv("RFQ_FAULT", "replica_exit:1")
    cfg = _cfg(max_num_seqs=2)
    router = DPRouter(cfg, 1)
    try:
        eng_tok = router.backend().tokenizer
        ids = eng_tok.chat_ids(build_messages(synth.make_rfq(1).text))
        params = dict(temperature=0.1, max_tokens=1200, grammar=True, min_items=0, profile=1)
        out = asyncio.run(router.generate(ids, params, timeout=300))
        assert out["finish"] == "stop"
        RFQResponse(**json.loads(out["text"]))
        # the replica exits after serving one request; the router restarts it
        import time

        deadline = time.time() + 300
        while router.restarts == 0 and time.time() < deadline:
            time.sleep(0.2)
        assert router.restarts >= 1
        while not router.healthy and time.time() < deadline:
            time.sleep(0.2)
        assert router.healthy
    finally:
        router.shutdown()


def test_request_deadline_aborts_and_frees_kv():
    """A request whose deadline expires is retired inside the engine (finish reason
    'timeout', KV released) instead of running to completion in the background."""
    eng = LLMEngine(_cfg())
    free0 = eng.kv.stats()["free"]
    eng.faults = FaultInjector("step_sleep:1:300,step_sleep:2:300,step_sleep:3:300")
    aeng = AsyncEngine(eng)

    async def run():
        return await aeng.generate(_prompt(eng, 11), timeout=0.5)

    with pytest.raises(asyncio.TimeoutError):
        asyncio.run(run())
    import time

    t0 = time.time()
    while eng.has_work() and time.time() - t0 < 30:
        time.sleep(0.05)
    assert not eng.has_work()
    assert eng.kv.stats()["free"] == free0
    aeng.shutdown()


@pytest.mark.slow
def test_router_custom_allreduce_error_restarts_on_rccl(monkeypatch):
    """a custom all-reduce flag timeout on TP rank 0 (simulated by
    the car_error fault, which fires only while the custom all-reduce is configured)
    fails that replica's requests, the rank-0 worker exits, and the router restarts
    the whole TP group with custom_allreduce=False -- which then serves."""
    from replisense_rfq_amd.engine.router import DPRouter

    monkeypatch.setenv("RFQ_FAULT", "car_error:8")
    cfg = _cfg(model="tiny-llama-tp", tp=2, max_num_seqs=2, custom_allreduce=True)
    router = DPRouter(cfg, 1, 2)
    try:
        tok = router.backend().tokenizer
        ids = tok.chat_ids(build_messages(synth.make_rfq(1).text))
        params = dict(temperature=0.1, max_tokens=1200, grammar=True, min_items=0, profile=1)
        import time

        try:
            out = asyncio.run(router.generate(ids, params, timeout=300))
            assert out["finish"] == "engine_error", out
        except RuntimeError as e:            # the replica died before replying
            assert "replica died" in str(e)
        deadline = time.time() + 300
        while router.restarts == 0 and time.time() < deadline:
            time.sleep(0.2)
        assert router.restarts >= 1
        assert router._cfg_dict["custom_allreduce"] is False
        while not router.healthy and time.time() < deadline:
            time.sleep(0.2)
        out = asyncio.run(router.generate(ids, params, timeout=300))
        assert out["finish"] == "stop"
        RFQResponse(**json.loads(out["text"]))
        assert router.restarts == 1
    finally:
        router.shutdown()


def test_timed_out_request_reports_a_nonempty_error():
    """the reference's 30 s LLM timeout (rfq_agent.py:69) surfaces as
    openai's APITimeoutError("Request timed out.") inside the error dict
    (rfq_agent.py:178-182).  The engine's deadline raises asyncio.TimeoutError, whose
    str() is empty; the service must still report a non-empty error."""
    from replisense_rfq_amd.service.extract import TIMEOUT_MESSAGE, error_text

    eng = LLMEngine(_cfg())
    eng.faults = FaultInjector(",".join(f"step_sleep:{eng.num_steps + i}:300" for i in range(4)))
    aeng = AsyncEngine(eng)
    svc = ExtractService(EngineBackend(eng, aeng, timeout_s=0.5))
    out = asyncio.run(svc.generate_async(synth.make_rfq(12).text, "email-body"))
    assert out["success"] is False and out["error"] == TIMEOUT_MESSAGE
    assert out["missing_fields"] == ["all"] and out["source_file"] == "unknown"
    assert error_text(asyncio.TimeoutError()) == TIMEOUT_MESSAGE
    assert error_text(ValueError("bad")) == "bad"
    aeng.shutdown()
