"""Data-parallel router: one engine replica per GPU (or TP group) in its own process.

SURVEY.md §2.3 DP row: whole-node docs/s with Llama-3-8B TP=1 = 8 independent
replicas behind a router.  Each worker process is pinned to its devices through
``HIP_VISIBLE_DEVICES`` *before* torch initialises HIP (spawned, never forked
from a GPU-initialised parent), builds an ``LLMEngine`` and serves requests from
a multiprocessing queue; the API process keeps one dispatcher thread that
resolves asyncio futures.  Routing is least-outstanding-tokens.  If a worker
dies, its in-flight requests fail (-> HTTP 500 "RFQ processing failed", the
reference semantics for exceptions escaping the generator) and the replica is
restarted.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time

log = logging.getLogger("replisense_rfq_amd.router")


def _worker(idx: int, devices: str, cfg_dict: dict, inq, outq):
    if devices:
        os.environ["HIP_VISIBLE_DEVICES"] = devices
    from ..utils.config import EngineConfig
    from ..utils.faults import FaultInjector
    from .engine import LLMEngine
    from .sequence import SamplingParams

    cfg = EngineConfig(**cfg_dict)
    eng = LLMEngine(cfg)
    exit_after = FaultInjector().replica_exit_after()
    outq.put(("ready", idx, None))
    pending = {}
    served = 0
    while True:
        try:
            while True:
                msg = inq.get_nowait() if eng.has_work() else inq.get(timeout=0.05)
                if msg is None:
                    return
                if msg[0] == "abort":               # the client's deadline expired
                    for sid, (r, s) in list(pending.items()):
                        if r == msg[1]:
                            eng.abort_request(s, "timeout")
                            pending.pop(sid, None)
                    continue
                rid, prompt, p = msg
                seq = eng.add_request(prompt, SamplingParams(**p))
                pending[seq.req_id] = (rid, seq)
        except queue.Empty:
            pass
        if not eng.has_work():
            continue
        try:
            finished = eng.step()
        except Exception:                      # fail this replica's in-flight work
            log.exception("replica %d step failed", idx)
            finished = eng.abort_all("engine_error")
        for s in finished:
            rid, _ = pending.pop(s.req_id, (None, None))
            if rid is not None:
                outq.put(("done", rid, {"text": eng.decode_text(s), "finish": s.finish_reason,
                                        "span": s.span()}))
                served += 1
        if exit_after is not None and served >= exit_after:
            outq.close()                       # flush what was served, then crash
            outq.join_thread()
            os._exit(3)                        # injected replica crash


class DPRouter:
    def __init__(self, cfg, n_replicas: int, devices_per_replica: int = 1,
                 restart: bool = True):
        self.cfg = cfg
        self.n = n_replicas
        self.dpr = devices_per_replica
        self.restart = restart
        self.ctx = mp.get_context("spawn")
        self.outq = self.ctx.Queue()
        self.inqs = [None] * n_replicas
        self.procs = [None] * n_replicas
        self.ready = [False] * n_replicas
        self.load = [0] * n_replicas
        self.where: dict[int, int] = {}
        self.futures: dict[int, tuple] = {}
        self._ids = itertools.count()
        self.completed = 0
        self.restarts = 0
        self._lock = threading.Lock()
        self._cfg_dict = dict(cfg.to_dict())
        self._cfg_dict["dp"] = 1
        for i in range(n_replicas):
            self._spawn(i)
        deadline = time.time() + 1800
        while not all(self.ready) and time.time() < deadline:
            kind, idx, _ = self.outq.get(timeout=1800)
            if kind == "ready":
                self.ready[idx] = True
        self._stop = False
        self._thread = threading.Thread(target=self._dispatch, daemon=True)
        self._thread.start()

    def _spawn(self, i: int) -> None:
        devs = ",".join(str(i * self.dpr + j) for j in range(self.dpr)) \
            if self.cfg.device != "cpu" else ""
        q = self.ctx.Queue()
        p = self.ctx.Process(target=_worker, args=(i, devs, self._cfg_dict, q, self.outq),
                             daemon=True)
        p.start()
        self.inqs[i], self.procs[i], self.ready[i] = q, p, False

    def _dispatch(self):
        while not self._stop:
            try:
                kind, rid, payload = self.outq.get(timeout=0.1)
            except queue.Empty:
                self._check_workers()
                continue
            if kind == "ready":
                self.ready[rid] = True             # (rid is the replica index here)
                log.info("replica %d ready", rid)
                continue
            with self._lock:
                loop, fut, cost = self.futures.pop(rid, (None, None, 0))
                r = self.where.pop(rid, None)
                if r is not None:
                    self.load[r] -= cost
                self.completed += 1
            if fut is not None:
                loop.call_soon_threadsafe(lambda f=fut, p=payload: f.done() or f.set_result(p))
            self._check_workers()

    def _check_workers(self):
        for i, p in enumerate(self.procs):
            if p is None or p.is_alive() or self._stop:
                continue
            log.error("replica %d died (exit %s); failing its requests", i, p.exitcode)
            with self._lock:
                self.ready[i] = False
                dead = [rid for rid, r in self.where.items() if r == i]
                for rid in dead:
                    loop, fut, _ = self.futures.pop(rid)
                    self.where.pop(rid)
                    loop.call_soon_threadsafe(
                        lambda f=fut: f.done() or f.set_exception(RuntimeError("replica died")))
                self.load[i] = 0
                if self.restart:
                    self.restarts += 1
                    self._spawn(i)
                else:
                    self.procs[i] = None

    @property
    def healthy(self) -> bool:
        return any(self.ready)

    async def generate(self, prompt: list[int], params: dict, timeout: float | None = None):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        cost = len(prompt) + params.get("max_tokens", 1200) // 4
        with self._lock:
            live = [i for i in range(self.n) if self.ready[i]]
            if not live:
                raise RuntimeError("no live engine replica")
            rid = next(self._ids)
            r = min(live, key=lambda i: self.load[i])
            self.load[r] += cost
            self.where[rid] = r
            self.futures[rid] = (loop, fut, cost)
        self.inqs[r].put((rid, prompt, params))
        if not timeout:
            return await fut
        try:
            return await asyncio.wait_for(asyncio.shield(fut), timeout)
        except asyncio.TimeoutError:
            with self._lock:
                _, _, cost = self.futures.pop(rid, (None, None, 0))
                if self.where.pop(rid, None) is not None:
                    self.load[r] -= cost
            self.inqs[r].put(("abort", rid))
            raise

    def backend(self):
        return RouterBackend(self)

    def stats(self) -> dict:
        return {"replicas": self.n, "ready": sum(self.ready), "restarts": self.restarts,
                "outstanding": len(self.where), "load": list(self.load),
                "completed": self.completed}

    def shutdown(self):
        self._stop = True
        for q, p in zip(self.inqs, self.procs):
            if p is not None and p.is_alive():
                q.put(None)
        for p in self.procs:
            if p is not None:
                p.join(timeout=10)


class RouterBackend:
    """ExtractService backend over the DP router."""

    def __init__(self, router: DPRouter):
        self.router = router
        from .tokenizer import flavor_for_vocab, get_tokenizer
        from ..models.config import get_config

        self.tokenizer = get_tokenizer(flavor_for_vocab(get_config(router.cfg.model).vocab_size))
        from ..service.prompt import register_prompt_prefix

        register_prompt_prefix(self.tokenizer)

    @property
    def healthy(self) -> bool:
        return self.router.healthy

    def complete(self, messages):
        return asyncio.run(self.acomplete(messages))

    async def acomplete(self, messages):
        from ..service.extract import document_of
        from ..service.hints import decode_hints_for

        ids = self.tokenizer.chat_ids(messages)
        cfg = self.router.cfg
        params = dict(temperature=cfg.temperature, max_tokens=cfg.max_tokens, grammar=cfg.grammar,
                      **decode_hints_for(document_of(messages), cfg.decode_hints))
        out = await self.router.generate(ids, params, timeout=cfg.request_timeout_s)
        if out["finish"] in ("engine_error", "grammar_error"):
            raise RuntimeError(f"generation failed: {out['finish']}")
        return out["text"]


def maybe_router(cfg):
    """A DPRouter when RFQ_DP > 1 (replicas of cfg.tp devices each) or when the
    single engine should live in its own process (RFQ_ENGINE_PROCESS=1: the API
    process then only parses HTTP, tokenises and validates), else None."""
    own_process = os.environ.get("RFQ_ENGINE_PROCESS", "0").lower() in ("1", "true", "on")
    if cfg.dp <= 1 and not own_process:
        return None
    return DPRouter(cfg, max(1, cfg.dp), max(1, cfg.tp))
