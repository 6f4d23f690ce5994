"""Data-parallel router: engine replicas (each a TP group of processes) behind
one dispatcher.

SURVEY.md §2.3: whole-node docs/s with Llama-3-8B TP=1 = 8 independent replicas
(DP=8); Llama-3-70B = one replica of TP=8 over RCCL/xGMI (the reference's own
model, ``llama3-70b-8192``, rfq_agent.py:62).  ``RFQ_DP`` x ``RFQ_TP`` processes
are spawned (never forked from a GPU-initialised parent), one per GPU.  Every
process of replica r sees the replica's devices through ``HIP_VISIBLE_DEVICES``
(set before torch initialises HIP) and joins the replica's own process group
(``init_process_group``: RCCL on GPUs, gloo on CPU; 127.0.0.1 rendezvous on a
per-replica port).  TP rank 0 builds the ``LLMEngine`` scheduler and serves
requests from a multiprocessing queue; TP ranks > 0 mirror its steps
(``LLMEngine.worker_loop``, shared-memory control plane).  The API process keeps
one dispatcher thread that resolves asyncio futures.  Routing is
least-outstanding-tokens.  If any process of a replica dies, the replica's
in-flight requests fail (-> HTTP 500 "RFQ processing failed", the reference
semantics for exceptions escaping the generator) and the whole TP group is
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


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _join_group(devices: str, tp_rank: int, tp: int, port: int):
    """Pin this process to the replica's devices and (TP > 1) join the replica's
    process group.  Runs before anything touches HIP."""
    if devices:
        os.environ["HIP_VISIBLE_DEVICES"] = devices
        from ..utils.affinity import pin_to_gpu

        pin_to_gpu(tp_rank)       # NUMA-local cores of this process's device (GPU replicas)
    if tp <= 1:
        from ..parallel.tp import SINGLE

        return SINGLE
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(tp_rank),
                      WORLD_SIZE=str(tp), LOCAL_RANK=str(tp_rank))
    from ..parallel.tp import init_distributed

    return init_distributed()


def _follower(idx: int, devices: str, tp_rank: int, tp: int, port: int, cfg_dict: dict):
    """TP rank > 0 of replica `idx`: mirror rank 0's steps until it stops."""
    ctx = _join_group(devices, tp_rank, tp, port)
    from ..utils.config import EngineConfig
    from .engine import LLMEngine

    eng = LLMEngine(EngineConfig(**cfg_dict), tp=ctx)
    eng.worker_loop()


def _worker(idx: int, devices: str, cfg_dict: dict, inq, outq, tp: int = 1, port: int = 0):
    ctx = _join_group(devices, 0, tp, port)
    from ..utils.config import EngineConfig
    from ..utils.faults import FaultInjector
    from .engine import LLMEngine

    cfg = EngineConfig(**cfg_dict)
    eng = LLMEngine(cfg, tp=ctx)
    from .engine import short_gil_switch

    short_gil_switch()                         # the inbox feeder thread shares the GIL
    exit_after = FaultInjector().replica_exit_after()
    outq.put(("ready", idx, None))
    serve_loop(eng, inq, outq, idx, exit_after)


def serve_loop(eng, inq, outq, idx: int = 0, exit_after=None,
               shutdown_engine: bool = True) -> None:
    """The engine side of the request queues: admit (rid, prompt, params) messages
    (also while a step runs on the device), step, and answer ("done", rid, result).
    Runs a replica worker process's engine (``_worker``) or, with
    ``shutdown_engine=False``, an engine that outlives the loop (the bench's
    separate-process HTTP phase).  A ``None`` message ends the loop."""
    from ..utils.faults import CustomAllReduceError
    from .sequence import SamplingParams

    pending = {}
    served = 0
    held = []                                  # inbox messages deferred to the loop top

    def apply(msg) -> bool:                    # False: shut down
        if msg is None:
            return False
        if msg[0] == "abort":                  # the client's deadline expired
            for sid, (r, s) in list(pending.items()):
                if r == msg[1]:
                    eng.abort_request(s, "timeout")
                    pending.pop(sid, None)
            return True
        rid, prompt, p = msg
        seq = eng.add_request(prompt, SamplingParams(**p))
        pending[seq.req_id] = (rid, seq)
        return True

    def admit_in_step():
        """runner.busy_hook: admit new requests while the step runs on the device;
        aborts and shutdown (which touch sequences of the running step), and an add
        that raised, wait for the loop top."""
        try:
            while True:
                msg = inq.get_nowait()
                if msg is not None and msg[0] != "abort":
                    try:
                        apply(msg)
                        continue
                    except Exception:  # noqa: BLE001 - replayed (and raised) at the loop top
                        pass
                held.append(msg)
        except queue.Empty:
            pass

    eng.runner.busy_hook = admit_in_step
    while True:
        try:
            while True:
                if held:
                    msg = held.pop(0)
                else:
                    msg = inq.get_nowait() if eng.has_work() else inq.get(timeout=0.05)
                try:
                    alive = apply(msg)
                except Exception:  # noqa: BLE001 - fail only this request, keep serving
                    log.exception("replica %d: request could not be admitted", idx)
                    if msg is not None and msg[0] != "abort":
                        outq.put(("done", msg[0], {"text": "", "finish": "engine_error",
                                                   "span": {}}))
                    continue
                if not alive:
                    if shutdown_engine:
                        eng.shutdown()             # release the TP followers
                    eng.runner.busy_hook = None
                    return
        except queue.Empty:
            pass
        if not eng.has_work():
            continue
        fatal = False
        try:
            finished = eng.step()
        except CustomAllReduceError:
            # the custom all-reduce's flag protocol failed: this replica's sums can no
            # longer be trusted (the error counter is sticky).  Fail what it holds and
            # exit, so _check_workers restarts the TP group on RCCL all-reduces.
            log.exception("replica %d: custom all-reduce failure, restarting on RCCL", idx)
            finished = eng.abort_all("engine_error")
            fatal = True
        except Exception:                      # fail this replica's in-flight work
            log.exception("replica %d step failed", idx)
            finished = eng.abort_all("engine_error")
        for s in finished:
            rid, _ = pending.pop(s.req_id, (None, None))
            if rid is not None:
                outq.put(("done", rid, {"text": eng.decode_text(s), "finish": s.finish_reason,
                                        "span": s.span()}))
                served += 1
        if fatal or (exit_after is not None and served >= exit_after):
            if not shutdown_engine:
                # an engine embedded in a bigger process (the bench's HTTP phase): end the
                # loop, never the process; what it held was failed above
                for _, (rid, _s) in list(pending.items()):
                    outq.put(("done", rid, {"text": "", "finish": "engine_error", "span": {}}))
                pending.clear()
                eng.runner.busy_hook = None
                return
            outq.close()                       # flush what was served, then leave
            outq.join_thread()
            os._exit(4 if fatal else 3)        # 3 = injected replica crash


class DPRouter:
    def __init__(self, cfg, n_replicas: int, devices_per_replica: int = 1,
                 restart: bool = True, queues=None):
        """``queues`` = (inq, outq): attach to ONE engine loop that another process
        already runs (``serve_loop``) instead of spawning replicas; it is taken as
        ready and is never restarted."""
        self.cfg = cfg
        self.n = n_replicas
        self.dpr = devices_per_replica
        self.tp = max(1, int(cfg.tp))
        if self.tp > 1 and self.dpr != self.tp:
            raise ValueError(f"TP={self.tp} replicas need {self.tp} devices each")
        self.restart = restart
        self.ctx = mp.get_context("spawn")
        self.outq = self.ctx.Queue()
        self.inqs = [None] * n_replicas
        self.procs = [None] * n_replicas          # TP rank 0 (the engine loop)
        self.followers: list[list] = [[] for _ in range(n_replicas)]
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
        if str(self._cfg_dict.get("device", "")).startswith("cuda:"):
            self._cfg_dict["device"] = "cuda"     # the replica sees only its own devices
        if queues is not None:
            if n_replicas != 1:
                raise ValueError("attached queues serve exactly one replica")
            self.inqs[0], self.outq = queues
            self.ready[0] = True
            self.restart = False
        for i in range(n_replicas if queues is None else 0):
            self._spawn(i)
        deadline = time.time() + 1800
        while not all(self.ready) and time.time() < deadline:
            kind, idx, _ = self.outq.get(timeout=1800)
            if kind == "ready":
                self.ready[idx] = True
        self._stop = False
        self._thread = threading.Thread(target=self._dispatch, daemon=True)
        self._thread.start()

    def _devices(self, i: int) -> str:
        """HIP_VISIBLE_DEVICES of replica i.  Logical device d of the replicas maps
        through ``RFQ_DEVICES`` when set, else through the parent's own
        HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (an operator's
        ``HIP_VISIBLE_DEVICES=3`` keeps the engine on physical GPU 3; a
        ROCR_VISIBLE_DEVICES mask is inherited and indexed inside).  A single replica of
        ``cfg.device = "cuda:N"`` starts at logical device N."""
        if self.cfg.device == "cpu":
            return ""
        phys = (os.environ.get("RFQ_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
                or os.environ.get("CUDA_VISIBLE_DEVICES"))
        ids = [x.strip() for x in phys.split(",") if x.strip()] if phys else None
        base = 0
        dev = str(self.cfg.device)
        if self.n == 1 and dev.startswith("cuda:"):
            base = int(dev.split(":", 1)[1])
        devs = [base + i * self.dpr + j for j in range(self.dpr)]
        if ids is not None and max(devs) >= len(ids):
            raise ValueError(f"replica {i} needs logical devices {devs} but only "
                             f"{len(ids)} are visible ({phys})")
        return ",".join(ids[d] if ids else str(d) for d in devs)

    def _spawn(self, i: int) -> None:
        devs = self._devices(i)
        port = _free_port() if self.tp > 1 else 0
        q = self.ctx.Queue()
        p = self.ctx.Process(target=_worker,
                             args=(i, devs, self._cfg_dict, q, self.outq, self.tp, port),
                             daemon=True)
        p.start()
        fol = []
        for r in range(1, self.tp):
            f = self.ctx.Process(target=_follower,
                                 args=(i, devs, r, self.tp, port, self._cfg_dict), daemon=True)
            f.start()
            fol.append(f)
        self.inqs[i], self.procs[i], self.ready[i] = q, p, False
        self.followers[i] = fol

    def _kill_replica(self, i: int) -> None:
        for f in [self.procs[i], *self.followers[i]]:
            if f is not None and f.is_alive():
                f.kill()
        for f in [self.procs[i], *self.followers[i]]:
            if f is not None:
                f.join(timeout=10)

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
            if p is None or self._stop:
                continue
            dead = [x for x in [p, *self.followers[i]] if not x.is_alive()]
            if not dead:
                continue
            log.error("replica %d: process %s died (exit %s); failing its requests", i,
                      dead[0].pid, dead[0].exitcode)
            self._kill_replica(i)                  # a TP group cannot run with a rank missing
            if self.tp > 1 and self._cfg_dict.get("custom_allreduce"):
                # a TP replica failed: restart it on RCCL all-reduces only (the custom
                # xGMI kernel fails a step on a flag timeout, see runner.py)
                log.error("replica %d restarts with custom all-reduce disabled", i)
                self._cfg_dict = dict(self._cfg_dict, custom_allreduce=False)
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
        return {"replicas": self.n, "tp": self.tp, "ready": sum(self.ready),
                "restarts": self.restarts,
                "outstanding": len(self.where), "load": list(self.load),
                "completed": self.completed}

    def shutdown(self):
        self._stop = True
        for q, p in zip(self.inqs, self.procs):
            if p is not None and p.is_alive():
                q.put(None)
        for i, p in enumerate(self.procs):
            if p is not None:
                p.join(timeout=30)
            for f in self.followers[i]:
                f.join(timeout=30)
                if f.is_alive():
                    f.kill()


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
    """A DPRouter when RFQ_DP > 1 or RFQ_TP > 1 (replicas of cfg.tp processes/devices
    each) or when the single engine should live in its own process
    (RFQ_ENGINE_PROCESS: the API process then only parses HTTP, tokenises and
    validates), else None.  RFQ_ENGINE_PROCESS defaults to "auto" = on for a GPU engine:
    with the API in the engine's process its Python (HTTP, parsing, chat template,
    validation) shares the engine thread's GIL and the service delivered 0.86x the
    engine's docs/s; in two processes 1.01x (profiles/r4_http_open_loop.md)."""
    v = os.environ.get("RFQ_ENGINE_PROCESS", "auto").lower()
    dev = cfg.device
    if dev == "auto":
        import torch

        # device_count() does not initialise HIP in this (API) process
        dev = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    own_process = v in ("1", "true", "on") or (v == "auto" and dev != "cpu")
    if cfg.dp <= 1 and cfg.tp <= 1 and not own_process:
        return None
    return DPRouter(cfg, max(1, cfg.dp), max(1, cfg.tp))
