"""LLM inference engine: continuous batching over the gfx950 model runner.

Replaces the reference's remote call chain (ag2 ConversableAgent -> openai ->
Groq, rfq_agent.py:112-118,163) with an on-node engine:

  add_request(prompt ids, SamplingParams) -> Sequence
  step(): schedule -> runner.execute (one forward + grammar-masked sampling)
          -> advance grammar automata (C++ batch_advance), append sampled +
             jump-forward tokens, publish prompt blocks to the prefix cache,
             retire finished sequences
  generate(prompts) -> finished Sequences            (blocking, used by bench)
  AsyncEngine.submit(...) -> awaitable               (service / HTTP path)

One engine owns one model replica (TP group).  With TP > 1 only TP-rank 0 runs
this loop; the other ranks sit in :meth:`LLMEngine.worker_loop`.
"""
from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time

import numpy as np
import torch

from ..models.config import get_config
from ..models.llama import DecoderLM
from ..parallel.tp import SINGLE, TPContext
from ..utils.config import EngineConfig
from ..utils.faults import FaultInjector
from ..utils.trace import trace_range
from .grammar import get_grammar
from .kv_cache import KVCache
from .runner import ModelRunner
from .scheduler import Scheduler
from .sequence import SamplingParams, Sequence, Status
from .tokenizer import flavor_for_vocab, get_tokenizer

log = logging.getLogger("replisense_rfq_amd.engine")


def resolve_device(spec: str, tp: TPContext) -> torch.device:
    if spec == "auto":
        if torch.cuda.is_available():
            import os

            local = int(os.environ.get("LOCAL_RANK", tp.rank))
            return torch.device("cuda", local % max(1, torch.cuda.device_count()))
        return torch.device("cpu")
    return torch.device(spec)


class LLMEngine:
    def __init__(self, cfg: EngineConfig | None = None, tp: TPContext = SINGLE,
                 model=None, capture: bool = True):
        self.cfg = cfg or EngineConfig()
        self.tp = tp
        self.device = resolve_device(self.cfg.device, tp)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.model_cfg = get_config(self.cfg.model)
        self.tokenizer = get_tokenizer(flavor_for_vocab(self.model_cfg.vocab_size))
        t0 = time.perf_counter()
        self.model = model or DecoderLM(self.model_cfg, self.device, tp, seed=self.cfg.seed)
        self.init_weights_s = time.perf_counter() - t0
        self.kv = KVCache(self.model_cfg, self.model.hkv, self._num_blocks(), self.device,
                          prefix_cache=self.cfg.prefix_cache)
        self.model.attach_kv_cache(self.kv.k, self.kv.v)
        self.grammar = get_grammar(self.tokenizer.flavor) if self.cfg.grammar else None
        self.runner = ModelRunner(self.model, self.kv, self.cfg,
                                  self.grammar.mask_table() if self.grammar else None, tp)
        self.scheduler = Scheduler(self.cfg, self.kv)
        self.capture_s = 0.0
        self.tune_s = 0.0
        if self.device.type == "cuda" and self.cfg.tune_gemm:
            self._tune_gemms()
        if capture and self.device.type == "cuda" and self.cfg.use_graphs:
            buckets = [b for b in self.cfg.graph_buckets if b <= self.cfg.max_num_seqs]
            if buckets:
                self.capture_s = self.runner.capture_graphs(buckets)
        self.num_steps = 0
        self.step_times: list[float] = []
        self.timers = {"schedule_s": 0.0, "execute_s": 0.0, "post_s": 0.0}
        self.faults = FaultInjector()

    # ------------------------------------------------------------------ setup
    def _tune_gemms(self) -> None:
        from ..ops.autotune import tune_model
        from .runner import TOKEN_MULTS

        t0 = time.perf_counter()
        nbs = [b for b in self.cfg.graph_buckets if b <= min(64, self.cfg.max_num_seqs)] or [1]
        ms = sorted({nb * m for nb in nbs for m in TOKEN_MULTS if nb * m <= 64})
        self.gemm_plan = tune_model(self.model, ms, nbs)
        self.tune_s = time.perf_counter() - t0

    def _num_blocks(self) -> int:
        cfg = self.cfg
        per_seq = (cfg.max_model_len + 31) // 32
        if self.device.type == "cuda":
            free, _ = torch.cuda.mem_get_info(self.device)
            n = KVCache.blocks_for_memory(self.model_cfg, self.model.hkv, free, cfg.kv_fraction)
        else:
            n = 64 + 8 * per_seq
        n = min(n, per_seq * cfg.max_num_seqs + 64)
        if cfg.max_kv_blocks:
            n = min(n, cfg.max_kv_blocks)
        if self.tp.enabled:          # every rank must size the pool identically
            t = torch.tensor([n], device=self.device if self.device.type == "cuda" else "cpu")
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=self.tp.group)
            n = int(t.item())
        return n

    # --------------------------------------------------------------- requests
    def add_request(self, prompt_ids: list[int], params: SamplingParams | None = None,
                    callback=None) -> Sequence:
        params = params or SamplingParams(temperature=self.cfg.temperature,
                                          max_tokens=self.cfg.max_tokens,
                                          grammar=self.grammar is not None)
        if len(prompt_ids) + params.max_tokens > self.cfg.max_model_len:
            params.max_tokens = max(1, self.cfg.max_model_len - len(prompt_ids))
        seq = Sequence(list(prompt_ids), params, callback=callback)
        if params.grammar and self.grammar is not None:
            seq.gstate, forced = self.grammar.initial(params.min_items)
            seq.tokens += forced
            seq.num_forced += len(forced)
            seq.mask_idx = self.grammar.mask(seq.gstate)
        self.scheduler.add(seq)
        return seq

    # ------------------------------------------------------------------- step
    def step(self) -> list[Sequence]:
        ts = time.perf_counter()
        with trace_range("schedule"):
            plan = self.scheduler.schedule()
        if plan.empty:
            return []
        if self.faults.active:
            self.faults.on_step(self.num_steps)
        t0 = time.perf_counter()
        with trace_range("execute"):
            rows, toks = self.runner.execute(plan)
        now = time.perf_counter()
        with trace_range("post"):
            return self._post(plan, rows, toks, now, t0, ts)

    def _post(self, plan, rows, toks, now, t0, ts) -> list[Sequence]:
        self.timers["schedule_s"] += t0 - ts
        self.timers["execute_s"] += now - t0
        self.step_times.append(now - t0)
        self.num_steps += 1
        for s in plan.decode:
            s.num_cached += 1
        for s, q in plan.extend:
            s.num_cached += q
            self.kv.publish(s)
            if not s.t_prefill_done and not s.in_prefill:
                s.t_prefill_done = now
        # gather sequences that sample this step
        samp = [(s, int(toks[k])) for k, (s, do) in enumerate(rows) if do]
        finished: list[Sequence] = []
        gseqs = [(s, t) for s, t in samp if s.gstate is not None]
        if gseqs:
            states = np.array([s.gstate for s, _ in gseqs], np.int32).reshape(-1, 5)
            tokens = np.array([t for _, t in gseqs], np.int32)
            masks, offs, forced, ok = self.grammar.batch_advance(states, tokens)
            for i, (s, t) in enumerate(gseqs):
                f = forced[offs[i]:offs[i + 1]].tolist()
                s.tokens.append(t)
                s.tokens.extend(f)
                s.num_sampled += 1
                s.num_forced += len(f)
                s.gstate = tuple(int(x) for x in states[i])
                s.mask_idx = int(masks[i])
                if not s.t_first_token:
                    s.t_first_token = now
                if not ok[i]:
                    self._finish(s, "grammar_error", finished)
                elif masks[i] < 0:
                    self._finish(s, "stop", finished)
                elif s.num_generated >= s.params.max_tokens:
                    self._finish(s, "length", finished)
        for s, t in samp:
            if s.gstate is not None:
                continue
            s.tokens.append(t)
            s.num_sampled += 1
            if not s.t_first_token:
                s.t_first_token = now
            if t in self.tokenizer.eos_ids:
                self._finish(s, "stop", finished)
            elif s.num_generated >= s.params.max_tokens:
                self._finish(s, "length", finished)
        self.timers["post_s"] += time.perf_counter() - now
        return finished

    def _finish(self, s: Sequence, reason: str, out: list):
        self.scheduler.finish(s, reason)
        out.append(s)
        if s.callback is not None:
            try:
                s.callback(s)
            except Exception:  # pragma: no cover - callbacks must not kill the loop
                log.exception("sequence callback failed")

    def has_work(self) -> bool:
        return self.scheduler.has_work

    def abort_all(self, reason: str) -> list[Sequence]:
        """Finish every queued/running sequence (releasing its KV blocks)."""
        out: list[Sequence] = []
        for s in list(self.scheduler.running) + list(self.scheduler.waiting):
            if s in self.scheduler.waiting:
                self.scheduler.waiting.remove(s)
            self._finish(s, reason, out)
        return out

    def generate(self, prompts: list[list[int]], params=None,
                 seeds: list[int] | None = None) -> list[Sequence]:
        """Blocking batch generation.  `params`: one SamplingParams for all, or a list."""
        seqs = []
        for i, p in enumerate(prompts):
            sp = params[i] if isinstance(params, (list, tuple)) else params
            if seeds is not None:
                base = sp or self.default_params()
                sp = SamplingParams(base.temperature, base.max_tokens, seeds[i], base.grammar,
                                    base.min_items)
            seqs.append(self.add_request(p, sp))
        while self.has_work():
            self.step()
        return seqs

    def default_params(self, **kw) -> SamplingParams:
        p = SamplingParams(temperature=self.cfg.temperature, max_tokens=self.cfg.max_tokens,
                           grammar=self.grammar is not None)
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def decode_text(self, seq: Sequence) -> str:
        return self.tokenizer.decode(seq.output_ids)

    # ------------------------------------------------------------------- TP
    def worker_loop(self) -> None:
        """Non-zero TP ranks: mirror rank 0's steps until told to stop."""
        while self.runner.worker_step():
            pass

    def shutdown(self) -> None:
        self.runner.stop_workers()

    def stats(self) -> dict:
        st = dict(self.runner.stats)
        st.update({k: round(v, 3) for k, v in self.timers.items()})
        st.update(self.kv.stats())
        st["preempted"] = self.scheduler.num_preempted
        st["running"] = len(self.scheduler.running)
        st["waiting"] = len(self.scheduler.waiting)
        return st


class AsyncEngine:
    """Thread-hosted engine loop with an asyncio front door.

    The HTTP handlers only enqueue; one background thread owns every mutable
    engine structure (single-owner design), so no locks are held
    across a GPU step.
    """

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        self._inbox: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._wake = threading.Event()
        self.error: BaseException | None = None
        self.step_started = 0.0
        self.stalled = False
        self._thread = threading.Thread(target=self._loop, name="rfq-engine", daemon=True)
        self._thread.start()
        self._watchdog = threading.Thread(target=self._watch, name="rfq-watchdog", daemon=True)
        self._watchdog.start()

    def _watch(self):
        """Step watchdog: a step running longer than ``step_timeout_s`` marks the
        engine stalled (``/health`` -> 503) so an orchestrator can restart it.
        A GPU step cannot be interrupted safely, so in-flight requests are left
        to their own request timeouts."""
        limit = self.engine.cfg.step_timeout_s
        while not self._stop.wait(min(1.0, limit / 4)):
            t = self.step_started
            if t and time.monotonic() - t > limit and not self.stalled:
                self.stalled = True
                log.error("engine step exceeded %.1fs watchdog", limit)

    @property
    def healthy(self) -> bool:
        return not self.stalled and self._thread.is_alive()

    def _loop(self):
        eng = self.engine
        while not self._stop.is_set():
            try:
                while True:
                    prompt, params, cb = self._inbox.get_nowait()
                    eng.add_request(prompt, params, cb)
            except queue.Empty:
                pass
            if eng.has_work():
                self.step_started = time.monotonic()
                try:
                    eng.step()
                except BaseException as e:  # engine failure: fail every in-flight request
                    log.exception("engine step failed")
                    self.error = e
                    eng.abort_all("engine_error")
                finally:
                    self.step_started = 0.0
            else:
                self._wake.wait(0.005)
                self._wake.clear()

    async def generate(self, prompt_ids: list[int], params: SamplingParams | None = None,
                       timeout: float | None = None) -> Sequence:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def done(seq):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(seq))

        self._inbox.put((prompt_ids, params, done))
        self._wake.set()
        if timeout:
            return await asyncio.wait_for(fut, timeout)
        return await fut

    def shutdown(self):
        self._stop.set()
        self._wake.set()
        self._thread.join(timeout=5)
