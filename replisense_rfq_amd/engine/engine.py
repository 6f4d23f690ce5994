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
import os
import queue
import sys
import threading
import time

import numpy as np
import torch

from .. import runtime
from ..models.config import get_config
from ..models.llama import DecoderLM
from ..parallel.tp import SINGLE, TPContext
from ..utils.config import EngineConfig
from ..utils.faults import CustomAllReduceError, FaultInjector
from ..utils.trace import trace_range
from .grammar import PROFILE_REFERENCE, PROFILE_SYNTHETIC, get_grammar
from .kv_cache import KVCache
from .runner import EXT_MAX, MAX_GRAPH_TOKENS, TOKEN_MULTS, ModelRunner
from .sequence import SamplingParams, Sequence, Status
from .tokenizer import flavor_for_vocab, get_tokenizer

log = logging.getLogger("replisense_rfq_amd.engine")

FINISH_REASONS = {1: "stop", 2: "length", 3: "grammar_error", 4: "abort", 5: "engine_error",
                  6: "timeout"}


def resolve_device(spec: str, tp: TPContext) -> torch.device:
    if spec == "auto":
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", tp.rank))
            return torch.device("cuda", local % max(1, torch.cuda.device_count()))
        return torch.device("cpu")
    return torch.device(spec)


def short_gil_switch() -> float:
    """Shorten the GIL switch interval for a process whose engine loop shares the
    interpreter with other threads (HTTP event loop, prompt tokenisers, the bench's
    admission hook).  Every native call of a step (schedule_and_pack, the token
    readback, post) releases the GIL, and taking it back waits up to one switch
    interval while another thread runs Python: at the default 5 ms that was several ms
    of idle GPU per step (bench: pack 5.2 ms of a 113 ms step with a tokenizer thread
    busy); 0.5 ms bounds it.  Called only by the loops that have such threads
    (AsyncEngine, DocStream, the DP router worker), never by a bare LLMEngine.
    Returns the previous interval so a temporary user can restore it."""
    prev = sys.getswitchinterval()
    sys.setswitchinterval(float(os.environ.get("RFQ_GIL_SWITCH_MS", "0.5")) / 1e3)
    return prev


class LLMEngine:
    def __init__(self, cfg: EngineConfig | None = None, tp: TPContext = SINGLE,
                 model=None, capture: bool = True):
        self.cfg = cfg or EngineConfig()
        self.tp = tp
        self.device = resolve_device(self.cfg.device, tp)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        if tp.enabled and self.cfg.custom_allreduce and self.device.type == "cuda":
            tp.enable_custom_allreduce()
        self.model_cfg = get_config(self.cfg.model)
        self.tokenizer = get_tokenizer(flavor_for_vocab(self.model_cfg.vocab_size),
                                       self._tokenizer_path())
        t0 = time.perf_counter()
        weights = None
        if model is None and self.cfg.weights_path:
            from ..models.weights import load_safetensors

            weights = load_safetensors(self.cfg.weights_path, self.model_cfg, tp, self.device,
                                       moe_ep=self.cfg.moe_parallel == "ep")
        self.model = model or DecoderLM(self.model_cfg, self.device, tp, seed=self.cfg.seed,
                                        weights=weights, moe_ep=self.cfg.moe_parallel == "ep")
        # the norm weights go into qkv / gate|up before anything copies those weights
        # (tiled copies below) or times them (start-up plans): models/llama.py fold_norms
        if self.device.type == "cuda":
            self.model.fold_norms()
        # before the KV pool is sized from the free memory: the tiled copies take theirs
        self.tiled_bytes = self.model.tile_decode_weights() if self.cfg.tune_gemm else 0
        self.init_weights_s = time.perf_counter() - t0
        self.kv = KVCache(self.model_cfg, self.model.hkv, self._num_blocks(), self.device,
                          prefix_cache=self.cfg.prefix_cache)
        self.model.attach_kv_cache(self.kv.k, self.kv.v)
        self.grammar = get_grammar(self.tokenizer.flavor, self.tokenizer) if self.cfg.grammar \
            else None
        self.runner = ModelRunner(self.model, self.kv, self.cfg,
                                  self.grammar.mask_table() if self.grammar else None, tp)
        self.core = self._make_core()
        self.kv.core = self.core
        self._live: dict[int, Sequence] = {}
        self.capture_s = 0.0
        self.tune_s = 0.0
        if self.device.type == "cuda" and self.cfg.tune_gemm:
            self._tune_gemms()
        if capture and self.device.type == "cuda" and self.cfg.use_graphs:
            buckets = [b for b in self.cfg.graph_buckets if b <= self.cfg.max_num_seqs]
            limit = MAX_GRAPH_TOKENS
            if self.model_cfg.is_moe:
                # MoE: graphs only where the per-expert skinny kernels run; larger
                # steps go eager (the grouped dense MFMA GEMM, models/moe.py, is
                # host-sync-free, but its token-count-dependent grid is not captured)
                from ..models.moe import SKINNY_MAX_TOKENS

                limit = int(os.environ.get("RFQ_MOE_GRAPH_TOKENS", SKINNY_MAX_TOKENS))
                buckets = [b for b in buckets if b <= limit]
            if buckets:
                self.capture_s = self.runner.capture_graphs(buckets, limit)
                self.core.set_graph_keys(sorted(self.runner.graphs))
        self.num_steps = 0
        self.step_times: list[float] = []
        self.timers = {"execute_s": 0.0, "post_s": 0.0}
        self.faults = FaultInjector()
        self.pinned_blocks = 0
        if self.cfg.prefix_cache and self.cfg.warm_prefix and tp.rank == 0:
            try:
                self.warm_prefix()
            except BaseException:
                # the followers are mirroring the warm-up: release them before the
                # caller sees the failure (it may rebuild the group, bench.py)
                self.runner.stop_workers()
                raise

    def warm_prefix(self, ids: list[int] | None = None) -> int:
        """prefill the shared system + template prefix once
        at start-up and pin its KV blocks, so the first wave of requests already
        hits the prefix cache and the template can never be evicted under load.
        TP followers mirror the warm-up step like any other."""
        if ids is None:
            from ..service.prompt import shared_prefix_ids

            ids = shared_prefix_ids(self.tokenizer)
        if len(ids) < 2 * self.kv.block_size:
            return 0
        # prompt = prefix + 1 token so every full prefix block is computed and published
        params = SamplingParams(temperature=0.0, max_tokens=1, grammar=False)
        self.generate([list(ids) + [ids[-1]]], params)
        self.pinned_blocks = int(self.core.pin_prefix(np.asarray(ids, np.int32)))
        return self.pinned_blocks

    # ------------------------------------------------------------------ setup
    def _tokenizer_path(self) -> str | None:
        if self.cfg.tokenizer_path:
            return self.cfg.tokenizer_path
        if self.cfg.weights_path and os.path.isdir(self.cfg.weights_path):
            cand = os.path.join(self.cfg.weights_path, "tokenizer.json")
            if os.path.exists(cand):
                return cand
        return None

    def _make_core(self):
        """Native scheduler / packer / post-processor (csrc/runtime/engine_core.cpp)."""
        c = self.cfg
        conf = dict(block_size=self.kv.block_size, num_blocks=self.kv.num_blocks - 1,
                    scratch_block=self.kv.scratch_block, max_num_seqs=c.max_num_seqs,
                    max_batched_tokens=c.max_batched_tokens, max_model_len=c.max_model_len,
                    ext_max=EXT_MAX, group=self.model.hq // self.model.hkv, hkv=self.model.hkv,
                    jump_forward=c.jump_forward, prefix_cache=c.prefix_cache,
                    is_cuda=self.device.type == "cuda", use_graphs=c.use_graphs,
                    token_mults=list(TOKEN_MULTS), eos_ids=list(self.tokenizer.eos_ids),
                    decode_tiles=c.decode_tiles, prefill_qblk=self.runner.prefill_qblk)
        g = self.grammar.native if self.grammar is not None else None
        if self.grammar is not None and g is None:
            raise RuntimeError("the native grammar automaton failed to build")
        return runtime.load().EngineCore(conf, g)

    def _tune_gemms(self) -> None:
        from ..ops.autotune import tune_model
        from .runner import TOKEN_MULTS

        t0 = time.perf_counter()
        nbs = [b for b in self.cfg.graph_buckets if b <= min(64, self.cfg.max_num_seqs)] or [1]
        ms = sorted({nb * m for nb in nbs for m in TOKEN_MULTS if nb * m <= 64})
        self.gemm_plan = tune_model(
            self.model, ms, nbs,
            max_tokens=min(self.cfg.max_batched_tokens, 16384) if self.cfg.gemm_split else 0,
            max_seqs=self.cfg.max_num_seqs)
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
        params = params or self.default_params()
        if len(prompt_ids) + params.max_tokens > self.cfg.max_model_len:
            params.max_tokens = max(1, self.cfg.max_model_len - len(prompt_ids))
        seq = Sequence(list(prompt_ids), params, callback=callback)
        seq.status = Status.WAITING
        seq.core_id = self.core.add(np.asarray(prompt_ids, np.int32), float(params.temperature),
                                    int(params.max_tokens), int(params.seed),
                                    bool(params.grammar and self.grammar is not None),
                                    int(params.min_items), int(params.profile), seq.t_arrival)
        self._live[seq.core_id] = seq
        return seq

    # ------------------------------------------------------------------- step
    def step(self) -> list[Sequence]:
        ts = time.perf_counter()
        if self.faults.active and self.core.has_work:
            self.faults.on_step(self.num_steps, self.tp.enabled and self.cfg.custom_allreduce)
        with trace_range("execute"):
            toks = self.runner.execute(self.core, ts)
        if toks is None:
            return [self._finalize(i) for i in self.core.drain_finished()]
        now = time.perf_counter()
        self.timers["execute_s"] += now - ts
        self.step_times.append(now - ts)
        self.num_steps += 1
        with trace_range("post"):
            done = self.core.post(np.ascontiguousarray(toks, np.int32), now)
            finished = [self._finalize(i) for i in done]
        self.timers["post_s"] += time.perf_counter() - now
        return finished

    def _finalize(self, cid: int) -> Sequence:
        """Copy a finished sequence out of the core, release its record, notify."""
        s = self._live.pop(cid)
        info = self.core.info(cid)
        s.tokens = self.core.tokens(cid).tolist()
        s.num_cached = info["num_cached"]
        s.prefix_hit_tokens = info["prefix_hit"]
        s.num_sampled = info["num_sampled"]
        s.num_forced = info["num_forced"]
        s.mask_idx = info["mask_idx"]
        s.finish_reason = FINISH_REASONS.get(info["finish"], "abort")
        s.status = Status.FINISHED
        s.t_first_sched = info["t_first_sched"]
        s.t_prefill_done = info["t_prefill_done"]
        s.t_first_token = info["t_first_token"]
        s.t_finish = info["t_finish"] or time.perf_counter()
        self.core.release(cid)
        if s.callback is not None:
            try:
                s.callback(s)
            except Exception:  # pragma: no cover - callbacks must not kill the loop
                log.exception("sequence callback failed")
        return s

    def has_work(self) -> bool:
        return self.core.has_work

    def abort_request(self, seq: Sequence, reason: str = "abort") -> bool:
        """Retire one request between steps (deadline expired, client gone); its KV
        blocks return to the pool immediately."""
        code = {v: k for k, v in FINISH_REASONS.items()}.get(reason, 4)
        cid = getattr(seq, "core_id", None)
        if cid is None or cid not in self._live or self._live[cid] is not seq:
            return False
        if not self.core.abort(cid, code, time.perf_counter()):
            return False
        self._finalize(cid)
        return True

    def abort_all(self, reason: str) -> list[Sequence]:
        """Finish every queued/running sequence (releasing its KV blocks)."""
        code = {v: k for k, v in FINISH_REASONS.items()}.get(reason, 4)
        return [self._finalize(i) for i in self.core.abort_all(code, time.perf_counter())]

    def generate(self, prompts: list[list[int]], params=None,
                 seeds: list[int] | None = None) -> list[Sequence]:
        """Blocking batch generation.  `params`: one SamplingParams for all, or a list."""
        seqs = []
        for i, p in enumerate(prompts):
            sp = params[i] if isinstance(params, (list, tuple)) else params
            if seeds is not None:
                base = sp or self.default_params()
                sp = SamplingParams(base.temperature, base.max_tokens, seeds[i], base.grammar,
                                    base.min_items, base.profile)
            seqs.append(self.add_request(p, sp))
        while self.has_work():
            self.step()
        return seqs

    def default_params(self, **kw) -> SamplingParams:
        p = SamplingParams(temperature=self.cfg.temperature, max_tokens=self.cfg.max_tokens,
                           grammar=self.grammar is not None,
                           profile=PROFILE_SYNTHETIC if self.cfg.decode_hints else PROFILE_REFERENCE)
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def decode_text(self, seq: Sequence) -> str:
        return self.tokenizer.decode(seq.output_ids)

    # ------------------------------------------------------------------- TP
    def worker_loop(self, tolerate_car_errors: bool = False) -> bool:
        """Non-zero TP ranks: mirror rank 0's steps until told to stop.

        ``tolerate_car_errors``: a custom all-reduce flag timeout on this rank (raised
        after the step's device work, so the rank is still in step with rank 0) is
        recorded and mirroring continues; rank 0, whose own all-reduces then time out
        on this rank's silent kernels, ends the group and the caller decides (bench.py
        re-forms it on RCCL).  Returns True if such an error was seen."""
        failed = False
        while True:
            try:
                if not self.runner.worker_step():
                    return failed
            except CustomAllReduceError:
                if not tolerate_car_errors:
                    raise
                failed = True

    def shutdown(self) -> None:
        self.runner.stop_workers()

    def stats(self) -> dict:
        st = dict(self.runner.stats)
        st.update({k: round(v, 3) for k, v in self.timers.items()})
        st.update(self.kv.stats(self.core))
        st["preempted"] = self.core.num_preempted
        st["pinned_blocks"] = self.core.num_pinned
        st["running"] = self.core.num_running
        st["waiting"] = self.core.num_waiting
        return st


class _Request:
    """Handle shared by the HTTP side and the engine thread (set once admitted)."""
    __slots__ = ("seq",)

    def __init__(self):
        self.seq = None


class AsyncEngine:
    """Thread-hosted engine loop with an asyncio front door.

    The HTTP handlers only enqueue; one background thread owns every mutable
    engine structure (single-owner design), so no locks are held
    across a GPU step.
    """

    def __init__(self, engine: LLMEngine):
        self.engine = engine
        short_gil_switch()            # the HTTP event loop shares this interpreter
        self._inbox: queue.Queue = queue.Queue()
        self._held: list = []                    # inbox messages deferred to the loop top
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

    def _drain(self, in_step: bool = False):
        """Apply the inbox.  ``in_step``: called by the runner while a step executes on
        the device (runner.busy_hook), so new requests are admitted during GPU time
        instead of between steps; aborts (which free KV blocks of sequences that may
        be in the running step) and any add that raised wait for the loop top."""
        if not in_step:
            held, self._held = self._held, []
            for msg in held:
                self._apply_or_fail(msg)
        try:
            while True:
                msg = self._inbox.get_nowait()
                if in_step and msg[0] == "add":
                    try:
                        self._apply(msg)
                    except Exception:  # noqa: BLE001 - replayed at the loop top
                        self._held.append(msg)
                elif in_step:
                    self._held.append(msg)
                else:
                    self._apply_or_fail(msg)
        except queue.Empty:
            pass

    def _apply_or_fail(self, msg):
        """Apply one inbox message at the loop top.  A message that raises fails only
        its own request (an add's caller gets a finished ``engine_error`` Sequence, the
        G8 error-dict path); the engine thread keeps serving everyone else."""
        try:
            self._apply(msg)
        except Exception:  # noqa: BLE001
            log.exception("request could not be admitted")
            if msg[0] == "add":
                _, prompt, params, cb, req = msg
                s = Sequence(list(prompt), params or self.engine.default_params(), callback=cb)
                s.status = Status.FINISHED
                s.finish_reason = "engine_error"
                s.t_finish = time.perf_counter()
                req.seq = s
                if cb is not None:
                    try:
                        cb(s)
                    except Exception:  # pragma: no cover - callbacks must not kill the loop
                        log.exception("sequence callback failed")

    def _in_step(self):
        self._drain(in_step=True)

    def _apply(self, msg):
        eng = self.engine
        if msg[0] == "add":
            _, prompt, params, cb, req = msg
            req.seq = eng.add_request(prompt, params, cb)
        elif msg[1].seq is not None:             # ("abort", req): deadline expired
            eng.abort_request(msg[1].seq, "timeout")

    def _loop(self):
        eng = self.engine
        runner = getattr(eng, "runner", None)
        if runner is not None:
            runner.busy_hook = self._in_step
        while not self._stop.is_set():
            self._drain()
            if eng.has_work():
                self.step_started = time.monotonic()
                try:
                    eng.step()
                except BaseException as e:  # engine failure: fail every in-flight request
                    # (including requests the busy hook admitted during this step: they
                    # are in the core already and are failed with it, like the rest)
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

        req = _Request()
        self._inbox.put(("add", prompt_ids, params, done, req))
        self._wake.set()
        if not timeout:
            return await fut
        try:
            return await asyncio.wait_for(asyncio.shield(fut), timeout)
        except asyncio.TimeoutError:
            self._inbox.put(("abort", req))      # stop computing it; free its KV
            self._wake.set()
            raise

    def shutdown(self):
        self._stop.set()
        self._wake.set()
        self._thread.join(timeout=5)
        runner = getattr(self.engine, "runner", None)
        if runner is not None and runner.busy_hook == self._in_step:
            runner.busy_hook = None
