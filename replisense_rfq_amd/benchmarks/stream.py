"""Closed-loop document streams over an LLMEngine and their measurements.

Used by bench.py (the driver's headline metric and its extra phases) and by
tools/bench_depth_sweep.py.  A stream keeps ``in_flight`` synthetic RFQ documents
admitted to the engine (production continuous batching: a finished document is
replaced by the next one at once) and records every completed Sequence, so a
timed window yields docs/s and the latency under load of exactly the documents it
completed.

Documents come either straight from the synthetic corpus (the /parse-text/ path:
email bodies) or, with ``formats``, as generated PDF / XLSX / DOCX attachments run
through the service's own parser first (the /upload/ path, BASELINE configs 3 and
5: app/file_parser.py's CPU stage feeding the prefill queue), parsed ahead of the
engine in a spawned process pool.
"""
from __future__ import annotations

import queue
import statistics
import threading
import time


_WORKER_TOK = {}


def _worker_tokenizer(flavor: str, path):
    """One tokenizer per parse worker process (prompt prefix registered, as in the
    engine process: token-identical prompts)."""
    key = (flavor, path)
    if key not in _WORKER_TOK:
        from ..engine.tokenizer import get_tokenizer
        from ..service.prompt import register_prompt_prefix

        tok = get_tokenizer(flavor, path)
        register_prompt_prefix(tok)
        _WORKER_TOK[key] = tok
    return _WORKER_TOK[key]


def _parsed_doc(args):
    """Worker: generate one synthetic attachment, parse it with the service parser,
    build the prompt and tokenise it (off the engine process's GIL); return (prompt
    ids, decode hints).  Module-level for the spawn pool."""
    seed, fmt, flavor, tok_path = args
    import os
    import tempfile
    from pathlib import Path

    from ..service.parser import FileParser
    from ..utils import docgen, synth

    d = synth.make_rfq(seed)
    p = Path(tempfile.gettempdir()) / f"rfq_bench_{os.getpid()}_{seed}.{fmt}"
    p.write_bytes(docgen.rfq_attachment(d, fmt))
    try:
        text = FileParser().parse_file(str(p))["raw_text"]       # file_parser.py:97-99
    finally:
        p.unlink(missing_ok=True)
    from ..service.prompt import build_messages

    return _worker_tokenizer(flavor, tok_path).chat_ids(build_messages(text)), \
        synth.decode_hints(d)


def _produce_proc(base: int, flavor: str, path, out_q, stop_evt) -> None:
    """Spawned producer process for the plain-text stream: synthesise each document,
    build the byte-identical prompt and tokenise it, away from the engine's GIL (a
    producer thread in the engine process took the GIL from the step loop every switch
    interval: the scheduler pack waited 5.2 ms per step at the default 5 ms interval and
    the forward launch +3 ms at 0.5 ms).  Imports no torch and never touches the GPU."""
    import queue as _q

    from ..engine.tokenizer import get_tokenizer
    from ..service.prompt import build_messages, register_prompt_prefix
    from ..utils import synth

    tok = get_tokenizer(flavor, path)
    register_prompt_prefix(tok)
    i = 0
    while not stop_evt.is_set():
        d = synth.make_rfq(base + i)
        item = (base + i, tok.chat_ids(build_messages(d.text)), synth.decode_hints(d))
        while not stop_evt.is_set():
            try:
                out_q.put(item, timeout=0.1)
                break
            except _q.Full:
                continue
        i += 1


class DocStream:
    """One replica's continuous document stream over an LLMEngine.

    A producer thread builds and tokenises prompts ahead of the engine (as the
    HTTP front-end does while the engine steps); the engine loop keeps
    ``in_flight`` documents admitted and counts completions.  ``run_until(n)``
    steps the engine until ``n`` documents have completed in total and returns,
    leaving the in-flight documents in place for the next call.
    """

    def __init__(self, engine, dp_rank: int, seed: int, in_flight: int,
                 formats: tuple | None = None, parse_procs: int = 4,
                 producer: str | None = None, overlap_admit: bool | None = None):
        from ..service.extract import build_messages
        from ..service.prompt import register_prompt_prefix
        from ..utils import synth

        self.engine = engine
        self.tok = engine.tokenizer
        register_prompt_prefix(self.tok)         # what the service's EngineBackend does
        self.in_flight = in_flight
        self.base = (seed * 7919 + dp_rank) * 1_000_003
        self.ready: queue.Queue = queue.Queue(maxsize=max(64, in_flight))
        self.stop = threading.Event()
        self.live = 0
        self.completed = 0
        self.finished = []                       # sequences completed in the current window
        self._build, self._synth = build_messages, synth
        self.formats = tuple(formats) if formats else None
        self._pool = None
        if self.formats:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor

            # spawn, never fork: this process owns a GPU context
            self._pool = ProcessPoolExecutor(parse_procs, mp_context=mp.get_context("spawn"))
        # plain-text stream: the prompts come from a spawned process (RFQ_BENCH_PRODUCER=
        # process, default) or, as before, from a thread of this process (=thread)
        import os

        mode = producer or os.environ.get("RFQ_BENCH_PRODUCER", "process")
        # admit new documents while a step runs on the device (runner.busy_hook)
        self.overlap_admit = (overlap_admit if overlap_admit is not None
                              else os.environ.get("RFQ_BENCH_OVERLAP_ADMIT", "1") != "0")
        self._proc = None
        self.thread = None
        if self.formats is None and mode == "process":
            import multiprocessing as mp

            ctx = mp.get_context("spawn")            # never fork: this process owns a GPU
            self.ready = ctx.Queue(maxsize=max(64, in_flight))
            self._stop_evt = ctx.Event()
            self._proc = ctx.Process(target=_produce_proc, name="bench-tokenize",
                                     args=(self.base, self.tok.flavor, getattr(self.tok, "path", None),
                                           self.ready, self._stop_evt), daemon=True)
            self._proc.start()
        else:
            self.thread = threading.Thread(target=self._produce, name="bench-tokenize",
                                           daemon=True)
            self.thread.start()

    def _docs(self):
        i = 0
        if self._pool is None:
            while True:
                d = self._synth.make_rfq(self.base + i)
                yield self.base + i, d.text, self._synth.decode_hints(d)
                i += 1
        chunk = 32
        flavor, path = self.tok.flavor, getattr(self.tok, "path", None)
        while not self.stop.is_set():
            args = [(self.base + i + k, self.formats[(i + k) % len(self.formats)], flavor, path)
                    for k in range(chunk)]
            for a, (ids, hints) in zip(args, self._pool.map(_parsed_doc, args)):
                yield a[0], ids, hints                  # already tokenised by the worker
            i += chunk

    def _produce(self):
        for s, doc, hints in self._docs():
            if self.stop.is_set():
                return
            ids = doc if self._pool is not None else self.tok.chat_ids(self._build(doc))
            params = self.engine.default_params(seed=s & 0xFFFFFF, **hints)
            while not self.stop.is_set():
                try:
                    self.ready.put((ids, params), timeout=0.1)
                    break
                except queue.Full:
                    continue

    def _top_up(self, block: bool):
        eng = self.engine
        while self.live < self.in_flight:
            try:
                item = self.ready.get(block=block and not eng.has_work(), timeout=1.0)
            except queue.Empty:
                if self._proc is not None and not self._proc.is_alive():
                    raise RuntimeError(f"bench producer process exited "
                                       f"(code {self._proc.exitcode}); no more documents")
                return
            if self._proc is not None:           # (doc seed, prompt ids, decode hints)
                s, ids, hints = item
                params = eng.default_params(seed=s & 0xFFFFFF, **hints)
            else:
                ids, params = item
            eng.add_request(ids, params)
            self.live += 1

    def run_until(self, target: int, deadline: float | None = None):
        """Step until ``target`` documents completed in total (or perf_counter passes
        ``deadline``; then returns False)."""
        eng = self.engine
        runner = getattr(eng, "runner", None)
        hooked = [False]

        def admit():                     # runs while the step executes on the device
            hooked[0] = True
            self._top_up(block=False)

        if runner is not None and self.overlap_admit:
            runner.busy_hook = admit
        try:
            while self.completed < target:
                if deadline is not None and time.perf_counter() > deadline:
                    return False
                # the documents retired by the previous step are replaced during this
                # step's device time (admit) instead of between steps, where the GPU
                # idles; only an empty engine (or a step that never launched) tops up here
                if not hooked[0] or not eng.has_work():
                    self._top_up(block=True)
                if not eng.has_work():
                    continue
                hooked[0] = False
                done = eng.step()
                self.live -= len(done)
                self.completed += len(done)
                self.finished.extend(done)
        finally:
            if runner is not None:
                runner.busy_hook = None
        return True

    def close(self):
        self.stop.set()
        if self._proc is not None:
            self._stop_evt.set()
        try:
            while True:
                self.ready.get_nowait()
        except queue.Empty:
            pass
        if self._proc is not None:
            self._proc.join(timeout=10)
            if self._proc.is_alive():
                self._proc.terminate()
                self._proc.join(timeout=5)
            self.ready.cancel_join_thread()
            self._proc = None
        if self.thread is not None:
            self.thread.join(timeout=10)
        if self._pool is not None:
            self._pool.shutdown(wait=False, cancel_futures=True)
        if self.engine.has_work():
            self.engine.abort_all("abort")
        self.live = 0


def validate(engine, seqs) -> dict:
    """Post-process a window's completions like the service does (rfq_agent.py:185-206)
    and report the per-document token shape."""
    from ..service.extract import parse_and_validate_response

    n = max(1, len(seqs))
    ok = 0
    for s in seqs:
        out = parse_and_validate_response(engine.decode_text(s), "direct_text_input")
        ok += bool(out.get("success")) and "validation warnings" not in out.get("message", "")
    return dict(
        prompt_tokens=sum(s.prompt_len for s in seqs) / n,
        completion_tokens=sum(s.num_generated for s in seqs) / n,
        sampled_tokens=sum(s.num_sampled for s in seqs) / n,
        prefix_hit_tokens=sum(s.prefix_hit_tokens for s in seqs) / n,
        valid=ok / n)


def pcts(vals) -> dict | None:
    """p50 / p90 / p99 / max / mean of a list of seconds (nearest-rank percentiles)."""
    if not vals:
        return None
    v = sorted(vals)

    def q(p):
        return v[min(len(v) - 1, max(0, int(round(p / 100.0 * len(v) + 0.5)) - 1))]
    return {"p50": round(q(50), 3), "p90": round(q(90), 3), "p99": round(q(99), 3),
            "max": round(v[-1], 3), "mean": round(sum(v) / len(v), 3), "n": len(v)}


def loaded_latency(seqs) -> dict:
    """Latency under load of the documents that completed inside a timed window:
    submission to the engine -> last token (``e2e``) and -> first sampled token
    (``ttft``), the server-side time a closed-loop client with this many requests
    in flight waits per document (the reference's only metric is per-request
    server time, /root/reference/app/rfq_agent.py:158-168; its LLM call times out
    at 30 s, rfq_agent.py:69)."""
    e2e = [s.t_finish - s.t_arrival for s in seqs if s.t_finish and s.t_arrival]
    ttft = [s.t_first_token - s.t_arrival for s in seqs if s.t_first_token and s.t_arrival]
    return {"e2e_s": pcts(e2e), "ttft_s": pcts(ttft)}


def latency(engine, dp_rank: int, runs: int):
    """Single-request end-to-end latency of the extraction path (idle engine)."""
    from ..service.extract import build_messages, parse_and_validate_response
    from ..utils import synth

    out, detail = [], []
    tok = engine.tokenizer
    for i in range(runs):
        d = synth.make_rfq(10_000_000 + dp_rank * 1000 + i)
        t0 = time.perf_counter()
        ids = tok.chat_ids(build_messages(d.text))
        s, = engine.generate([ids], engine.default_params(**synth.decode_hints(d)))
        r = parse_and_validate_response(engine.decode_text(s), "direct_text_input")
        out.append(time.perf_counter() - t0)
        ok = bool(r.get("success")) and "validation warnings" not in r.get("message", "")
        detail.append((s.num_generated, s.num_sampled, s.span().get("ttft_ms") or 0.0, out[-1],
                       ok))
    return out, detail


def single_stream(detail):
    """Single-request decode rates (Groq 350 tok/s per stream): output
    tokens/s after the first token, and the sampled (non-jump-forward) step rate."""
    if not detail:
        return None
    rates, steps, ttft = [], [], []
    for gen, sampled, ttft_ms, total, _ in detail:
        dec = max(total - ttft_ms / 1e3, 1e-6)
        rates.append(gen / dec)
        steps.append(sampled / dec)
        ttft.append(ttft_ms)
    return {"completion_tok_s_p50": round(statistics.median(rates), 1),
            "sampled_steps_per_s_p50": round(statistics.median(steps), 1),
            "ttft_ms_p50": round(statistics.median(ttft), 1),
            "baseline_decode_tok_s": 350.0,
            "valid": round(sum(d[4] for d in detail) / len(detail), 3)}
