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


def _postprocess_proc(flavor: str, path, in_q, out_q) -> None:
    """Spawned post-processing process: the service's extraction epilogue for every
    completed document of the stream -- detokenise, JSON recovery and pydantic
    validation (``parse_and_validate_response``, rfq_agent.py:185-206) -- off the
    engine process's GIL, as the HTTP layer does it off the engine thread.  Receives
    (key, output token ids), returns (key, validated, fallback).  ``None`` ends it.
    Imports no torch and never touches the GPU."""
    from ..engine.tokenizer import get_tokenizer
    from ..service.extract import parse_and_validate_response

    tok = get_tokenizer(flavor, path)
    while True:
        item = in_q.get()
        if item is None:
            return
        key, ids = item
        try:
            out = parse_and_validate_response(tok.decode(ids), "direct_text_input")
            ok = bool(out.get("success"))
            fb = ok and "validation warnings" in out.get("message", "")
        except Exception:  # noqa: BLE001 - a failed document is reported, never fatal
            ok, fb = False, False
        out_q.put((key, ok, fb))


class DocStream:
    """One replica's continuous document stream over an LLMEngine.

    A producer thread builds and tokenises prompts ahead of the engine (as the
    HTTP front-end does while the engine steps); the engine loop keeps
    ``in_flight`` documents admitted.  A document *completes* only when the
    service's post-processing has run on it: every finished sequence goes to a
    spawned post-processing process (detokenise -> JSON recovery -> pydantic
    validation, rfq_agent.py:185-206) and is counted when its validated result comes
    back.  ``run_until(n)`` steps the engine until ``n`` documents have completed in
    total and returns, leaving the in-flight documents in place for the next call.
    ``post="inline"`` validates in this process instead (tests, tools).
    """

    def __init__(self, engine, dp_rank: int, seed: int, in_flight: int,
                 formats: tuple | None = None, parse_procs: int = 4,
                 producer: str | None = None, overlap_admit: bool | None = None,
                 post: str | None = None):
        from ..engine.engine import short_gil_switch
        from ..service.extract import build_messages
        from ..service.prompt import register_prompt_prefix
        from ..utils import synth

        self._prev_switch = short_gil_switch()   # producer / post threads share the GIL
        self.engine = engine
        self.tok = engine.tokenizer
        register_prompt_prefix(self.tok)         # what the service's EngineBackend does
        self.in_flight = in_flight
        self.base = (seed * 7919 + dp_rank) * 1_000_003
        self.ready: queue.Queue = queue.Queue(maxsize=max(64, in_flight))
        self.stop = threading.Event()
        self.live = 0
        self.completed = 0                       # documents validated (post-processed)
        self.retired = 0                         # sequences the engine finished
        self.finished = []                       # sequences completed in the current window
        self.valid = 0                           # of ``finished``: validated, no fallback
        self.fallback = 0                        # validated through the G12 fallback
        self._pending: dict = {}                 # key -> finished Sequence awaiting post
        self._key = 0
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
        # post-processing: a spawned process (default) or inline
        self.post_mode = post or os.environ.get("RFQ_BENCH_POST", "process")
        self._post = None
        if self.post_mode == "process":
            import multiprocessing as mp

            ctx = mp.get_context("spawn")
            self._post_in, self._post_out = ctx.Queue(), ctx.Queue()
            self._post = ctx.Process(target=_postprocess_proc, name="bench-postprocess",
                                     args=(self.tok.flavor, getattr(self.tok, "path", None),
                                           self._post_in, self._post_out), daemon=True)
            self._post.start()

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

    def _submit_post(self, done) -> None:
        """Hand the engine's finished sequences to the post-processing stage."""
        for s in done:
            if self._post is None:
                from ..service.extract import parse_and_validate_response

                try:
                    out = parse_and_validate_response(self.engine.decode_text(s),
                                                      "direct_text_input")
                    ok = bool(out.get("success"))
                    fb = ok and "validation warnings" in out.get("message", "")
                except Exception:  # noqa: BLE001
                    ok, fb = False, False
                self._complete(s, ok, fb)
            else:
                self._key += 1
                self._pending[self._key] = s
                self._post_in.put((self._key, s.output_ids))

    def _complete(self, s, ok: bool, fb: bool) -> None:
        s.t_valid = time.perf_counter()
        s.valid = ok and not fb
        self.completed += 1
        self.valid += s.valid
        self.fallback += fb
        self.finished.append(s)

    def _collect(self, block: bool = False) -> None:
        """Count the documents whose post-processing has come back."""
        if self._post is None:
            return
        while self._pending:
            try:
                key, ok, fb = (self._post_out.get(timeout=1.0) if block
                               else self._post_out.get_nowait())
            except queue.Empty:
                if block and not self._post.is_alive():
                    raise RuntimeError(f"bench post-processing process exited "
                                       f"(code {self._post.exitcode})")
                return
            self._complete(self._pending.pop(key), ok, fb)
            block = False

    def run_until(self, target: int, deadline: float | None = None):
        """Step until ``target`` documents completed in total -- finished by the engine
        AND post-processed (detokenised, JSON-recovered, validated) -- or perf_counter
        passes ``deadline`` (then returns False)."""
        eng = self.engine
        runner = getattr(eng, "runner", None)
        hooked = [False]

        def admit():                     # runs while the step executes on the device
            hooked[0] = True
            self._top_up(block=False)
            self._collect()

        if runner is not None and self.overlap_admit:
            runner.busy_hook = admit
        try:
            while self.completed < target:
                if deadline is not None and time.perf_counter() > deadline:
                    return False
                self._collect()
                if self.completed >= target:
                    break
                # the documents retired by the previous step are replaced during this
                # step's device time (admit) instead of between steps, where the GPU
                # idles; only an empty engine (or a step that never launched) tops up here
                if not hooked[0] or not eng.has_work():
                    self._top_up(block=True)
                if not eng.has_work():
                    # everything in flight has left the engine: wait for its validation
                    self._collect(block=True)
                    continue
                hooked[0] = False
                done = eng.step()
                self.live -= len(done)
                self.retired += len(done)
                self._submit_post(done)
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
        if self._post is not None:
            self._post_in.put(None)
            self._post.join(timeout=10)
            if self._post.is_alive():
                self._post.terminate()
                self._post.join(timeout=5)
            self._post_in.cancel_join_thread()
            self._post_out.cancel_join_thread()
            self._post = None
        self._pending.clear()
        if self.engine.has_work():
            self.engine.abort_all("abort")
        self.live = 0
        import sys

        sys.setswitchinterval(self._prev_switch)

    def clear_window(self) -> None:
        """Start a new measurement window: forget the completed documents so far."""
        self.finished.clear()
        self.valid = 0
        self.fallback = 0

    def window_valid(self) -> float:
        """Share of the window's documents that validated on the schema's first path
        (no G12 fallback): the post-processing result of EVERY counted document."""
        return self.valid / max(1, len(self.finished))


def token_shape(seqs) -> dict:
    """Per-document token shape of a window's completions.  ``sampled_share`` = sampled /
    completion tokens (the reference's recorded completions: 0.524 on this grammar and
    tokenizer, tests/engine/test_decode_shape.py); ``completion_tokens_p50`` /
    ``sampled_tokens_p50`` compare with the recorded rows' 341.5 / 160."""
    import statistics

    from ..engine.grammar import PROFILE_SYNTHETIC, Limits

    n = max(1, len(seqs))
    gen = sum(s.num_generated for s in seqs)
    samp = sum(s.num_sampled for s in seqs)
    # documents whose part-count hint exceeds the SYNTHETIC item cap decode
    # fewer line items than they mention -- report how many
    cap = Limits.from_env().max_items
    synth = [s for s in seqs if s.params.profile == PROFILE_SYNTHETIC]
    trunc = sum(1 for s in synth if s.params.min_items > cap)
    return dict(
        items_hint_cap=cap,
        items_hint_truncated_share=trunc / max(1, len(synth)),
        items_hint_p50=statistics.median([s.params.min_items for s in synth]) if synth else 0,
        prompt_tokens=sum(s.prompt_len for s in seqs) / n,
        completion_tokens=gen / n,
        sampled_tokens=samp / n,
        sampled_share=samp / max(1, gen),
        completion_tokens_p50=statistics.median([s.num_generated for s in seqs]) if seqs else 0,
        sampled_tokens_p50=statistics.median([s.num_sampled for s in seqs]) if seqs else 0,
        prefix_hit_tokens=sum(s.prefix_hit_tokens for s in seqs) / n)


def validate(engine, seqs) -> dict:
    """Per-document token shape plus the share that validated (no G12 fallback).
    Sequences a DocStream already post-processed carry their result (``s.valid``);
    any other sequence is post-processed here like the service does
    (rfq_agent.py:185-206)."""
    from ..service.extract import parse_and_validate_response

    n = max(1, len(seqs))
    ok = 0
    for s in seqs:
        v = getattr(s, "valid", None)
        if v is None:
            out = parse_and_validate_response(engine.decode_text(s), "direct_text_input")
            v = bool(out.get("success")) and "validation warnings" not in out.get("message", "")
        ok += bool(v)
    return dict(token_shape(seqs), valid=ok / n)


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
    submission to the engine -> validated result (``e2e``: last token plus the
    post-processing stage when the stream ran it) and -> first sampled token
    (``ttft``), the server-side time a closed-loop client with this many requests
    in flight waits per document (the reference's only metric is per-request
    server time, /root/reference/app/rfq_agent.py:158-168; its LLM call times out
    at 30 s, rfq_agent.py:69)."""
    e2e = [getattr(s, "t_valid", 0.0) or s.t_finish for s in seqs]
    e2e = [t - s.t_arrival for t, s in zip(e2e, seqs) if t and s.t_arrival]
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


def reference_requests() -> list[dict]:
    """The reference's 14 recorded requests to llama3-70b-8192 (cache.db rows 1-14):
    system + user message exactly as the reference sent them, the document inside the
    user message (for the decoding hint), and Groq's usage telemetry."""
    import json
    import os

    with open(os.path.join(os.path.dirname(__file__), "reference_prompts.json")) as f:
        return json.load(f)["rows"]


def latency_reference(engine, runs: int = 14, deadline: float | None = None):
    """Single-request latency over a FIXED set: the reference's own recorded prompts
    (the same prefill Groq saw), decoded with the bench's hints (SYNTHETIC profile, item
    count from the document) so random-init weights produce the reference's decode shape.
    Deterministic per (weights seed, prompt), so two runs differ only by timing noise.
    Returns (latencies, detail) like ``latency``, plus the per-row (row, sampled steps,
    completion tokens) list."""
    from ..engine.grammar import PROFILE_SYNTHETIC
    from ..service.extract import parse_and_validate_response
    from ..service.hints import estimate_line_items

    out, detail, rows = [], [], []
    tok = engine.tokenizer
    for r in reference_requests()[:runs]:
        if deadline is not None and time.perf_counter() > deadline:
            break
        msgs = [{"role": "system", "content": r["system"]}, {"role": "user", "content": r["user"]}]
        t0 = time.perf_counter()
        ids = tok.chat_ids(msgs)
        params = engine.default_params(min_items=estimate_line_items(r["document"]),
                                       profile=PROFILE_SYNTHETIC)
        s, = engine.generate([ids], params)
        res = parse_and_validate_response(engine.decode_text(s), "direct_text_input")
        out.append(time.perf_counter() - t0)
        ok = bool(res.get("success")) and "validation warnings" not in res.get("message", "")
        detail.append((s.num_generated, s.num_sampled, s.span().get("ttft_ms") or 0.0, out[-1],
                       ok))
        rows.append((r["row"], s.num_sampled, s.num_generated, len(ids)))
    return out, detail, rows


PDF_SET_SEEDS = tuple(range(9000, 9012))


def pdf_set_requests(n: int = 12) -> list[dict]:
    """BASELINE config 4's prefill-heavy workload: a FIXED set of
    multi-page PDF RFQs (utils/synth.make_long_rfq, rendered by utils/docgen) whose
    parsed text (service/parser.py, the reference's file_parser.py contract) runs past the
    8,000-character cap of rfq_agent.py:147-149.  Returns the chat messages, the parsed
    text length, the page count and the item hint per document."""
    import os
    import tempfile
    from pathlib import Path

    from ..service.hints import estimate_line_items
    from ..service.parser import FileParser
    from ..service.prompt import build_messages, truncate
    from ..utils import docgen, synth

    out = []
    for seed in PDF_SET_SEEDS[:n]:
        d = synth.make_long_rfq(seed)
        p = Path(tempfile.gettempdir()) / f"rfq_pdfset_{os.getpid()}_{seed}.pdf"
        p.write_bytes(docgen.rfq_attachment(d, "pdf"))
        try:
            text = FileParser().parse_file(str(p))["raw_text"]
        finally:
            p.unlink(missing_ok=True)
        out.append({"seed": seed, "messages": build_messages(text), "chars": len(text),
                    "pages": text.count("=== Page "),
                    "min_items": estimate_line_items(truncate(text))})
    return out


def latency_pdf_set(engine, n: int = 12, deadline: float | None = None) -> dict | None:
    """Single-request latency over the fixed PDF set (one request at a time, bench hints
    as for the reference set): TTFT (prefill of ~2.3-2.6 K new tokens after the shared
    prefix) and end-to-end seconds per document."""
    from ..engine.grammar import PROFILE_SYNTHETIC
    from ..service.extract import parse_and_validate_response

    tok = engine.tokenizer
    rows = []
    for r in pdf_set_requests(n):
        if deadline is not None and time.perf_counter() > deadline:
            break
        t0 = time.perf_counter()
        ids = tok.chat_ids(r["messages"])
        params = engine.default_params(min_items=r["min_items"], profile=PROFILE_SYNTHETIC)
        s, = engine.generate([ids], params)
        res = parse_and_validate_response(engine.decode_text(s), "upload.pdf")
        dt = time.perf_counter() - t0
        rows.append({"seed": r["seed"], "pages": r["pages"], "chars": r["chars"],
                     "prompt_tokens": len(ids), "prefix_hit": s.span().get("prefix_hit"),
                     "ttft_ms": round(s.span().get("ttft_ms") or 0.0, 1),
                     "sampled": s.num_sampled, "tokens": s.num_generated, "s": round(dt, 3),
                     "valid": bool(res.get("success"))})
    if not rows:
        return None
    med = lambda k: statistics.median(x[k] for x in rows)  # noqa: E731
    return {"set": "multi-page PDF RFQs past the 8,000-char cap (synth.make_long_rfq seeds "
                   f"{PDF_SET_SEEDS[0]}-{PDF_SET_SEEDS[-1]}), parsed by service/parser.py",
            "docs": len(rows), "pages_p50": med("pages"), "chars_p50": med("chars"),
            "prompt_tokens_p50": med("prompt_tokens"), "ttft_ms_p50": med("ttft_ms"),
            "e2e_s_p50": round(med("s"), 4), "sampled_steps_p50": med("sampled"),
            "valid": round(sum(x["valid"] for x in rows) / len(rows), 3), "per_doc": rows}


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
