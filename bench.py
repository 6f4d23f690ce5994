#!/usr/bin/env python
"""RFQ extraction benchmark — BASELINE.json metric:
"RFQ docs/sec whole-node + p50 /parse-text/ latency, Llama-3-8B TP=1 and 70B TP=8".

One process per GPU.  Each TP group is one engine replica (default Llama-3-8B,
TP=1 => DP=N replicas; weak scaling: every replica serves the same stream).

Workload: every replica serves ONE continuous stream of synthetic RFQ documents
through the full extraction path — prompt build (8,000-char truncation +
byte-identical template, rfq_agent.py:147-151) -> Llama-3 chat tokenisation ->
continuous-batching engine (chunked prefill, prefix cache, grammar-constrained
Gumbel sampling at T=0.1, jump-forward, hipGraph decode) -> detokenise -> JSON
recovery + pydantic validation (rfq_agent.py:185-206).  ``--max-num-seqs``
documents are kept in flight; a finished document is immediately replaced by
the next one (production continuous batching).

A *step* is one fixed slice of that stream: ``--docs-per-step`` completed
documents per replica.  ``--warmup`` steps absorb the ramp-up (first prefill
wave, survivorship bias of the in-flight mix); then exactly ``--steps`` steps
are timed, bracketed by barrier + ``torch.cuda.synchronize()`` on both sides,
and the MAX over ranks is reported.  Documents count only when they complete
inside the timed window (the stream's in-flight state carries across the
boundaries, as in a running server).  After the timed region the in-flight
remainder is aborted and the single-request p50 latency of the same path (the
reference's 0.883 s p50 Groq server time) is measured on replica 0.

Weights are random-init (no checkpoints offline); documents are synthetic with
the reference's length distribution.  ``--gpus N`` without a
torchrun environment re-launches this script under torch.distributed.run with N
ranks (before any GPU call).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

from replisense_rfq_amd.benchmarks.stream import (DocStream, latency, latency_pdf_set,
                                                  latency_reference, loaded_latency,
                                                  single_stream as _single_stream, token_shape,
                                                  validate)

BASELINE_P50_S = 0.883          # Groq llama3-70b p50 server time per request
REFERENCE_SAMPLED_STEPS_P50 = 160   # the reference's recorded completions (r5_decode_shape.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--docs-per-step", type=int, default=512,
                    help="completed documents per replica that make one step")
    ap.add_argument("--max-num-seqs", type=int, default=1536,
                    help="documents in flight per replica: the headline operating point is the "
                         "deepest whose loaded p99 stays inside the service's 30 s request "
                         "deadline (profiles/r3_depth_sweep.md)")
    ap.add_argument("--latency-slo", type=float, default=30.0,
                    help="per-document deadline the loaded p99 is checked against "
                         "(rfq_agent.py:69 timeout; utils/config.py request_timeout_s)")
    ap.add_argument("--latency-runs", type=int, default=15)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-jump-forward", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--prefill-chunk", type=int, default=16384)
    ap.add_argument("--kv-fraction", type=float, default=0.85,
                    help="fraction of free HBM for the paged KV pool (288 GB per MI355X)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--time-budget", type=float, default=0.0,
                    help="seconds; if > 0 the latency phase is skipped once this much wall "
                         "time has passed (the JSON line is always printed)")
    ap.add_argument("--tp-latency-model", default="auto",
                    help="after the timed region, serve single requests of this model with "
                         "ONE TP group over all N ranks (BASELINE config 4: 70B TP=8). "
                         "'auto' = llama3-70b on the driver's 8-GPU run of the default "
                         "8B DP bench; 'none' = off")
    ap.add_argument("--phases", default="auto",
                    help="extra phases after the timed window: comma list of http, mixtral, "
                         "70b; 'auto' = all on the 1-GPU run of the 8B bench, 'none' = off")
    ap.add_argument("--phase-budget", type=float, default=310.0,
                    help="seconds for all extra phases together (each is bounded; a watchdog "
                         "prints the JSON line if they overrun)")
    ap.add_argument("--http-open-rate", type=float, default=0.0,
                    help="open-loop HTTP phase: offered requests/s (0 = 90 %% of the "
                         "timed window's docs/s per replica)")
    ap.add_argument("--http-open-warm", type=float, default=20.0)
    ap.add_argument("--http-open-measure", type=float, default=30.0)
    ap.add_argument("--http-open-burst", type=float, default=0.75,
                    help="open-loop HTTP phase: initial burst as a fraction of the "
                         "in-flight depth (starts the queue near its steady state)")
    ap.add_argument("--http-idle-requests", type=int, default=20,
                    help="open-loop HTTP phase: idle single /parse-text/ requests sent one at "
                         "a time after the window (the metric's p50 /parse-text/ latency)")
    ap.add_argument("--http-docs", type=int, default=512)
    ap.add_argument("--http-clients", type=int, default=64)
    ap.add_argument("--depth-in-flight", type=int, default=160,
                    help="latency-bounded depth phase: documents in flight (loaded p50 ~2 s)")
    ap.add_argument("--depth-docs", type=int, default=640)
    ap.add_argument("--mixtral-model", default="mixtral-8x7b")
    ap.add_argument("--mixtral-in-flight", type=int, default=768)
    ap.add_argument("--mixtral-warm", type=int, default=512)
    ap.add_argument("--mixtral-docs", type=int, default=1024)
    ap.add_argument("--big-model", default="llama3-70b")
    ap.add_argument("--big-latency-runs", type=int, default=14,
                    help="70B phase: single requests over the reference's 14 recorded prompts "
                         "(a fixed set; fewer if the phase budget runs out)")
    ap.add_argument("--tp-latency-runs", type=int, default=14)
    ap.add_argument("--pdf-set", type=int, default=12,
                    help="multi-page PDF RFQs past the 8,000-char cap run one at a time in "
                         "the 70B phase (BASELINE config 4, prefill-heavy); 0 = off")
    ap.add_argument("--tp-docs", type=int, default=256,
                    help="TP phase: documents timed in a continuous stream (0 = skip)")
    ap.add_argument("--tp-in-flight", type=int, default=128,
                    help="TP phase: documents in flight during that stream")
    ap.add_argument("--tp-latency-budget", type=float, default=240.0,
                    help="seconds for the whole TP latency phase; a watchdog prints the "
                         "JSON line (phase marked timeout) and ends every rank past it")
    return ap.parse_args()


def _tp_latency_model(args, world: int) -> str | None:
    m = os.environ.get("RFQ_BENCH_TP_LATENCY", args.tp_latency_model)
    if m in ("", "none", "0"):
        return None
    if m == "auto":
        return "llama3-70b" if (world == 8 and args.tp == 1 and args.model == "llama3-8b"
                                and args.latency_runs > 0) else None
    return m


def _phase_list(args, world: int) -> list:
    """Extra phases after the timed window (benchmarks/phases.py).  'auto': on the
    driver's 1-GPU run of the default 8B bench, all three."""
    v = args.phases
    if v in ("", "none", "0"):
        return []
    if v == "auto":
        return (["http_open", "http", "depth", "mixtral", "70b"]
                if (world == 1 and args.tp == 1 and args.model == "llama3-8b") else [])
    return [p for p in v.split(",") if p]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _self_launch(args) -> int:
    """`bench.py --gpus N` outside torchrun: start N ranks under torch.distributed.run
    as a child process (never exec: no GPU has been touched in this process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def _gemm_plan_summary() -> dict:
    """Which large-M projections the start-up plan put on the hand-written MFMA GEMM
    (ops/autotune.py tune_split): buckets won per projection."""
    try:
        from replisense_rfq_amd.ops.autotune import SPLIT_REPORT
    except Exception:  # noqa: BLE001
        return {}
    return {r[0].split(":", 1)[1]: r[5] for r in SPLIT_REPORT
            if r[0].startswith("dense:") and isinstance(r[5], str) and "buckets" in r[5]}


def _host_timers(engine) -> dict:
    st = engine.runner.stats
    return {"pack_s": st.get("pack_s", 0.0), "launch_s": st.get("launch_s", 0.0),
            "overlap_s": st.get("overlap_s", 0.0),
            "wait_s": st.get("wait_s", 0.0), "post_s": engine.timers.get("post_s", 0.0),
            "execute_s": engine.timers.get("execute_s", 0.0)}


class _Heartbeat:
    """Rank 0 prints a progress line to stderr every ``period`` seconds, so a long
    silent phase (engine init, the timed window, the TP phase) never looks hung to
    a supervisor watching the output.  stdout keeps exactly the one JSON line."""

    def __init__(self, t_start: float, period: float = 30.0):
        self.t_start = t_start
        self.phase = "init"
        self.stream = None
        self.stop = threading.Event()
        self.thread = threading.Thread(target=self._run, args=(period,), daemon=True)
        self.thread.start()

    def _run(self, period: float):
        while not self.stop.wait(period):
            done = self.stream.completed if self.stream is not None else 0
            print(f"[bench] t={time.perf_counter() - self.t_start:.0f}s phase={self.phase} "
                  f"docs_completed={done}", file=sys.stderr, flush=True)


class _Emitter:
    """Rank 0's ONE JSON line, printed exactly once: by the main thread at the end,
    or by the TP-phase watchdog if that phase overruns its budget."""

    def __init__(self):
        self.lock = threading.Lock()
        self.done = False

    def emit(self, out: dict) -> None:
        with self.lock:
            if not self.done:
                print(json.dumps(out), flush=True)
                self.done = True


def tp_latency_phase(model: str, args, wctx, rank: int, on_timeout) -> dict | None:
    """BASELINE config 4 on the same node: one TP group spanning all N ranks serves
    ``model`` (default Llama-3-70B at TP=8: RCCL + the custom xGMI all-reduce fused
    with the residual-add RMSNorm, hipGraph decode).  Runs after the timed region (the
    8B DP engine is freed first), so it never touches the docs/s measurement.

      1. single /parse-text/-path requests on the idle group (p50, decode rates);
      2. ``--tp-docs`` documents of a continuous stream with ``--tp-in-flight`` in
         flight, after a warm-up of half that many (docs/s of the TP group).

    Bounded: a watchdog on every rank ends the process after ``--tp-latency-budget``
    seconds (rank 0 first prints the JSON line with whatever the phase measured so
    far, marked ``timeout``); an exception on any rank is reported instead of failing
    the whole bench.  A custom all-reduce flag timeout on any rank (never seen on this
    node's xGMI before the run) re-forms the group once on RCCL all-reduces and measures
    again; ``car_fallback`` says why."""
    import gc

    import torch

    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.utils.config import EngineConfig
    from replisense_rfq_amd.utils.faults import CustomAllReduceError

    res = {"model": model, "parallelism": f"tp{wctx.world}"}
    timer = threading.Timer(args.tp_latency_budget, lambda: on_timeout(res))
    timer.daemon = True
    timer.start()
    t0 = time.perf_counter()
    for attempt in range(2):
        car_err = None
        eng = None
        try:
            nseq = max(8, args.tp_in_flight)
            buckets = tuple(b for b in (1, 2, 4, 8, 16, 32, 64, 128, 256) if b <= nseq)
            cfg = EngineConfig.from_env(
                model=model, tp=wctx.world, seed=args.seed, max_num_seqs=nseq,
                max_kv_blocks=max(4096, nseq * 48), graph_buckets=buckets,
                use_graphs=not args.no_graphs, jump_forward=not args.no_jump_forward,
                prefix_cache=not args.no_prefix_cache)
            if attempt:
                cfg.custom_allreduce = False
            eng = LLMEngine(cfg, tp=wctx)
            res["init_s"] = round(time.perf_counter() - t0, 1)
            res["custom_allreduce"] = wctx.car is not None
            # why the custom xGMI all-reduce is (not) in use: "ok", "set-up failed ...",
            # "self-test failed ...", a runtime fallback, or off on CPU / by config
            res["car_status"] = wctx.car_status or ("ok" if wctx.car is not None else
                                                    "off" if not cfg.custom_allreduce else
                                                    "not enabled on this device")
            if wctx.rank == 0:
                try:
                    # the same FIXED set as the one-GPU 70B phase: the
                    # reference's 14 recorded prompts, per-row sampled steps reported
                    lat, detail, rows = latency_reference(eng, args.tp_latency_runs)
                    res["latency_set"] = "reference prompts (cache.db rows 1-14), bench hints"
                    res["p50_parse_text_latency_s"] = round(statistics.median(lat), 4)
                    res["latency_vs_baseline_p50"] = round(BASELINE_P50_S / statistics.median(lat), 2)
                    ss = res["single_stream"] = _single_stream(detail)
                    res["runs"] = len(lat)
                    res["sampled_steps_p50"] = statistics.median(r[1] for r in rows)
                    if ss and ss.get("sampled_steps_per_s_p50"):    # see phases.model_phase
                        res["p50_at_reference_steps_s"] = round(
                            ss["ttft_ms_p50"] / 1e3 + REFERENCE_SAMPLED_STEPS_P50
                            / ss["sampled_steps_per_s_p50"], 4)
                    res["per_row"] = [{"row": a, "sampled": b, "tokens": c, "prompt": d,
                                       "s": round(t, 3)} for (a, b, c, d), t in zip(rows, lat)]
                    if args.pdf_set and time.perf_counter() - t0 < args.tp_latency_budget - 90:
                        # BASELINE config 4's prefill-heavy documents on the real TP group
                        # (the one-GPU 70B phase runs the same fixed set at TP = 1)
                        res["pdf_set"] = latency_pdf_set(
                            eng, args.pdf_set, deadline=time.perf_counter() + 60.0)
                    if args.tp_docs > 0:
                        stream = DocStream(eng, 0, args.seed + 1, args.tp_in_flight)
                        warm = max(1, args.tp_in_flight // 2)
                        stream.run_until(warm)
                        stream.clear_window()
                        if eng.device.type == "cuda":
                            torch.cuda.synchronize()
                        t1 = time.perf_counter()
                        stream.run_until(warm + args.tp_docs)
                        if eng.device.type == "cuda":
                            torch.cuda.synchronize()
                        dt = time.perf_counter() - t1
                        res["docs_per_s"] = round(args.tp_docs / dt, 3)
                        res["docs"], res["in_flight"] = args.tp_docs, args.tp_in_flight
                        res["per_doc"] = {k: round(v, 3)
                                          for k, v in validate(eng, stream.finished).items()}
                        stream.close()
                finally:
                    if wctx.enabled:
                        eng.shutdown()
            elif eng.worker_loop(tolerate_car_errors=True):
                car_err = "custom all-reduce flag timeouts on a follower rank"
            if eng.device.type == "cuda":
                torch.cuda.synchronize()
            res["status"] = "ok"
        except CustomAllReduceError as e:
            car_err = f"{type(e).__name__}: {str(e)[:200]}"
            res["status"] = f"error: {car_err}"
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line, never fatal
            res["status"] = f"error: {type(e).__name__}: {str(e)[:300]}"
        eng = None
        if attempt == 0 and wctx.enabled and _any_rank(wctx, car_err is not None):
            # a custom all-reduce flag timed out on some rank (its sums may be stale):
            # every rank drops the custom kernels and the group measures again on RCCL
            note = car_err or "custom all-reduce flag timeouts on a peer rank"
            res.clear()
            res.update({"model": model, "parallelism": f"tp{wctx.world}",
                        "car_fallback": note})
            if wctx.car is not None:
                wctx.car.close()
                wctx.car = None
            wctx.car_status = "runtime flag timeouts: group re-formed on RCCL"
            gc.collect()
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
            continue
        break
    timer.cancel()
    res["phase_s"] = round(time.perf_counter() - t0, 1)
    return res


def _any_rank(wctx, flag: bool) -> bool:
    """True on every rank of the TP group if ``flag`` is set on any of them."""
    import torch
    import torch.distributed as dist

    dev = "cuda" if dist.get_backend(wctx.group) == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=wctx.group)
    return int(t.item()) == 1


def main():
    args = parse()
    t_start = time.perf_counter()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args))

    # before anything touches HIP: this rank (and the producer / post-processing
    # processes it spawns) runs on its GPU's NUMA-local cores
    from replisense_rfq_amd.utils.affinity import pin_to_gpu

    affinity = pin_to_gpu(int(os.environ.get("LOCAL_RANK", "0")))

    import torch
    import torch.distributed as dist

    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.parallel.tp import init_distributed, split_groups
    from replisense_rfq_amd.utils.config import EngineConfig

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    wctx = init_distributed()
    tp, dp_rank, dp_world = split_groups(args.tp) if world > 1 else (wctx, 0, 1)
    cfg = EngineConfig.from_env(
        model=args.model, tp=args.tp, seed=args.seed, max_num_seqs=args.max_num_seqs,
        use_graphs=not args.no_graphs, jump_forward=not args.no_jump_forward,
        prefix_cache=not args.no_prefix_cache, max_batched_tokens=args.prefill_chunk,
        kv_fraction=args.kv_fraction)
    t_init = time.perf_counter()
    hb = _Heartbeat(t_start) if rank == 0 else None

    def mark(name):
        if hb is not None:
            hb.phase = name

    engine = LLMEngine(cfg, tp=tp)
    t_init = time.perf_counter() - t_init
    on_gpu = engine.device.type == "cuda"

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def phase(fn):
        """TP rank 0 drives `fn`; the other ranks of its group mirror the steps
        until rank 0 releases them (engine.shutdown)."""
        if tp.rank == 0:
            r = fn()
            if tp.enabled:
                engine.shutdown()
            return r
        engine.worker_loop()
        return None

    stream = DocStream(engine, dp_rank, args.seed, args.max_num_seqs) if tp.rank == 0 else None
    per = args.docs_per_step
    if hb is not None:
        hb.stream = stream
    mark("warmup")
    phase(lambda: stream.run_until(args.warmup * per))
    if stream is not None:
        stream.clear_window()
    steps0 = engine.num_steps
    gsteps0 = engine.stats().get("graph_steps", 0)
    host0 = _host_timers(engine)
    barrier()
    sync()
    mark("timed")
    t0 = time.perf_counter()
    phase(lambda: stream.run_until((args.warmup + args.steps) * per))
    sync()
    barrier()
    dt = time.perf_counter() - t0
    steps_timed = engine.num_steps - steps0
    gsteps_timed = engine.stats().get("graph_steps", 0) - gsteps0
    host = {k: round(v - host0[k], 3) for k, v in _host_timers(engine).items()}
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=engine.device if on_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    shape, loaded = {}, {"e2e_s": None, "ttft_s": None}
    done_in_window = 0
    post = {}
    if stream is not None:
        done_in_window = stream.completed - args.warmup * per
        # every document counted in the window was post-processed inside it (detokenise
        # -> JSON recovery -> pydantic validation, rfq_agent.py:185-206)
        shape = dict(token_shape(stream.finished), valid=stream.window_valid())
        post = {"mode": stream.post_mode, "validated": len(stream.finished),
                "fallback": stream.fallback,
                "failed": len(stream.finished) - stream.valid - stream.fallback}
        loaded = loaded_latency(stream.finished)
        stream.close()
    stats = engine.stats()

    lat, detail = [], []
    run_lat = bool(args.latency_runs) and (
        not args.time_budget or time.perf_counter() - t_start < args.time_budget)
    if world > 1:                 # every rank must take the same branch
        f = torch.tensor([int(run_lat)], device=engine.device if on_gpu else "cpu")
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        run_lat = bool(f.item())
    mark("latency")
    if run_lat and dp_rank == 0:
        r = phase(lambda: latency(engine, dp_rank, args.latency_runs))
        if r is not None:
            lat, detail = r
    barrier()

    out = None
    if rank == 0:
        docs = per * dp_world * args.steps
        value = docs / dt
        p50 = statistics.median(lat) if lat else None
        out = {
            "metric": "rfq_docs_per_sec_whole_node",
            "value": round(value, 3),
            "unit": "docs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.md has no docs/s number (the reference never measured one)
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic RFQ documents (reference length distribution), random-init weights",
            "config": {"model": args.model, "global_batch": per * dp_world,
                       "seq_len": int(shape.get("prompt_tokens", 0) +
                                      shape.get("completion_tokens", 0)),
                       "parallelism": f"dp{dp_world}" + (f"-tp{args.tp}" if args.tp > 1 else ""),
                       "step": f"{per} completed documents per replica of a continuous stream",
                       "in_flight_per_replica": args.max_num_seqs,
                       "temperature": cfg.temperature, "grammar": cfg.grammar,
                       "profile": "synthetic", "decode_hints": True,
                       "jump_forward": cfg.jump_forward,
                       # hipGraphs are captured for decode-only steps of up to the largest
                       # bucket of sequences; the count says how many timed steps used one
                       "graphs": (f"{gsteps_timed} of {steps_timed} timed steps (captured for "
                                  f"decode-only steps <= {max(cfg.graph_buckets)} sequences)"
                                  if cfg.use_graphs else "off"),
                       # prompts built + tokenised in a spawned process (benchmarks.stream)
                       "producer": os.environ.get("RFQ_BENCH_PRODUCER", "process"),
                       "admit": ("during step" if os.environ.get("RFQ_BENCH_OVERLAP_ADMIT", "1")
                                 != "0" else "between steps"),
                       # a document counts once its post-processing (detokenise, JSON
                       # recovery, pydantic validation) has run inside the timed window
                       "counted": "validated in window"},
            "postprocess": post,
            # latency under load of the documents completed in the timed window
            # (submission -> last token, closed loop at in_flight_per_replica)
            "loaded_latency_s": loaded["e2e_s"],
            "loaded_ttft_s": loaded["ttft_s"],
            "latency_slo_s": args.latency_slo,
            "slo_met_p99": bool(loaded["e2e_s"] and loaded["e2e_s"]["p99"] <= args.latency_slo),
            # replaced by the HTTP measurement of the http_open phase when it runs
            "p50_parse_text_latency_s": round(p50, 4) if p50 is not None else None,
            "p50_parse_text_source": "engine.generate on the service path (no HTTP hop)",
            "p50_engine_latency_s": round(p50, 4) if p50 is not None else None,
            "single_stream": _single_stream(detail),
            "latency_vs_baseline_p50": round(BASELINE_P50_S / p50, 2) if p50 else None,
            "baseline": "BASELINE.md publishes no docs/s (vs_baseline null).  "
                        "latency_vs_baseline_p50 = 0.883 s / p50 of an idle single request: "
                        "Llama-3-8B here vs the reference's Groq llama3-70b-8192 (a different "
                        "model); the same-model (70B) comparison is in the 70b phase",
            "per_doc": {k: round(v, 3) for k, v in shape.items()},
            "engine": {"init_s": round(t_init, 1), "graph_capture_s": round(engine.capture_s, 1),
                       "gemm_tune_s": round(engine.tune_s, 1),
                       "gemm_plan": _gemm_plan_summary(),
                       # decode-tiled projection weights: extra copy (bytes) or in place
                       "tiled_weights": getattr(engine.model, "tiled_plan", None) or "off",
                       "timed_engine_steps": steps_timed,
                       "docs_completed_in_window_rank0": done_in_window,
                       "graph_steps": stats.get("graph_steps"), "steps": stats.get("steps"),
                       # host seconds inside the timed window (rank 0): scheduler pack,
                       # forward launch, device wait, post-processing (grammar, retire)
                       "host_s": host,
                       "kv_blocks": stats.get("blocks"), "preempted": stats.get("preempted"),
                       "affinity": affinity,
                       "wall_s": round(time.perf_counter() - t_start, 1)},
        }

    emitter = _Emitter()
    phases = _phase_list(args, world)
    if phases:
        # BASELINE configs 3 and 5 and the reference's own model, driver-clocked in the
        # same JSON line (world == 1: every rank is rank 0)
        from replisense_rfq_amd.benchmarks import phases as ph

        out["phases"] = {}
        t_ph = time.perf_counter()

        def left():
            return args.phase_budget - (time.perf_counter() - t_ph)

        def on_overrun():
            out["phases"]["status"] = f"timeout after {args.phase_budget:.0f} s"
            out["engine"]["wall_s"] = round(time.perf_counter() - t_start, 1)
            emitter.emit(out)
            os._exit(0)

        guard = threading.Timer(args.phase_budget + 120.0, on_overrun)
        guard.daemon = True
        guard.start()
        if "http_open" in phases:
            mark("phase:http_open")
            rate = args.http_open_rate or 0.9 * out["value"] / max(1, dp_world)
            r = ph.http_open_loop_phase(
                engine, rate=rate, warm_s=args.http_open_warm,
                measure_s=args.http_open_measure,
                budget_s=min(args.http_open_warm + args.http_open_measure + 60.0, left()),
                seed=args.seed, burst_depth=int(args.http_open_burst * args.max_num_seqs),
                idle_requests=args.http_idle_requests)
            r["engine_docs_per_s"] = round(out["value"] / max(1, dp_world), 3)
            if r.get("docs_per_s"):
                r["http_vs_engine"] = round(r["docs_per_s"] / r["engine_docs_per_s"], 3)
            out["phases"]["http_open_loop"] = r
            idle = r.get("idle") or {}
            if idle.get("client_p50_s"):
                # the metric's p50 /parse-text/ latency, through
                # /parse-text/ (client clock) and the service's X-Process-Time header
                out["p50_parse_text_latency_s"] = idle["client_p50_s"]
                out["p50_x_process_time_s"] = idle["x_process_time_p50_s"]
                out["p50_parse_text_source"] = (
                    f"HTTP POST /parse-text/ through uvicorn (api process + engine process), "
                    f"{idle['valid']} idle single requests, client clock")
        if "http" in phases:
            mark("phase:http")
            out["phases"]["http_upload"] = ph.http_upload_phase(
                engine, n_docs=args.http_docs, clients=args.http_clients,
                budget_s=min(120.0, left()), seed=args.seed)
        if "depth" in phases:
            mark("phase:depth")
            d = ph.depth_phase(engine, in_flight=args.depth_in_flight,
                               warm_docs=args.depth_in_flight, docs=args.depth_docs,
                               budget_s=min(60.0, left()), seed=args.seed)
            d["headline_in_flight"] = args.max_num_seqs
            out["phases"]["latency_bounded_depth"] = d
        import gc

        if hb is not None:
            hb.stream = None
        del stream, engine
        gc.collect()
        if on_gpu:
            torch.cuda.empty_cache()
        if "mixtral" in phases and left() > 60:
            mark("phase:mixtral")
            out["phases"]["mixtral"] = ph.model_phase(
                args.mixtral_model, seed=args.seed, in_flight=args.mixtral_in_flight,
                warm_docs=args.mixtral_warm, docs=args.mixtral_docs, formats=("pdf", "xlsx"),
                budget_s=min(160.0, left() - 120 if "70b" in phases else left()),
                max_batched_tokens=args.prefill_chunk)
        if "70b" in phases and left() > 30:
            mark("phase:70b")
            out["phases"]["llama3_70b"] = ph.model_phase(
                args.big_model, seed=args.seed, latency_runs=args.big_latency_runs,
                budget_s=left(), in_flight=8, reference_set=True, pdf_set=args.pdf_set,
                # one request at a time: decode graphs / start-up plans for one sequence
                # (M = 1..8 with jump-forward extends) -- the 64-row plans took 86 s
                graph_buckets=(1,),
                # 14 prompts of <= 640 new tokens each: their prefills run on the library
                # GEMMs without the large-M split plans (the plans' start-up timing of
                # the 70B projections took 65 s of this phase for 14 prefill steps)
                max_batched_tokens=min(args.prefill_chunk, 1024), gemm_split=False)
        guard.cancel()
        out["phases"]["phase_s"] = round(time.perf_counter() - t_ph, 1)
        out["engine"]["wall_s"] = round(time.perf_counter() - t_start, 1)
        emitter.emit(out)
        return
    tpl = _tp_latency_model(args, world)
    if tpl is not None:
        # free the DP replica (weights, KV pool, graph pools) before the TP group loads
        import gc

        if hb is not None:
            hb.stream = None          # the heartbeat must not keep the DP engine alive
        del stream, engine
        gc.collect()
        if on_gpu:
            torch.cuda.empty_cache()
        barrier()

        def on_timeout(partial):
            if out is not None:
                emitter.emit(dict(out, tp_latency=dict(
                    partial, status=f"timeout after {args.tp_latency_budget:.0f} s")))
            os._exit(0)

        mark(f"tp_latency:{tpl}")
        res = tp_latency_phase(tpl, args, wctx, rank, on_timeout)
        if out is not None:
            out["tp_latency"] = res
            out["engine"]["wall_s"] = round(time.perf_counter() - t_start, 1)
        if res["status"] != "ok":
            # the other ranks may be stuck mirroring a step that never comes: report
            # and leave (their own watchdogs end them)
            if out is not None:
                emitter.emit(out)
            sys.stdout.flush()
            os._exit(0)
    if out is not None:
        emitter.emit(out)
    if world > 1:
        if tpl is not None:
            # a peer whose TP phase failed has already left: never wait on it forever
            guard = threading.Timer(60.0, lambda: os._exit(0))
            guard.daemon = True
            guard.start()
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
