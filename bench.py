#!/usr/bin/env python
"""RFQ extraction benchmark — BASELINE.json metric:
"RFQ docs/sec whole-node + p50 /parse-text/ latency, Llama-3-8B TP=1 and 70B TP=8".

One process per GPU (torchrun).  Each TP group is one engine replica (default
Llama-3-8B, TP=1 => DP=N replicas, weak scaling: every replica processes the same
number of documents per step).  A *step* = one wave of ``--docs-per-step``
synthetic RFQ documents per replica pushed through the full extraction path:
prompt build (8,000-char truncation + byte-identical template) -> Llama-3 chat
tokenisation -> continuous-batching engine (chunked prefill, prefix cache,
grammar-constrained Gumbel sampling at T=0.1, jump-forward, hipGraph decode) ->
detokenise -> JSON recovery + pydantic validation (rfq_agent.py:185-206).
Weights are random-init (no checkpoints offline); documents are synthetic with
the reference's length distribution.

Timed region: exactly --steps steps (= steps x docs-per-step documents per replica),
bracketed by barrier + cuda synchronize on both sides; the max over ranks is
reported.  Default ``--mode stream`` feeds those documents as one continuous
stream (at most --max-num-seqs in flight, new documents admitted as others
finish — production continuous batching); ``--mode wave`` drains each step's
batch before starting the next.  After it, the single-request p50
latency of the same path (the reference's 0.883 s p50 Groq server time,
BASELINE.md) is measured on replica 0.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import statistics
import sys
import threading
import time

import torch
import torch.distributed as dist

from replisense_rfq_amd.engine.engine import LLMEngine
from replisense_rfq_amd.parallel.tp import init_distributed, split_groups
from replisense_rfq_amd.service.extract import build_messages, parse_and_validate_response
from replisense_rfq_amd.service.hints import estimate_line_items
from replisense_rfq_amd.service.prompt import register_prompt_prefix
from replisense_rfq_amd.utils import synth
from replisense_rfq_amd.utils.config import EngineConfig

BASELINE_P50_S = 0.883          # Groq llama3-70b p50 server time per request
BASELINE_DOCS_PER_S = 1.0 / BASELINE_P50_S


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--docs-per-step", type=int, default=3072)
    ap.add_argument("--max-num-seqs", type=int, default=3072)
    ap.add_argument("--latency-runs", type=int, default=15)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-jump-forward", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--prefill-chunk", type=int, default=16384)
    ap.add_argument("--kv-fraction", type=float, default=0.85,
                    help="fraction of free HBM for the paged KV pool (288 GB per MI355X)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--mode", choices=("stream", "wave"), default="stream",
                    help="stream: the K*docs-per-step documents of the timed region are one "
                         "continuous-batching stream (max-num-seqs in flight); wave: each step "
                         "is a closed batch that drains before the next starts")
    return ap.parse_args()


class Replica:
    def __init__(self, engine: LLMEngine, dp_rank: int, seed: int):
        self.engine = engine
        self.tok = engine.tokenizer
        register_prompt_prefix(self.tok)         # what the service's EngineBackend does
        self.dp_rank = dp_rank
        self.seed = seed
        self.wave = 0
        self.last = {}

    def docs(self, n: int):
        base = (self.seed * 7919 + self.dp_rank) * 1_000_003 + self.wave * 10_007
        self.wave += 1
        return [synth.make_rfq(base + i) for i in range(n)]

    def run_wave(self, n: int, waves: int = 1) -> int:
        """Push n * waves documents through the service path.  As in the HTTP server
        (requests are tokenised by the API front-end while the engine steps), a
        producer thread builds and tokenises the prompts and the engine admits each
        one as soon as it is ready, so prompt preparation overlaps GPU execution."""
        t0 = time.perf_counter()
        docs = [d for _ in range(waves) for d in self.docs(n)]
        n = len(docs)
        eng = self.engine
        wave = self.wave
        ready: queue.SimpleQueue = queue.SimpleQueue()
        prep = {}

        def produce():
            ts = time.perf_counter()
            for i, d in enumerate(docs):
                ids = self.tok.chat_ids(build_messages(d.text))
                ready.put((ids, eng.default_params(seed=(wave * 100_003 + i) & 0xFFFFFF,
                                                   min_items=estimate_line_items(d.text))))
            prep["s"] = time.perf_counter() - ts
            ready.put(None)

        old_switch = sys.getswitchinterval()
        sys.setswitchinterval(2e-4)        # the step loop re-takes the GIL promptly
        th = threading.Thread(target=produce, name="bench-tokenize", daemon=True)
        th.start()
        seqs, producing = [], True
        try:
            while True:
                while producing:
                    try:
                        item = ready.get() if not eng.has_work() else ready.get_nowait()
                    except queue.Empty:
                        break
                    if item is None:
                        producing = False
                    else:
                        seqs.append(eng.add_request(*item))
                if eng.has_work():
                    eng.step()
                elif not producing:
                    break
        finally:
            sys.setswitchinterval(old_switch)
            th.join()
        t1 = t0 + prep.get("s", 0.0)
        t2 = time.perf_counter()
        ok = 0
        for s in seqs:
            out = parse_and_validate_response(eng.decode_text(s), "direct_text_input")
            ok += bool(out.get("success")) and "validation warnings" not in out.get("message", "")
        eng.runner.tp.enabled and eng.shutdown()
        self.phases = {"prep_s_overlapped": round(t1 - t0, 2), "engine_s": round(t2 - t0, 2),
                       "post_s": round(time.perf_counter() - t2, 2)}
        self.last = dict(
            prompt_tokens=sum(s.prompt_len for s in seqs) / n,
            completion_tokens=sum(s.num_generated for s in seqs) / n,
            sampled_tokens=sum(s.num_sampled for s in seqs) / n,
            prefix_hit_tokens=sum(s.prefix_hit_tokens for s in seqs) / n,
            valid=ok / n)
        return ok

    def latency(self, runs: int) -> list[float]:
        out = []
        self.lat_detail = []
        eng = self.engine
        for i in range(runs):
            d = synth.make_rfq(10_000_000 + self.dp_rank * 1000 + i)
            t0 = time.perf_counter()
            ids = self.tok.chat_ids(build_messages(d.text))
            s, = eng.generate([ids], eng.default_params(min_items=estimate_line_items(d.text)))
            parse_and_validate_response(eng.decode_text(s), "direct_text_input")
            out.append(time.perf_counter() - t0)
            sp = s.span()
            self.lat_detail.append((s.num_generated, s.num_sampled, sp.get("ttft_ms") or 0.0,
                                    out[-1]))
        eng.runner.tp.enabled and eng.shutdown()      # release the TP workers' loop
        return out


def _single_stream(detail):
    """Single-request decode rates (Groq 350 tok/s per stream): output
    tokens/s after the first token, and the sampled (non-jump-forward) step rate."""
    if not detail:
        return None
    rates, steps, ttft = [], [], []
    for gen, sampled, ttft_ms, total in detail:
        dec = max(total - ttft_ms / 1e3, 1e-6)
        rates.append(gen / dec)
        steps.append(sampled / dec)
        ttft.append(ttft_ms)
    return {"completion_tok_s_p50": round(statistics.median(rates), 1),
            "sampled_steps_per_s_p50": round(statistics.median(steps), 1),
            "ttft_ms_p50": round(statistics.median(ttft), 1),
            "baseline_decode_tok_s": 350.0}


def sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    wctx = init_distributed()
    tp, dp_rank, dp_world = split_groups(args.tp) if world > 1 else (wctx, 0, 1)
    cfg = EngineConfig.from_env(
        model=args.model, tp=args.tp, seed=args.seed, max_num_seqs=args.max_num_seqs,
        use_graphs=not args.no_graphs, jump_forward=not args.no_jump_forward,
        prefix_cache=not args.no_prefix_cache, max_batched_tokens=args.prefill_chunk,
        kv_fraction=args.kv_fraction)
    t_init = time.perf_counter()
    engine = LLMEngine(cfg, tp=tp)
    t_init = time.perf_counter() - t_init
    rep = Replica(engine, dp_rank, args.seed)

    def barrier():
        if world > 1:
            dist.barrier()

    def phase(fn):
        """TP rank 0 drives `fn`; the other ranks of its group mirror the steps."""
        if tp.rank == 0:
            r = fn()
        else:
            engine.worker_loop()
            r = None
        return r

    for _ in range(args.warmup):
        phase(lambda: rep.run_wave(args.docs_per_step))
    barrier()
    sync()
    t0 = time.perf_counter()
    if args.mode == "stream":
        phase(lambda: rep.run_wave(args.docs_per_step, waves=args.steps))
    else:
        for _ in range(args.steps):
            phase(lambda: rep.run_wave(args.docs_per_step))
    sync()
    barrier()
    dt = time.perf_counter() - t0
    steps_before = engine.num_steps
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64,
                         device=engine.device if engine.device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    lat = []
    if args.latency_runs and dp_rank == 0:
        lat = phase(lambda: rep.latency(args.latency_runs)) or []
    barrier()

    if rank == 0:
        docs = args.docs_per_step * dp_world * args.steps
        value = docs / dt
        p50 = statistics.median(lat) if lat else None
        st = engine.stats()
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
            "vs_baseline": round(value / BASELINE_DOCS_PER_S, 2),
            "dtype": "bf16",
            "data": "synthetic RFQ documents (reference length distribution), random-init weights",
            "config": {"model": args.model, "global_batch": args.docs_per_step * dp_world,
                       "seq_len": int(rep.last.get("prompt_tokens", 0) +
                                      rep.last.get("completion_tokens", 0)),
                       "parallelism": f"dp{dp_world}" + (f"-tp{args.tp}" if args.tp > 1 else ""),
                       "docs_per_step_per_replica": args.docs_per_step,
                       "temperature": cfg.temperature, "grammar": cfg.grammar,
                       "jump_forward": cfg.jump_forward, "graphs": cfg.use_graphs,
                       "mode": args.mode, "max_num_seqs": args.max_num_seqs},
            "p50_parse_text_latency_s": round(p50, 4) if p50 is not None else None,
            "single_stream": _single_stream(getattr(rep, "lat_detail", [])),
            "latency_vs_baseline_p50": round(BASELINE_P50_S / p50, 2) if p50 else None,
            "baseline": "vs_baseline = docs/s / (1 / 0.883 s), the reference's single-stream "
                        "Groq llama3-70b p50 server time (BASELINE.md)",
            "per_doc": {k: round(v, 2) for k, v in rep.last.items()},
            "engine": {"init_s": round(t_init, 1), "graph_capture_s": round(engine.capture_s, 1),
                       "gemm_tune_s": round(engine.tune_s, 1),
                       "wave_phases": getattr(rep, "phases", None),
                       "engine_steps": steps_before, "graph_steps": st.get("graph_steps"),
                       "kv_blocks": st.get("blocks"), "preempted": st.get("preempted"),
                       "host_s": {k: round(st.get(k, 0), 2) for k in
                                  ("schedule_s", "pack_s", "forward_s", "post_s")}},
        }
        for r in getattr(engine, "gemm_plan", None) or []:
            print("[bench] gemm plan %s M=%d N=%d K=%d hipblaslt %.1fus -> %s %.1fus"
                  % (r[0], r[1], r[2], r[3], r[4], "lib" if r[5] < 0 else f"skinny{r[5]}", r[6]),
                  file=sys.stderr)
        from replisense_rfq_amd.ops.autotune import SPLIT_REPORT
        for r in SPLIT_REPORT:
            print("[bench] gemm split %s M=%d N=%d K=%d one call %.1fus -> %s %.1fus" % r,
                  file=sys.stderr)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
