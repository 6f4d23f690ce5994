"""Llama-3-70B TP=8, one rank emulated on one MI355X: the per-step compute of rank 0
(BASELINE config 4; the reference's own model, /root/reference/app/rfq_agent.py:62),
with a committed model of the xGMI all-reduce cost on top.

Rank 0's exact shard is built (Hq 8, Hkv 1, d_ff 3,584 per rank, vocab shard 16,032,
17.6 GB of bf16 weights) through ``parallel.tp.EmulatedTP``: every collective is a
local no-op (the row-parallel epilogue keeps its residual add + RMSNorm), so the
hipGraph-captured decode step runs exactly the kernels one rank of the real group
runs, minus the 160 all-reduces and the sampler's partial all-gather.

The engine serves real RFQ prompts (the byte-identical reference prompt, prefix
cache warm) at batch 1.  Sampling is unconstrained (grammar off): rank 0 holds only
1/8 of the vocabulary, so the schema automaton cannot run without its peers; the
emulation times ``--decode-tokens`` plain decode steps per request, which is what
the grammar-constrained request does per sampled step (jump-forward extends ride in
the same graph-launched steps at no measurable extra cost at batch 1: the 70B TP=1
phase of bench.py runs 26.3 ms per sampled step vs 26.2 ms per plain decode step).

Projection (printed as JSON, and as markdown with --md):
  step_tp8  = step_rank0 - 2 L * t_norm + 2 L * t_ar(16 KB) + t_gather
  ttft_tp8  = ttft_rank0 + 2 L * t_ar(T * 16 KB)
  p50_tp8   = ttft_tp8 + steps_p50 * step_tp8
where t_norm is the emulation's own residual-add RMSNorm launch (the real group runs
the custom all-reduce's fused add + RMSNorm kernel in its place, so t_ar is the cost
of that fused kernel)
with steps_p50 the sampled steps of the reference-like p50 document (default from
the 70B TP=1 bench phase: 38.0 sampled steps/s x (3.97 s - 0.06 s TTFT) = 149) and
t_ar swept over a range of one-shot custom all-reduce latencies.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import logging

    logging.basicConfig(level=logging.INFO, stream=sys.stderr)   # start-up plan lines
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--decode-tokens", type=int, default=150)
    ap.add_argument("--steps-p50", type=float, default=149.0)
    ap.add_argument("--ar-us", default="4,6,8,12,25",
                    help="one-shot all-reduce latencies (us) for a 16 KB decode message")
    ap.add_argument("--gather-us", type=float, default=10.0,
                    help="the sampler's (value, index) partial all-gather per step")
    ap.add_argument("--prefill-ar-gbps", type=float, default=300.0,
                    help="effective two-shot all-reduce bandwidth for prefill messages")
    ap.add_argument("--norm-us", type=float, default=4.9,
                    help="the emulated step's fused_add_rms_norm launch (rocprof window)")
    ap.add_argument("--pdf-set", type=int, default=0,
                    help="also prefill N multi-page PDF RFQs past the 8,000-char cap "
                         "(benchmarks/stream.pdf_set_requests) and report their TTFT")
    ap.add_argument("--md", default="")
    ap.add_argument("--reproject", default="",
                    help="recompute the projection of an earlier run's JSON (no GPU)")
    a = ap.parse_args()
    if a.reproject:
        with open(a.reproject) as f:
            prev = json.load(f)
        runs = prev["runs"]
        pf = statistics.median(r["prompt_tokens"] - r["prefix_hit"] for r in runs)
        proj = project(prev["rank0_step_ms_p50"], prev["rank0_ttft_ms_p50"], pf, 80, 8192 * 2, a)
        prev["projection"] = proj
        prev["projection_formula"] = "step - 2L*t_norm + 2L*t_ar + t_gather"
        print(json.dumps(prev), flush=True)
        if a.md:
            write_md(a.md, proj)
        return

    import torch

    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.engine.sequence import SamplingParams
    from replisense_rfq_amd.models.config import get_config
    from replisense_rfq_amd.models.llama import DecoderLM
    from replisense_rfq_amd.parallel.tp import EmulatedTP
    from replisense_rfq_amd.service.extract import build_messages
    from replisense_rfq_amd.service.prompt import register_prompt_prefix
    from replisense_rfq_amd.utils import synth
    from replisense_rfq_amd.utils.config import EngineConfig

    mc = get_config(a.model)
    tp = EmulatedTP(rank=a.rank, world=a.world)
    t0 = time.perf_counter()
    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    model = DecoderLM(mc, dev, tp, seed=0)
    cfg = EngineConfig.from_env(model=a.model, max_num_seqs=8, grammar=False,
                                graph_buckets=(1, 2, 4, 8), device=str(dev))
    eng = LLMEngine(cfg, model=model)
    init_s = time.perf_counter() - t0
    tok = eng.tokenizer
    register_prompt_prefix(tok)
    res_runs = []
    for i in range(a.runs + 1):                        # run 0: warm-up
        d = synth.make_rfq(10_000_000 + i)
        ids = tok.chat_ids(build_messages(d.text))
        sp = SamplingParams(temperature=0.1, max_tokens=a.decode_tokens, seed=i, grammar=False)
        t1 = time.perf_counter()
        s, = eng.generate([ids], sp)
        if gpu:
            torch.cuda.synchronize()
        e2e = time.perf_counter() - t1
        ttft = (s.t_first_token - s.t_arrival)
        n = s.num_generated
        if i == 0:
            continue
        res_runs.append({"prompt_tokens": s.prompt_len, "prefix_hit": s.prefix_hit_tokens,
                         "generated": n, "ttft_ms": round(1e3 * ttft, 2),
                         "step_ms": round(1e3 * (e2e - ttft) / max(1, n - 1), 3)})
    pdf_rows = []
    if a.pdf_set:
        # BASELINE config 4's prefill-heavy documents: TTFT of ~2.4 K
        # new tokens after the shared prefix, one request at a time
        from replisense_rfq_amd.benchmarks.stream import pdf_set_requests

        for j, r in enumerate(pdf_set_requests(a.pdf_set)):
            ids = tok.chat_ids(r["messages"])
            sp = SamplingParams(temperature=0.1, max_tokens=4, seed=j, grammar=False)
            s, = eng.generate([ids], sp)
            if gpu:
                torch.cuda.synchronize()
            pdf_rows.append({"seed": r["seed"], "pages": r["pages"], "prompt_tokens": s.prompt_len,
                             "prefix_hit": s.prefix_hit_tokens,
                             "ttft_ms": round(1e3 * (s.t_first_token - s.t_arrival), 2)})
    step = statistics.median(r["step_ms"] for r in res_runs)
    ttft = statistics.median(r["ttft_ms"] for r in res_runs)
    prefill_tokens = statistics.median(r["prompt_tokens"] - r["prefix_hit"] for r in res_runs)
    L = mc.n_layers
    msg_decode = mc.hidden * 2                       # one token's hidden row, bf16
    w_bytes = sum(t.numel() * t.element_size() for lw in model.w["layers"] for t in lw.values())
    w_bytes += model.w["lm_head"].numel() * 2
    proj = project(step, ttft, prefill_tokens, L, msg_decode, a)
    out = {"model": a.model, "emulated": f"rank {a.rank} of TP={a.world}",
           "shard": {"hq": model.hq, "hkv": model.hkv, "ffn": model.ffn_local,
                     "vocab": model.vocab_local, "weight_gb": round(w_bytes / 1e9, 2)},
           "init_s": round(init_s, 1), "runs": res_runs,
           "rank0_step_ms_p50": step, "rank0_ttft_ms_p50": ttft,
           "hbm_floor_ms": round(w_bytes / 6.3e12 * 1e3, 3),
           "graph_steps": eng.stats().get("graph_steps"),
           "all_reduces_per_step": 2 * L, "steps_p50": a.steps_p50, "projection": proj}
    if pdf_rows:
        pf = statistics.median(r["prompt_tokens"] - r["prefix_hit"] for r in pdf_rows)
        pttft = statistics.median(r["ttft_ms"] for r in pdf_rows)
        out["pdf_set"] = {"docs": len(pdf_rows), "new_tokens_p50": pf, "rank0_ttft_ms_p50": pttft,
                          "projection": project(step, pttft, pf, L, msg_decode, a),
                          "per_doc": pdf_rows}
    print(json.dumps(out), flush=True)
    if a.md:
        write_md(a.md, proj)


def project(step, ttft, prefill_tokens, L, msg_decode, a):
    proj = []
    for ar in (float(x) for x in a.ar_us.split(",")):
        step8 = step + (2 * L * (ar - a.norm_us) + a.gather_us) / 1e3
        pf_ar_us = max(ar, prefill_tokens * msg_decode / (a.prefill_ar_gbps * 1e3))
        ttft8 = ttft + 2 * L * pf_ar_us / 1e3
        p50 = (ttft8 + a.steps_p50 * step8) / 1e3
        proj.append({"ar_us": ar, "step_ms": round(step8, 3), "ttft_ms": round(ttft8, 2),
                     "p50_s": round(p50, 3), "vs_0.883s": round(0.883 / p50, 2)})
    return proj


def write_md(path, proj):
    lines = ["| t_AR+norm (16 KB) | step ms | TTFT ms | projected p50 s | 0.883 s / p50 |",
             "|---|---|---|---|---|"]
    for p in proj:
        lines.append(f"| {p['ar_us']} us | {p['step_ms']} | {p['ttft_ms']} | {p['p50_s']} | "
                     f"{p['vs_0.883s']}x |")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
