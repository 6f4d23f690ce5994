"""Throughput vs. latency-under-load of the bench's document stream, one engine.

For every (prefill chunk, in-flight depth) pair: ramp the closed-loop stream of
bench.py to that depth, then time a window of completed documents and report
docs/s plus the e2e / TTFT percentiles of exactly those documents.  The engine is
built once; the token budget is changed at run time
(``EngineCore.set_max_batched_tokens``).  Used to choose the headline operating
point of bench.py: the highest docs/s whose loaded p99 stays inside the service's
30 s request deadline (/root/reference/app/rfq_agent.py:69).

Prints one JSON line per window (stdout) and writes them all to --out.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--depths", default="1024,1536,2048,3072")
    ap.add_argument("--chunks", default="16384,8192")
    ap.add_argument("--window-mult", type=float, default=1.5,
                    help="timed documents per window = max(min-docs, mult * depth)")
    ap.add_argument("--min-docs", type=int, default=768)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "depth_sweep.json"))
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()

    import torch

    from replisense_rfq_amd.benchmarks import stream as bench
    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.utils.config import EngineConfig

    depths = [int(x) for x in a.depths.split(",")]
    chunks = [int(x) for x in a.chunks.split(",")]
    cfg = EngineConfig.from_env(model=a.model, seed=a.seed, max_num_seqs=max(depths),
                                max_batched_tokens=max(chunks))
    t0 = time.perf_counter()
    eng = LLMEngine(cfg)
    init_s = time.perf_counter() - t0
    stream = bench.DocStream(eng, 0, a.seed, depths[0])
    rows = []
    order = list(depths)
    for ci, chunk in enumerate(chunks):
        eng.core.set_max_batched_tokens(chunk)
        for d in order:
            stream.in_flight = d
            # ramp: drain down to the new depth (no admissions while above it), then
            # one full turnover of documents at that depth
            stream.run_until(stream.completed + max(0, stream.live - d) + d)
            stream.clear_window()
            steps0 = eng.num_steps
            if eng.device.type == "cuda":
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            n = max(a.min_docs, int(a.window_mult * d))
            stream.run_until(stream.completed + n)
            if eng.device.type == "cuda":
                torch.cuda.synchronize()
            dt = time.perf_counter() - t1
            lat = bench.loaded_latency(stream.finished)
            shape = bench.validate(eng, stream.finished[:1024])
            row = {"chunk": chunk, "in_flight": d, "docs": n, "seconds": round(dt, 2),
                   "docs_per_s": round(n / dt, 2), "steps": eng.num_steps - steps0,
                   "ms_per_engine_step": round(1e3 * dt / max(1, eng.num_steps - steps0), 1),
                   "loaded_latency": lat,
                   "per_doc": {k: round(v, 2) for k, v in shape.items()}}
            rows.append(row)
            print(json.dumps(row), flush=True)
        order = order[::-1]
    stream.close()
    out = {"model": a.model, "init_s": round(init_s, 1), "windows": rows,
           "data": "synthetic RFQ documents, random-init weights, bench.py stream"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
