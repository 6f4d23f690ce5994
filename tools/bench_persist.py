"""Batch-1 decode step: persistent layers (csrc/kernels/decode_persist.hip) vs the
multi-launch small-step path, on one GPU, hipGraph-captured like the engine's decode
graphs.  VERDICT r5 item 1.

Shapes: ``8b`` (Llama-3-8B, 32 layers) and ``tp8`` (Llama-3-70B TP=8 rank shard: d 8192,
8 q heads / 1 kv head, d_ff 3,584, vocab shard 16,032, 80 layers).  Random-init weights,
random KV context of ``--ctx`` tokens, one decode row (``--T`` rows of one sequence
each).  Modes: ``0`` (row-streaming launches, _forward_fold), ``ao`` (attention + o per
layer in one persistent launch), ``all`` (every layer in one launch).  Prints one JSON
line per (shape, mode): ms per step, µs per layer, and the relative logits error against
mode 0.

  python tools/bench_persist.py --shape 8b --ctx 512,1024,2048
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from dataclasses import replace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from replisense_rfq_amd import ops
    from replisense_rfq_amd.models.config import LLAMA3_8B, ModelConfig
    from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="8b")
    ap.add_argument("--ctx", default="512,1024")
    ap.add_argument("--T", type=int, default=1)
    ap.add_argument("--splits", type=int, default=16)
    ap.add_argument("--modes", default="0,ao,all")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--layers", type=int, default=0, help="override the layer count")
    ap.add_argument("--flags", type=int, default=0, help="RFQ_PERSIST_FLAGS for the kernel")
    a = ap.parse_args()

    dev = torch.device("cuda:0")
    if a.shape == "8b":
        cfg = LLAMA3_8B
    else:
        cfg = ModelConfig("70b-tp8-rank", vocab_size=16032, hidden=8192, n_layers=80, n_heads=8,
                          n_kv_heads=1, ffn=3584)
    if a.layers:
        cfg = replace(cfg, n_layers=a.layers)
    import replisense_rfq_amd.models.llama as llama

    llama.PERSIST_FLAGS = a.flags
    model = DecoderLM(cfg, dev, seed=1)
    model.fold_norms()
    ctxs = [int(c) for c in a.ctx.split(",")]
    T = a.T
    nb_seq = (max(ctxs) + T + 31) // 32
    nblocks = T * nb_seq + 1
    shape = (cfg.n_layers, nblocks, model.hkv, 32, 128)
    g = torch.Generator(device=dev).manual_seed(3)
    model.attach_kv_cache(torch.randn(shape, generator=g, device=dev).to(torch.bfloat16),
                          torch.randn(shape, generator=g, device=dev).to(torch.bfloat16))
    ops.kernel_errors()
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
    for ctx in ctxs:
        slots = [(i * nb_seq + ctx // 32) * 32 + ctx % 32 for i in range(T)]
        m = ForwardMeta(
            input_ids=i32([7] * T), positions=i32([ctx] * T), slot_mapping=i32(slots),
            num_decode=T, dec_block_tables=i32([[i * nb_seq + j for j in range(nb_seq)]
                                                for i in range(T)]),
            dec_q_start=i32(list(range(T))), dec_q_len=i32([1] * T),
            dec_kv_len=i32([ctx + 1] * T), dec_work_seq=i32(list(range(T))),
            dec_work_ct=i32([0] * T), logits_idx=torch.arange(T, dtype=torch.int64, device=dev),
            decode_splits=a.splits)
        ref = None
        for mode in a.modes.split(","):
            if mode.startswith(("raw:", "rows:")):
                bench_parts(model, m, mode, a, cfg, ctx)
                continue
            model.persist = mode
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                model.forward(m)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = model.forward(m)
            for _ in range(3):
                graph.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                graph.replay()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            lo = out.float().clone()
            if ref is None:
                ref = lo
            rel = float((lo - ref).norm() / ref.norm())
            print(json.dumps({"shape": a.shape, "layers": cfg.n_layers, "ctx": ctx, "T": T,
                              "splits": a.splits, "mode": mode, "flags": a.flags,
                              "ms_per_step": round(ms, 4),
                              "us_per_layer": round(1000 * ms / cfg.n_layers, 2),
                              "rel_vs_first": round(rel, 5),
                              "kernel_errors": ops.kernel_errors()}), flush=True)
            del graph


def bench_parts(model, m, mode, a, cfg, ctx):
    """Timing pieces: ``raw:<mask>`` = one persistent launch of every layer with only the
    stages in <mask> (1 qkv, 2 attention, 4 o, 8 gate|up, 16 down; no embed / LM head);
    ``rows:<qkv|o|gu|down|attn>`` = the same projection on its multi-launch kernel for every
    layer (the fold path's row-streaming GEMVs / decode attention)."""
    import torch

    from replisense_rfq_amd import ops

    T = m.num_tokens
    w = model.w
    eps = cfg.rms_eps
    qd, F = model.hq * cfg.head_dim, model.ffn_local
    res = torch.randn((T, cfg.hidden), device=model.device).to(torch.bfloat16)
    attn = torch.randn((T, qd), device=model.device).to(torch.bfloat16) * 0.1
    act = torch.randn((T, F), device=model.device).to(torch.bfloat16) * 0.1
    qbuf = torch.randn((T, qd), device=model.device).to(torch.bfloat16)
    tab, tk, cnt = model._persist_state()
    S = m.decode_splits
    po = torch.empty(T * model.hq * S * 128, device=model.device)
    pm = torch.empty(T * model.hq * S * 2, device=model.device)
    kind, arg = mode.split(":")

    def body():
        if kind == "raw":
            ops.decode_persist(res, tab, qbuf, attn, act, m.positions, model.cos_sin,
                               m.slot_mapping, m.dec_block_tables, m.dec_q_start, m.dec_q_len,
                               m.dec_kv_len, m.dec_work_seq, m.dec_work_ct, po, pm, tk, cnt, 0,
                               cfg.n_layers, int(arg), model.hq, model.hkv, F,
                               model.kv_k.shape[3], S, model.scale, eps, a.flags)
            return
        for li in range(cfg.n_layers):
            lw = w["layers"][li]
            if arg == "qkv":
                ops.rows_rope_normx(res, lw["qkv"], m.positions, model.cos_sin, m.slot_mapping,
                                    model.kv_k[li], model.kv_v[li], model.hq, model.hkv, eps)
            elif arg == "o":
                ops.rows_residual_add(attn, lw["o"], res)
            elif arg == "gu":
                ops.rows_swiglu_normx(res, lw["gate_up"], eps)
            elif arg == "down":
                ops.rows_residual_add(act, lw["down"], res)
            elif arg == "attn":
                model._attend(li, None, attn, m, (po, pm), None, qkv=qbuf)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        body()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(json.dumps({"shape": a.shape, "layers": cfg.n_layers, "ctx": ctx, "T": T,
                      "splits": S, "mode": mode, "flags": a.flags, "ms": round(ms, 4),
                      "us_per_layer": round(1000 * ms / cfg.n_layers, 2),
                      "kernel_errors": ops.kernel_errors()}), flush=True)


if __name__ == "__main__":
    main()
