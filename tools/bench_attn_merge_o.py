"""Decode attention -> o projection per layer at batch 1, as the latency path's graph runs
it: split-K decode attention + its merge launch + the o GEMV (+ residual-add RMSNorm on
the 8B shape) vs the attention leaving its split partials and the o GEMV merging them in
its prologue (gemv_splitk_merge).  L layers with their own weights and KV captured in one
hipGraph, µs per layer; every o cfg of the fold and the unfused o path's cfgs are timed.

Usage: python tools/bench_attn_merge_o.py [--ctx 700] [--models 8b,tp8]
"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

# Hq, Hkv, hidden, layers, norm epilogue (TP = 1 only)
SHAPES = {"8b": (32, 8, 4096, 32, True), "tp8": (8, 1, 8192, 80, False)}
CFGS = (8, 9, 12, 13, 0, 1)


def graph_us(body, reps=20):
    body()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def run(name, ctx, splits):
    Hq, Hkv, H, L, norm = SHAPES[name]
    dev = torch.device("cuda")
    K = Hq * 128
    pages = (ctx + 31) // 32 + 1
    wos = [(torch.randn(H, K, device=dev) / math.sqrt(K)).to(torch.bfloat16) for _ in range(L)]
    for w in wos:
        ops.register_tiled(w, ops.tile_weight(w))
    kcs = [torch.randn(pages, Hkv, 32, 128, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    vcs = [torch.randn_like(k) for k in kcs]
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)  # noqa: E731
    bt = torch.arange(pages, dtype=torch.int32, device=dev).view(1, pages)
    qs, ql, kvl = i32([0]), i32([1]), i32([ctx])
    G = Hq // Hkv
    tiles = 2
    items = ((G + 15) // 16 + tiles - 1) // tiles
    wseq, wct = i32([0] * items), i32(list(range(items)))
    q = torch.randn(1, (Hq + 2 * Hkv) * 128, device=dev, dtype=torch.bfloat16)
    attn = torch.empty(1, K, device=dev, dtype=torch.bfloat16)
    po = torch.empty(Hq * splits * 128, device=dev)
    pm = torch.empty(Hq * splits * 2, device=dev)
    part, tls = ops.splitk_ws(dev)
    y = torch.empty(1, H, device=dev, dtype=torch.bfloat16)
    res = torch.randn(1, H, device=dev, dtype=torch.bfloat16)
    out = torch.empty(1, H, device=dev, dtype=torch.bfloat16)
    nw = torch.ones(H, device=dev, dtype=torch.bfloat16)
    cnt = ops.norm_counter(dev)
    scale = 1 / math.sqrt(128)
    T = ops.SPLITK_TILED | ops.SPLITK_NT
    row = {"model": name, "ctx": ctx, "splits": splits, "norm": norm}

    def attention(li, reduce):
        ops.attn_decode(q, kcs[li], vcs[li], bt, qs, ql, kvl, wseq, wct, attn, po, pm, Hq, Hkv,
                        scale, splits, tiles, None, 1, reduce=reduce)

    def o_unfused(li, c):
        w = ops._wsel(wos[li], c)
        if norm:
            torch.ops.rfq_amd.gemv_splitk_norm(attn, w, y, res, nw, 1e-5, out, cnt, part, tls, c)
        else:
            torch.ops.rfq_amd.gemv_splitk(attn, w, y, part, tls, c)

    def o_fold(li, c):
        w = ops._wsel(wos[li], c)
        if norm:
            torch.ops.rfq_amd.gemv_splitk_merge(po, pm, splits, w, y, part, tls, c, res, nw, 1e-5,
                                                out, cnt)
        else:
            torch.ops.rfq_amd.gemv_splitk_merge(po, pm, splits, w, y, part, tls, c, None, None,
                                                0.0, None, None)

    row["attn_merge_us"] = round(graph_us(lambda: [attention(li, True) for li in range(L)]) / L, 2)
    row["attn_nomerge_us"] = round(graph_us(lambda: [attention(li, False) for li in range(L)]) / L,
                                   2)
    best_u, best_f = (None, 1e9), (None, 1e9)
    for c in CFGS:
        c |= T
        t = graph_us(lambda c=c: [(attention(li, True), o_unfused(li, c)) for li in range(L)]) / L
        row[f"unfused{c}_us"] = round(t, 2)
        best_u = min(best_u, (c, t), key=lambda p: p[1])
        if ops.gemv_merge_fits(1, K, c, splits):
            t = graph_us(lambda c=c: [(attention(li, False), o_fold(li, c)) for li in range(L)]) / L
            row[f"fold{c}_us"] = round(t, 2)
            best_f = min(best_f, (c, t), key=lambda p: p[1])
    # the unfused path's best o alone vs the fold's best o alone (no attention)
    row["o_only_us"] = round(graph_us(lambda: [o_unfused(li, best_u[0]) for li in range(L)]) / L, 2)
    row["best_unfused"] = [best_u[0], round(best_u[1], 2)]
    row["best_fold"] = [best_f[0], round(best_f[1], 2)]
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=700)
    ap.add_argument("--splits", type=int, default=16)
    ap.add_argument("--models", default="8b,tp8")
    a = ap.parse_args()
    _native.require()
    for name in a.models.split(","):
        run(name, a.ctx, a.splits)


if __name__ == "__main__":
    main()
