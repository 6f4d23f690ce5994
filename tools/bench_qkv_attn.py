"""Fused QKV + RoPE + KV append + decode attention (decode_fused.hip) vs the launches it
replaces -- the split-K QKV GEMV with the RoPE epilogue, the split-K decode attention
and its merge -- per layer at batch 1, as the latency path's decode graph runs them:
L layers with their own weights and KV caches captured in one hipGraph (every weight
streams from HBM), µs per layer.  Shapes: Llama-3-8B (Hq 32 / Hkv 8, K 4096) and the
Llama-3-70B TP=8 rank shard (Hq 8 / Hkv 1, K 8192).

Usage: python tools/bench_qkv_attn.py [--ctx 700] [--splits 16] [--cfgs 56,60,...]
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
from replisense_rfq_amd.ops import reference as ref  # noqa: E402

SHAPES = {"8b": (32, 8, 4096, 32), "tp8": (8, 1, 8192, 80)}


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


def run(name, ctx, splits, cfgs):
    Hq, Hkv, K, L = SHAPES[name]
    dev = torch.device("cuda")
    N = (Hq + 2 * Hkv) * 128
    pages = (ctx + 31) // 32 + 1
    ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(L)]
    for w in ws:
        ops.register_tiled(w, ops.tile_weight(w))
    kcs = [torch.randn(pages, Hkv, 32, 128, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    vcs = [torch.randn_like(k) for k in kcs]
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=dev)  # noqa: E731
    bt = torch.arange(pages, dtype=torch.int32, device=dev).view(1, pages)
    pos, slots = i32([ctx - 1]), i32([ctx - 1])
    qs, ql, kvl = i32([0]), i32([1]), i32([ctx])
    G = Hq // Hkv
    tiles = 2
    items = ((G + 15) // 16 + tiles - 1) // tiles
    wseq, wct = i32([0] * items), i32(list(range(items)))
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin(8192, 128, 500000.0, device=dev)
    out = torch.empty(1, Hq * 128, device=dev, dtype=torch.bfloat16)
    po = torch.empty(Hq * splits * 128, device=dev)
    pm = torch.empty(Hq * splits * 2, device=dev)
    part, tls = ops.splitk_ws(dev)
    done, err = ops.fuse_ws(dev)
    scale = 1 / math.sqrt(128)
    qkv = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
    row = {"model": name, "ctx": ctx, "splits": splits}

    def attn():
        ops.attn_decode(qkv, kcs[0], vcs[0], bt, qs, ql, kvl, wseq, wct, out, po, pm, Hq, Hkv,
                        scale, splits, tiles)

    # the attention launch alone (same KV per layer is fine: the split kernel's cost is
    # its latency chain, the pages are a few hundred KB)
    row["attn_only_us"] = round(graph_us(lambda: [attn() for _ in range(L)]) / L, 2)
    for c in cfgs:
        wsel = [ops._wsel(w, c | ops.SPLITK_BIT) for w in ws]

        def two():
            for li in range(L):
                torch.ops.rfq_amd.gemv_splitk_rope(x, wsel[li], qkv, pos, cs, slots, kcs[li],
                                                   vcs[li], Hq, Hkv, part, tls, c)
                ops.attn_decode(qkv, kcs[li], vcs[li], bt, qs, ql, kvl, wseq, wct, out, po, pm,
                                Hq, Hkv, scale, splits, tiles)

        def rope_only():
            for li in range(L):
                torch.ops.rfq_amd.gemv_splitk_rope(x, wsel[li], qkv, pos, cs, slots, kcs[li],
                                                   vcs[li], Hq, Hkv, part, tls, c)

        def fused():
            for li in range(L):
                ops.qkv_attn(x, ws[li], pos, cs, slots, kcs[li], vcs[li], Hq, Hkv, c | 4, bt, qs,
                             ql, kvl, wseq, wct, tiles, 1, out, po, pm, scale, splits, li, L)
                if splits > 1:
                    ops.attn_decode_merge(po, pm, out, Hq, splits)

        def fused_last():
            for li in range(L):
                ops.qkv_attn(x, ws[li], pos, cs, slots, kcs[li], vcs[li], Hq, Hkv, c | 4 | 64,
                             bt, qs, ql, kvl, wseq, wct, tiles, 1, out, po, pm, scale, splits,
                             li, L)
                if splits > 1:
                    ops.attn_decode_merge(po, pm, out, Hq, splits)

        wpad = i32([-1] * items)

        def fused_gemv_only():       # every work item padding: the GEMV in the fused binary
            for li in range(L):
                ops.qkv_attn(x, ws[li], pos, cs, slots, kcs[li], vcs[li], Hq, Hkv, c | 4, bt, qs,
                             ql, kvl, wpad, wct, tiles, 1, out, po, pm, scale, splits, li, L)

        def fused_nomerge():
            for li in range(L):
                ops.qkv_attn(x, ws[li], pos, cs, slots, kcs[li], vcs[li], Hq, Hkv, c | 4, bt, qs,
                             ql, kvl, wseq, wct, tiles, 1, out, po, pm, scale, splits, li, L)

        def merge_only():
            for li in range(L):
                ops.attn_decode_merge(po, pm, out, Hq, splits)

        row[f"fgemv{c | 4}_us"] = round(graph_us(fused_gemv_only) / L, 2)
        row[f"fnomerge{c | 4}_us"] = round(graph_us(fused_nomerge) / L, 2)
        row["merge_us"] = round(graph_us(merge_only) / L, 2)
        row[f"rope{c}_us"] = round(graph_us(rope_only) / L, 2)
        row[f"two{c}_us"] = round(graph_us(two) / L, 2)
        row[f"fused{c | 4}_us"] = round(graph_us(fused) / L, 2)
        row[f"fusedlast{c | 4}_us"] = round(graph_us(fused_last) / L, 2)
        torch.cuda.synchronize()
        row["fuse_err"] = int(err[0])
    print(json.dumps(row), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=700)
    ap.add_argument("--splits", default="16")
    ap.add_argument("--cfgs", default="60,61,52")
    ap.add_argument("--models", default="8b,tp8")
    a = ap.parse_args()
    _native.require()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for name in a.models.split(","):
        for sp in (int(s) for s in a.splits.split(",")):
            run(name, a.ctx, sp, cfgs)


if __name__ == "__main__":
    main()
