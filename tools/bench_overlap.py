"""Does a memory-bound decode attention overlap with a compute-bound GEMM on MI355X?

Two halves of the throughput step's batch (micro-batches) could run their layers on two
streams so one half's decode attention (HBM-bound, ~25 % of the step) runs beside the
other half's projections (MFMA-bound, ~70 %).  This measures the premise on bare
kernels: attention over B sequences (ctx C, shared P-token prefix, Llama-3-8B heads) and
the gate|up / o GEMMs at M rows, each alone, back to back on one stream, and on two
streams at once.  Prints one JSON line per case; µs per iteration.

Usage: python tools/bench_overlap.py
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402


def attn_case(B, C, P, Hq=32, Hkv=8, q=1, tiles=2):
    dev = torch.device("cuda")
    pages_per = (C + 31) // 32
    pp = P // 32
    uniq = pages_per - pp
    nblocks = pp + B * uniq + 1
    k = torch.randn(nblocks, Hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    bt = torch.empty(B, pages_per, dtype=torch.int32)
    nxt = pp
    for b in range(B):
        bt[b, :pp] = torch.arange(pp)
        bt[b, pp:] = torch.arange(nxt, nxt + uniq)
        nxt += uniq
    bt = bt.to(dev)
    G = Hq // Hkv
    T = B * q
    qs = torch.arange(0, T, q, dtype=torch.int32, device=dev)
    ql = torch.full((B,), q, dtype=torch.int32, device=dev)
    kvl = torch.full((B,), C, dtype=torch.int32, device=dev)
    items = ((q * G + 15) // 16 + tiles - 1) // tiles
    ws = torch.arange(B, dtype=torch.int32, device=dev).repeat_interleave(items)
    wct = torch.arange(items, dtype=torch.int32, device=dev).repeat(B)
    qt = torch.randn(T, Hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(qt)
    return lambda: ops.attn_decode(qt, k, v, bt, qs, ql, kvl, ws, wct, out, out, out, Hq, Hkv,
                                   1 / math.sqrt(128), 1, tiles)


def gemm_case(M, N, K):
    dev = torch.device("cuda")
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    return lambda: torch.matmul(x, w.t(), out=y)


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e3)
    return best


def main():
    _native.require()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for (B, C, P), (M, N, K, name) in [((768, 832, 416), (3840, 28672, 4096, "gate_up")),
                                      ((768, 832, 416), (3840, 4096, 14336, "down")),
                                      ((768, 832, 416), (3840, 6144, 4096, "qkv")),
                                      ((1536, 832, 416), (7680, 28672, 4096, "gate_up"))]:
        fa = attn_case(B, C, P)
        fg = gemm_case(M, N, K)
        ta, tg = timed(fa), timed(fg)

        def serial():
            fa()
            fg()

        def both():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                fa()
            with torch.cuda.stream(s2):
                fg()
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        ts, tb = timed(serial), timed(both)
        print(json.dumps({"attn": {"B": B, "ctx": C, "prefix": P}, "gemm": name, "M": M,
                          "N": N, "K": K, "attn_us": round(ta, 1), "gemm_us": round(tg, 1),
                          "serial_us": round(ts, 1), "two_streams_us": round(tb, 1),
                          "overlap_gain": round(1 - tb / ts, 3)}), flush=True)


if __name__ == "__main__":
    main()
