"""Decode attention cost vs. prefix sharing: B sequences with context C where the
first P tokens are (a) the same physical KV pages for every sequence (prefix-cache
hit) or (b) distinct pages.  Tells how much of the shared-prefix traffic the
L2/MALL already absorbs (i.e. what cascade attention could still save)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()


def run(B, C, P, shared, Hq=32, Hkv=8, q=1, tiles=2, splits=2, iters=20):
    dev = torch.device("cuda")
    pages_per = (C + 31) // 32
    pp = P // 32
    uniq = pages_per - pp
    nblocks = (pp if shared else B * pp) + B * uniq + 1
    k = torch.randn(nblocks, Hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    bt = torch.empty(B, pages_per, dtype=torch.int32)
    nxt = pp if shared else 0
    for b in range(B):
        if shared:
            bt[b, :pp] = torch.arange(pp)
        else:
            bt[b, :pp] = torch.arange(nxt, nxt + pp)
            nxt += pp
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
    po = torch.empty(T * Hq * splits * 128, device=dev)
    pm = torch.empty(T * Hq * splits * 2, device=dev)
    f = lambda: ops.attn_decode(qt, k, v, bt, qs, ql, kvl, ws, wct, out, po, pm, Hq, Hkv,  # noqa
                                1 / math.sqrt(128), splits, tiles)
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    kv_bytes = B * C * Hkv * 128 * 2 * 2
    return us, kv_bytes / us / 1e6


def run_cascade(B, C, P, Hq=32, Hkv=8, q=1, tiles=2, iters=20):
    """Throughput-shape decode attention (one split) over a shared prompt prefix: the
    per-sequence kernel reading the prefix pages once per sequence (L2 hits) vs the
    cascade form (attn_decode_shared: prefix pass once per 8 rows + suffix pass that
    merges it).  Meta pass excluded (the engine runs it once per step, layer 0).
    Returns (per-sequence µs, cascade µs, max |diff|)."""
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
    out_a, out_b = torch.empty_like(qt), torch.empty_like(qt)
    wsi = torch.empty(2 + B + T, dtype=torch.int32, device=dev)
    pre_o = torch.empty(T * Hq * 128, device=dev)
    pre_ml = torch.empty(T * Hq * 2, device=dev)
    sc = 1 / math.sqrt(128)
    fa = lambda: ops.attn_decode(qt, k, v, bt, qs, ql, kvl, ws, wct, out_a, out_a, out_a,  # noqa
                                 Hq, Hkv, sc, 1, tiles)
    fb = lambda: ops.attn_decode_shared(qt, k, v, bt, qs, ql, kvl, ws, wct, out_b, wsi,  # noqa
                                        pre_o, pre_ml, Hq, Hkv, sc, tiles, False)
    ops.attn_decode_shared(qt, k, v, bt, qs, ql, kvl, ws, wct, out_b, wsi, pre_o, pre_ml,
                           Hq, Hkv, sc, tiles, True)
    fa()
    torch.cuda.synchronize()
    diff = (out_a.float() - out_b.float()).abs().max().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for f in (fa, fb, fa, fb):
        f()
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e3)
    return min(res[0], res[2]), min(res[1], res[3]), diff


def run_latency(C, Hq, Hkv, splits, tiles=2, L=32, reps=20, single=False):
    """Batch-1 decode attention as the latency path runs it: L layers with their own
    KV caches, the L (split kernel [+ reduce]) launches captured in one hipGraph;
    returns µs per layer."""
    dev = torch.device("cuda")
    pages = (C + 31) // 32
    ks = [torch.randn(pages + 1, Hkv, 32, 128, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    vs = [torch.randn_like(k) for k in ks]
    bt = torch.arange(pages, dtype=torch.int32, device=dev).view(1, pages)
    G = Hq // Hkv
    qs = torch.zeros(1, dtype=torch.int32, device=dev)
    ql = torch.ones(1, dtype=torch.int32, device=dev)
    kvl = torch.full((1,), C, dtype=torch.int32, device=dev)
    items = ((G + 15) // 16 + tiles - 1) // tiles
    ws = torch.zeros(items, dtype=torch.int32, device=dev)
    wct = torch.arange(items, dtype=torch.int32, device=dev)
    qt = torch.randn(1, Hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(qt)
    po = torch.empty(Hq * splits * 128, device=dev)
    pm = torch.empty(Hq * splits * 2, device=dev)
    tickets = torch.zeros(items * Hkv, dtype=torch.int32, device=dev) if single else None

    def body():
        for k, v in zip(ks, vs):
            ops.attn_decode(qt, k, v, bt, qs, ql, kvl, ws, wct, out, po, pm, Hq, Hkv,
                            1 / math.sqrt(128), splits, tiles, tickets)

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
        best = min(best, e0.elapsed_time(e1) * 1e3 / (reps * L))
    return best


def run_floor(Hq, L=32, reps=20):
    """The graph's per-launch floor at this latency shape: L dependent one-row elementwise
    kernels (an add into the [1, Hq*128] output) captured and replayed like run_latency."""
    dev = torch.device("cuda")
    out = torch.zeros(1, Hq * 128, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(L):
            out.add_(1)
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
        best = min(best, e0.elapsed_time(e1) * 1e3 / (reps * L))
    return best


def main():
    if os.environ.get("LAT"):
        # batch-1 latency path: split count vs context (8B 32/8 heads, 70B 64/8)
        for Hq in (32, 64):
            for C in (256, 512, 1024, 2048):
                row = {"Hq": Hq, "Hkv": 8, "ctx": C}
                for sp in (8, 16, 32):
                    row[f"s{sp}_us"] = round(run_latency(C, Hq, 8, sp), 2)
                for sp in (8, 16):                 # one column tile per work item
                    row[f"s{sp}_t1_us"] = round(run_latency(C, Hq, 8, sp, tiles=1), 2)
                print(json.dumps(row), flush=True)
        return
    if os.environ.get("LAT_SP"):
        # one wave per split: the reduce launch vs the in-kernel merge by the last split wave
        # (tickets; whole-wave merge, every split's loads in flight at once)
        shapes = ((8, 1, 80), (32, 8, 32), (64, 8, 80))   # 70B TP=8 rank, 8B, 70B TP=1
        for Hq, Hkv, L in shapes:
            for C in (512, 1024, 2048):
                row = {"Hq": Hq, "Hkv": Hkv, "ctx": C}
                for sp in (8, 16):
                    for t in (1, 2):
                        row[f"s{sp}_t{t}_reduce_us"] = round(run_latency(C, Hq, Hkv, sp, t, L=L), 2)
                        row[f"s{sp}_t{t}_single_us"] = round(
                            run_latency(C, Hq, Hkv, sp, t, L=L, single=True), 2)
                print(json.dumps(row), flush=True)
        return
    if os.environ.get("LAT_S32"):
        # 32 splits (two-kernel merge; the in-kernel merge serves <= 16) vs 16, every shape
        for Hq, Hkv, L in ((8, 1, 80), (32, 8, 32), (64, 8, 80)):
            for C in (512, 1024, 2048, 4096):
                print(json.dumps({"Hq": Hq, "Hkv": Hkv, "ctx": C,
                                  "graph_floor_us": round(run_floor(Hq, L=L), 2),
                                  "s16_t1_reduce_us": round(run_latency(C, Hq, Hkv, 16, 1, L=L), 2),
                                  "s16_t1_single_us": round(run_latency(C, Hq, Hkv, 16, 1, L=L,
                                                                        single=True), 2),
                                  "s32_t1_reduce_us": round(run_latency(C, Hq, Hkv, 32, 1, L=L), 2)}),
                      flush=True)
        return
    if os.environ.get("LAT_TP8"):
        # Llama-3-70B TP=8 rank shape (Hq 8, Hkv 1): only splits x 1 kv head waves
        for C in (512, 1024, 2048, 4096):
            row = {"Hq": 8, "Hkv": 1, "ctx": C}
            for sp in (8, 16, 32):
                row[f"s{sp}_us"] = round(run_latency(C, 8, 1, sp, L=80), 2)
            print(json.dumps(row), flush=True)
        return
    if os.environ.get("CASCADE"):
        # the headline's operating point: ~1,536 decode rows, 407-token shared prompt
        # prefix (13 pages), ~815-token contexts; extend rows q 3-9 (jump-forward)
        for B, C, P, q in [(1536, 832, 416, 1), (1536, 832, 416, 3), (2048, 800, 416, 1),
                           (1024, 1024, 416, 1)]:
            a, b, d = run_cascade(B, C, P, q=q)
            print(json.dumps({"B": B, "ctx": C, "prefix": P, "q": q, "per_seq_us": round(a, 1),
                              "cascade_us": round(b, 1), "max_diff": d}), flush=True)
        return
    if os.environ.get("TILES_AB"):
        # column tiles per work item: 1 (138 VGPRs) vs 2 (242 VGPRs, fewer waves per SIMD)
        for B, C, P, q in [(2048, 800, 416, 1), (2048, 800, 416, 3), (3072, 800, 416, 1)]:
            for tiles in (1, 2):
                for splits in (1, 2):
                    us, _ = run(B, C, P, True, q=q, tiles=tiles, splits=splits)
                    print(json.dumps({"B": B, "ctx": C, "q": q, "tiles": tiles, "splits": splits,
                                      "us": round(us, 1)}), flush=True)
        return
    for B, C, P, q in [(2048, 800, 416, 1), (2048, 800, 416, 3), (1024, 1000, 416, 1)]:
        a = run(B, C, P, True, q=q)
        b = run(B, C, P, False, q=q)
        c = run(B, C - P, 0, False, q=q)      # the suffix alone: cascade attention's floor
        print(json.dumps({"B": B, "ctx": C, "shared_prefix": P, "q": q,
                          "shared_us": round(a[0], 1), "shared_logical_TBps": round(a[1], 2),
                          "distinct_us": round(b[0], 1), "distinct_TBps": round(b[1], 2),
                          "suffix_only_us": round(c[0], 1)}),
              flush=True)


if __name__ == "__main__":
    main()
