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


def main():
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
