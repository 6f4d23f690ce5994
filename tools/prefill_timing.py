"""Where the time of a small-grid prefill attention launch goes: per-workgroup phase
stamps (attn_prefill_kernel ts, s_memrealtime at 100 MHz) of one launch at the TP=8
rank shape (Hq 8 / Hkv 1, one sequence).  Prints, per shape and form, the launch span
(first entry to last end), the critical (last-ending) workgroup's phases and the
medians over workgroups:

  meta   entry -> work item metadata read
  first  -> first key tiles landed in LDS
  loop   -> key loop done (per-tile µs = loop / tiles)
  hand   -> split hand-off (partials published, ticket drawn)
  tail   -> merge + output written

Usage: SHAPES=1x2048x8x1,1x512x8x1 SMALL=0 python tools/prefill_timing.py
"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402


def run(B, S, Hq, Hkv, small):
    qblk = ops.prefill_qblk(Hq, Hkv)
    dev = torch.device("cuda")
    pages = (S + 31) // 32
    k = torch.randn(B * pages + 1, Hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    bt = torch.arange(B * pages, dtype=torch.int32, device=dev).view(B, pages)
    T = B * S
    q = torch.randn(T, Hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    qs = torch.arange(0, T, S, dtype=torch.int32, device=dev)
    ql = torch.full((B,), S, dtype=torch.int32, device=dev)
    kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
    nqb = (S + qblk - 1) // qblk
    ws = torch.arange(B, dtype=torch.int32, device=dev).repeat_interleave(nqb)
    wq = torch.arange(nqb, dtype=torch.int32, device=dev).repeat(B)
    ts = torch.zeros(4096 * 8, dtype=torch.int64, device=dev)

    def f():
        ops.attn_prefill(q, k, v, bt, qs, ql, kvl, ws, wq, out, Hq, Hkv, 1 / math.sqrt(128), qblk,
                         small_mode=small)

    for _ in range(5):
        f()
    torch.cuda.synchronize()
    rows = []
    for rep in range(3):
        ts.zero_()
        torch.ops.rfq_amd.attn_prefill_timing(ts)
        f()
        torch.ops.rfq_amd.attn_prefill_timing(ts[:0])
        torch.cuda.synchronize()
        t = ts.view(-1, 8).cpu()
        act = t[(t[:, 0] > 0) & (t[:, 1] > 0)]
        ent = t[t[:, 0] > 0]
        t0 = int(ent[:, 0].min())
        us = lambda a, b: (int(a) - int(b)) / 100.0  # noqa: E731 (100 MHz ticks -> µs)
        ends = [(int(r[5]) if r[5] > 0 else int(r[4]) if r[4] > 0 else int(r[3])) for r in act]
        crit = act[max(range(len(act)), key=lambda i: ends[i])]
        span = (max(ends) - t0) / 100.0
        phases = lambda r: {  # noqa: E731
            "start": us(r[0], t0), "meta": us(r[1], r[0]), "first": us(r[2], r[1]),
            "loop": us(r[3], r[2]), "tiles": int(r[6]) & 0xFFFF,
            "hand": us(r[4], r[3]) if r[4] > 0 else None,
            "tail": us(r[5], r[4] if r[4] > 0 else r[3]) if r[5] > 0 else None,
            "merger": bool(int(r[6]) >> 17 & 1)}
        med = {}
        for key in ("meta", "first", "loop", "hand", "tail", "start"):
            vals = [phases(r)[key] for r in act if phases(r)[key] is not None]
            med[key] = round(statistics.median(vals), 2) if vals else None
        per_tile = [phases(r)["loop"] / phases(r)["tiles"] for r in act if phases(r)["tiles"] > 0]
        rows.append({"B": B, "S": S, "Hq": Hq, "Hkv": Hkv, "small": small, "rep": rep,
                     "wgs": len(ent), "active": len(act), "span_us": round(span, 2),
                     "critical": {k2: (round(v2, 2) if isinstance(v2, float) else v2)
                                  for k2, v2 in phases(crit).items()},
                     "median": med,
                     "tile_us_median": round(statistics.median(per_tile), 2) if per_tile else None,
                     "last_start_us": round(max(us(r[0], t0) for r in ent), 2)})
    if os.environ.get("RAW"):
        # per workgroup of the last launch: blockIdx, start µs, tiles (-1 = left early), end µs
        print(json.dumps({"raw": [[i, us(r[0], t0), (int(r[6]) & 0xFFFF) if r[1] > 0 else -1,
                                   us(max(int(r[3]), int(r[4]), int(r[5])), t0) if r[1] > 0
                                   else None] for i, r in enumerate(t.tolist()) if r[0] > 0]}),
              flush=True)
    for r in rows:
        print(json.dumps(r), flush=True)


def main():
    _native.require()
    shapes = [tuple(int(v) for v in t.split("x"))
              for t in os.environ.get("SHAPES", "1x2048x8x1,1x1024x8x1,1x512x8x1").split(",")]
    for small in [int(s) for s in os.environ.get("SMALL", "0,1,2").split(",")]:
        for B, S, Hq, Hkv in shapes:
            run(B, S, Hq, Hkv, small)


if __name__ == "__main__":
    main()
