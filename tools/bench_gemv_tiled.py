"""Split-K GEMV at M = 1: row-major weights vs the decode-tiled layout (ops.tile_weight).

Each case captures L distinct weight matrices (so the stream never sits in the 256 MiB
Infinity Cache, as in a real decode step) in one hipGraph and reports the best cfg per
layout, us per call and TB/s.  Tiled outputs are checked bit for bit against the
row-major kernel of the same cfg (same loads, same MFMA order).

Usage (GPU box): python tools/bench_gemv_tiled.py > gpurun_out/gemv_tiled.jsonl
"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, ".")
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

# name: (rows of W, K, kind)  kind: plain | swi (rows = 2F) | rope (rows = (Hq + 2Hkv) * 128)
SHAPES = {
    "8b_qkv": (6144, 4096, "plain"), "8b_o": (4096, 4096, "plain"),
    "8b_gate_up": (28672, 4096, "swi"), "8b_down": (4096, 14336, "plain"),
    "tp8_qkv": (1280, 8192, "plain"), "tp8_o": (8192, 1024, "plain"),
    "tp8_gate_up": (7168, 8192, "swi"), "tp8_down": (8192, 3584, "plain"),
    "70b_o": (8192, 8192, "plain"), "70b_down": (8192, 28672, "plain"),
}


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    part, tiles = ops.splitk_ws(dev)
    for name, (rows, K, kind) in SHAPES.items():
        L = max(2, min(16, int(2.0e9 // (rows * K * 2))))
        ws = [((torch.rand((rows, K), device=dev) - 0.5) / K ** 0.5).to(torch.bfloat16)
              for _ in range(L)]
        wts = [ops.tile_weight(w) for w in ws]
        x = (torch.rand((1, K), device=dev) - 0.5).to(torch.bfloat16)
        ncol = rows // 2 if kind == "swi" else rows
        ys = [torch.empty((1, ncol), device=dev, dtype=torch.bfloat16) for _ in range(L)]

        def call(w, y, cfg):
            if kind == "swi":
                _native.ops().gemv_splitk_swiglu(x, w, y, part, tiles, cfg)
            else:
                _native.ops().gemv_splitk(x, w, y, part, tiles, cfg)

        res = {"shape": name, "rows": rows, "K": K, "layers": L, "MB": round(rows * K * 2 / 1e6, 1)}
        layouts = [(False, False, False), (True, False, False), (True, True, False),
                   (True, True, True)]
        if os.environ.get("GEMV_BENCH_ALL") == "1":
            layouts.insert(2, (False, True, False))
        for tiled, nt, pe in layouts:
            best = None
            for c in ops.SPLITK_CFGS:
                cfg = (c | (ops.SPLITK_TILED if tiled else 0) | (ops.SPLITK_NT if nt else 0)
                       | (ops.SPLITK_PERSIST if pe else 0))
                ntile = ncol // 16
                if not ops.splitk_fits(dev, c, 1, rows, ntile) or K // 128 < (2 << (c & 3)):
                    continue
                wl = wts if tiled else ws
                for i in range(L):
                    call(wl[i], ys[i], cfg)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for i in range(L):
                        call(wl[i], ys[i], cfg)
                g.replay()
                torch.cuda.synchronize()
                ts = []
                for _ in range(7):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    g.replay()
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3 / L)
                t = statistics.median(ts)
                if tiled or nt:
                    ref = torch.empty_like(ys[0])
                    call(ws[0], ref, c)
                    call((wts if tiled else ws)[0], ys[0], cfg)
                    torch.cuda.synchronize()
                    assert torch.equal(ref, ys[0]), f"{name} cfg {cfg}: tiled != row-major"
                if best is None or t < best[1]:
                    best = (cfg, t)
                del g
            key = ("tiled" if tiled else "rowmajor") + ("_nt" if nt else "") + ("_p" if pe else "")
            res[key] = {"cfg": best[0], "us": round(best[1], 2),
                        "TBps": round(rows * K * 2 / best[1] / 1e6, 2)}
        res["speedup"] = round(res["rowmajor"]["us"] / res["tiled"]["us"], 3)
        res["speedup_nt"] = round(res["rowmajor"]["us"] / res["tiled_nt"]["us"], 3)
        res["speedup_nt_p"] = round(res["rowmajor"]["us"] / res["tiled_nt_p"]["us"], 3)
        print(json.dumps(res), flush=True)
        del ws, wts


if __name__ == "__main__":
    main()
