"""Probe: does a batch-1 weight-streaming GEMV run faster when its weights are already
resident in the 256 MiB Infinity Cache (MALL), and do two streams / two graph
branches run concurrently on this stack?  Decides whether a side-stream weight
prefetch can hide the per-kernel ramp of the decode step (profiles/r3_mall_probe.md).

Usage (GPU box): python tools/probe_mall.py > gpurun_out/mall.json
"""
from __future__ import annotations

import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402


def _ev():
    return torch.cuda.Event(enable_timing=True)


def time_fn(fn, pre=None, reps=20):
    out = []
    for _ in range(reps):
        if pre is not None:
            pre()
        a, b = _ev(), _ev()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return statistics.median(out)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    flush = torch.empty(1 << 29, dtype=torch.int32, device=dev)        # 2 GiB
    part, tiles = ops.splitk_ws(dev)
    res = {}

    def do_flush():
        flush.fill_(1)

    shapes = {"tp8_gate_up": (3584, 8192, "swi"), "tp8_down": (8192, 3584, "plain"),
              "tp8_o": (8192, 1024, "plain"), "8b_gate_up": (14336, 4096, "swi"),
              "8b_down": (4096, 14336, "plain")}
    for name, (n, k, kind) in shapes.items():
        rows = 2 * n if kind == "swi" else n
        w = (torch.rand((rows, k), device=dev, dtype=torch.float32) - 0.5).to(torch.bfloat16)
        x = (torch.rand((1, k), device=dev, dtype=torch.float32) - 0.5).to(torch.bfloat16)
        y = torch.empty((1, n), device=dev, dtype=torch.bfloat16)
        scratch = torch.empty((), device=dev, dtype=torch.float32)

        def warm():
            do_flush()
            torch.sum(w, dim=(0, 1), dtype=torch.float32, out=scratch)

        best = None
        for cfg in ops.SPLITK_CFGS:
            if not ops.splitk_fits(dev, cfg, 1, rows, rows // 16):
                continue
            if kind == "swi":
                fn = (lambda c=cfg: _native.ops().gemv_splitk_swiglu(x, w, y, part, tiles, c))
            else:
                fn = (lambda c=cfg: _native.ops().gemv_splitk(x, w, y, part, tiles, c))
            fn()
            cold = time_fn(fn, do_flush, reps=8)
            if best is None or cold < best[1]:
                best = (cfg, cold, fn)
        cfg, _, fn = best
        cold = time_fn(fn, do_flush)
        hot = time_fn(fn, warm)
        back = time_fn(fn, None)                     # back-to-back replays of the same W
        mb = w.numel() * 2 / 1e6
        res[name] = {"cfg": cfg, "MB": round(mb, 1), "cold_us": round(cold, 2),
                     "mall_warm_us": round(hot, 2), "back_to_back_us": round(back, 2),
                     "cold_TBps": round(mb / cold, 2), "warm_TBps": round(mb / hot, 2)}
        print(json.dumps({name: res[name]}), file=sys.stderr, flush=True)
        del w

    # concurrency: two independent matmuls on two streams, eager and as graph branches
    a = torch.randn((4096, 4096), device=dev, dtype=torch.bfloat16)
    b = torch.randn((4096, 4096), device=dev, dtype=torch.bfloat16)
    c1 = torch.empty_like(a)
    c2 = torch.empty_like(a)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def one():
        torch.matmul(a, b, out=c1)

    def serial():
        torch.matmul(a, b, out=c1)
        torch.matmul(a, b, out=c2)

    def par():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            torch.matmul(a, b, out=c1)
        with torch.cuda.stream(s2):
            torch.matmul(a, b, out=c2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    for f in (one, serial, par):
        f()
    torch.cuda.synchronize()
    res["eager_one_us"] = round(time_fn(one), 1)
    res["eager_serial_us"] = round(time_fn(serial), 1)
    res["eager_two_streams_us"] = round(time_fn(par), 1)
    graphs = {}
    for nm, f in (("serial", serial), ("branches", par)):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            f()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            f()
        graphs[nm] = g
        res[f"graph_{nm}_us"] = round(time_fn(g.replay), 1)

    # concurrent prefetch beside a GEMV: the GEMV streams W1 while a side stream reads
    # W2 (the next projection's weights); then the GEMV on W2
    n, k = 3584, 8192
    w1 = torch.randn((2 * n, k), device=dev, dtype=torch.bfloat16)
    w2 = torch.randn((8192, 3584), device=dev, dtype=torch.bfloat16)
    x1 = torch.randn((1, k), device=dev, dtype=torch.bfloat16)
    y1 = torch.empty((1, n), device=dev, dtype=torch.bfloat16)
    y2 = torch.empty((1, 8192), device=dev, dtype=torch.bfloat16)
    scratch = torch.empty((), device=dev, dtype=torch.float32)
    cfg1 = res["tp8_gate_up"]["cfg"]
    cfg2 = res["tp8_down"]["cfg"]

    def chain():
        _native.ops().gemv_splitk_swiglu(x1, w1, y1, part, tiles, cfg1)
        _native.ops().gemv_splitk(y1, w2, y2, part, tiles, cfg2)

    def chain_pf():
        cur = torch.cuda.current_stream()
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            torch.sum(w2, dim=(0, 1), dtype=torch.float32, out=scratch)
        _native.ops().gemv_splitk_swiglu(x1, w1, y1, part, tiles, cfg1)
        cur.wait_stream(s2)
        _native.ops().gemv_splitk(y1, w2, y2, part, tiles, cfg2)

    for nm, f in (("chain", chain), ("chain_prefetch", chain_pf)):
        f()
        res[f"{nm}_eager_us"] = round(time_fn(f, do_flush), 1)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            f()
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            f()
        res[f"{nm}_graph_us"] = round(time_fn(g.replay, do_flush), 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
