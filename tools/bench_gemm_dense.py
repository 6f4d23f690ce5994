"""Hand-written dense GEMM (csrc/kernels/gemm_dense.hip) vs hipBLASLt (torch.matmul):
numerics against an fp32 torch oracle, then interleaved timing in one process
(cdna_hip_programming.md §5.4 rule 24) on uniform random [-1, 1) operands scaled like
projection activations / weights (rule 25: never zero-filled).

Shapes: the Llama-3-8B projections (qkv, o, gate_up (+SwiGLU), down) and the 70B
TP=8 rank shards at the token counts of the throughput path.  Prints one JSON line
per shape and a summary table (markdown) to --out.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {                     # name: (N, K, swiglu)
    "qkv": (6144, 4096, False),
    "o": (4096, 4096, False),
    "gate_up": (28672, 4096, False),
    "gate_up+swiglu": (28672, 4096, True),
    "down": (4096, 14336, False),
    "70b_tp8_qkv": (1280, 8192, False),
    "70b_tp8_o": (8192, 1024, False),
    "70b_tp8_gate_up+swiglu": (7168, 8192, True),
    "70b_tp8_down": (8192, 3584, False),
    # K sweeps of the gate_up panel: the intercept of time vs K is the per-tile
    # prologue / epilogue cost (a K-independent part of every output tile)
    "gu_k1024": (28672, 1024, False),
    "gu_k2048": (28672, 2048, False),
    "gu_k8192": (28672, 8192, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1024,2048,4096,6000,7168,8192")
    ap.add_argument("--shapes", default="qkv,o,gate_up,gate_up+swiglu,down")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--cfg", type=int, default=0, help="numerics check variant")
    ap.add_argument("--cfgs", default="0,1,2,3", help="kernel variants timed")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "gemm_dense.md"))
    a = ap.parse_args()
    a.cfgs = [int(c) for c in a.cfgs.split(",")]

    import torch

    from replisense_rfq_amd import ops
    from replisense_rfq_amd.ops import reference as ref

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    for name in a.shapes.split(","):
        N, K, swi = SHAPES[name]
        w = ((torch.rand(N, K, device=dev) * 2 - 1) * (1.0 / K ** 0.5)).to(torch.bfloat16)
        for M in (int(m) for m in a.ms.split(",")):
            x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            # numerics vs fp32 oracle (first / last 512 rows: covers the M tail)
            y = ops.gemm_dense(x, w, swiglu=swi, cfg=a.cfg)
            sel = torch.cat([torch.arange(0, min(M, 512)), torch.arange(max(0, M - 512), M)]).unique()
            yr = x[sel].float() @ w.float().t()
            if swi:
                F = N // 2
                g = yr[:, :F].to(torch.bfloat16).float()
                u = yr[:, F:].to(torch.bfloat16).float()
                yr = ((g * torch.sigmoid(g)).to(torch.bfloat16).float() * u)
            err = (y[sel].float() - yr).abs().max().item()
            scale = yr.abs().max().item()
            ok = err <= 0.02 * scale + 1e-2
            row = {"shape": name, "M": M, "N": N, "K": K, "swiglu": swi, "max_abs_err": err,
                   "ref_max": scale, "ok": ok}
            if not a.check_only:
                out = torch.empty_like(y)
                gu = torch.empty((M, N), dtype=torch.bfloat16, device=dev) if swi else None

                def mk(c):
                    return lambda: ops.gemm_dense(x, w, out=out, swiglu=swi, cfg=c)

                def blt():
                    if swi:
                        torch.matmul(x, w.t(), out=gu)
                        ops.silu_mul(gu, out)
                    else:
                        torch.matmul(x, w.t(), out=out)
                fns = [("cfg%d" % c, mk(c)) for c in a.cfgs] + [("blt", blt)]
                for _, f in fns:
                    for _ in range(3):
                        f()
                ts = {k: [] for k, _ in fns}
                for _ in range(a.rounds):
                    for k, f in fns:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(a.iters):
                            f()
                        e1.record()
                        torch.cuda.synchronize()
                        ts[k].append(e0.elapsed_time(e1) * 1e3 / a.iters)
                med = {k: statistics.median(v) for k, v in ts.items()}
                best = min((k for k in med if k != "blt"), key=lambda k: med[k])
                tm, tb = ts[best], ts["blt"]
                row["us"] = {k: round(v, 1) for k, v in med.items()}
                row["best_cfg"] = best
                flops = 2.0 * M * N * K
                us_m, us_b = statistics.median(tm), statistics.median(tb)
                row.update(us_mine=round(us_m, 1), us_hipblaslt=round(us_b, 1),
                           pf_mine=round(flops / us_m / 1e9, 3),
                           pf_hipblaslt=round(flops / us_b / 1e9, 3),
                           speedup=round(us_b / us_m, 3))
            rows.append(row)
            print(json.dumps(row), flush=True)
    bad = [r for r in rows if not r["ok"]]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write("| shape | M | N | K | best cfg | us | PF/s | hipBLASLt(+silu_mul) us | PF/s | speedup | max err |\n")
        f.write("|---|---|---|---|---|---|---|---|---|---|---|\n")
        for r in rows:
            f.write(f"| {r['shape']} | {r['M']} | {r['N']} | {r['K']} | {r.get('best_cfg', '')} | {r.get('us_mine', '')} | "
                    f"{r.get('pf_mine', '')} | {r.get('us_hipblaslt', '')} | "
                    f"{r.get('pf_hipblaslt', '')} | {r.get('speedup', '')} | "
                    f"{r['max_abs_err']:.3g} |\n")
    if bad:
        print(f"NUMERICS FAILED: {len(bad)} shapes", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
