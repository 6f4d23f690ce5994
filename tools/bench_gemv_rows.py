"""Row-streaming GEMV (gemv_rows.hip) against the latency-path kernels the start-up
plans choose today: the split-K GEMV on the decode-tiled layout with non-temporal loads
(gemv_core.h, cfg | 16 | 32) and its row-major form, the skinny GEMM and hipBLASLt.
Shapes: the Llama-3-70B TP=8 rank shard and Llama-3-8B, M = 1, 2, 4.  Weights rotate
through > 1 GiB so every call streams from HBM; µs per call from captured hipGraphs.

Usage: python tools/bench_gemv_rows.py [--model tp8|8b|both] [M ...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402
from replisense_rfq_amd.ops import reference as ref  # noqa: E402
from replisense_rfq_amd.ops.autotune import _time  # noqa: E402

SHAPES = {
    "tp8": {"hidden": 8192, "hq": 8, "hkv": 1, "ffn": 3584},
    "8b": {"hidden": 4096, "hq": 32, "hkv": 8, "ffn": 14336},
    "70b": {"hidden": 8192, "hq": 64, "hkv": 8, "ffn": 28672},     # TP = 1
}
ROWS_PLAIN = (4, 8, 12, 5, 9, 2, 6, 3)
ROWS_PAIRED = (4, 8, 12, 68, 72, 76)
SPLIT_TN = ops.SPLITK_TILED | ops.SPLITK_NT


def weights(N, K):
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
    tiled = {w.data_ptr(): ops.tile_weight(w) for w in ws}
    return ws, tiled


def best(row):
    keys = [k for k in row if isinstance(row[k], float)]
    b = min(keys, key=lambda k: row[k])
    return b, row[b]


def emit(model, shape, M, N, K, row, nbytes):
    old = {k: v for k, v in row.items() if not k.startswith("rows")}
    new = {k: v for k, v in row.items() if k.startswith("rows")}
    bo, to = best(old)
    bn, tn = best(new)
    print(json.dumps({"model": model, "shape": shape, "M": M, "N": N, "K": K,
                      "us": {k: round(v, 2) for k, v in row.items()},
                      "best_old": bo, "old_us": round(to, 2), "best_rows": bn,
                      "rows_us": round(tn, 2), "speedup": round(to / tn, 3),
                      "rows_TBps": round(nbytes / tn / 1e6, 2)}), flush=True)


def run(model, Ms):
    OPS = torch.ops.rfq_amd
    sh = SHAPES[model]
    d, hq, hkv, F = sh["hidden"], sh["hq"], sh["hkv"], sh["ffn"]
    part, tiles = ops.splitk_ws("cuda")
    plain = {"qkv": ((hq + 2 * hkv) * 128, d), "o": (d, hq * 128), "down": (d, F)}
    for name, (N, K) in plain.items():
        ws, tl = weights(N, K)
        for M in Ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"lib": _time(lambda w: torch.matmul(x, w.t(), out=y), ws, 2)}
            for c in (12, 13, 14, 15):
                if c & 1 and N % 32:
                    continue
                row[f"sk{c}"] = _time(lambda w, c=c: OPS.skinny_gemm(x, w, y, c), ws, 2)
            for c in ops.SPLITK_CFGS:
                if K // 128 >= (2 << (c & 3)) and ops.splitk_fits("cuda", c, M, N, N // 16):
                    row[f"sp{c}"] = _time(lambda w, c=c: OPS.gemv_splitk(x, w, y, part, tiles, c),
                                          ws, 2)
                    row[f"sptn{c}"] = _time(lambda w, c=c: OPS.gemv_splitk(
                        x, tl[w.data_ptr()], y, part, tiles, c | SPLIT_TN), ws, 2)
            for c in ROWS_PLAIN:
                row[f"rows{c}"] = _time(lambda w, c=c: OPS.gemv_rows(x, w, y, c), ws, 2)
            emit(model, name, M, N, K, row, N * K * 2)
        del ws, tl
    ws, tl = weights(2 * F, d)
    for M in Ms:
        x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
        gu = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
        act = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
        row = {"lib+silu": _time(lambda w: OPS.silu_mul(torch.matmul(x, w.t(), out=gu), act), ws, 2)}
        for c in (0, 2):
            row[f"swi{c}"] = _time(lambda w, c=c: OPS.skinny_gemm_swiglu(x, w, act, c), ws, 2)
        for c in ops.SPLITK_CFGS:
            if d // 128 >= (2 << (c & 3)) and ops.splitk_fits("cuda", c, M, 2 * F, F // 16):
                row[f"spswi{c}"] = _time(
                    lambda w, c=c: OPS.gemv_splitk_swiglu(x, w, act, part, tiles, c), ws, 2)
                row[f"spswitn{c}"] = _time(lambda w, c=c: OPS.gemv_splitk_swiglu(
                    x, tl[w.data_ptr()], act, part, tiles, c | SPLIT_TN), ws, 2)
        for c in ROWS_PAIRED:
            row[f"rowsswi{c}"] = _time(lambda w, c=c: OPS.gemv_rows_swiglu(x, w, act, c), ws, 2)
        emit(model, "gate_up+swiglu", M, 2 * F, d, row, 2 * F * d * 2)
    del ws, tl
    N = (hq + 2 * hkv) * 128
    ws, tl = weights(N, d)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device="cuda")
    for M in Ms:
        x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
        qkv = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        kc = torch.zeros(M // 32 + 2, hkv, 32, 128, device="cuda", dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        pos = torch.arange(100, 100 + M, device="cuda", dtype=torch.int32)
        slots = torch.arange(M, device="cuda", dtype=torch.int32)
        row = {}
        for c in (13, 15):
            row[f"skrope{c}"] = _time(lambda w, c=c: OPS.skinny_gemm_rope(
                x, w, qkv, pos, cos_sin, slots, kc, vc, hq, hkv, c), ws, 2)
        for c in ops.SPLITK_CFGS:
            if d // 128 >= (2 << (c & 3)) and ops.splitk_fits("cuda", c, M, N, N // 32):
                row[f"sprope{c}"] = _time(lambda w, c=c: OPS.gemv_splitk_rope(
                    x, w, qkv, pos, cos_sin, slots, kc, vc, hq, hkv, part, tiles, c), ws, 2)
                row[f"spropetn{c}"] = _time(lambda w, c=c: OPS.gemv_splitk_rope(
                    x, tl[w.data_ptr()], qkv, pos, cos_sin, slots, kc, vc, hq, hkv, part, tiles,
                    c | SPLIT_TN), ws, 2)
        for c in ROWS_PAIRED:
            row[f"rowsrope{c}"] = _time(lambda w, c=c: OPS.gemv_rows_rope(
                x, w, qkv, pos, cos_sin, slots, kc, vc, hq, hkv, c), ws, 2)
        emit(model, "qkv+rope", M, N, d, row, N * d * 2)
    del ws, tl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="both", choices=sorted(SHAPES) + ["both"])
    ap.add_argument("ms", nargs="*", type=int)
    a = ap.parse_args()
    _native.require()
    for model in (sorted(SHAPES, reverse=True) if a.model == "both" else [a.model]):
        run(model, a.ms or [1, 2, 4])


if __name__ == "__main__":
    main()
