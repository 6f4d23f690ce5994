"""Latency-path projections at M <= 16, every candidate the start-up plans time
(ops/autotune.py), on the Llama-3-70B TP=8 rank shard and the Llama-3-8B shapes:
hipBLASLt, the skinny kernel (gemm_skinny.hip), the split-K GEMV with its in-launch
reduction, and the fused epilogues (gate|up + SwiGLU, QKV + RoPE + KV append) in
their skinny and split-K forms.  Weights rotate through > 1 GiB so every call
streams from HBM; times from captured hipGraphs (µs per call).

Usage: python tools/bench_decode_gemv.py [--model tp8|8b] [M ...]
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
    # hidden 8192, Hq 64 / Hkv 8 / d_ff 28672 over 8 ranks
    "tp8": {"hidden": 8192, "hq": 8, "hkv": 1, "ffn": 3584},
    "8b": {"hidden": 4096, "hq": 32, "hkv": 8, "ffn": 14336},
}


def weights(N, K):
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    return [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]


def best_of(row):
    keys = [k for k in row if isinstance(row[k], float)]
    b = min(keys, key=lambda k: row[k])
    return b, row[b]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="tp8", choices=sorted(SHAPES))
    ap.add_argument("ms", nargs="*", type=int)
    a = ap.parse_args()
    _native.require()
    OPS = torch.ops.rfq_amd
    sh = SHAPES[a.model]
    d, hq, hkv, F = sh["hidden"], sh["hq"], sh["hkv"], sh["ffn"]
    Ms = a.ms or [1, 4]
    part, tiles = ops.splitk_ws("cuda")
    plain = {"qkv": ((hq + 2 * hkv) * 128, d), "o": (d, hq * 128), "down": (d, F)}
    for name, (N, K) in plain.items():
        ws = weights(N, K)
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
            b, t = best_of(row)
            print(json.dumps({"model": a.model, "shape": name, "M": M, "N": N, "K": K,
                              "us": {k: round(v, 1) for k, v in row.items()}, "best": b,
                              "best_TBps": round(N * K * 2 / t / 1e6, 2)}), flush=True)
        del ws
    # gate|up + SwiGLU
    ws = weights(2 * F, d)
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
        b, t = best_of(row)
        print(json.dumps({"model": a.model, "shape": "gate_up+swiglu", "M": M, "N": 2 * F, "K": d,
                          "us": {k: round(v, 1) for k, v in row.items()}, "best": b,
                          "best_TBps": round(2 * F * d * 2 / t / 1e6, 2)}), flush=True)
    del ws
    # QKV + RoPE + KV append
    N = (hq + 2 * hkv) * 128
    ws = weights(N, d)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device="cuda")
    for M in Ms:
        x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
        qkv = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        kc = torch.zeros(M // 32 + 2, hkv, 32, 128, device="cuda", dtype=torch.bfloat16)
        vc = torch.zeros_like(kc)
        pos = torch.arange(100, 100 + M, device="cuda", dtype=torch.int32)
        slots = torch.arange(M, device="cuda", dtype=torch.int32)

        def unfused(w):
            torch.matmul(x, w.t(), out=qkv)
            OPS.rope_kv(qkv, pos, cos_sin, slots, kc, vc, hq, hkv)

        def sk_unfused(w):
            OPS.skinny_gemm(x, w, qkv, 14)
            OPS.rope_kv(qkv, pos, cos_sin, slots, kc, vc, hq, hkv)

        row = {"lib+rope": _time(unfused, ws, 2), "sk14+rope": _time(sk_unfused, ws, 2)}
        for c in (13, 15):
            row[f"skrope{c}"] = _time(lambda w, c=c: OPS.skinny_gemm_rope(
                x, w, qkv, pos, cos_sin, slots, kc, vc, hq, hkv, c), ws, 2)
        for c in ops.SPLITK_CFGS:
            if d // 128 >= (2 << (c & 3)) and ops.splitk_fits("cuda", c, M, N, N // 32):
                row[f"sprope{c}"] = _time(lambda w, c=c: OPS.gemv_splitk_rope(
                    x, w, qkv, pos, cos_sin, slots, kc, vc, hq, hkv, part, tiles, c), ws, 2)
        b, t = best_of(row)
        print(json.dumps({"model": a.model, "shape": "qkv+rope", "M": M, "N": N, "K": d,
                          "us": {k: round(v, 1) for k, v in row.items()}, "best": b,
                          "best_TBps": round(N * d * 2 / t / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
