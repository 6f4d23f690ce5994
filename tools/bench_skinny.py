"""Skinny-M GEMM (csrc/kernels/gemm_skinny.hip) vs hipBLASLt at the latency-path
shapes.  Weights are rotated through > 1 GiB of copies so every call streams
from HBM (the 256 MB Infinity Cache would otherwise hold a single 32 MB W)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336), "lm_head": (128256, 4096),
          "70b_qkv": (10240, 8192), "70b_gate_up": (57344, 8192), "70b_down": (8192, 28672)}


def timeit(fn, iters):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


CFGS = [int(c) for c in os.environ.get("SK_CFGS", "0,1,2,3").split(",")]


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [1, 4, 8, 16, 32, 64]
    for name, (N, K) in SHAPES.items():
        nbytes = N * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"shape": name, "M": M, "N": N, "K": K}
            us = timeit(lambda i: torch.matmul(x, ws[i % copies].t(), out=out), 30)
            row["hipblaslt_us"] = round(us, 1)
            row["hipblaslt_TBps"] = round(nbytes / us / 1e6, 2)
            for cfg in CFGS:
                us = timeit(lambda i: torch.ops.rfq_amd.skinny_gemm(x, ws[i % copies], out, cfg), 30)
                row[f"sk{cfg}_us"] = round(us, 1)
            best = min(CFGS, key=lambda c: row[f"sk{c}_us"])
            row["best"] = best
            row["best_TBps"] = round(nbytes / row[f"sk{best}_us"] / 1e6, 2)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
