"""Latency-path GEMV variants at M <= 16 (weights rotated through > 1 GiB so every
call streams from HBM), timed from captured hipGraphs like ops/autotune.py:
hipBLASLt, the skinny kernel (csrc/kernels/gemm_skinny.hip), the split-K GEMV with
its in-launch reduction (gemv_splitk, cfg = KS | NW | U bits), and for the MLP the
gate|up projection with the SwiGLU epilogue vs skinny gate|up + silu_mul.
Prints one JSON line per (shape, M)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402
from replisense_rfq_amd.ops.autotune import _time  # noqa: E402

_native.require()
OPS = torch.ops.rfq_amd
SHAPES = {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096),
          "70b_o": (8192, 8192), "70b_down": (8192, 28672)}


def weights(N, K):
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    return [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [1, 4, 16]
    part = torch.empty(16 * 16 * 16384, device="cuda")
    tiles = torch.zeros(2048, dtype=torch.int32, device="cuda")
    for name, (N, K) in SHAPES.items():
        ws = weights(N, K)
        nbytes = N * K * 2
        for M in Ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            row = {"shape": name, "M": M, "N": N, "K": K}
            row["lib"] = round(_time(lambda w: torch.matmul(x, w.t(), out=y), ws, 2), 1)
            for c in (12, 13, 14, 15):
                row[f"sk{c}"] = round(_time(lambda w, c=c: OPS.skinny_gemm(x, w, y, c), ws, 2), 1)
            ref = (x.float() @ ws[0].float().t())
            for c in range(16):
                KS = 2 << (c & 3)
                if K // 128 < KS:
                    continue
                OPS.gemv_splitk(x, ws[0], y, part, tiles, c)
                err = float((y.float() - ref).abs().max())
                assert err < 0.05 + 0.02 * float(ref.abs().max()), (name, M, c, err)
                row[f"sp{c}"] = round(_time(lambda w, c=c: OPS.gemv_splitk(x, w, y, part, tiles, c),
                                            ws, 2), 1)
            best = min((k for k in row if k.startswith(("sk", "sp", "lib"))), key=lambda k: row[k])
            row["best"] = best
            row["best_TBps"] = round(nbytes / row[best] / 1e6, 2)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()
    # gate|up + SwiGLU
    N2, K = 2 * 14336, 4096
    ws = weights(N2, K)
    for M in Ms:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        gu = torch.empty(M, N2, device="cuda", dtype=torch.bfloat16)
        act = torch.empty(M, N2 // 2, device="cuda", dtype=torch.bfloat16)
        row = {"shape": "gate_up+silu", "M": M}
        for c in (12, 13, 14, 15):
            row[f"sk{c}+silu"] = round(_time(lambda w, c=c: (OPS.skinny_gemm(x, w, gu, c),
                                                             OPS.silu_mul(gu, act)), ws, 2), 1)
        for c in (0, 2):
            ref_gu = torch.empty_like(gu)
            OPS.skinny_gemm(x, ws[0], ref_gu, 13 if c == 0 else 15)   # same tile / wave split
            ref = torch.empty_like(act)
            OPS.silu_mul(ref_gu, ref)
            OPS.skinny_gemm_swiglu(x, ws[0], act, c)
            assert torch.equal(act, ref), ("swiglu differs", M, c)
            row[f"swi{c}"] = round(_time(lambda w, c=c: OPS.skinny_gemm_swiglu(x, w, act, c),
                                         ws, 2), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
