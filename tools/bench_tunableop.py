"""How much does PyTorch TunableOp (hipBLASLt / rocBLAS solution search per GEMM shape)
gain over the default hipBLASLt heuristic on the throughput step's projection shapes?

Run once with PYTORCH_TUNABLEOP_ENABLED=0 (default heuristic) and once with
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 (search, results to
PYTORCH_TUNABLEOP_FILENAME).  Prints one JSON line per shape: µs per call of
torch.matmul(x, w.t(), out=y) with weights rotated through > 1 GiB.

Usage: python tools/bench_tunableop.py [tag]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd.ops import _native  # noqa: E402

PROJ = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}
MS = (5120, 6144, 7168, 7680, 8192, 9216)
# (name, M, N, K): Llama-3-8B projections at throughput-step row counts
SHAPES = [(n, m, *PROJ[n]) for n in ("down", "o", "qkv") for m in MS]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0")
    dev = torch.device("cuda")
    for name, M, N, K in SHAPES:
        copies = max(2, (1 << 30) // (N * K * 2) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for w in ws:
            torch.matmul(x, w.t(), out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def timed(fn):
            fn(ws[0])
            torch.cuda.synchronize()
            best = float("inf")
            for _ in range(3):
                e0.record()
                for _ in range(5):
                    for w in ws:
                        fn(w)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / (5 * len(ws)))
            return best

        t_lib = timed(lambda w: torch.matmul(x, w.t(), out=y))
        row = {"tag": tag, "gemm": name, "M": M, "N": N, "K": K, "lib_us": round(t_lib, 1),
               "lib_tflops": round(2 * M * N * K / t_lib / 1e6, 1)}
        if tag == "default":      # the hand-written persistent GEMM (cfg 13960), once
            t_w4 = timed(lambda w: _native.ops().gemm_dense(x, w, y, False, 13960))
            row["w4p_us"] = round(t_w4, 1)
        print(json.dumps(row), flush=True)
        del ws


if __name__ == "__main__":
    main()
