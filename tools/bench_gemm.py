"""hipBLASLt GEMM throughput at the Llama-3-8B projection shapes (x @ W^T, bf16)."""
import json
import sys
import time

import torch


def bench(M, N, K, iters=20):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        y = x @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        y = x @ w.t()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms * 1e3, 2 * M * N * K / ms / 1e9


def main():
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
              "down": (4096, 14336), "lm_head": (128256, 4096)}
    Ms = [int(a) for a in sys.argv[1:]] or [1, 16, 64, 256, 512, 768, 1024, 1536, 2048, 4096, 16384]
    out = []
    for M in Ms:
        row = {"M": M}
        for name, (N, K) in shapes.items():
            if name == "lm_head" and M > 1024:
                continue
            us, tf = bench(M, N, K)
            row[name] = (round(us, 1), round(tf, 1))
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
