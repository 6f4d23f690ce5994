"""hipBLASLt efficiency vs. token count M at the Llama-3-8B projection shapes.

Throughput steps have arbitrary M (decode rows + jump-forward extends + prefill
chunks), so the default heuristic's choice at *unaligned* M matters as much as at
round sizes.  Prints one JSON line per (M, shape) with µs and PFLOP/s; the first
line is a large square GEMM as the practical bf16 ceiling on this box.
"""
import json
import sys

import torch


def bench(M, N, K, iters=20):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        x @ w.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        x @ w.t()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    return us, 2.0 * M * N * K / (us * 1e-6) / 1e15


def main():
    us, pf = bench(8192, 8192, 8192)
    print(json.dumps({"M": 8192, "shape": "square8192", "us": round(us, 1), "pflops": round(pf, 3)}))
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
              "down": (4096, 14336)}
    Ms = [int(a) for a in sys.argv[1:]] or [3000, 3072, 4000, 4096, 5000, 5120, 6000, 6144,
                                            6500, 6656, 7000, 7168]
    for M in Ms:
        for name, (N, K) in shapes.items():
            us, pf = bench(M, N, K)
            print(json.dumps({"M": M, "shape": name, "us": round(us, 1), "pflops": round(pf, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
