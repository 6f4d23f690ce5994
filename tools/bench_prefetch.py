"""Does a weight prefetch into the MALL (Infinity Cache, 256 MB) speed up a latency-path
GEMV that follows it?  For each projection shape: the skinny GEMV at M = 1 on weights
evicted from L2/MALL (1 GiB of other reads first) vs the same GEMV right after a
strided read of its weights (one element per 64-B line).  Times the GEMV alone (events).
A large gap would make overlapping next-kernel weight prefetch with the
latency-bound attention / norm kernels of a decode step worth building."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()
OPS = torch.ops.rfq_amd
SHAPES = {"o": (4096, 4096, 14), "qkv": (6144, 4096, 15), "down": (4096, 14336, 14),
          "gate_up": (28672, 4096, 12)}


def main():
    flush = torch.empty(1 << 29, device="cuda", dtype=torch.bfloat16)   # 1 GiB
    sink = torch.empty(1, device="cuda")
    for name, (N, K, cfg) in SHAPES.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(1, N, device="cuda", dtype=torch.bfloat16)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        res = {"shape": name, "MB": round(N * K * 2 / 1e6, 1)}
        for mode in ("cold", "prefetched", "cold", "prefetched"):
            tot = 0.0
            for _ in range(10):
                sink += flush.sum(dtype=torch.float32)          # evict: 1 GiB read only
                if mode == "prefetched":
                    sink += w.view(-1)[::32].sum(dtype=torch.float32)
                torch.cuda.synchronize()
                e0.record()
                OPS.skinny_gemm(x, w, y, cfg)
                e1.record()
                torch.cuda.synchronize()
                tot += e0.elapsed_time(e1) * 1e3
            res[mode] = round(tot / 10, 1)
        res["speedup"] = round(res["cold"] / res["prefetched"], 2)
        print(json.dumps(res), flush=True)
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
