"""Weight-streaming GEMM (gemm_skinny.hip) vs weight row stride: is the long-K
slowdown (down 4096x14336 at ~4.4 TB/s vs gate_up at ~5.6) a row-stride / DRAM
mapping effect?  Weights are rotated through > 1 GiB so each call streams from HBM;
graph-replayed timing; hipBLASLt (torch.matmul) for reference."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()
ops = _native.ops()


def gtime(fn, n_inner, reps=3):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n_inner)
    return best


def main():
    dev = torch.device("cuda:0")
    for (N, K) in ((4096, 14336), (28672, 4096), (8192, 28672), (4096, 4096)):
        nbytes = N * K * 2
        L = max(2, (3 << 30) // nbytes)
        for pad in (0, 64, 256):
            buf = [torch.randn(N, K + pad, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
            ws = [b[:, :K] for b in buf]
            for M in (1, 4):
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                res = {"N": N, "K": K, "pad": pad, "M": M}
                for cfg in (12, 13, 14, 15):
                    t = gtime(lambda: [ops.skinny_gemm(x, w, out, cfg) for w in ws], L)
                    res[f"sk{cfg}_us"] = round(t, 1)
                t = gtime(lambda: [torch.matmul(x, w.t(), out=out) for w in ws], L)
                res["lib_us"] = round(t, 1)
                best = min(v for k, v in res.items() if k.endswith("_us") and k.startswith("sk"))
                res["best_TBps"] = round(nbytes / best / 1e6, 2)
                print(json.dumps(res), flush=True)
            del buf, ws


if __name__ == "__main__":
    main()
