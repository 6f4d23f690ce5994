"""Latency-path MoE weight streaming (gemm_skinny.hip moe_skinny_kernel) on full-size
Mixtral-8x7B expert weights: µs per call and effective TB/s of the routed experts'
weights, for 1-3 tokens (2-6 routed experts).  Four layer copies are rotated so
every call streams from HBM, as in a decode step."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.models.moe import BLOCK_S, MoEBuffers  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()


def main():
    d, F, E, k, L = 4096, 14336, 8, 2, 4
    dev = torch.device("cuda:0")
    w13 = [torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    w2 = [torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
    router = torch.randn(E, d, device=dev, dtype=torch.bfloat16) * 0.05
    for T in (1, 2, 3):
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        bufs = MoEBuffers.allocate(T, k, E, d, F, dev)
        n = T * k
        w, ids = bufs.weights[:T], bufs.ids[:T]
        ops.moe_route(x, router, k, True, w, ids)
        cap = (n + E * (BLOCK_S - 1) + BLOCK_S - 1) // BLOCK_S * BLOCK_S
        sorted_ids = bufs.sorted_ids[:cap]
        ops.moe_align(ids, E, BLOCK_S, sorted_ids, bufs.inv_pos[:n],
                      bufs.expert_of_block[:cap // BLOCK_S], bufs.expert_offsets, bufs.num_blocks)
        act, y = bufs.act[:cap], bufs.y[:cap]
        yf = torch.empty(4, cap, d, device=dev, dtype=torch.float32)
        n_exp = int(ids.unique().numel())
        res = {"T": T, "experts": n_exp}
        for name, fn, wbytes in (
                ("w13", lambda i: ops.moe_skinny(x, sorted_ids, k, bufs.expert_offsets, w13[i],
                                                 act, True, True, n), 2 * F * d * 2),
                ("w2", lambda i: ops.moe_skinny(act, sorted_ids, k, bufs.expert_offsets, w2[i],
                                                y, False, False, n), F * d * 2),
                ("w2s2", lambda i: ops.moe_skinny_splitk(act, sorted_ids, k, bufs.expert_offsets,
                                                         w2[i], yf, n, 2), F * d * 2),
                ("w2s4", lambda i: ops.moe_skinny_splitk(act, sorted_ids, k, bufs.expert_offsets,
                                                         w2[i], yf, n, 4), F * d * 2)):
            for i in range(L):
                fn(i)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                for _ in range(4):
                    for i in range(L):
                        fn(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(3):
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1e3 / (4 * L))
            res[name + "_us"] = round(best, 1)
            res[name + "_TBps"] = round(n_exp * wbytes / best / 1e6, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
