"""Mixtral throughput-path w2 + top-k combine (ops.moe_w2_combine): never split (cus 0)
vs the device-side split-K rule (cus = the CU count; gemm_w4.hip GROUPED KS = 2, fp32
partial slabs summed in the combine) vs the round-5 path (moe_gemm_dense + moe_combine).
Random weights, routed rows from a random router; numerics against an fp32 torch
reference of the same routed MLP tail.  One JSON line per token count."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers, _cus  # noqa: E402


def timeit(fn, iters=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / iters * 1e3)
    return statistics.median(best)


def main():
    d, F, E, k = 4096, 14336, 8, 2
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    w13 = ((torch.rand(E, 2 * F, d, device=dev) * 2 - 1) / 64).to(torch.bfloat16)
    w2 = ((torch.rand(E, d, F, device=dev) * 2 - 1) / 120).to(torch.bfloat16)
    for T in [int(a) for a in sys.argv[1:]] or [768, 1024, 1536, 2048, 2600, 3072, 4096, 5120, 6144, 8192]:
        x = (torch.rand(T, d, device=dev) * 2 - 1).to(torch.bfloat16)
        logits = torch.randn(T, E, device=dev, dtype=torch.bfloat16)
        bufs = MoEBuffers.allocate(T, k, E, d, F, dev)
        yf2 = bufs.yf2 if bufs.yf2 is not None else torch.empty(2, bufs.xs.shape[0], d,
                                                                   dtype=torch.float32, device=dev)
        n = T * k
        cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
        nb = cap // BLOCK_M
        w, ids = bufs.weights[:T], bufs.ids[:T]
        ops.moe_topk(logits, k, True, w, ids)
        ops.moe_align(ids, E, BLOCK_M, bufs.sorted_ids[:cap], bufs.inv_pos[:n],
                      bufs.expert_of_block[:nb], bufs.expert_offsets, bufs.num_blocks)
        xs, act, y = bufs.xs[:cap], bufs.act[:cap], bufs.y[:cap]
        ops.moe_gather(x, bufs.sorted_ids[:cap], k, xs)
        off = bufs.expert_offsets
        ops.moe_gemm_dense(xs, w13, act, off, True)
        out0 = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
        out1, out2 = torch.empty_like(out0), torch.empty_like(out0)
        cus = _cus(dev)

        def r5():
            ops.moe_gemm_dense(act, w2, y, off, False)
            ops.moe_combine(y, bufs.inv_pos[:n], w, k, out0)

        def one():
            ops.moe_w2_combine(act, w2, y, yf2, off, bufs.inv_pos[:n], w, k, out1, 0)

        def two():
            ops.moe_w2_combine(act, w2, y, yf2, off, bufs.inv_pos[:n], w, k, out2, cus)

        r5()
        one()
        two()
        torch.cuda.synchronize()
        # fp32 reference: per expert act . w2^T, then the weighted top-k sum
        offl = off.tolist()
        yr = torch.zeros(cap, d, dtype=torch.float32, device=dev)
        for e in range(E):
            a, b = offl[e], offl[e + 1]
            if b > a:
                yr[a:b] = act[a:b].float() @ w2[e].float().t()
        pos = bufs.inv_pos[:n].long().view(T, k)
        ref = (yr[pos] * w.float().unsqueeze(-1)).sum(1)
        scale = ref.abs().max().item()
        err0 = (out0.float() - ref).abs().max().item() / scale
        err1 = (out1.float() - ref).abs().max().item() / scale
        err2 = (out2.float() - ref).abs().max().item() / scale
        t0, t1, t2 = timeit(r5), timeit(one), timeit(two)
        rows_e = [offl[e + 1] - offl[e] for e in range(E)]
        tiles = sum(((r // BLOCK_M) + 1) // 2 for r in rows_e) * (d // 256)
        fl = 2.0 * n * d * F
        full, part = divmod(tiles, cus)
        split = 2 if 0 < part <= cus // 2 and full <= 2 else 1
        print(json.dumps({"T": T, "pairs": n, "live_tiles": tiles, "rounds": round(tiles / cus, 3),
                          "auto_slices": split, "us_r5": round(t0, 1), "us_never": round(t1, 1),
                          "us_auto": round(t2, 1), "speedup_auto_vs_r5": round(t0 / t2, 3),
                          "pf_r5": round(fl / t0 / 1e9, 3), "pf_auto": round(fl / t2 / 1e9, 3),
                          "rel_err_r5": round(err0, 5), "rel_err_never": round(err1, 5),
                          "rel_err_auto": round(err2, 5)}),
              flush=True)
        del bufs, yf2


if __name__ == "__main__":
    main()
