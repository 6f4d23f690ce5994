"""Mixtral MoE MLP GEMMs at throughput-step token counts, three ways (one process,
interleaved, random data): the hand-written grouped GEMM on the dense kernel's
ping-pong structure (ops.moe_gemm_dense, host-sync free), round 2's 256x256 grouped
kernel (ops.moe_gemm8, tile 256) and one hipBLASLt GEMM per routed expert with the
host reading the segment offsets (+ silu_mul).  w13 with the SwiGLU epilogue, then
w2.  TF/s count the routed pairs only."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers  # noqa: E402


def timeit(fn, iters=5, rounds=3):
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
    w13 = ((torch.rand(E, 2 * F, d, device=dev) * 2 - 1) / 64).to(torch.bfloat16)
    w2 = ((torch.rand(E, d, F, device=dev) * 2 - 1) / 120).to(torch.bfloat16)
    for T in [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192, 16384]:
        x = (torch.rand(T, d, device=dev) * 2 - 1).to(torch.bfloat16)
        logits = torch.randn(T, E, device=dev, dtype=torch.bfloat16)
        bufs = MoEBuffers.allocate(T, k, E, d, F, dev)
        n = T * k
        cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
        nb = cap // BLOCK_M
        w, ids = bufs.weights[:T], bufs.ids[:T]
        ops.moe_topk(logits, k, True, w, ids)
        ops.moe_align(ids, E, BLOCK_M, bufs.sorted_ids[:cap], bufs.inv_pos[:n],
                      bufs.expert_of_block[:nb], bufs.expert_offsets, bufs.num_blocks)
        xs = bufs.xs[:cap]
        ops.moe_gather(x, bufs.sorted_ids[:cap], k, xs)
        h13, act, y = bufs.h13[:cap], bufs.act[:cap], bufs.y[:cap]
        eob = bufs.expert_of_block[:nb]
        off = bufs.expert_offsets
        # numerics: dense grouped vs the per-expert torch oracle on the real rows
        offl = off.tolist()
        act_d = torch.empty_like(act)
        ops.moe_gemm_dense(xs, w13, act_d, off, True, 8)
        y_d = torch.empty_like(y)
        ops.moe_gemm_dense(act_d, w2, y_d, off, False, 8)
        err13 = err2 = 0.0
        for e in range(E):
            a, b = offl[e], offl[e + 1]
            if b <= a:
                continue
            r = xs[a:b].float() @ w13[e].float().t()
            gg, u = r[:, :F].to(torch.bfloat16).float(), r[:, F:].to(torch.bfloat16).float()
            ref = (gg * torch.sigmoid(gg)).to(torch.bfloat16).float() * u
            err13 = max(err13, (act_d[a:b].float() - ref).abs().max().item() / ref.abs().max().item())
            r2 = act_d[a:b].float() @ w2[e].float().t()
            err2 = max(err2, (y_d[a:b].float() - r2).abs().max().item() / r2.abs().max().item())

        def dense():
            ops.moe_gemm_dense(xs, w13, act, off, True, 0)
            ops.moe_gemm_dense(act, w2, y, off, False, 0)

        def w4():
            ops.moe_gemm_dense(xs, w13, act, off, True, 8)
            ops.moe_gemm_dense(act, w2, y, off, False, 8)

        def gemm8():
            ops.moe_gemm8(xs, w13, act, eob, bufs.num_blocks, off, True, 256)
            ops.moe_gemm8(act, w2, y, eob, bufs.num_blocks, off, False, 256)

        def per_expert():
            o = off.tolist()
            for e in range(E):
                a, b = o[e], o[e + 1]
                if b > a:
                    torch.matmul(xs[a:b], w13[e].t(), out=h13[a:b])
            ops.silu_mul(h13[:o[E]], act[:o[E]])
            for e in range(E):
                a, b = o[e], o[e + 1]
                if b > a:
                    torch.matmul(act[a:b], w2[e].t(), out=y[a:b])

        ts = {name: timeit(fn) for name, fn in (("dense", dense), ("w4", w4), ("gemm8", gemm8),
                                                ("per_expert", per_expert))}
        fl = 2.0 * n * (2 * F * d + d * F)
        print(json.dumps({"T": T, "pairs": n, "rows_padded": offl[E],
                          "us": {k_: round(v, 1) for k_, v in ts.items()},
                          "pf": {k_: round(fl / v / 1e9, 3) for k_, v in ts.items()},
                          "rel_err_w13": round(err13, 4), "rel_err_w2": round(err2, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
