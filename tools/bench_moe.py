"""Grouped-GEMM throughput for the Mixtral MoE at throughput-step token counts:
the hand-written grouped GEMMs (8-wave 128x256 with the fused SwiGLU epilogue, and
the older 4-wave 128x128) vs hipBLASLt called once per expert (with the host
reading the expert counts).  TF/s count the routed pairs only (2 * pairs * N * K),
not the block padding."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    d, F, E, k = 4096, 14336, 8, 2
    dev = torch.device("cuda:0")
    w13 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
    w2 = torch.randn(E, d, F, device=dev, dtype=torch.bfloat16) * 0.02
    for T in [int(a) for a in sys.argv[1:]] or [256, 512, 1024, 1536, 3072]:
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
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
        t13 = timeit(lambda: ops.moe_grouped_gemm(xs, w13, h13, eob, bufs.num_blocks))
        t2 = timeit(lambda: ops.moe_grouped_gemm(act, w2, y, eob, bufs.num_blocks))
        tsm = timeit(lambda: ops.silu_mul(h13, act))
        g13 = timeit(lambda: ops.moe_gemm8(xs, w13, act, eob, bufs.num_blocks, bufs.expert_offsets,
                                           True, 128))
        g2 = timeit(lambda: ops.moe_gemm8(act, w2, y, eob, bufs.num_blocks, bufs.expert_offsets,
                                          False, 128))
        q13 = timeit(lambda: ops.moe_gemm8(xs, w13, act, eob, bufs.num_blocks, bufs.expert_offsets,
                                           True, 256))
        q2 = timeit(lambda: ops.moe_gemm8(act, w2, y, eob, bufs.num_blocks, bufs.expert_offsets,
                                          False, 256))
        off = bufs.expert_offsets.cpu().tolist()
        cnt = torch.bincount(ids.flatten().long(), minlength=E).cpu().tolist()

        def per_expert13():
            for e in range(E):
                a, c = off[e], cnt[e]
                if c:
                    torch.matmul(xs[a:a + c], w13[e].t(), out=h13[a:a + c])

        def per_expert2():
            for e in range(E):
                a, c = off[e], cnt[e]
                if c:
                    torch.matmul(act[a:a + c], w2[e].t(), out=y[a:a + c])

        b13 = timeit(per_expert13)
        b2 = timeit(per_expert2)
        fl13 = 2 * n * 2 * F * d
        fl2 = 2 * n * F * d
        print(json.dumps({"T": T, "pairs": n, "rows_padded": int(bufs.num_blocks.item()) * BLOCK_M,
                          "gemm8_w13_swiglu_us": round(g13, 1),
                          "gemm8_w13_TF": round(fl13 / g13 / 1e6, 1),
                          "gemm8_w2_us": round(g2, 1), "gemm8_w2_TF": round(fl2 / g2 / 1e6, 1),
                          "gemm256_w13_swiglu_us": round(q13, 1),
                          "gemm256_w13_TF": round(fl13 / q13 / 1e6, 1),
                          "gemm256_w2_us": round(q2, 1), "gemm256_w2_TF": round(fl2 / q2 / 1e6, 1),
                          "silu_mul_us": round(tsm, 1),
                          "grouped_w13_us": round(t13, 1),
                          "grouped_w13_TF": round(fl13 / t13 / 1e6, 1),
                          "blt_w13_us": round(b13, 1), "blt_w13_TF": round(fl13 / b13 / 1e6, 1),
                          "grouped_w2_us": round(t2, 1), "grouped_w2_TF": round(fl2 / t2 / 1e6, 1),
                          "blt_w2_us": round(b2, 1), "blt_w2_TF": round(fl2 / b2 / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
