"""Run one kernel configuration repeatedly for a rocprofv3 --pmc pass, or summarise
the counters of such a pass.

  python tools/prof_one_kernel.py run prefill B S Hq Hkv      # the profiled program
  python tools/prof_one_kernel.py run moe T [tile]             # Mixtral w13+SwiGLU grouped GEMM
  python tools/prof_one_kernel.py sum <prof dir> <kernel substring>
"""
import csv
import glob
import math
import os
import sys
from collections import defaultdict


def run(kind, *a):
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools import bench_prefill

    if kind == "prefill":
        B, S, Hq, Hkv = (int(x) for x in a)
        bench_prefill.run(B, S, Hq, Hkv, iters=5)
    elif kind == "moe":
        from replisense_rfq_amd import ops
        from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers

        T = int(a[0])
        tile = int(a[1]) if len(a) > 1 else 256
        d, F, E, k = 4096, 14336, 8, 2
        dev = torch.device("cuda:0")
        w13 = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        logits = torch.randn(T, E, device=dev, dtype=torch.bfloat16)
        bufs = MoEBuffers.allocate(T, k, E, d, F, dev)
        n = T * k
        cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
        nb = cap // BLOCK_M
        ops.moe_topk(logits, k, True, bufs.weights[:T], bufs.ids[:T])
        ops.moe_align(bufs.ids[:T], E, BLOCK_M, bufs.sorted_ids[:cap], bufs.inv_pos[:n],
                      bufs.expert_of_block[:nb], bufs.expert_offsets, bufs.num_blocks)
        ops.moe_gather(x, bufs.sorted_ids[:cap], k, bufs.xs[:cap])
        for _ in range(5):
            ops.moe_gemm8(bufs.xs[:cap], w13, bufs.act[:cap], bufs.expert_of_block[:nb],
                          bufs.num_blocks, bufs.expert_offsets, True, tile)
    elif kind == "gemm":
        # python tools/prof_one_kernel.py run gemm M N K swiglu(0|1) cfg
        from replisense_rfq_amd import ops

        M, N, K, swi, cfg = (int(x) for x in a)
        dev = torch.device("cuda:0")
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        for _ in range(10):
            ops.gemm_dense(x, w, swiglu=bool(swi), cfg=cfg)
        for _ in range(10):
            torch.matmul(x, w.t())
    torch.cuda.synchronize()


def summarise(d, sub):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        print("no counter_collection.csv under", d)
        return
    tot = defaultdict(float)
    n = defaultdict(int)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if sub not in r.get("Kernel_Name", ""):
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    for k in sorted(tot):
        print(f"{k:32s} {tot[k]:16.0f}  (dispatch rows {n[k]})")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*sys.argv[2:])
    else:
        summarise(sys.argv[2], sys.argv[3])
