"""Prefill attention (csrc/kernels/attn_prefill.hip) throughput: causal GQA over a
paged KV cache, q_len = kv_len = S per sequence, B sequences; TFLOP/s counts the
causal half (2 * S^2 * dh * Hq FLOPs per sequence: QK^T and PV).  Shapes: Llama-3
8B / Mixtral per GPU (Hq 32, Hkv 8) and 70B TP=8 per rank (Hq 8, Hkv 1)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()


def run(B, S, Hq, Hkv, iters=10, P=0):
    """P > 0: the first P keys of each sequence are a cached prefix (q_len = S - P)."""
    qblk = int(os.environ.get("QBLK", 0)) or ops.prefill_qblk(Hq, Hkv)
    dev = torch.device("cuda")
    pages = (S + 31) // 32
    k = torch.randn(B * pages + 1, Hkv, 32, 128, device=dev, dtype=torch.bfloat16)
    v = torch.randn_like(k)
    bt = torch.arange(B * pages, dtype=torch.int32, device=dev).view(B, pages)
    Q = S - P
    T = B * Q
    q = torch.randn(T, Hq * 128, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(q)
    qs = torch.arange(0, T, Q, dtype=torch.int32, device=dev)
    ql = torch.full((B,), Q, dtype=torch.int32, device=dev)
    kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
    nqb = (Q + qblk - 1) // qblk
    ws = torch.arange(B, dtype=torch.int32, device=dev).repeat_interleave(nqb)
    wq = torch.arange(nqb, dtype=torch.int32, device=dev).repeat(B)
    hs = int(os.environ["HSPLIT"]) if "HSPLIT" in os.environ else None
    kvs = os.environ["KVSPLIT"] != "0" if "KVSPLIT" in os.environ else None
    sm = int(os.environ["SMALL"]) if "SMALL" in os.environ else None
    f = lambda: ops.attn_prefill(q, k, v, bt, qs, ql, kvl, ws, wq, out, Hq, Hkv,  # noqa: E731
                                 1 / math.sqrt(128), qblk, hsplit_below=hs, kvsplit=kvs,
                                 small_mode=sm)
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    # QK^T + PV over the visible keys: query i sees P + i + 1 of them
    flops = B * 4.0 * 128 * Hq * (Q * P + Q * (Q + 1) / 2)
    # numerics spot check of the first sequence against an fp32 torch reference
    if B <= 4:
        from replisense_rfq_amd.ops import reference as ref

        exp = torch.zeros(Q, Hq * 128, dtype=torch.bfloat16)
        ref.attn_prefill(q[:Q].cpu(), k.cpu(), v.cpu(), bt[:1].cpu(), qs[:1].cpu(), ql[:1].cpu(),
                         kvl[:1].cpu(), None, None, exp, Hq, Hkv, 1 / math.sqrt(128))
        err = float((out[:Q].float().cpu() - exp.float()).abs().max())
        assert err < 0.05, ("prefill numerics", err)
    return us, flops / us / 1e6


SHAPES = [(1, 2048, 32, 8), (4, 2048, 32, 8), (1, 2048, 8, 1), (8, 2048, 8, 1),
          (16, 512, 32, 8), (1, 8192, 32, 8), (1, 1024, 8, 1), (1, 4096, 8, 1), (2, 2048, 8, 1)]


def main():
    # SHAPES=BxSxHqxHkv,...  (env) overrides the default list; HSPLIT / KVSPLIT / SMALL
    # pick the small-grid forms (ops.attn_prefill); PREFIX=P: P cached keys per sequence
    shapes = SHAPES
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["SHAPES"].split(",")]
    P = int(os.environ.get("PREFIX", 0))
    for B, S, Hq, Hkv in shapes:
        us, tf = run(B, S, Hq, Hkv, P=P)
        print(json.dumps({"B": B, "S": S, "prefix": P, "Hq": Hq, "Hkv": Hkv, "us": round(us, 1),
                          "TFLOPs": round(tf, 1), "pct_of_2.5PF": round(tf / 25.0, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
