"""Streaming-op roofline check: SwiGLU (act.hip silu_mul) and residual-add RMSNorm
(norm.hip fused_add_rms_norm) at the Llama-3-8B shapes of the throughput path
(F=14336, d=4096) over the decode batch sizes the bench runs.  Prints achieved
HBM bandwidth (bytes the op must move / kernel time) and the max error against a
plain fp32 PyTorch oracle."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from replisense_rfq_amd import ops  # noqa: E402
from replisense_rfq_amd.ops import _native  # noqa: E402

_native.require()


def _time(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def silu(M, F=14336):
    gu = torch.randn(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    us = _time(lambda: ops.silu_mul(gu, out))
    g, u = gu[:, :F].float(), gu[:, F:].float()
    ref = torch.nn.functional.silu(g) * u
    err = (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
    return {"op": "silu_mul", "M": M, "us": round(us, 2),
            "TBps": round(3 * M * F * 2 / us / 1e6, 2), "rel_err": err}


def norm(M, d=4096):
    x = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    res0 = torch.randn(M, d, device="cuda", dtype=torch.bfloat16)
    w = torch.rand(d, device="cuda", dtype=torch.bfloat16) + 0.5
    res = res0.clone()
    out = torch.empty_like(x)
    us = _time(lambda: ops.fused_add_rms_norm(x, res, w, 1e-5, out))
    res.copy_(res0)
    ops.fused_add_rms_norm(x, res, w, 1e-5, out)
    h = (x.float() + res0.float()).bfloat16().float()
    ref = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    return {"op": "fused_add_rms_norm", "M": M, "us": round(us, 2),
            "TBps": round(4 * M * d * 2 / us / 1e6, 2), "rel_err": err}


if __name__ == "__main__":
    for M in (64, 256, 1024, 2048, 3072):
        print(json.dumps(silu(M)), flush=True)
    for M in (64, 256, 1024, 2048, 3072):
        print(json.dumps(norm(M)), flush=True)
