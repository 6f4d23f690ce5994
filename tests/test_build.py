"""The in-tree native libraries build for gfx950 and load on a CPU-only host
(catches undefined symbols, e.g. a template kernel whose host stub was never
instantiated, before anything reaches a GPU box)."""
import torch

from replisense_rfq_amd import _build, runtime


def test_native_libraries_build_and_load():
    so = _build.build_kernels()
    torch.ops.load_library(str(so))
    for op in ("rms_norm", "attn_decode", "attn_prefill", "skinny_gemm", "moe_skinny",
               "moe_grouped_gemm", "car_allreduce", "sample_partial"):
        assert hasattr(torch.ops.rfq_amd, op), op
    rt = runtime.load()
    assert hasattr(rt, "EngineCore") and hasattr(rt, "Grammar")
