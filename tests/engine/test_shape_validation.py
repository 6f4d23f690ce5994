"""a GQA group the prefill kernel has no instance for is rejected
when the model / runner is built (a clear ValueError), not by a TORCH_CHECK at the
first prefill on the GPU."""
from dataclasses import replace

import pytest

from replisense_rfq_amd import ops
from replisense_rfq_amd.engine.engine import LLMEngine
from replisense_rfq_amd.models.config import TINY_LLAMA, get_config
from replisense_rfq_amd.utils.config import EngineConfig


@pytest.mark.parametrize("hq,hkv,qblk", [(32, 8, 64), (64, 8, 32), (8, 1, 32), (16, 8, 64),
                                          (4, 1, 64)])
def test_supported_groups(hq, hkv, qblk):
    assert ops.prefill_qblk(hq, hkv) == qblk
    assert qblk * (hq // hkv) // 32 in (4, 8)          # the kernel's wave counts


@pytest.mark.parametrize("hq,hkv", [(16, 1), (12, 1), (8, 8), (6, 4), (4, 0)])
def test_unsupported_groups_rejected(hq, hkv):
    with pytest.raises(ValueError, match="GQA groups"):
        ops.prefill_qblk(hq, hkv)


def test_engine_build_rejects_group16(monkeypatch):
    bad = replace(TINY_LLAMA, name="tiny-g16", n_heads=16, n_kv_heads=1)
    import replisense_rfq_amd.engine.engine as E

    monkeypatch.setattr(E, "get_config", lambda name: bad if name == "tiny-g16" else get_config(name))
    with pytest.raises(ValueError, match="GQA groups"):
        LLMEngine(EngineConfig(model="tiny-g16", device="cpu", max_num_seqs=2))


def test_tile_weight_layout():
    """Decode-tiled weight layout of the split-K GEMV (gemm_skinny.hip TL): element
    ((T * K/128 + B) * 4 + j) * 512 + lane * 8 + e = W[16T + lane%16][128B + 32j +
    8(lane//16) + e]; untile_weight inverts it; shapes outside the tiling rejected."""
    import torch

    w = torch.randn(48, 384)
    t = ops.tile_weight(w)
    assert t.shape == w.shape and torch.equal(ops.untile_weight(t), w)
    flat = t.reshape(-1)
    for T, B, j, lane, e in [(0, 0, 0, 0, 0), (2, 1, 3, 37, 5), (1, 2, 1, 63, 7)]:
        off = ((T * 3 + B) * 4 + j) * 512 + lane * 8 + e
        assert flat[off] == w[16 * T + lane % 16, 128 * B + 32 * j + 8 * (lane // 16) + e]
    with pytest.raises(ValueError):
        ops.tile_weight(torch.randn(40, 384))


def test_tiled_registry_lifetime():
    """ops.register_tiled: a copy is found only for the exact tensor object it was
    registered for (not a view at the same address), in-place entries (None) report
    the tensor itself as tiled-only, and entries die with their weight."""
    import gc

    import torch

    w = torch.randn(32, 256)
    wt = ops.tile_weight(w)
    ops.register_tiled(w, wt)
    assert ops.tiled_of(w) is wt and not ops.tiled_only(w)
    assert ops.tiled_of(w.view(32, 256)) is None
    v = ops.tile_weight(torch.randn(16, 128))
    ops.register_tiled(v, None)
    assert ops.tiled_of(v) is v and ops.tiled_only(v)
    n = len(ops._TILED)
    del w, wt, v
    gc.collect()
    assert len(ops._TILED) == n - 2
