"""Folded RMSNorm weights (DecoderLM.fold_norms) + the small-step forward that reads the
un-normalised residual (_forward_fold): the same logits as the plain forward.

CPU: the fold path runs through the torch oracles of the row-streaming kernels
(ops.rows_rope_normx / rows_swiglu_normx / rows_residual_add).  GPU: the kernels
themselves (gemv_rows.hip kRwNormX / kRwResAdd), decode steps of 1-4 tokens."""
import copy

import pytest
import torch

from replisense_rfq_amd.models.config import get_config
from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta


def _meta(T, device):
    g = torch.Generator().manual_seed(99)
    ids = torch.randint(0, 1000, (T,), dtype=torch.int32, generator=g)
    pos = torch.arange(T, dtype=torch.int32)
    m = dict(input_ids=ids, positions=pos, slot_mapping=pos.clone(), num_decode=0,
             num_prefill_tokens=T, pf_block_tables=torch.zeros(1, 1, dtype=torch.int32),
             pf_q_start=torch.tensor([0], dtype=torch.int32),
             pf_q_len=torch.tensor([T], dtype=torch.int32),
             pf_kv_len=torch.tensor([T], dtype=torch.int32),
             work_seq=torch.zeros(1, dtype=torch.int32),
             work_qblk=torch.zeros(1, dtype=torch.int32),
             logits_idx=torch.arange(T, dtype=torch.int64))
    return ForwardMeta(**{k: (v.to(device) if isinstance(v, torch.Tensor) else v)
                          for k, v in m.items()})


def _pair(device):
    cfg = get_config("tiny-llama")
    a = DecoderLM(cfg, device, seed=3)
    # non-trivial norm weights, so folding them actually changes the projections
    for lw in a.w["layers"]:
        lw["attn_norm"].copy_((1 + 0.2 * torch.randn_like(lw["attn_norm"].float())).to(torch.bfloat16))
        lw["mlp_norm"].copy_((1 + 0.2 * torch.randn_like(lw["mlp_norm"].float())).to(torch.bfloat16))
    w = dict(a.w)
    w["layers"] = [{k: t.clone() for k, t in lw.items()} for lw in a.w["layers"]]
    b = DecoderLM(cfg, device, weights=w)
    shape = (cfg.n_layers, 2, a.hkv, 32, 128)
    for m in (a, b):
        m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16, device=device),
                          torch.zeros(shape, dtype=torch.bfloat16, device=device))
    assert b.fold_norms() and b.norms_folded
    return a, b


def test_fold_norms_cpu_matches_plain_forward():
    torch.manual_seed(0)
    a, b = _pair("cpu")
    for T in (1, 2):
        la = a.forward(_meta(T, "cpu")).float()
        assert b._fold_step(_meta(T, "cpu"), T)
        lb = b.forward(_meta(T, "cpu")).float()
        rel = (la - lb).norm() / la.norm()
        assert rel < 2e-2, (T, rel)
    # steps above the fold path's size run the plain forward on the folded weights with
    # unit norm weights: exact algebra, same logits
    T = 8
    assert not b._fold_step(_meta(T, "cpu"), T)
    la = a.forward(_meta(T, "cpu")).float()
    lb = b.forward(_meta(T, "cpu")).float()
    assert (la - lb).norm() / la.norm() < 2e-2


def test_fold_is_skipped_for_tp_and_moe(monkeypatch):
    cfg = get_config("tiny-mixtral")
    m = DecoderLM(cfg, "cpu", seed=1)
    assert not m.fold_norms()
    monkeypatch.setenv("RFQ_NORM_FOLD", "0")
    m2 = DecoderLM(get_config("tiny-llama"), "cpu", seed=1)
    assert not m2.fold_norms()


@pytest.mark.gpu
def test_fold_norms_gpu_matches_plain_forward(gpu):
    from replisense_rfq_amd import ops

    ops.reset_plans()            # bare models: no plan of an earlier engine applies
    torch.manual_seed(0)
    a, b = _pair(gpu)
    for T in (1, 2, 3, 4):
        la = a.forward(_meta(T, gpu)).float()
        # steps of up to FOLD_MAX_M tokens take the folded path, larger ones the plain
        # forward on the folded weights (unit norm weights): the same logits either way
        assert b._fold_step(_meta(T, gpu), T) == (T <= ops.FOLD_MAX_M)
        lb = b.forward(_meta(T, gpu)).float()
        rel = (la - lb).norm() / la.norm()
        assert rel < 3e-2, (T, rel)


def _decode_meta(tok, pos, device):
    """One decode row at position ``pos`` of sequence 0 (KV blocks 0, 1)."""
    i32 = lambda v: torch.tensor(v, dtype=torch.int32)  # noqa: E731
    m = dict(input_ids=i32([tok]), positions=i32([pos]), slot_mapping=i32([pos]), num_decode=1,
             dec_block_tables=i32([[0, 1]]), dec_q_start=i32([0]), dec_q_len=i32([1]),
             dec_kv_len=i32([pos + 1]), dec_work_seq=i32([0]), dec_work_ct=i32([0]),
             logits_idx=torch.tensor([0], dtype=torch.int64))
    return ForwardMeta(**{k: (v.to(device) if isinstance(v, torch.Tensor) else v)
                          for k, v in m.items()})


def test_fold_norms_logits_parity_prefill_then_decode():
    """the fold rounds W' = bf16(W diag(g)) once, so it is not bit-exact; pin
    the logits of the folded model (prefill on the plain forward with unit norms, then
    decode steps on _forward_fold) against the unfolded model over a whole sequence:
    relative L2 error <= 2e-2 per step and the same greedy token on every step."""
    torch.manual_seed(0)
    a, b = _pair("cpu")
    T = 12
    la = a.forward(_meta(T, "cpu")).float()
    lb = b.forward(_meta(T, "cpu")).float()
    assert (la - lb).norm() / la.norm() < 2e-2
    tok = int(la[-1].argmax())
    for step in range(6):
        ma, mb = _decode_meta(tok, T + step, "cpu"), _decode_meta(tok, T + step, "cpu")
        assert b._fold_step(mb, 1)
        la = a.forward(ma).float()
        lb = b.forward(mb).float()
        rel = (la - lb).norm() / la.norm()
        assert rel < 2e-2, (step, rel)
        assert int(la.argmax()) == int(lb.argmax()), step
        tok = int(la.argmax())
