"""Timeline of the engine form's CU 0 (flags bit 8 stamps, s_memrealtime at 100 MHz) for
one persistent launch of 8B layers: wave start / end, staging, rs, each ring slot's
issue / publish / consume, the epilogue.  Usage: diag_engine.py <stage mask> <flags>
[layers]."""
import json
import os
import sys
from dataclasses import replace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from replisense_rfq_amd import ops
    from replisense_rfq_amd.models.config import LLAMA3_8B
    from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta

    mask, flags = int(sys.argv[1]), int(sys.argv[2]) | 16 | 256
    L = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    dev = torch.device("cuda:0")
    cfg = replace(LLAMA3_8B, n_layers=L, vocab_size=4096)
    model = DecoderLM(cfg, dev, seed=1)
    model.fold_norms()
    ctx, T = 1024, 1
    nb = (ctx + 32) // 32
    shape = (cfg.n_layers, nb, model.hkv, 32, 128)
    model.attach_kv_cache(torch.randn(shape, device=dev).to(torch.bfloat16),
                          torch.randn(shape, device=dev).to(torch.bfloat16))
    i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
    m = ForwardMeta(input_ids=i32([1]), positions=i32([ctx]), slot_mapping=i32([ctx]),
                    num_decode=1, dec_block_tables=i32([list(range(nb))]), dec_q_start=i32([0]),
                    dec_q_len=i32([1]), dec_kv_len=i32([ctx + 1]), dec_work_seq=i32([0]),
                    dec_work_ct=i32([0]), decode_splits=16)
    qd, F = model.hq * cfg.head_dim, model.ffn_local
    res = torch.randn((T, cfg.hidden), device=dev).to(torch.bfloat16)
    attn = torch.randn((T, qd), device=dev).to(torch.bfloat16) * 0.1
    act = torch.randn((T, F), device=dev).to(torch.bfloat16) * 0.1
    qbuf = torch.randn((T, qd), device=dev).to(torch.bfloat16)
    tab, tk, cnt = model._persist_state()
    S = 16
    po = torch.empty(T * model.hq * S * 128, device=dev)
    pm = torch.zeros(2048, device=dev)

    def run():
        ops.decode_persist(res, tab, qbuf, attn, act, m.positions, model.cos_sin, m.slot_mapping,
                           m.dec_block_tables, m.dec_q_start, m.dec_q_len, m.dec_kv_len,
                           m.dec_work_seq, m.dec_work_ct, po, pm, tk, cnt, 0, L, mask, model.hq,
                           model.hkv, F, model.kv_k.shape[3], S, model.scale, cfg.rms_eps, flags)

    for _ in range(5):
        run()
    pm.zero_()
    torch.cuda.synchronize()
    run()
    torch.cuda.synchronize()
    st = pm.view(torch.int64).cpu().tolist()
    t0 = min(v for v in st if v > 0)
    us = lambda v: round((v - t0) / 100.0, 2) if v > 0 else None  # noqa: E731
    out = {"mask": mask, "flags": flags, "layers": L,
           "wave_start": [us(st[i]) for i in range(4)], "wave_end": [us(st[4 + i]) for i in range(4)],
           "after_staging": [us(st[8 + i]) for i in range(3)], "after_rs": [us(st[12 + i]) for i in range(3)],
           "epilogue": [us(st[16]), us(st[17])],
           "issue_start": [us(st[64 + n]) for n in range(64)],
           "issued": [us(st[256 + n]) for n in range(64)], "published": [us(st[128 + n]) for n in range(64)],
           "consumed": [us(st[192 + n]) for n in range(64)], "clock_mhz": round((st[27] - st[25]) / max(1, st[26] - st[24]) * 100.0, 1),
           "kernel_errors": ops.kernel_errors()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
