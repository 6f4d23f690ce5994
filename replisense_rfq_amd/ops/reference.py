"""Plain PyTorch (fp32-accumulating) reference implementations of every HIP op.

These are (a) the numerics oracles the kernel tests compare against and (b) the
CPU execution path used by the engine when no GPU is present (unit tests of the
scheduler / grammar / service layers run the whole model on CPU through them).
They mirror the kernels' exact contracts: paged KV layout
``[num_blocks, Hkv, BS, D]``, in-place q rotation inside the fused QKV buffer,
Gumbel-max sampling with the same counter-based hash, etc.
"""
from __future__ import annotations

import math

import torch

MASK64 = (1 << 64) - 1


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor) -> None:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    out.copy_((xf * r * w.float()).to(out.dtype))


def fused_add_rms_norm(x, residual, w, eps, out) -> None:
    s = (x.float() + residual.float()).to(residual.dtype)
    residual.copy_(s)
    rms_norm(s, w, eps, out)


def silu_mul(gate_up: torch.Tensor, out: torch.Tensor) -> None:
    F = out.shape[1]
    g, u = gate_up[:, :F], gate_up[:, F:]
    out.copy_((torch.nn.functional.silu(g.float()).to(g.dtype).float() * u.float()).to(out.dtype))


def embed(ids, table, out, vocab_start: int = 0) -> None:
    V = table.shape[0]
    local = ids.long() - vocab_start
    ok = (local >= 0) & (local < V)
    rows = table[local.clamp(0, V - 1)]
    out.copy_(torch.where(ok[:, None], rows, torch.zeros_like(rows)))


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device="cpu") -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq: int, Hkv: int) -> None:
    D = 128
    T = qkv.shape[0]
    if T == 0:
        return
    BS = k_cache.shape[2]
    cs = cos_sin[positions[:T].long()]
    c, s = cs[:, None, : D // 2], cs[:, None, D // 2:]

    def rot(x):
        x1, x2 = x[..., : D // 2].float(), x[..., D // 2:].float()
        return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).to(x.dtype)

    q = qkv[:, : Hq * D].view(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(T, Hkv, D)
    q.copy_(rot(q))
    kr = rot(k)
    slots = slot_mapping[:T].long()
    ok = slots >= 0
    if ok.any():
        sl = slots[ok]
        blk, off = sl // BS, sl % BS
        k_cache[blk, :, off] = kr[ok]
        v_cache[blk, :, off] = v[ok]


def _gather_kv(cache, block_table, n: int):
    BS = cache.shape[2]
    nb = (n + BS - 1) // BS
    pages = cache[block_table[:nb].long()]             # [nb, Hkv, BS, D]
    return pages.permute(1, 0, 2, 3).reshape(cache.shape[1], nb * BS, -1)[:, :n]


def attn_prefill(q, k_cache, v_cache, block_tables, seq_q_start, seq_q_len, seq_kv_len,
                 work_seq, work_qblk, out, Hq: int, Hkv: int, scale: float) -> None:
    G = Hq // Hkv
    for b in range(seq_q_len.shape[0]):
        ql, kl, t0 = int(seq_q_len[b]), int(seq_kv_len[b]), int(seq_q_start[b])
        if ql == 0:
            continue
        k = _gather_kv(k_cache, block_tables[b], kl).float()
        v = _gather_kv(v_cache, block_tables[b], kl).float()
        k = k.repeat_interleave(G, 0)
        v = v.repeat_interleave(G, 0)
        qb = q[t0:t0 + ql, : Hq * 128].view(ql, Hq, 128).permute(1, 0, 2).float()
        s = torch.einsum("hqd,hkd->hqk", qb, k) * scale
        qpos = torch.arange(kl - ql, kl, device=q.device)[:, None]
        kpos = torch.arange(kl, device=q.device)[None, :]
        s = s.masked_fill(kpos > qpos, float("-inf"))
        o = torch.einsum("hqk,hkd->hqd", torch.softmax(s, -1), v)
        out[t0:t0 + ql, : Hq * 128].copy_(o.permute(1, 0, 2).reshape(ql, -1).to(out.dtype))


def _mix64(x: torch.Tensor) -> torch.Tensor:
    """splitmix-style finaliser on int64 tensors (wrapping arithmetic)."""
    def lsr(v, n):
        return (v >> n) & ((1 << (64 - n)) - 1)
    x = x ^ lsr(x, 33)
    x = x * torch.tensor(0xff51afd7ed558ccd - (1 << 64), dtype=torch.int64)
    x = x ^ lsr(x, 33)
    x = x * torch.tensor(0xc4ceb9fe1a85ec53 - (1 << 64), dtype=torch.int64)
    x = x ^ lsr(x, 33)
    return x


def gumbel_noise(seed: int, cols: torch.Tensor) -> torch.Tensor:
    """Same noise as the kernel's hash_u32(seed, 0x9e3779b9, col) -> Gumbel(0,1)."""
    s = seed & MASK64
    s = s - (1 << 64) if s >= (1 << 63) else s
    base = (0x9E3779B9 << 32)
    base = base - (1 << 64) if base >= (1 << 63) else base
    x = torch.tensor(s, dtype=torch.int64) ^ (torch.tensor(base, dtype=torch.int64) | cols.long())
    h = _mix64(x) & 0xFFFFFFFF
    u = ((h >> 8).double() + 0.5) * (1.0 / 16777216.0)
    return (-torch.log(-torch.log(u))).float()


def sample(logits: torch.Tensor, mask_table: torch.Tensor | None, mask_idx: torch.Tensor,
           temps: torch.Tensor, seeds: torch.Tensor, v0: int = 0):
    """Returns (best_val[B], best_idx[B]) over the local vocab shard (global ids)."""
    B, Vl = logits.shape
    cols = torch.arange(v0, v0 + Vl)
    vals = torch.empty(B)
    idxs = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        sc = logits[b].float().cpu()
        t = float(temps[b])
        if t > 0:
            sc = sc / t + gumbel_noise(int(seeds[b]), cols)
        mi = int(mask_idx[b])
        if mask_table is not None and mi >= 0:
            words = mask_table[mi].cpu().long() & 0xFFFFFFFF
            bits = (words[cols >> 5] >> (cols & 31)) & 1
            sc = sc.masked_fill(bits == 0, float("-inf"))
        j = int(torch.argmax(sc))
        vals[b] = sc[j]
        idxs[b] = v0 + j
    return vals, idxs


def moe_topk(router_logits, topk: int, renorm: bool):
    p = torch.softmax(router_logits.float(), -1)
    # ties (equal bf16 logits) go to the lower expert index, as in moe_topk_kernel
    order = torch.sort(router_logits.float(), dim=-1, descending=True, stable=True).indices
    ids = order[..., :topk]
    w = p.gather(-1, ids)
    if renorm:
        w = w / w.sum(-1, keepdim=True)
    return w, ids.int()


def moe_forward(x, w13, w2, router_logits, topk: int, expert_offset: int = 0):
    """Mixtral sparse MLP oracle: x [T,d], w13 [E, 2F, d], w2 [E, d, F].  With expert
    parallelism w13/w2 hold experts [expert_offset, expert_offset + E) only and the
    result is this rank's partial sum."""
    w, ids = moe_topk(router_logits, topk, True)
    out = torch.zeros(x.shape, dtype=torch.float32, device=x.device)
    F = w2.shape[2]
    for e in range(w13.shape[0]):
        tok, slot = torch.nonzero(ids == e + expert_offset, as_tuple=True)
        if tok.numel() == 0:
            continue
        h = x[tok].float() @ w13[e].float().t()
        a = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
        y = a.to(x.dtype).float() @ w2[e].float().t()
        out.index_add_(0, tok, y * w[tok, slot, None])
    return out.to(x.dtype)


def softmax_scale(head_dim: int = 128) -> float:
    return 1.0 / math.sqrt(head_dim)
