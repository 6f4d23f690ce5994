"""Seeded random-init weights, generated directly as this rank's TP shard.

BASELINE.json runs the benchmark on random-init weights of the real
architectures (no checkpoints, no network).  Each tensor is drawn on the target
device from a generator seeded by (seed, layer, name, tp_rank), so TP workers
build their shards independently with no weight broadcast
and a replica restart regenerates identical weights.

Layout (torch Linear convention, out = x @ W^T):
  qkv     [(Hq + 2 Hkv)/TP * 128, d]      column-parallel (q heads | k heads | v heads)
  o       [d, Hq/TP * 128]                row-parallel
  gate_up [2 F/TP, d]                     column-parallel (gate | up)
  down    [d, F/TP]                       row-parallel
  MoE:    router [E, d]; w13 [E, 2F/TP, d]; w2 [E, d, F/TP]
  embed   [V, d] replicated; lm_head [V/TP, d] vocab-parallel

A safetensors loader with the same names is provided for real checkpoints.
"""
from __future__ import annotations

import hashlib

import torch

from ..parallel.tp import TPContext
from .config import ModelConfig


def _seed(*parts) -> int:
    h = hashlib.blake2b(repr(parts).encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") & ((1 << 63) - 1)


def _randn(shape, std, seed_parts, device, dtype):
    g = torch.Generator(device=device)
    g.manual_seed(_seed(*seed_parts))
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=g)
    return t.to(dtype)


class LayerWeights(dict):
    __getattr__ = dict.__getitem__


def init_weights(cfg: ModelConfig, tp: TPContext, device, dtype=torch.bfloat16, seed: int = 0,
                 moe_ep: bool = False):
    """moe_ep: experts are split across the TP group (each rank holds E/TP whole
    experts) instead of every expert's FFN being column/row split."""
    d, D = cfg.hidden, cfg.head_dim
    R = tp.world
    if cfg.n_heads % R or cfg.n_kv_heads % R or cfg.ffn % R or cfg.vocab_size % R:
        raise ValueError(f"{cfg.name} is not divisible by TP={R}")
    if moe_ep and cfg.n_experts % R:
        raise ValueError(f"{cfg.n_experts} experts are not divisible by EP={R}")
    hq, hkv, F = cfg.n_heads // R, cfg.n_kv_heads // R, cfg.ffn // R
    std = cfg.init_std
    r = tp.rank
    ones = lambda n: torch.ones(n, dtype=dtype, device=device)  # noqa: E731
    layers = []
    for li in range(cfg.n_layers):
        lw = LayerWeights(
            attn_norm=ones(d),
            mlp_norm=ones(d),
            qkv=_randn(((hq + 2 * hkv) * D, d), std, (seed, li, "qkv", r), device, dtype),
            o=_randn((d, hq * D), std, (seed, li, "o", r), device, dtype),
        )
        if cfg.is_moe:
            E = cfg.n_experts
            lw["router"] = _randn((E, d), std, (seed, li, "router"), device, dtype)
            if moe_ep:
                El, Ff = E // R, cfg.ffn
                lw["w13"] = _randn((El, 2 * Ff, d), std, (seed, li, "w13e", r), device, dtype)
                lw["w2"] = _randn((El, d, Ff), std, (seed, li, "w2e", r), device, dtype)
            else:
                lw["w13"] = _randn((E, 2 * F, d), std, (seed, li, "w13", r), device, dtype)
                lw["w2"] = _randn((E, d, F), std, (seed, li, "w2", r), device, dtype)
        else:
            lw["gate_up"] = _randn((2 * F, d), std, (seed, li, "gate_up", r), device, dtype)
            lw["down"] = _randn((d, F), std, (seed, li, "down", r), device, dtype)
        layers.append(lw)
    v0, v1 = tp.shard(cfg.vocab_size)
    return dict(
        embed=_randn((cfg.vocab_size, d), std, (seed, "embed"), device, dtype),
        final_norm=ones(d),
        lm_head=_randn((v1 - v0, d), std, (seed, "lm_head", r), device, dtype),
        layers=layers,
        vocab_start=v0,
    )


class _LazyCheckpoint:
    """Tensor name -> file index over a set of safetensors files; reads only the
    requested slice of each tensor (memory-mapped), so a TP rank of a 141 GB
    Llama-3-70B checkpoint touches ~1/8 of it and never holds the whole file."""

    def __init__(self, files):
        from safetensors import safe_open

        self._handles = [safe_open(f, framework="pt", device="cpu") for f in files]
        self._where = {}
        for h in self._handles:
            for k in h.keys():
                self._where[k] = h

    def __contains__(self, name):
        return name in self._where

    def full(self, name):
        return self._where[name].get_tensor(name)

    def rows(self, name, a, b):          # W[a:b]
        return self._where[name].get_slice(name)[a:b]

    def cols(self, name, a, b):          # W[:, a:b]
        return self._where[name].get_slice(name)[:, a:b]


def load_safetensors(path: str, cfg: ModelConfig, tp: TPContext, device, dtype=torch.bfloat16,
                     moe_ep: bool = False):
    """Load HF-style Llama/Mixtral safetensors shards into this rank's layout
    (Megatron TP split, or whole experts per rank with moe_ep), reading only this
    rank's slices; each layer is moved to the device as it is assembled."""
    import glob
    import os

    files = sorted(glob.glob(os.path.join(path, "*.safetensors"))) if os.path.isdir(path) else [path]
    ck = _LazyCheckpoint(files)

    def cols(name, n):        # column-parallel: this rank's rows of W
        a, b = tp.shard(n)
        return ck.rows(name, a, b)

    def rows(name, n):        # row-parallel: this rank's columns of W
        a, b = tp.shard(n)
        return ck.cols(name, a, b)

    D, F = cfg.head_dim, cfg.ffn
    layers = []
    for li in range(cfg.n_layers):
        p = f"model.layers.{li}."
        q = cols(p + "self_attn.q_proj.weight", cfg.n_heads * D)
        k = cols(p + "self_attn.k_proj.weight", cfg.n_kv_heads * D)
        v = cols(p + "self_attn.v_proj.weight", cfg.n_kv_heads * D)
        lw = LayerWeights(
            attn_norm=ck.full(p + "input_layernorm.weight"),
            mlp_norm=ck.full(p + "post_attention_layernorm.weight"),
            qkv=torch.cat([q, k, v]),
            o=rows(p + "self_attn.o_proj.weight", cfg.n_heads * D),
        )
        if cfg.is_moe and moe_ep and tp.world > 1:
            ex = p + "block_sparse_moe."
            El = cfg.n_experts // tp.world
            mine = range(tp.rank * El, (tp.rank + 1) * El)
            lw["router"] = ck.full(ex + "gate.weight")
            lw["w13"] = torch.stack([torch.cat([ck.full(f"{ex}experts.{e}.w1.weight"),
                                                ck.full(f"{ex}experts.{e}.w3.weight")])
                                     for e in mine])
            lw["w2"] = torch.stack([ck.full(f"{ex}experts.{e}.w2.weight") for e in mine])
        elif cfg.is_moe:
            ex = p + "block_sparse_moe."
            lw["router"] = ck.full(ex + "gate.weight")
            lw["w13"] = torch.stack([torch.cat([cols(f"{ex}experts.{e}.w1.weight", F),
                                                cols(f"{ex}experts.{e}.w3.weight", F)])
                                     for e in range(cfg.n_experts)])
            lw["w2"] = torch.stack([rows(f"{ex}experts.{e}.w2.weight", F)
                                    for e in range(cfg.n_experts)])
        else:
            lw["gate_up"] = torch.cat([cols(p + "mlp.gate_proj.weight", F),
                                       cols(p + "mlp.up_proj.weight", F)])
            lw["down"] = rows(p + "mlp.down_proj.weight", F)
        layers.append(LayerWeights({k: t.to(device=device, dtype=dtype).contiguous()
                                    for k, t in lw.items()}))
    v0, v1 = tp.shard(cfg.vocab_size)
    head_name = "lm_head.weight" if "lm_head.weight" in ck else "model.embed_tokens.weight"
    return dict(
        embed=ck.full("model.embed_tokens.weight").to(device=device, dtype=dtype),
        final_norm=ck.full("model.norm.weight").to(device=device, dtype=dtype),
        lm_head=ck.rows(head_name, v0, v1).to(device=device, dtype=dtype).contiguous(),
        layers=layers,
        vocab_start=v0,
    )


def shard_weights(full: dict, cfg: ModelConfig, tp: TPContext, moe_ep: bool = False) -> dict:
    """Slice full (TP=1) weights into this rank's Megatron shard (same layout as
    init_weights), e.g. to check TP numerics against the single-device model.
    moe_ep: whole experts per rank instead of FFN-split experts."""
    D, R, r = cfg.head_dim, tp.world, tp.rank
    hq, hkv, F = cfg.n_heads // R, cfg.n_kv_heads // R, cfg.ffn // R
    Hq, Hkv = cfg.n_heads, cfg.n_kv_heads
    layers = []
    for lw in full["layers"]:
        q = lw["qkv"][: Hq * D][r * hq * D:(r + 1) * hq * D]
        k = lw["qkv"][Hq * D:(Hq + Hkv) * D][r * hkv * D:(r + 1) * hkv * D]
        v = lw["qkv"][(Hq + Hkv) * D:][r * hkv * D:(r + 1) * hkv * D]
        out = LayerWeights(attn_norm=lw["attn_norm"], mlp_norm=lw["mlp_norm"],
                           qkv=torch.cat([q, k, v]).contiguous(),
                           o=lw["o"][:, r * hq * D:(r + 1) * hq * D].contiguous())
        if cfg.is_moe and moe_ep:
            El = cfg.n_experts // R
            out["router"] = lw["router"]
            out["w13"] = lw["w13"][r * El:(r + 1) * El].contiguous()
            out["w2"] = lw["w2"][r * El:(r + 1) * El].contiguous()
        elif cfg.is_moe:
            Ff = cfg.ffn
            out["router"] = lw["router"]
            out["w13"] = torch.cat([lw["w13"][:, r * F:(r + 1) * F],
                                    lw["w13"][:, Ff + r * F:Ff + (r + 1) * F]], 1).contiguous()
            out["w2"] = lw["w2"][:, :, r * F:(r + 1) * F].contiguous()
        else:
            Ff = cfg.ffn
            out["gate_up"] = torch.cat([lw["gate_up"][r * F:(r + 1) * F],
                                        lw["gate_up"][Ff + r * F:Ff + (r + 1) * F]]).contiguous()
            out["down"] = lw["down"][:, r * F:(r + 1) * F].contiguous()
        layers.append(out)
    v0, v1 = tp.shard(cfg.vocab_size)
    return dict(embed=full["embed"], final_norm=full["final_norm"],
                lm_head=full["lm_head"][v0:v1].contiguous(), layers=layers, vocab_start=v0)


def export_hf(full: dict, cfg: ModelConfig) -> dict[str, torch.Tensor]:
    """Inverse of load_safetensors for TP=1 weights: HF tensor names -> tensors
    (used to write test checkpoints and to round-trip the loader)."""
    D, F, Hq, Hkv = cfg.head_dim, cfg.ffn, cfg.n_heads, cfg.n_kv_heads
    out = {"model.embed_tokens.weight": full["embed"], "model.norm.weight": full["final_norm"],
           "lm_head.weight": full["lm_head"]}
    from .. import ops

    for li, lw in enumerate(full["layers"]):
        p = f"model.layers.{li}."
        # an engine's in-place decode-tiled projections (DecoderLM.tile_decode_weights)
        lw = {k: ops.untile_weight(v) if isinstance(v, torch.Tensor) and ops.tiled_only(v)
              else v for k, v in lw.items()}
        out[p + "input_layernorm.weight"] = lw["attn_norm"]
        out[p + "post_attention_layernorm.weight"] = lw["mlp_norm"]
        out[p + "self_attn.q_proj.weight"] = lw["qkv"][: Hq * D]
        out[p + "self_attn.k_proj.weight"] = lw["qkv"][Hq * D:(Hq + Hkv) * D]
        out[p + "self_attn.v_proj.weight"] = lw["qkv"][(Hq + Hkv) * D:]
        out[p + "self_attn.o_proj.weight"] = lw["o"]
        if cfg.is_moe:
            ex = p + "block_sparse_moe."
            out[ex + "gate.weight"] = lw["router"]
            for e in range(cfg.n_experts):
                out[f"{ex}experts.{e}.w1.weight"] = lw["w13"][e, :F]
                out[f"{ex}experts.{e}.w3.weight"] = lw["w13"][e, F:]
                out[f"{ex}experts.{e}.w2.weight"] = lw["w2"][e]
        else:
            out[p + "mlp.gate_proj.weight"] = lw["gate_up"][:F]
            out[p + "mlp.up_proj.weight"] = lw["gate_up"][F:]
            out[p + "mlp.down_proj.weight"] = lw["down"]
    return {k: v.contiguous() for k, v in out.items()}
