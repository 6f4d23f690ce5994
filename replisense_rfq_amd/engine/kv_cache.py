"""Paged KV cache: device pools + native block manager + prefix cache.

Pools are two tensors ``[L, num_blocks, Hkv_local, 32, 128]`` (bf16), sized from a
fraction of free HBM (288 GB per MI355X: a Llama-3-8B replica gets ~100 GB of
KV = ~800K tokens, far beyond the ≤3.7K-token RFQ sequences × max batch).  The
last block is a scratch page for padded graph rows and is never handed out.
Block bookkeeping (refcounts, free list, LRU of cached prefix blocks, chained
block hashes) lives in the C++ runtime (csrc/runtime/block_manager.cpp).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import runtime
from ..models.config import ModelConfig
from .sequence import Sequence


class KVCache:
    def __init__(self, cfg: ModelConfig, hkv_local: int, num_blocks: int, device,
                 block_size: int = 32, dtype=torch.bfloat16, prefix_cache: bool = True):
        if block_size != 32:
            raise ValueError("the gfx950 attention kernels use 32-token pages")
        self.cfg = cfg
        self.block_size = block_size
        self.num_blocks = num_blocks
        shape = (cfg.n_layers, num_blocks, hkv_local, block_size, cfg.head_dim)
        self.k = torch.empty(shape, dtype=dtype, device=device)
        self.v = torch.empty(shape, dtype=dtype, device=device)
        if not self.k.is_cuda:
            self.k.zero_()
            self.v.zero_()
        self.scratch_block = num_blocks - 1
        self.bm = runtime.load().BlockManager(num_blocks - 1, block_size)
        self.prefix_cache = prefix_cache

    @staticmethod
    def bytes_per_block(cfg: ModelConfig, hkv_local: int, block_size: int = 32) -> int:
        return 2 * cfg.n_layers * hkv_local * block_size * cfg.head_dim * 2

    @classmethod
    def blocks_for_memory(cls, cfg, hkv_local, free_bytes, fraction, block_size=32) -> int:
        return max(16, int(free_bytes * fraction) // cls.bytes_per_block(cfg, hkv_local, block_size))

    # ------------------------------------------------------------ sequences
    @property
    def num_free(self) -> int:
        return self.bm.num_free

    def blocks_needed(self, seq: Sequence, upto: int) -> int:
        need = (upto + self.block_size - 1) // self.block_size
        return max(0, need - len(seq.blocks))

    def admit(self, seq: Sequence) -> bool:
        """Prefix-match the prompt and reserve its first chunk lazily (grow())."""
        bs = self.block_size
        if self.prefix_cache and seq.prompt_len > bs:
            toks = np.asarray(seq.prompt, np.int32)
            seq.block_hashes = list(self.bm.hash_blocks(toks, bs, 0))
            # keep >= 1 prompt token to compute so the first sampled token has logits
            usable = seq.block_hashes[: (seq.prompt_len - 1) // bs]
            hit = self.bm.match_prefix(usable)
            if hit:
                seq.blocks = list(hit)
                seq.num_cached = len(hit) * bs
                seq.num_registered = len(hit)
                seq.prefix_hit_tokens = seq.num_cached
        return True

    def grow(self, seq: Sequence, upto: int) -> bool:
        n = self.blocks_needed(seq, upto)
        if n == 0:
            return True
        got = self.bm.allocate(n)
        if got is None:
            return False
        seq.blocks.extend(got)
        return True

    def publish(self, seq: Sequence) -> None:
        """Register prompt blocks that are now completely written."""
        if not self.prefix_cache or not seq.block_hashes:
            return
        full = min(seq.num_cached, seq.prompt_len) // self.block_size
        full = min(full, len(seq.block_hashes))
        for i in range(seq.num_registered, full):
            self.bm.register_block(seq.blocks[i], seq.block_hashes[i])
        seq.num_registered = max(seq.num_registered, full)

    def free(self, seq: Sequence) -> None:
        if seq.blocks:
            self.bm.release(seq.blocks)
        seq.blocks = []

    def slot(self, seq: Sequence, pos: int) -> int:
        return seq.blocks[pos // self.block_size] * self.block_size + pos % self.block_size

    def stats(self) -> dict:
        return {"blocks": self.num_blocks, "free": self.bm.num_free, "cached": self.bm.num_cached,
                "prefix_queries": self.bm.queries, "prefix_hits": self.bm.hits,
                "evictions": self.bm.evictions}
