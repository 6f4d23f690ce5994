"""Paged KV cache: device pools + native block manager + prefix cache.

Pools are two tensors ``[L, num_blocks, Hkv_local, 32, 128]`` (bf16), sized from a
fraction of free HBM (288 GB per MI355X: a Llama-3-8B replica gets ~100 GB of
KV = ~800K tokens, far beyond the ≤3.7K-token RFQ sequences × max batch).  The
last block is a scratch page for padded graph rows and is never handed out.
Block bookkeeping (refcounts, free list, LRU of cached prefix blocks, chained
block hashes) lives in the native engine core (csrc/runtime/engine_core.cpp over
block_manager.cpp); this class owns the device pools.
"""
from __future__ import annotations

import torch

from ..models.config import ModelConfig


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
        self.scratch_block = num_blocks - 1      # blocks [0, num_blocks-1) belong to the core
        self.prefix_cache = prefix_cache
        self.core = None                         # set by the engine (block accounting)

    @staticmethod
    def bytes_per_block(cfg: ModelConfig, hkv_local: int, block_size: int = 32) -> int:
        return 2 * cfg.n_layers * hkv_local * block_size * cfg.head_dim * 2

    @classmethod
    def blocks_for_memory(cls, cfg, hkv_local, free_bytes, fraction, block_size=32) -> int:
        return max(16, int(free_bytes * fraction) // cls.bytes_per_block(cfg, hkv_local, block_size))

    def stats(self, core=None) -> dict:
        core = core if core is not None else self.core
        return {"blocks": self.num_blocks, "free": core.num_free_blocks,
                "cached": core.num_cached_blocks, "prefix_queries": core.prefix_queries,
                "prefix_hits": core.prefix_hits, "evictions": core.evictions}
