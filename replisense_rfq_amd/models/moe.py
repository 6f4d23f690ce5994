"""Mixtral sparse-MoE MLP on the gfx950 kernels (BASELINE.json config 5).

The routed computation runs entirely in hand-written kernels
(``csrc/kernels/moe.hip``): top-2 router softmax, counting-sort alignment of the
(token, slot) pairs into 128-row expert blocks, row gather, MFMA grouped GEMM for
the fused w1|w3 projection, SwiGLU, grouped GEMM for w2 and the weighted combine.
Buffers are sized from upper bounds once per batch size so the chain can be
captured into a hipGraph.  On CPU the torch oracle (:func:`ops.reference.moe_forward`)
is used instead.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import torch

from .. import ops
from ..ops import reference as ref

BLOCK_M = 128
BLOCK_S = 16            # expert segment padding on the small-batch path
SKINNY_MAX_TOKENS = 64  # T <= this: per-expert weight-streaming kernels
# K slices of the latency-path w2 (gemm_skinny.hip moe_skinny_kernel SPLIT): 0/1 = off
W2_SPLITS = int(os.environ.get("RFQ_MOE_W2_SPLITS", "2"))
# Throughput-path grouped w2 split-K (gemm_w4.hip GROUPED KS = 2): "auto" lets the GEMM
# and the combine decide on the device from the live tile count (common.h moe_w2_ksplit);
# "0" never splits
W2_KSPLIT = os.environ.get("RFQ_MOE_W2_KSPLIT", "auto")


@dataclass
class MoEBuffers:
    max_tokens: int
    topk: int
    E: int
    weights: torch.Tensor
    ids: torch.Tensor
    sorted_ids: torch.Tensor
    inv_pos: torch.Tensor
    expert_of_block: torch.Tensor
    expert_offsets: torch.Tensor
    num_blocks: torch.Tensor
    xs: torch.Tensor
    h13: torch.Tensor
    act: torch.Tensor
    y: torch.Tensor
    yf: torch.Tensor | None = None     # [W2_SPLITS, rows, d] fp32 split-K w2 partials
    yf2: torch.Tensor | None = None    # [2, cap, d] fp32 throughput-path split-K w2 partials

    @classmethod
    def allocate(cls, max_tokens: int, topk: int, E: int, d: int, F: int, device,
                 dtype=torch.bfloat16) -> "MoEBuffers":
        n = max_tokens * topk
        cap = n + E * (BLOCK_M - 1)
        cap = (cap + BLOCK_M - 1) // BLOCK_M * BLOCK_M
        nb = cap // BLOCK_M
        i32 = dict(dtype=torch.int32, device=device)
        return cls(
            max_tokens=max_tokens, topk=topk, E=E,
            weights=torch.empty(max_tokens, topk, dtype=torch.float32, device=device),
            ids=torch.empty(max_tokens, topk, **i32),
            sorted_ids=torch.empty(cap, **i32),
            inv_pos=torch.empty(n, **i32),
            expert_of_block=torch.empty(max(nb, (n + E * (BLOCK_S - 1)) // BLOCK_S + 1), **i32),
            expert_offsets=torch.empty(E + 1, **i32),
            num_blocks=torch.empty(1, **i32),
            xs=torch.empty(cap, d, dtype=dtype, device=device),
            h13=torch.empty(cap, 2 * F, dtype=dtype, device=device),
            act=torch.empty(cap, F, dtype=dtype, device=device),
            y=torch.empty(cap, d, dtype=dtype, device=device),
            yf=(torch.empty(W2_SPLITS, n + (E + 2) * BLOCK_S, d, dtype=torch.float32,
                            device=device)
                if max_tokens <= SKINNY_MAX_TOKENS and W2_SPLITS > 1 else None),
            yf2=(torch.empty(2, cap, d, dtype=torch.float32, device=device)
                 if max_tokens > SKINNY_MAX_TOKENS and W2_KSPLIT != "0" else None),
        )


def moe_mlp(x: torch.Tensor, router_w: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor,
            topk: int, bufs: MoEBuffers | None, out: torch.Tensor | None = None,
            expert_offset: int = 0) -> torch.Tensor:
    """x [T, d] -> [T, d].  w13 [E, 2F, d] (gate|up), w2 [E, d, F], router_w [E_all, d].

    Expert parallelism: when this rank holds experts [expert_offset, expert_offset +
    E) of E_all, pairs routed elsewhere are sent to a dummy expert segment that no
    kernel computes and get combine weight 0; the TP all-reduce after the MLP sums
    the ranks' partial outputs (each expert runs on exactly one rank)."""
    T = x.shape[0]
    if not x.is_cuda:
        return ref.moe_forward(x, w13, w2, x @ router_w.t(), topk, expert_offset)
    E = w13.shape[0]
    ep = E != router_w.shape[0]
    assert bufs is not None and T <= bufs.max_tokens
    out = torch.empty_like(x) if out is None else out
    # buffers are sliced to this step's token count but keep their capacity-based
    # padding so the grouped GEMM grid is fixed for a given bucket
    n = T * topk
    w, ids = bufs.weights[:T], bufs.ids[:T]
    if ep:
        E = E + 1                  # + the dummy segment for remote experts
    if T <= SKINNY_MAX_TOKENS:
        # decode / short-extend steps: router GEMV + top-k in one kernel, stream only
        # the routed experts' weights, gather rows on the fly, SwiGLU fused into w13
        ops.moe_route(x, router_w, topk, True, w, ids)
        if ep:
            _localize(ids, w, expert_offset, E - 1)
        cap = (n + E * (BLOCK_S - 1) + BLOCK_S - 1) // BLOCK_S * BLOCK_S
        sorted_ids = bufs.sorted_ids[:cap]
        ops.moe_align(ids, E, BLOCK_S, sorted_ids, bufs.inv_pos[:n],
                      bufs.expert_of_block[:cap // BLOCK_S], bufs.expert_offsets,
                      bufs.num_blocks)
        F = w2.shape[2]
        act = bufs.act[:cap]
        y = bufs.y[:cap]
        ops.moe_skinny(x, sorted_ids, topk, bufs.expert_offsets, w13, act, True, True, n)
        assert act.shape[1] == F
        if bufs.yf is not None:
            # split-K w2: fp32 partial slabs, summed inside the top-k combine
            ops.moe_skinny_splitk(act, sorted_ids, topk, bufs.expert_offsets, w2, bufs.yf, n,
                                  W2_SPLITS)
            ops.moe_combine_splitk(bufs.yf, W2_SPLITS, bufs.inv_pos[:n], w, topk, out)
            return out
        ops.moe_skinny(act, sorted_ids, topk, bufs.expert_offsets, w2, y, False, False, n)
        ops.moe_combine(y, bufs.inv_pos[:n], w, topk, out)
        return out
    logits = x @ router_w.t()
    cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
    nb = cap // BLOCK_M
    ops.moe_topk(logits, topk, True, w, ids)
    if ep:
        _localize(ids, w, expert_offset, E - 1)
    sorted_ids, eob = bufs.sorted_ids[:cap], bufs.expert_of_block[:nb]
    ops.moe_align(ids, E, BLOCK_M, sorted_ids, bufs.inv_pos[:n], eob, bufs.expert_offsets,
                  bufs.num_blocks)
    xs, h13, act, y = bufs.xs[:cap], bufs.h13[:cap], bufs.act[:cap], bufs.y[:cap]
    ops.moe_gather(x, sorted_ids, topk, xs)
    if ops.moe_gemm_dense_ok(w13, True) and ops.moe_gemm_dense_ok(w2, False):
        # grouped GEMMs on the dense kernel's 8-wave ping-pong MFMA structure
        # (gemm_dense.hip GROUPED): the segment offsets are read on the device, the
        # grid is fixed by the capacity, w13's epilogue applies SwiGLU.  Measured
        # (profiles/r3_moe_dense_grouped.md) faster than round 2's grouped kernel and
        # than one hipBLASLt GEMM per expert at every step size from 512 to 16K tokens,
        # so no step reads the offsets back to the host
        ops.moe_gemm_dense(xs, w13, act, bufs.expert_offsets, True)
        if bufs.yf2 is not None and ops.MOE_W4 and w2_split_ok(w2):
            # w2 + combine with the split-K decision taken on the device (the live tile
            # count depends on the routing): fp32 K-slice slabs in yf2 or bf16 rows in y
            ops.moe_w2_combine(act, w2, y, bufs.yf2, bufs.expert_offsets, bufs.inv_pos[:n], w,
                               topk, out, _cus(x.device))
            return out
        ops.moe_gemm_dense(act, w2, y, bufs.expert_offsets, False)
    elif ops.moe_gemm8_ok(w13, True) and ops.moe_gemm8_ok(w2, False):
        w2_tile = 256 if n >= 320 * w13.shape[0] else 128
        ops.moe_gemm8(xs, w13, act, eob, bufs.num_blocks, bufs.expert_offsets, True, 256)
        ops.moe_gemm8(act, w2, y, eob, bufs.num_blocks, bufs.expert_offsets, False, w2_tile)
    else:
        ops.moe_grouped_gemm(xs, w13, h13, eob, bufs.num_blocks)
        ops.silu_mul(h13, act)
        ops.moe_grouped_gemm(act, w2, y, eob, bufs.num_blocks)
    ops.moe_combine(y, bufs.inv_pos[:n], w, topk, out)
    return out


def w2_split_ok(w2: torch.Tensor) -> bool:
    """Shapes the split-K grouped w2 takes (w2 [E, d, F]: d % 256, F % 256, F >= 512)."""
    d, F = w2.shape[1], w2.shape[2]
    return d % 256 == 0 and F % 256 == 0 and F >= 512


_CUS: dict = {}


def _cus(device) -> int:
    if device not in _CUS:
        _CUS[device] = torch.cuda.get_device_properties(device).multi_processor_count
    return _CUS[device]


def _localize(ids: torch.Tensor, w: torch.Tensor, e0: int, e_local: int) -> None:
    """Global expert ids -> this rank's local ids; remote pairs -> dummy id e_local
    with weight 0 (graph-capturable tensor ops)."""
    loc = ids - e0
    mine = (loc >= 0) & (loc < e_local)
    ids.copy_(torch.where(mine, loc, torch.full_like(loc, e_local)))
    w.mul_(mine.to(w.dtype))

