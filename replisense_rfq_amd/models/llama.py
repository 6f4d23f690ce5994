"""Llama-3 / Mixtral decoder on the gfx950 kernels.

One class serves Llama-3-8B, Llama-3-70B (TP=1..8) and Mixtral-8x7B (sparse MoE
MLP).  A forward pass consumes a *mixed* token batch laid out as
``[decode tokens (one per running sequence) | prefill/extend tokens]``:

  embed -> for each layer:
     fused_add_rms_norm -> QKV GEMM (hipBLASLt) -> rope_kv (q in place, k/v into
     the paged cache; on the latency path one skinny GEMM does both) -> attn_decode (split-K MFMA; decode rows and short grammar
     jump-forward extends) + attn_prefill (varlen causal MFMA flash; prompt
     chunks) -> O GEMM -> [all-reduce]
     -> fused_add_rms_norm -> gate|up GEMM -> silu_mul -> down GEMM -> [all-reduce]
       (TP=1 latency path, when the start-up plan measured it faster: gate|up GEMM with
        the SwiGLU epilogue, down GEMM with the residual-add RMSNorm in-launch)
        (MoE: router -> top-2 -> align -> grouped MFMA GEMMs -> combine)
  -> final norm on the rows that need logits -> vocab-parallel LM head.

Residual adds are fused into the following RMSNorm, the q rotation happens in
place inside the QKV GEMM output, and attention writes straight into the O-GEMM
input, so a layer is 5 GEMMs + 5 custom kernels with no extra copies.  Every op
is stream-ordered and allocation-stable, so the decode path is captured into a
hipGraph by the engine (ModelRunner.capture_graphs, engine/runner.py).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from .. import ops
from ..ops import reference as ref
from ..parallel.tp import SINGLE, TPContext
from .config import ModelConfig
from .moe import MoEBuffers, moe_mlp
from .weights import init_weights

# RFQ_SINGLE_PASS_DECODE: split-K decode attention merges its partials in-kernel (the
# last split wave of each work item, Guideline-16 sc1 hand-off; the whole wave merges
# 4 columns at a time with every split's loads in flight) instead of a second reduce
# launch.  "auto" (default): on where a kv head has at most 4 query columns (8B,
# Mixtral: 8.3 / 9.2 / 11.0 µs vs 8.9 / 9.8 / 11.8 with the reduce launch at ctx
# 512 / 1024 / 2048), off with 8 columns per kv head (70B at TP=8 and TP=1: two merge
# rounds, the reduce launch is 0.6-0.9 µs faster) -- profiles/r5_tp8_rank_emulation.md.
SINGLE_PASS_DECODE = os.environ.get("RFQ_SINGLE_PASS_DECODE", "auto").lower()


# RFQ_PERSIST: persistent decode layers (csrc/kernels/decode_persist.hip) for steps whose
# rows are all decode / short-extend rows, at most PERSIST_MAX_M of them, on folded norm
# weights:
#   "1" / "all"  every layer of the step in ONE launch (qkv -> attention -> o -> gate|up ->
#                down, next layer ...; each stage's first weights in flight across its seam)
#   "ao"         per layer: the qkv and MLP row-streaming launches, with attention + o in
#                one persistent launch (the o weights stream while the attention runs)
#   "0"          off: the multi-launch path (_forward_fold)
PERSIST = os.environ.get("RFQ_PERSIST", "0").lower()
PERSIST_MAX_M = 4
PERSIST_FLAGS = int(os.environ.get("RFQ_PERSIST_FLAGS", "0"))


@dataclass
class ForwardMeta:
    """Device-side description of one engine step (all int32 unless noted)."""
    input_ids: torch.Tensor            # [T]
    positions: torch.Tensor            # [T]
    slot_mapping: torch.Tensor         # [T]
    num_decode: int                    # rows [0, num_decode): decode + short-extend section
    dec_block_tables: torch.Tensor | None = None   # [NA, maxb]
    dec_q_start: torch.Tensor | None = None        # [NA] first row of each sequence
    dec_q_len: torch.Tensor | None = None          # [NA]
    dec_kv_len: torch.Tensor | None = None         # [NA]
    dec_work_seq: torch.Tensor | None = None       # [WA] (-1 = padding)
    dec_work_ct: torch.Tensor | None = None        # [WA] 16-column tile index
    num_prefill_tokens: int = 0
    pf_block_tables: torch.Tensor | None = None    # [P, maxb]
    pf_q_start: torch.Tensor | None = None         # [P] offset inside the prefill rows
    pf_q_len: torch.Tensor | None = None           # [P]
    pf_kv_len: torch.Tensor | None = None          # [P]
    work_seq: torch.Tensor | None = None           # [W]
    work_qblk: torch.Tensor | None = None          # [W]
    prefill_qblk: int = 32                         # queries per prefill work item
    logits_idx: torch.Tensor | None = None         # [S] int64 rows needing logits
    decode_splits: int = 1
    decode_tiles: int = 1          # column tiles per decode work item (attn_decode.hip)
    extra: dict = field(default_factory=dict)

    @property
    def num_tokens(self) -> int:
        return self.num_decode + self.num_prefill_tokens


class DecoderLM:
    def __init__(self, cfg: ModelConfig, device, tp: TPContext = SINGLE, seed: int = 0,
                 weights: dict | None = None, dtype=torch.bfloat16, moe_ep: bool = False):
        self.cfg = cfg
        self.tp = tp
        self.device = torch.device(device)
        self.dtype = dtype
        self.hq = cfg.n_heads // tp.world
        self.hkv = cfg.n_kv_heads // tp.world
        # MoE expert parallelism over the TP group: whole experts per rank
        self.moe_ep = bool(moe_ep and cfg.is_moe and tp.world > 1)
        self.ffn_local = cfg.ffn if self.moe_ep else cfg.ffn // tp.world
        self.expert_offset = tp.rank * (cfg.n_experts // tp.world) if self.moe_ep else 0
        self.w = weights if weights is not None else init_weights(cfg, tp, self.device, dtype, seed,
                                                                  moe_ep=self.moe_ep)
        self.vocab_start = self.w["vocab_start"]
        self.vocab_local = self.w["lm_head"].shape[0]
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                        device=self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.kv_k = None
        self.kv_v = None
        self._moe_bufs: dict[int, MoEBuffers] = {}
        self._tickets: torch.Tensor | None = None     # single-pass split decode attention
        # Megatron sequence parallelism for steps of >= sp_min_tokens tokens (TP > 1):
        # the residual stream lives sharded by token rows; each all-reduce becomes a
        # reduce-scatter (then the residual-add RMSNorm runs on 1/W of the rows) and an
        # all-gather before the next column-parallel GEMM.  0 = off (SURVEY.md §2.3 SP).
        self.sp_min_tokens = int(os.environ.get("RFQ_SP_MIN_TOKENS", "0"))
        self.tiled_inplace = False      # some projection stored only in the decode-tiled layout
        self.tiled_plan: dict = {}      # projection -> copy | inplace | off
        self.norms_folded = False       # fold_norms: attn / mlp RMSNorm weights in qkv / gate|up
        self.single_pass = (SINGLE_PASS_DECODE in ("1", "on", "true")
                            or (SINGLE_PASS_DECODE == "auto" and self.hq // self.hkv <= 4))
        self.persist = PERSIST if PERSIST in ("0", "1", "all", "ao", "engine") else "0"
        self._persist_tab = None        # int64 [L, 8] device table of layer pointers
        self._persist_key = None
        self._persist_tk = None         # split-merge tickets of the persistent attention
        self._persist_cnt = None        # seam counters (zeroed; each launch re-zeroes them)

    # ------------------------------------------------------------ folded norms
    def fold_norms(self) -> bool:
        """Fold each layer's attention / MLP RMSNorm weight into the columns of the
        projection that consumes the normalised activations:

            rmsnorm(x) diag(g) W^T = rsqrt(mean(x^2) + eps) * (x W'^T),   W' = W diag(g)

        qkv <- qkv * attn_norm, gate|up <- gate|up * mlp_norm (in place), and both norm
        weights become ones.  The algebra is the same on every path of the forward, but the
        numerics are not bit-identical: W' = bf16(W diag(g)) is rounded once, where the
        unfolded model rounds the normalised activations bf16(rmsnorm(x) g) instead.  The
        logits of the folded model stay within bf16 rounding of the unfolded one (pinned
        at <= 2e-2 relative over a prefill + decode sequence, tests/engine/
        test_fold_norms.py).  What it buys is the TP = 1 small-step path (_forward_fold): the qkv and
        gate|up row-streaming GEMVs read the UN-normalised residual and apply the norm's
        scale themselves (each wave reads the whole row anyway), and the o / down GEMVs add
        into the residual in their epilogue -- no norm launch and no cross-workgroup
        reduction left in a decode layer (2 launches fewer per layer).  Dense models at
        TP = 1 only (RFQ_NORM_FOLD=0 turns it off); the final norm before the LM head
        stays.  Returns whether the weights were folded."""
        # TP > 1: only the one-GPU rank emulation with the persistent path folds (a real
        # group's row-parallel epilogue is the all-reduce + add + RMSNorm kernel, so the
        # emulation keeps that structure unless it runs the persistent layers)
        tp_ok = not self.tp.enabled or (self.tp.emulated and self.persist != "0")
        if (self.norms_folded or self.cfg.is_moe or not tp_ok
                or os.environ.get("RFQ_NORM_FOLD", "1") == "0"):
            return self.norms_folded
        with torch.no_grad():
            for lw in self.w["layers"]:
                lw["qkv"].mul_(lw["attn_norm"][None, :])
                lw["gate_up"].mul_(lw["mlp_norm"][None, :])
                lw["attn_norm_folded"], lw["mlp_norm_folded"] = lw["attn_norm"], lw["mlp_norm"]
                lw["attn_norm"] = torch.ones_like(lw["attn_norm"])
                lw["mlp_norm"] = torch.ones_like(lw["mlp_norm"])
        self.norms_folded = True
        return True

    # ------------------------------------------------------- persistent decode layers
    def _persist_step(self, m: "ForwardMeta", T: int) -> bool:
        """Run this step through _forward_persist (RFQ_PERSIST): GPU, folded norms, dense,
        every row a decode / short-extend row (no prefill section), at most PERSIST_MAX_M
        rows, no cascade attention, row-major projections, no real collectives (TP = 1 or
        the one-GPU rank emulation), and the step's rows fit the kernel's LDS."""
        if self.persist == "0" or not self.norms_folded or self.device.type != "cuda":
            return False
        if self.tp.enabled and not self.tp.emulated:
            return False
        if m.num_prefill_tokens or T < 1 or T > PERSIST_MAX_M or T != m.num_decode:
            return False
        if 0 < ops.SHARED_PREFIX_MIN_ROWS <= m.num_decode or m.decode_splits > 16:
            return False
        lw = self.w["layers"][0]
        if any(ops.tiled_only(lw[k]) for k in ("qkv", "o", "gate_up", "down")):
            return False
        d, qd, F = self.cfg.hidden, self.hq * self.cfg.head_dim, self.ffn_local
        if d % 512 or qd % 512 or F % 512:
            return False
        if self.persist == "engine":
            # loader / consumer form: M <= 2, a row within 3 ring slots, >= 5 slots in LDS
            return (T <= 2 and max(d, qd, F) // 512 <= 33
                    and ops.decode_engine_info(T, d, self.hq, self.hkv, F)[0] > 0)
        mm = 1 if T <= 1 else 2 if T <= 2 else 4
        return 2112 + mm * (d + max(qd, F)) * 2 <= 160 * 1024

    def _persist_state(self):
        """Layer pointer table, tickets and counters of the persistent launch (built once,
        outside graph capture: the engine's warm-up step runs before any capture)."""
        layers = self.w["layers"]
        key = (self.kv_k.data_ptr(), self.kv_v.data_ptr(),
               tuple(lw[k].data_ptr() for lw in layers for k in ("qkv", "o", "gate_up", "down")))
        if self._persist_key != key:
            rows = [[lw["qkv"].data_ptr(), lw["o"].data_ptr(), lw["gate_up"].data_ptr(),
                     lw["down"].data_ptr(), self.kv_k[li].data_ptr(), self.kv_v[li].data_ptr(),
                     0, 0] for li, lw in enumerate(layers)]
            self._persist_tab = torch.tensor(rows, dtype=torch.int64, device=self.device)
            self._persist_key = key
        if self._persist_tk is None:
            self._persist_tk = torch.zeros(4096 * self.hkv, dtype=torch.int32, device=self.device)
            qd = self.hq * self.cfg.head_dim
            words, _, _ = ops.decode_persist_info(1, self.cfg.hidden, max(qd, self.ffn_local),
                                                  self.cfg.n_layers * 5)
            self._persist_cnt = torch.zeros(words, dtype=torch.int32, device=self.device)
        return self._persist_tab, self._persist_tk, self._persist_cnt

    def _forward_persist(self, m: ForwardMeta) -> torch.Tensor:
        """Small decode step on the persistent kernel (csrc/kernels/decode_persist.hip):
        "all" runs every layer in one launch, "engine" the same on the loader / consumer
        form (LDS-DMA weight ring, M <= 2), "ao" keeps qkv / MLP on the row-streaming
        launches and fuses attention + o per layer.  Same numerics as _forward_fold except
        the attention's split boundaries (one wave per (kv head, split), in-kernel merge)."""
        cfg, w = self.cfg, self.w
        T = m.num_tokens
        eps, L = cfg.rms_eps, cfg.n_layers
        qd, F = self.hq * cfg.head_dim, self.ffn_local
        tab, tk, cnt = self._persist_state()
        residual = ops.embed(m.input_ids[:T], w["embed"])
        attn = torch.empty((T, qd), dtype=self.dtype, device=self.device)
        act = torch.empty((T, F), dtype=self.dtype, device=self.device)
        S = max(1, m.decode_splits)
        if S > 1:
            po = torch.empty(T * self.hq * S * 128, device=self.device)
            pm = torch.empty(T * self.hq * S * 2, device=self.device)
        else:
            po = pm = torch.empty(1, device=self.device)
        meta = (m.positions, self.cos_sin, m.slot_mapping, m.dec_block_tables, m.dec_q_start,
                m.dec_q_len, m.dec_kv_len, m.dec_work_seq, m.dec_work_ct, po, pm, tk, cnt)
        if self.persist == "ao":
            for li in range(L):
                lw = w["layers"][li]
                qkv = ops.rows_rope_normx(residual, lw["qkv"], m.positions, self.cos_sin,
                                          m.slot_mapping, self.kv_k[li], self.kv_v[li], self.hq,
                                          self.hkv, eps)
                ops.decode_persist(residual, tab, qkv, attn, act, *meta, li, li + 1,
                                   ops.PERSIST_ATTN | ops.PERSIST_O, self.hq, self.hkv, F,
                                   self.kv_k.shape[3], S, self.scale, eps, PERSIST_FLAGS)
                a = ops.rows_swiglu_normx(residual, lw["gate_up"], eps)
                ops.rows_residual_add(a, lw["down"], residual)
        else:
            qbuf = torch.empty((T, qd), dtype=self.dtype, device=self.device)
            flags = PERSIST_FLAGS | (ops.PERSIST_ENGINE if self.persist == "engine" else 0)
            ops.decode_persist(residual, tab, qbuf, attn, act, *meta, 0, L, ops.PERSIST_STAGES,
                               self.hq, self.hkv, F, self.kv_k.shape[3], S, self.scale, eps,
                               flags)
        x = ops.rms_norm(residual, w["final_norm"], eps)
        xs = x if m.logits_idx is None else x.index_select(0, m.logits_idx)
        return ops.linear(xs, w["lm_head"])

    def _fold_step(self, m: "ForwardMeta", T: int) -> bool:
        """Run this step through _forward_fold: folded weights, a small step whose
        projections all fit the row-streaming GEMV, no cascade (shared-prefix) attention
        (_forward_fold has no normalised activations for it to read)."""
        if not self.norms_folded or T < 1:
            return False
        if 0 < ops.SHARED_PREFIX_MIN_ROWS <= m.num_decode:
            return False
        lw = self.w["layers"][0]
        d = self.cfg.hidden
        return (ops.fold_ok(T, d, lw["qkv"]) and ops.fold_ok(T, self.hq * self.cfg.head_dim, lw["o"])
                and ops.fold_ok(T, self.ffn_local, lw["down"])
                and not ops.tiled_only(lw["qkv"]) and not ops.tiled_only(lw["gate_up"])
                and not ops.tiled_only(lw["o"]) and not ops.tiled_only(lw["down"]))

    # ------------------------------------------------------- decode weight layout
    TILED_PROJ = ("qkv", "o", "gate_up", "down")

    def tile_decode_weights(self, mode: str | None = None) -> int:
        """Decode-tiled layout (ops.tile_weight) of the per-layer projections for the
        split-K GEMVs of small-batch decode steps: each wave load is then 1 KB of
        contiguous weight bytes.  Per projection, one of:

          copy     a tiled copy next to the row-major weight (large-M GEMMs keep
                   hipBLASLt / the plan's kernels);
          inplace  the row-major weight is replaced: small steps run the tiled split-K
                   GEMVs, large ones the hand-written dense GEMM on the tiled layout
                   (gemm_dense cfg 2|4; no library GEMM can read it).

        ``auto`` (RFQ_TILED_WEIGHTS, default) copies projections, smallest first, while
        the copies stay within 25 % of the device's memory (and 40 % of what is free;
        ranks sharing one GPU in a rehearsal set RFQ_TILED_WEIGHTS=0) and tiles the rest
        in place -- unless the norms are folded (the row-streaming decode path needs the
        row-major weight; then the rest stays row-major): 8B and the 70B TP=8 shard copy
        all four, 70B at TP=1 copies o and qkv and keeps gate|up and down row-major.  ``copy`` / ``inplace`` force one mode for all.  Dense models
        only.  The start-up plan (ops.autotune) times the tiled cfgs.  Returns the bytes
        of the extra copies."""
        mode = (mode or os.environ.get("RFQ_TILED_WEIGHTS", "auto")).lower()
        if mode in ("0", "off", "false") or self.cfg.is_moe or self.device.type != "cuda":
            return 0
        layers = self.w["layers"]
        names = [k for k in self.TILED_PROJ if k in layers[0]]
        size = {k: sum(lw[k].numel() * lw[k].element_size() for lw in layers) for k in names}

        def inplace_ok(k):           # the tiled dense GEMM's shape constraints
            t = layers[0][k]
            return t.shape[0] % 256 == 0 and t.shape[1] % 128 == 0

        if mode == "auto":
            free, total = torch.cuda.mem_get_info(self.device)
            budget = min(0.25 * total, 0.40 * free)
            plan, used = {}, 0
            for k in sorted(names, key=lambda n: size[n]):
                if used + size[k] <= budget:
                    plan[k], used = "copy", used + size[k]
                elif self.norms_folded:
                    # the folded-norm decode path streams row-major weights (gemv_rows);
                    # a tiled-only projection would send every small step to the split-K
                    # GEMVs instead: 70B TP=1 single stream 44.4 vs 42.5 sampled steps/s
                    # with gate|up row-major (profiles/r6/llama70b_tp1_tiling_ab.txt)
                    plan[k] = "off"
                else:
                    plan[k] = "inplace" if inplace_ok(k) else "off"
        elif mode == "inplace":
            plan = {k: "inplace" if inplace_ok(k) else "off" for k in names}
        else:
            plan = {k: "copy" for k in names}
        copied = 0
        for k in names:
            if plan[k] == "copy":
                for lw in layers:
                    t = lw[k]
                    if t.shape[0] % 16 == 0 and t.shape[1] % 128 == 0:
                        ops.register_tiled(t, ops.tile_weight(t))
                copied += size[k]
            elif plan[k] == "inplace":
                for lw in layers:
                    lw[k] = ops.tile_weight(lw[k])          # the row-major tensor is freed
                    ops.register_tiled(lw[k], None)
        self.tiled_plan = plan
        self.tiled_inplace = any(v == "inplace" for v in plan.values())
        return copied

    # ------------------------------------------------------------------ KV pool
    def attach_kv_cache(self, k_pool: torch.Tensor, v_pool: torch.Tensor) -> None:
        """Pools shaped [L, num_blocks, Hkv_local, 32, 128]."""
        assert k_pool.shape[0] == self.cfg.n_layers and k_pool.shape[2] == self.hkv
        self.kv_k, self.kv_v = k_pool, v_pool

    def moe_buffers(self, max_tokens: int) -> MoEBuffers:
        cap = 1
        while cap < max_tokens:
            cap *= 2
        if cap not in self._moe_bufs:
            self._moe_bufs[cap] = MoEBuffers.allocate(cap, self.cfg.moe_topk, self.cfg.n_experts,
                                                      self.cfg.hidden, self.ffn_local,
                                                      self.device, self.dtype)
        return self._moe_bufs[cap]

    # ------------------------------------------------------------------ forward
    def forward(self, m: ForwardMeta) -> torch.Tensor:
        cfg, w = self.cfg, self.w
        T = m.num_tokens
        eps = cfg.rms_eps
        qd = self.hq * cfg.head_dim

        if self.tp.enabled and 0 < self.sp_min_tokens <= T:
            return self._forward_sp(m)
        if self._persist_step(m, T):
            return self._forward_persist(m)
        if self._fold_step(m, T):
            return self._forward_fold(m)
        h = ops.embed(m.input_ids[:T], w["embed"])
        residual = h
        x = ops.rms_norm(h, w["layers"][0]["attn_norm"], eps)
        attn = torch.empty((T, qd), dtype=self.dtype, device=self.device)
        dec_parts, shared = self._attn_scratch(m, x)
        moe_bufs = self.moe_buffers(T) if (cfg.is_moe and x.is_cuda) else None
        L = cfg.n_layers
        # TP = 1 latency path: the o / down skinny GEMM runs the residual-add
        # RMSNorm in its last workgroup when the start-up plan measured it faster
        fuse = not self.tp.enabled and T <= ops.NORM_FUSE_MAX_M
        for li in range(L):
            lw = w["layers"][li]
            self._attend(li, x, attn, m, dec_parts, shared)
            if not (fuse and ops.linear_add_norm(attn, lw["o"], residual, lw["mlp_norm"], eps,
                                                 x)):
                o = ops.linear(attn, lw["o"])
                self.tp.all_reduce_add_norm_(o, residual, lw["mlp_norm"], eps, x)
            nxt = w["layers"][li + 1]["attn_norm"] if li + 1 < L else w["final_norm"]
            if cfg.is_moe:
                mo = moe_mlp(x, lw["router"], lw["w13"], lw["w2"], cfg.moe_topk, moe_bufs,
                             expert_offset=self.expert_offset)
            else:
                # latency path (any TP degree): gate|up with the SwiGLU epilogue (one
                # kernel, [M, F] out); TP = 1 may also fold the norm into down
                act = ops.linear_swiglu(x, lw["gate_up"]) if T <= ops.NORM_FUSE_MAX_M else None
                if act is not None:
                    if fuse and ops.linear_add_norm(act, lw["down"], residual, nxt, eps, x):
                        continue
                    mo = ops.linear(act, lw["down"])
                else:
                    # throughput path: gate|up with the SwiGLU epilogue in the hand-written
                    # large-M MFMA GEMM when the start-up plan measured it faster
                    act = ops.swiglu_large(x, lw["gate_up"])
                    if act is not None:
                        mo = ops.linear(act, lw["down"])
                        self.tp.all_reduce_add_norm_(mo, residual, nxt, eps, x)
                        continue
                    gu = ops.linear(x, lw["gate_up"])
                    if fuse and ops.linear_add_norm(gu, lw["down"], residual, nxt, eps, x,
                                                    gated=True):
                        continue
                    mo = ops.silu_linear(gu, lw["down"])
            self.tp.all_reduce_add_norm_(mo, residual, nxt, eps, x)
        xs = x if m.logits_idx is None else x.index_select(0, m.logits_idx)
        return ops.linear(xs, w["lm_head"])

    def _forward_fold(self, m: ForwardMeta) -> torch.Tensor:
        """Small-step forward over folded norm weights (fold_norms; TP = 1): the residual
        stream itself is every layer's input, so a layer is

            qkv + RoPE + KV append (norm scale in-kernel) -> attention -> o (+= residual)
            -> gate|up + SwiGLU (norm scale in-kernel) -> down (+= residual)

        four row-streaming GEMVs and the attention launches, with no RMSNorm launch and no
        cross-workgroup reduction (csrc/kernels/gemv_rows.hip kRwNormX / kRwResAdd)."""
        cfg, w = self.cfg, self.w
        T = m.num_tokens
        eps = cfg.rms_eps
        qd = self.hq * cfg.head_dim
        residual = ops.embed(m.input_ids[:T], w["embed"])
        attn = torch.empty((T, qd), dtype=self.dtype, device=self.device)
        dec_parts, shared = self._attn_scratch(m, residual)
        for li in range(cfg.n_layers):
            lw = w["layers"][li]
            qkv = ops.rows_rope_normx(residual, lw["qkv"], m.positions, self.cos_sin,
                                      m.slot_mapping, self.kv_k[li], self.kv_v[li], self.hq,
                                      self.hkv, eps)
            # x = None: with qkv precomputed _attend reads no activations (the residual
            # here is not normalised)
            self._attend(li, None, attn, m, dec_parts, shared, qkv=qkv)
            ops.rows_residual_add(attn, lw["o"], residual)
            act = ops.rows_swiglu_normx(residual, lw["gate_up"], eps)
            ops.rows_residual_add(act, lw["down"], residual)
        x = ops.rms_norm(residual, w["final_norm"], eps)
        xs = x if m.logits_idx is None else x.index_select(0, m.logits_idx)
        return ops.linear(xs, w["lm_head"])

    def _forward_sp(self, m: ForwardMeta) -> torch.Tensor:
        """Sequence-parallel forward (TP group of W ranks, T tokens padded to Tp = W*n).

        Per layer: AG(x shard) -> QKV / attention / O (rows [0, T) real) -> RS ->
        residual-add RMSNorm on this rank's n rows -> AG -> gate|up / down -> RS ->
        residual-add RMSNorm.  Same bytes on the wire as two all-reduces, but the
        norms and the residual stream cost 1/W; padding rows are zero and never read
        back.  The final shard is gathered once before the vocab-parallel LM head."""
        cfg, w, tp = self.cfg, self.w, self.tp
        T, W, eps = m.num_tokens, tp.world, cfg.rms_eps
        n = -(-T // W)
        Tp, lo = n * W, tp.rank * n
        d = cfg.hidden
        h = torch.zeros((Tp, d), dtype=self.dtype, device=self.device)
        ops.embed(m.input_ids[:T], w["embed"], out=h[:T])
        residual = h[lo:lo + n].clone()
        xs = ops.rms_norm(residual, w["layers"][0]["attn_norm"], eps)
        x = torch.empty((Tp, d), dtype=self.dtype, device=self.device)
        part = torch.empty((Tp, d), dtype=self.dtype, device=self.device)
        shard = torch.empty((n, d), dtype=self.dtype, device=self.device)
        attn = torch.zeros((Tp, self.hq * cfg.head_dim), dtype=self.dtype, device=self.device)
        dec_parts, shared = self._attn_scratch(m, x)
        moe_bufs = self.moe_buffers(Tp) if (cfg.is_moe and x.is_cuda) else None
        L = cfg.n_layers
        for li in range(L):
            lw = w["layers"][li]
            tp.all_gather_rows(x, xs)
            self._attend(li, x, attn, m, dec_parts, shared)
            ops.linear(attn, lw["o"], out=part)
            tp.reduce_scatter_rows(shard, part)
            ops.fused_add_rms_norm(shard, residual, lw["mlp_norm"], eps, out=xs)
            tp.all_gather_rows(x, xs)
            nxt = w["layers"][li + 1]["attn_norm"] if li + 1 < L else w["final_norm"]
            if cfg.is_moe:
                mo = moe_mlp(x, lw["router"], lw["w13"], lw["w2"], cfg.moe_topk, moe_bufs,
                             expert_offset=self.expert_offset)
            else:
                mo = ops.silu_linear(ops.linear(x, lw["gate_up"]), lw["down"])
            tp.reduce_scatter_rows(shard, mo)
            ops.fused_add_rms_norm(shard, residual, nxt, eps, out=xs)
        tp.all_gather_rows(x, xs)
        x = x[:T]
        xs = x if m.logits_idx is None else x.index_select(0, m.logits_idx)
        return ops.linear(xs, w["lm_head"])

    def _dec_tickets(self, work_items: int):
        """Zeroed int32 tickets for single-pass split decode attention (the kernel resets
        each entry it uses, so one persistent buffer serves every layer and graph replay).
        Sized once, before any capture: split decode only runs below 1024 (work item, kv
        head) waves (engine/runner.py _decode_splits), extend rows at most 4x that.
        Used where the single-pass merge is on (RFQ_SINGLE_PASS_DECODE)."""
        if self.device.type != "cuda" or not self.single_pass:
            return None
        if self._tickets is None:
            self._tickets = torch.zeros(4096 * self.hkv, dtype=torch.int32, device=self.device)
        return self._tickets if work_items * self.hkv <= self._tickets.numel() else None

    def _attn_scratch(self, m: ForwardMeta, x: torch.Tensor):
        """Split-K partials for decode attention and cascade-attention scratch."""
        D, hq = m.num_decode, self.hq
        dec_parts = None
        if D > 0 and m.decode_splits > 1 and x.is_cuda:
            dec_parts = (torch.empty(D * hq * m.decode_splits * 128, device=self.device),
                         torch.empty(D * hq * m.decode_splits * 2, device=self.device))
        shared = None
        if (D >= ops.SHARED_PREFIX_MIN_ROWS and dec_parts is None and x.is_cuda
                and ops.SHARED_PREFIX_MIN_ROWS > 0):
            # cascade attention over the shared prompt pages (meta computed in layer 0)
            nseq = m.dec_q_len.shape[0]
            shared = (torch.empty(2 + nseq + D, dtype=torch.int32, device=self.device),
                      torch.empty(D * hq * 128, device=self.device),
                      torch.empty(D * hq * 2, device=self.device))
        return dec_parts, shared

    def _attend(self, li: int, x, attn, m: ForwardMeta, dec_parts, shared, qkv=None) -> None:
        """QKV GEMM + RoPE + paged-KV append (unless ``qkv`` comes precomputed, as on the
        folded-norm path), then decode / prefill attention into ``attn`` (rows [0, T) of x
        and attn; rows past T are SP padding)."""
        T, D = m.num_tokens, m.num_decode
        hq, hkv = self.hq, self.hkv
        lw = self.w["layers"][li]
        kc, vc = self.kv_k[li], self.kv_v[li]
        if qkv is None:
            assert x is not None, "_attend: activations required without a precomputed qkv"
            qkv = ops.qkv_rope(x[:T], lw["qkv"], m.positions, self.cos_sin, m.slot_mapping, kc,
                               vc, hq, hkv)
        if shared is not None:
            ops.attn_decode_shared(qkv[:D], kc, vc, m.dec_block_tables, m.dec_q_start,
                                   m.dec_q_len, m.dec_kv_len, m.dec_work_seq, m.dec_work_ct,
                                   attn[:D], *shared, hq, hkv, self.scale, m.decode_tiles,
                                   li == 0)
        elif D > 0:
            po, pm = dec_parts if dec_parts is not None else (attn, attn)
            ns = m.decode_splits if dec_parts is not None else 1
            # every decode row one query (D rows = D sequences) and 8-16 query columns per
            # kv head: one column tile per work item is the whole work list already, and
            # the one-tile kernel's lighter register set is faster at batch 1 (TP = 8 rank
            # shape: 8.0 / 9.6 / 11.4 vs 8.2 / 10.1 / 12.7 µs at ctx 512 / 1K / 2K,
            # profiles/r5/attn_single_pass_lat.jsonl); the work list is the same, so
            # graphs captured this way replay any pure-decode step of their bucket
            tiles = m.decode_tiles
            if tiles > 1 and D == m.dec_q_len.shape[0] and 8 <= hq // hkv <= 16:
                tiles = 1
            ops.attn_decode(qkv[:D], kc, vc, m.dec_block_tables, m.dec_q_start, m.dec_q_len,
                            m.dec_kv_len, m.dec_work_seq, m.dec_work_ct, attn[:D], po, pm,
                            hq, hkv, self.scale, ns, tiles,
                            self._dec_tickets(m.dec_work_seq.numel()))
        if m.num_prefill_tokens > 0:
            ops.attn_prefill(qkv[D:T], kc, vc, m.pf_block_tables, m.pf_q_start, m.pf_q_len,
                             m.pf_kv_len, m.work_seq, m.work_qblk, attn[D:T], hq, hkv,
                             self.scale, m.prefill_qblk)

    # ------------------------------------------------------------- conveniences
    def weight_bytes(self) -> int:
        tot = 0
        for k, v in self.w.items():
            if isinstance(v, torch.Tensor):
                tot += v.numel() * v.element_size()
        for lw in self.w["layers"]:
            tot += sum(t.numel() * t.element_size() for t in lw.values())
        return tot
