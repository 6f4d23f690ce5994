"""Device ops: thin dispatch from tensor device to the gfx950 kernel or the torch oracle.

GPU tensors always go to ``torch.ops.rfq_amd.*`` (hand-written HIP kernels in
``csrc/kernels``); the library is loaded on first use and a GPU call fails loudly
if it cannot be.  CPU tensors use :mod:`.reference` (tests / CPU engine).
"""
from __future__ import annotations

import os

import torch

from . import _native
from . import reference as ref

__all__ = [
    "rms_norm", "fused_add_rms_norm", "silu_mul", "embed", "rope_kv", "attn_decode",
    "attn_prefill", "sample", "moe_topk", "moe_align", "moe_gather", "moe_grouped_gemm", "moe_gemm8", "count_nonfinite",
    "moe_combine", "moe_skinny", "native_available", "linear", "linear_plan",
    "set_linear_plan", "silu_linear", "set_silu_plan", "set_split_plan", "split_chunks",
    "set_norm_plan", "norm_plan", "norm_counter", "norm_partials", "linear_add_norm",
    "set_rope_plan", "set_swiglu_plan", "linear_swiglu", "splitk_ws",
    "rope_plan", "qkv_rope", "moe_route", "attn_decode_shared", "SHARED_PREFIX_MIN_ROWS",
    "gemm_dense", "gemm_dense_ok", "swiglu_large", "tile_weight", "untile_weight",
    "register_tiled", "tiled_of", "tiled_only", "clear_tiled", "SPLITK_TILED", "SPLITK_NT", "SPLITK_PERSIST",
    "ROWS_BIT", "ROWS_MAX_M", "ROWS_CFGS", "ROWS_CFGS_PAIRED", "rows_ok",
    "set_rows_best", "rows_rope_normx", "rows_swiglu_normx", "rows_residual_add", "fold_ok",
    "kernel_errors", "decode_persist", "decode_persist_info", "PERSIST_STAGES",
    "PERSIST_ENGINE", "decode_engine_info",
]

# Tokens per step up to which projections use the skinny weight-streaming GEMM
# (csrc/kernels/gemm_skinny.hip) instead of hipBLASLt; 0 disables it.
SKINNY_MAX_M = int(os.environ.get("RFQ_SKINNY_MAX_M", "64"))


def native_available() -> bool:
    return _native.available()


def kernel_errors() -> list[int]:
    """Counts of the bounded in-launch waits that gave up (csrc/kernels/kerr.hip):
    [stream-K slab waits, persistent decode stage waits, first failing persistent
    (layer << 8 | stage) + 1].  The first call allocates the words (do it before any graph
    capture); all zeros without the native library."""
    if not _native.available():
        return [0, 0, 0]
    return list(torch.ops.rfq_amd.kernel_errors())


# Persistent decode layers (csrc/kernels/decode_persist.hip): stage bits
PERSIST_QKV, PERSIST_ATTN, PERSIST_O, PERSIST_GU, PERSIST_DOWN = 1, 2, 4, 8, 16
PERSIST_STAGES = 31
PERSIST_ENGINE = 16      # flags bit: the loader / consumer (LDS-DMA ring) form, M <= 2


def decode_engine_info(M: int, d: int, Hq: int, Hkv: int, F: int) -> tuple[int, int]:
    """(LDS bytes, ring slots) of the engine form on this device; bytes 0 = does not fit."""
    return tuple(_native.ops().decode_engine_info(M, d, Hq, Hkv, F))


def decode_persist_info(M: int, d: int, Kx: int, nst: int) -> tuple[int, int, int]:
    """(counter words, LDS bytes, grid) of a persistent launch of ``nst`` stages."""
    return tuple(_native.ops().decode_persist_info(M, d, Kx, nst))


def decode_persist(residual, layers, qbuf, attn, act, positions, cos_sin, slots, block_tables,
                   q_start, q_len, kv_len, work_seq, work_ct, part_o, part_ml, tickets, counters,
                   l0, l1, stages, Hq, Hkv, F, BS, splits, scale, eps, flags=0) -> None:
    """Layers [l0, l1) of a small decode step in one launch (GPU only): qkv + RoPE + KV
    append -> attention + split merge -> o (+= residual) -> gate|up + SwiGLU -> down
    (+= residual), each stage present in the ``stages`` mask.  ``layers`` is the int64
    [L, 8] device table of (qkv, o, gate_up, down, k_cache, v_cache, 0, 0) pointers; the
    norms are folded into qkv / gate|up (DecoderLM.fold_norms).  ``residual`` [M, d] is
    updated in place; ``counters`` (int32 zeros, decode_persist_info words) are left
    zeroed by the launch."""
    _native.ops().decode_persist(residual, layers, qbuf, attn, act, positions, cos_sin, slots,
                                 block_tables, q_start, q_len, kv_len, work_seq, work_ct,
                                 part_o, part_ml, tickets, counters, l0, l1, stages, Hq, Hkv, F,
                                 BS, splits, scale, eps, flags)


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# (M, N, K) -> skinny cfg, or -1 for hipBLASLt.  Filled by ops.autotune at engine
# start (measured on the model's own weights); _default_plan covers untuned shapes.
_LINEAR_PLAN: dict[tuple[int, int, int], int] = {}
_TUNED_MS: list[int] = []


def set_linear_plan(plan: dict, ms) -> None:
    _LINEAR_PLAN.clear()
    _LINEAR_PLAN.update(plan)
    _TUNED_MS[:] = sorted(set(ms))


def _default_plan(M: int, N: int, K: int) -> int:
    """Measured on MI355X (profiles/skinny_gemm.md): the contiguous-k, plain-load
    variants beat hipBLASLt up to M=16 on every 8B/70B projection except down."""
    if M > 16:
        return -1
    return 14 if N <= 4096 else 13


def linear_plan(M: int, N: int, K: int) -> int:
    if M < 1 or M > SKINNY_MAX_M or K % 128 or N % 16:
        return -1
    if _TUNED_MS:
        for m in _TUNED_MS:
            if m >= M:
                c = _LINEAR_PLAN.get((m, N, K))
                if c is not None:
                    return c if (c < 0 or c >= SPLITK_BIT or c & 1 == 0 or N % 32 == 0) else -1
                break
    return _default_plan(M, N, K)


_SILU_PLAN: dict[tuple[int, int, int], int] = {}


def set_silu_plan(plan: dict) -> None:
    _SILU_PLAN.clear()
    _SILU_PLAN.update(plan)


def silu_linear(gu, w, out=None):
    """out = (silu(gate) * up) @ w^T for gu = [M, 2F] gate|up.  Small M: one skinny
    kernel computes SwiGLU while loading its operand (gemm_skinny.hip, gated X) when
    the start-up plan found it faster; otherwise act.hip silu_mul + linear."""
    M, F2 = gu.shape
    F, N = F2 // 2, w.shape[0]
    if _gpu(gu) and _TUNED_MS and M <= SKINNY_MAX_M and gu.stride(1) == 1 and not tiled_only(w):
        for m in _TUNED_MS:
            if m >= M:
                cfg = _SILU_PLAN.get((m, N, F), -1)
                if cfg >= 0:
                    if out is None:
                        out = torch.empty((M, N), dtype=gu.dtype, device=gu.device)
                    _native.ops().skinny_gemm(gu, w, out, cfg)
                    return out
                break
    return linear(silu_mul(gu), w, out=out)


# (M, N, K, gated) -> skinny cfg whose kernel also runs the following residual-add +
# RMSNorm in its last workgroup (gemm_skinny.hip NormEpi), or absent = unfused.
# Filled by ops.autotune.tune_norm for TP = 1 engines; M <= 16 only.
_NORM_PLAN: dict[tuple[int, int, int, bool], int] = {}
_NORM_COUNTERS: dict = {}
NORM_FUSE_MAX_M = 16


def set_norm_plan(plan: dict) -> None:
    _NORM_PLAN.clear()
    _NORM_PLAN.update(plan)


def norm_counter(device) -> torch.Tensor:
    """The zero-initialised ticket counter of the fused-norm GEMM (one per device; the
    kernels of a stream run in order and each leaves it at zero).  Allocated before
    any graph capture (ops.autotune) so captured graphs bake in a stable pointer."""
    return _norm_ws(device)[0]


def norm_partials(device) -> torch.Tensor:
    """fp32 workspace for the split-K fused-norm variant: 2 K slices x 16 rows x 8192."""
    return _norm_ws(device)[1]


def _norm_ws(device):
    d = torch.device(device)
    ws = _NORM_COUNTERS.get(d)
    if ws is None:
        ws = _NORM_COUNTERS[d] = (torch.zeros(64, dtype=torch.int32, device=d),
                                  torch.empty(2 * NORM_FUSE_MAX_M * 8192, dtype=torch.float32,
                                              device=d))
    return ws


def norm_plan(M: int, N: int, K: int, gated: bool) -> int:
    if not _NORM_PLAN or M > NORM_FUSE_MAX_M:
        return -1
    for m in _TUNED_MS:
        if m >= M:
            return _NORM_PLAN.get((m, N, K, gated), -1)
    return -1


def splitk_ws(device):
    """(fp32 partial slabs [16 slices x 16 rows x 16384], zeroed int32 tile tickets
    [16384]) of the split-K GEMV (gemm_skinny.hip gemv_splitk); allocated before any
    graph capture so captured graphs bake in stable pointers; tickets left at zero."""
    d = torch.device(device)
    key = ("splitk", d)
    ws = _NORM_COUNTERS.get(key)
    if ws is None:
        ws = _NORM_COUNTERS[key] = (torch.empty(16 * 16 * 16384, dtype=torch.float32, device=d),
                                    torch.zeros(16384, dtype=torch.int32, device=d))
    return ws


SPLITK_BIT = 128          # plan cfg bit: the split-K GEMV kernel (low bits = its cfg)
# split-K GEMV cfgs timed by the start-up plans: KS = 2 << (c & 3), bit 2 = 8 waves,
# bit 3 = U 2 (gemm_skinny.hip launch_gemv_splitk_epi)
SPLITK_CFGS = (0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14)


SPLITK_TILED = 16        # split-K GEMV cfg bit: W in the decode-tiled layout (tile_weight)
SPLITK_NT = 32           # split-K GEMV cfg bit: non-temporal weight loads
SPLITK_PERSIST = 64      # split-K GEMV cfg bit: persistent grid (tiled layout only)

# plan cfg bit: the row-streaming GEMV (csrc/kernels/gemv_rows.hip; low 4 bits = its cfg:
# [1:0] rows per wave = 1 << b, [3:2] 1 KB chunks in flight = 2 << b).  One wave per
# weight row over the full K, no cross-workgroup hand-off; M <= ROWS_MAX_M, K % 512 == 0,
# row-major weights.  Measured on MI355X at M = 1 (profiles/r5_gemv_rows.md): 1.2-1.5x
# the split-K GEMV on the 70B TP=8 shard and 8B shapes.
ROWS_BIT = 256
ROWS_MAX_M = 4
ROWS_CFGS = (4, 8, 12, 5, 9, 2, 6, 3)      # (RW, CU) = (1,4) (1,8) (1,16) (2,4) (2,8) (4,2) (4,4) (8,2)
# SwiGLU / RoPE epilogues: one row per wave (4, 8, 12), or both rows of the pair in one
# wave (| 64: X read once per pair, the better form at M = 3-4)
ROWS_CFGS_PAIRED = (4, 8, 12, 68, 72, 76)


def rows_ok(M: int, K: int, w: torch.Tensor) -> bool:
    """Shapes the row-streaming GEMV takes (host mirror of torch_ops.cpp check_rows)."""
    return 1 <= M <= ROWS_MAX_M and K % 512 == 0 and w.is_contiguous() and not tiled_only(w)


def tile_weight(w: torch.Tensor) -> torch.Tensor:
    """Decode-tiled copy of a [N, K] weight (gemm_skinny.hip gemv_splitk, TL): for each
    16-row tile and 128-wide k block, the four 16x32 MFMA A-fragments in lane order, so
    every wave-wide load of the split-K GEMV reads 1 KB of contiguous memory.  Same
    shape and dtype as ``w``; only the element order differs."""
    N, K = w.shape
    if N % 16 or K % 128:
        raise ValueError(f"tile_weight: N % 16 == 0 and K % 128 == 0 required, got {N}x{K}")
    return (w.view(N // 16, 16, K // 128, 4, 4, 8).permute(0, 2, 3, 4, 1, 5)
            .contiguous().view(N, K))


# data_ptr of a row-major projection weight -> its decode-tiled copy.  Filled when the
# model is built (DecoderLM.tile_decode_weights); split-K GEMV plan entries with the
# SPLITK_TILED bit read the copy, everything else the row-major original.
# Entries die with their weight (weakref finalizer), so an engine torn down in the
# same process frees its copies and a later weight at a reused address never matches.
_TILED: dict[int, tuple] = {}


def register_tiled(w: torch.Tensor, wt: torch.Tensor | None) -> None:
    """``wt``: the tiled copy of row-major ``w``; None: ``w`` itself is stored tiled
    (in-place mode, no row-major copy: every GEMM on it runs a tiled-layout kernel)."""
    import weakref

    key = w.data_ptr()
    _TILED[key] = (weakref.ref(w), wt)
    weakref.finalize(w, _TILED.pop, key, None)


def tiled_of(w: torch.Tensor) -> torch.Tensor | None:
    e = _TILED.get(w.data_ptr())
    if e is None or e[0]() is not w:
        return None
    return w if e[1] is None else e[1]


def tiled_only(w: torch.Tensor) -> bool:
    """``w`` is stored in the decode-tiled layout and has no row-major copy."""
    e = _TILED.get(w.data_ptr())
    return e is not None and e[1] is None and e[0]() is w


TILED_GEMV_DEFAULT = 8 | 16 | 32        # KS 2, 4 waves, U 2, tiled, nt (untuned shapes)


def _gemv_tiled(x, w, out, cfg: int | None = None):
    """out = x w^T for an in-place tiled ``w``: split-K GEMV in 16-row chunks for
    M <= SKINNY_MAX_M (the M = 16 plan entry), the dense MFMA GEMM on the tiled layout
    (gemm_dense cfg 2 | 4) above."""
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if M > SKINNY_MAX_M:
        _native.ops().gemm_dense(x, w, out, False, 2 | 4)
        return out
    part, tiles = splitk_ws(x.device)
    for a in range(0, M, 16):
        xm = x[a:a + 16]
        c = cfg if cfg is not None else linear_plan(xm.shape[0], N, K)
        if c < 0 or not (c & SPLITK_BIT) or not (c & SPLITK_TILED):
            c = TILED_GEMV_DEFAULT
        _native.ops().gemv_splitk(xm, w, out[a:a + 16], part, tiles, c & 127)
    return out


def clear_tiled() -> None:
    _TILED.clear()


def _wsel(w: torch.Tensor, cfg: int) -> torch.Tensor:
    """The weight a split-K GEMV cfg reads: the tiled copy under SPLITK_TILED."""
    if cfg & SPLITK_TILED:
        wt = tiled_of(w)
        if wt is None:
            raise RuntimeError("split-K plan selects the tiled layout but the weight has no "
                               "tiled copy (ops.register_tiled)")
        return wt
    return w


def untile_weight(wt: torch.Tensor) -> torch.Tensor:
    """Inverse of :func:`tile_weight`."""
    N, K = wt.shape
    return (wt.view(N // 16, K // 128, 4, 4, 16, 8).permute(0, 4, 1, 2, 3, 5)
            .contiguous().view(N, K))


def splitk_fits(device, cfg: int, M: int, n_rows: int, tiles: int) -> bool:
    """Whether the shared split-K workspace holds a launch (KS*M*n_rows partial floats,
    ``tiles`` ticket counters)."""
    part, cnt = splitk_ws(device)
    return (2 << (cfg & 3)) * M * n_rows <= part.numel() and tiles <= cnt.numel()


def linear_add_norm(x, w, residual, norm_w, eps, out, gated: bool = False) -> bool:
    """Try the fused path for ``y = x w^T`` (``gated``: x = gate|up, y = down(SwiGLU(x)))
    followed by ``fused_add_rms_norm(y, residual, norm_w, eps, out)``.  Returns False
    (nothing done) when the start-up plan has no fused kernel for this shape."""
    if not _gpu(x) or x.stride(1) != 1:
        return False
    M = x.shape[0]
    K = x.shape[1] // 2 if gated else x.shape[1]
    N = w.shape[0]
    cfg = norm_plan(M, N, K, gated)
    if cfg < 0 or (tiled_only(w) and not (cfg & SPLITK_BIT and cfg & SPLITK_TILED)):
        return False
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    if cfg & SPLITK_BIT:
        part, tiles = splitk_ws(x.device)
        _native.ops().gemv_splitk_norm(x, _wsel(w, cfg), y, residual, norm_w, eps, out,
                                       norm_counter(x.device), part, tiles, cfg & 127)
        return True
    _native.ops().skinny_gemm_norm(x, w, y, residual, norm_w, eps, out,
                                   norm_counter(x.device), norm_partials(x.device), cfg)
    return True


# (M, F, K) -> skinny cfg of the gate|up projection with the SwiGLU epilogue
# (gemm_skinny.hip SWI: out [M, F] = silu(x Wg^T) * (x Wu^T)), or absent = unfused.
_SWI_PLAN: dict[tuple[int, int, int], int] = {}


def set_swiglu_plan(plan: dict) -> None:
    _SWI_PLAN.clear()
    _SWI_PLAN.update(plan)


def linear_swiglu(x, w):
    """act[M, F] = silu(x Wg^T) * (x Wu^T) for w = gate|up [2F, K] in one skinny kernel
    when the start-up plan measured it faster than gate|up GEMM + silu_mul; None
    otherwise (the caller runs the unfused path)."""
    if not _SWI_PLAN or not _gpu(x) or x.stride(1) != 1 or x.stride(0) % 8:
        return None
    M, K = x.shape
    F = w.shape[0] // 2
    for m in _TUNED_MS:
        if m >= M:
            cfg = _SWI_PLAN.get((m, F, K), -1)
            if cfg < 0 or (tiled_only(w) and not (cfg & SPLITK_BIT and cfg & SPLITK_TILED)):
                return None
            out = torch.empty((M, F), dtype=x.dtype, device=x.device)
            if cfg & ROWS_BIT:
                _native.ops().gemv_rows_swiglu(x, w, out, cfg & 15)
            elif cfg & SPLITK_BIT:
                part, tiles = splitk_ws(x.device)
                _native.ops().gemv_splitk_swiglu(x, _wsel(w, cfg), out, part, tiles, cfg & 127)
            else:
                _native.ops().skinny_gemm_swiglu(x, w, out, cfg)
            return out
    return None


# ---------------------------------------------------------------- folded-norm latency path
# Best row-streaming cfg per (kind, M, N, K) measured by the start-up plans, whether or
# not it won its plan: the folded-norm path (models/llama.py _forward_fold) has no
# other kernel for its epilogues.  kind: "plain" | "swiglu" | "rope".
_ROWS_BEST: dict[tuple, int] = {}
ROWS_DEFAULT = {"plain": 9, "swiglu": 8, "rope": 8}
# folded path up to 2 tokens: at M = 3-4 the dot2 GEMV re-reads X per token and the
# gate|up + SwiGLU launch loses ~12 µs to the split-K MFMA GEMV (8B), more than the two
# norm launches the fold saves (profiles/r5_gemv_rows.md)
FOLD_MAX_M = int(os.environ.get("RFQ_FOLD_MAX_M", "2"))


def set_rows_best(best: dict) -> None:
    _ROWS_BEST.update(best)


def _rows_cfg(kind: str, M: int, N: int, K: int) -> int:
    for m in _TUNED_MS or [M]:
        if m >= M:
            c = _ROWS_BEST.get((kind, m, N, K))
            if c is not None:
                return c
            break
    return ROWS_DEFAULT[kind]


def rows_rope_normx(res, w, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, eps):
    """qkv = rmsnorm(res) @ w'^T with the norm weight folded into w' (DecoderLM.fold_norms),
    RoPE on q / k, k / v appended to the paged cache; only q columns are written (GPU).
    One row-streaming launch reading the UN-normalised residual (gemv_rows.hip kRwNormX)."""
    M, K = res.shape
    N = w.shape[0]
    qkv = torch.empty((M, N), dtype=res.dtype, device=res.device)
    if _gpu(res):
        _native.ops().gemv_rows_rope(res, w, qkv, positions, cos_sin, slot_mapping, k_cache,
                                     v_cache, Hq, Hkv, _rows_cfg("rope", M, N, K) | 16, eps)
        return qkv
    xn = torch.empty_like(res)
    ref.rms_norm(res, torch.ones(K, dtype=res.dtype), eps, xn)
    qkv.copy_(xn @ w.t())
    ref.rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv)
    return qkv


def rows_swiglu_normx(res, w, eps):
    """act = SwiGLU(rmsnorm(res) @ w'^T) with the norm weight folded into w' (gate|up)."""
    M, K = res.shape
    F = w.shape[0] // 2
    out = torch.empty((M, F), dtype=res.dtype, device=res.device)
    if _gpu(res):
        _native.ops().gemv_rows_swiglu(res, w, out, _rows_cfg("swiglu", M, F, K) | 16, eps)
        return out
    xn = torch.empty_like(res)
    ref.rms_norm(res, torch.ones(K, dtype=res.dtype), eps, xn)
    ref.silu_mul(xn @ w.t(), out)
    return out


def rows_residual_add(x, w, residual):
    """residual <- bf16(bf16(x @ w^T) + residual) (o / down + the residual add)."""
    M, K = x.shape
    N = w.shape[0]
    if _gpu(x):
        _native.ops().gemv_rows(x, w, residual, _rows_cfg("plain", M, N, K) | 32)
        return residual
    residual.copy_(((x @ w.t()).float() + residual.float()).to(residual.dtype))
    return residual


def fold_ok(M: int, K: int, w: torch.Tensor) -> bool:
    """The folded-norm path can run a projection of this step on the row-streaming
    kernel (GPU: rows_ok; CPU: always, through the oracles)."""
    if not w.is_cuda:
        return 1 <= M <= FOLD_MAX_M
    return 1 <= M <= min(FOLD_MAX_M, ROWS_MAX_M) and K % 512 == 0


# (M, N, K) -> skinny cfg (NT = 2) whose epilogue applies RoPE to q/k and appends k/v
# to the paged cache (gemm_skinny.hip RopeEpi), or absent = linear + rope_kv.
_ROPE_PLAN: dict[tuple[int, int, int], int] = {}
ROPE_FUSE_MAX_M = 16


def set_rope_plan(plan: dict) -> None:
    _ROPE_PLAN.clear()
    _ROPE_PLAN.update(plan)


def rope_plan(M: int, N: int, K: int) -> int:
    if not _ROPE_PLAN or M > ROPE_FUSE_MAX_M:
        return -1
    for m in _TUNED_MS:
        if m >= M:
            return _ROPE_PLAN.get((m, N, K), -1)
    return -1


def qkv_rope(x, w, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv):
    """qkv = x w^T, then NeoX RoPE on q (in place) and k, k/v appended to the paged
    cache.  Small M: one skinny kernel does all of it in its epilogue when the start-up
    plan measured that faster (then only the q columns of the result are written)."""
    if _gpu(x) and x.stride(1) == 1 and x.stride(0) % 8 == 0:
        cfg = rope_plan(x.shape[0], w.shape[0], x.shape[1])
        if tiled_only(w) and not (cfg & SPLITK_BIT and cfg & SPLITK_TILED):
            cfg = -1
        if cfg >= 0:
            qkv = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
            if cfg & ROWS_BIT:
                _native.ops().gemv_rows_rope(x, w, qkv, positions, cos_sin, slot_mapping,
                                             k_cache, v_cache, Hq, Hkv, cfg & 15)
            elif cfg & SPLITK_BIT:
                part, tiles = splitk_ws(x.device)
                _native.ops().gemv_splitk_rope(x, _wsel(w, cfg), qkv, positions, cos_sin,
                                               slot_mapping, k_cache, v_cache, Hq, Hkv, part,
                                               tiles, cfg & 127)
            else:
                _native.ops().skinny_gemm_rope(x, w, qkv, positions, cos_sin, slot_mapping,
                                               k_cache, v_cache, Hq, Hkv, cfg)
            return qkv
    qkv = linear(x, w)
    rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv)
    return qkv


def attn_decode_merge(part_o, part_ml, out, Hq, num_splits):
    """Merge split-K decode-attention partials into bf16 rows of ``out``."""
    _native.ops().attn_decode_merge(part_o, part_ml, out, Hq, num_splits)


# (N, K) -> (quantum q, table) where table[j] is the row-chunk split (in units of q
# rows, largest first) for M in ((j-1)q, jq], or None to keep one GEMM.  Filled by
# ops.autotune.tune_split at engine start: hipBLASLt's heuristic is uneven across
# M (e.g. down 4096x14336 runs at 0.9 PFLOP/s at M=6656 but 1.6 at M=4096), so
# large steps are cut into chunks whose measured times sum to less.
_SPLIT_PLAN: dict[tuple[int, int], tuple[int, list]] = {}


def set_split_plan(plan: dict) -> None:
    _SPLIT_PLAN.clear()
    _SPLIT_PLAN.update(plan)


def split_chunks(M: int, N: int, K: int) -> list[int] | None:
    """Row counts of the hipBLASLt calls for an [M, K] x [K, N] GEMM (None = one call)."""
    p = _SPLIT_PLAN.get((N, K))
    if p is None:
        return None
    q, table = p[0], p[1]
    j = -(-M // q)
    if j >= len(table) or table[j] is None:
        return None
    rows, left = [], M
    for c in table[j]:
        r = min(left, c * q)
        if r > 0:
            rows.append(r)
        left -= r
    return rows


_LT_BAD: set = set()        # (algo, M) pairs hipBLASLt rejected: plain matmul for those


def _dense_cfg(M: int, N: int, K: int, swiglu: bool = False) -> int:
    """gemm_dense cfg the start-up plan chose for this M bucket, or -1 (library)."""
    p = _SPLIT_PLAN.get((N, K))
    if p is None or len(p) < 5:
        return -1
    q, sel = p[0], p[4 if swiglu else 3]
    j = -(-M // q)
    if j < len(sel):
        return sel[j]
    return sel[-1] if len(sel) > 1 else -1        # past the tuned range: the largest bucket


def _hybrid_rows(M: int, N: int, K: int) -> tuple[int, int]:
    """(rows on the hand-written kernel, its cfg) for the plan's hybrid split of this M
    bucket (ops.autotune.plan_hybrid), or (0, -1)."""
    p = _SPLIT_PLAN.get((N, K))
    if p is None or len(p) < 6:
        return 0, -1
    q, hyb = p[0], p[5]
    j = -(-M // q)
    h = hyb[j] if j < len(hyb) else 0
    if not h:
        return 0, -1
    m1 = h[0] * q
    return (m1, h[1]) if 0 < m1 < M else (0, -1)


def swiglu_large(x, w):
    """act[M, F] = silu(x Wg^T) * (x Wu^T) for large M in one hand-written MFMA GEMM with
    the SwiGLU epilogue (gemm_dense.hip) when the start-up plan measured it faster than
    the library GEMM + silu_mul; None otherwise (the caller runs that unfused path)."""
    if not _gpu(x) or x.stride(1) != 1 or x.stride(0) % 8:
        return None
    M, K = x.shape
    N = w.shape[0]
    if M <= SKINNY_MAX_M:
        return None
    if tiled_only(w):                 # no row-major copy: the tiled dense kernel, fused
        out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device)
        _native.ops().gemm_dense(x, w, out, True, 2 | 4)
        return out
    cfg = _dense_cfg(M, N, K, swiglu=True)
    if cfg < 0:
        return None
    out = torch.empty((M, N // 2), dtype=x.dtype, device=x.device)
    _native.ops().gemm_dense(x, w, out, True, cfg)
    return out


def _lt_or_torch(x, w, out) -> None:
    """out = x w^T with the algorithm the start-up plan measured fastest for this
    M bucket (csrc/bindings/gemm_lt.cpp), else torch.matmul."""
    M, N, K = x.shape[0], w.shape[0], x.shape[1]
    p = _SPLIT_PLAN.get((N, K))
    if p is not None and len(p) > 2:
        q, algos = p[0], p[2]
        j = -(-M // q)
        a = algos[j] if j < len(algos) else -1
        if a >= 0 and (a, M) not in _LT_BAD:
            if _native.ops().lt_matmul(x, w, out, a) == 0:
                return
            _LT_BAD.add((a, M))
    torch.matmul(x, w.t(), out=out)


def linear(x, w, out=None, plan: int | None = None):
    """out[M, N] = x[M, K] . w[N, K]^T (bf16).  Small M streams W through the skinny
    MFMA kernel (csrc/kernels/gemm_skinny.hip) when the tuning plan says it beats
    hipBLASLt; large M goes to hipBLASLt, split into row chunks where the start-up
    M-split plan measured that to be faster."""
    M, K = x.shape
    N = w.shape[0]
    if M == 0:
        # a chunked-prefill step whose chunk ends no prompt selects no logits rows
        return out if out is not None else torch.empty((0, N), dtype=x.dtype, device=x.device)
    if _gpu(x) and tiled_only(w):
        return _gemv_tiled(x, w, out, plan)
    if _gpu(x) and x.stride(1) == 1 and x.stride(0) % 8 == 0:
        cfg = linear_plan(M, N, K) if plan is None else plan
        if cfg >= 0:
            if out is None:
                out = torch.empty((M, N), dtype=x.dtype, device=x.device)
            if cfg & ROWS_BIT:
                _native.ops().gemv_rows(x, w, out, cfg & 15)
                return out
            if cfg & SPLITK_BIT:
                part, tiles = splitk_ws(x.device)
                _native.ops().gemv_splitk(x, _wsel(w, cfg), out, part, tiles, cfg & 127)
                return out
            _native.ops().skinny_gemm(x, w, out, cfg)
            return out
        if _SPLIT_PLAN and M > SKINNY_MAX_M and (N, K) in _SPLIT_PLAN:
            if out is None:
                out = torch.empty((M, N), dtype=x.dtype, device=x.device)
            dc = _dense_cfg(M, N, K)
            if dc >= 0 and out.stride(1) == 1 and out.stride(0) % 4 == 0:
                _native.ops().gemm_dense(x, w, out, False, dc)
                return out
            m1, hc = _hybrid_rows(M, N, K)
            if m1 > 0 and out.stride(1) == 1 and out.stride(0) % 4 == 0:
                # whole rounds of the hand-written kernel's tiles, the rest on the library
                _native.ops().gemm_dense(x[:m1], w, out[:m1], False, hc)
                _lt_or_torch(x[m1:], w, out[m1:])
                return out
            rows = split_chunks(M, N, K) or [M]
            a = 0
            for r in rows:
                _lt_or_torch(x[a:a + r], w, out[a:a + r])
                a += r
            return out
    if out is None:
        return x @ w.t()
    torch.matmul(x, w.t(), out=out)
    return out


def gemm_dense_ok(M: int, N: int, K: int, swiglu: bool = False) -> bool:
    """Shapes the hand-written 256x256 MFMA GEMM (csrc/kernels/gemm_dense.hip) takes:
    K % 64 == 0, N % 256 == 0 (N = 2F with F % 128 == 0 under swiglu)."""
    return M >= 1 and K % 64 == 0 and K >= 64 and N % 256 == 0


def gemm_w4_ok(M: int, N: int, K: int) -> bool:
    """gemm_w4 / gemm_w4p (gemm_dense cfg bit 3) address every operand with 32-bit byte
    offsets through buffer resources: K % 128 == 0 and each operand under 2 GiB."""
    lim = (1 << 31) - 1
    return K % 128 == 0 and N * K * 2 < lim and M * max(K, N) * 2 < lim


def w4p_stream_k_applies(M: int, N: int, K: int, cus: int) -> bool:
    """Whether gemm_dense cfg bit 14 (stream-K over gemm_w4p's last rounds) changes the
    launch for this shape; the launcher's rule (gemm_w4.hip launch_gemm_w4): a partly
    filled last round of 256 x 256 tiles (N = 2F under SwiGLU: F / 128 column tiles) on
    ``cus`` (rounded down to 8) persistent workgroups, each with >= 2 chunks of 4
    K-tiles.  Otherwise the plain persistent kernel runs."""
    ncu = cus // 8 * 8
    if K % 256 or ncu <= 0:
        return False
    grid = -(-M // 256) * (N // 256)
    r, rounds = grid % ncu, grid // ncu
    sk = 0 if r == 0 else (r if 2 * r >= ncu else (r + ncu if rounds >= 1 else 0))
    return sk > 0 and sk * (K // 256) >= 2 * ncu


def gemm_dense(x, w, out=None, swiglu: bool = False, cfg: int = 0):
    """out[M, N] = x[M, K] . w[N, K]^T on the 8-wave ping-pong MFMA kernel; swiglu:
    w = gate|up [2F, K] and out[M, F] = silu(x Wg^T) * (x Wu^T) (rounded like the
    unfused GEMM -> bf16 -> silu_mul).  GPU only; CPU tensors use the torch oracle."""
    M, N = x.shape[0], w.shape[0]
    n_out = N // 2 if swiglu else N
    if out is None:
        out = torch.empty((M, n_out), dtype=x.dtype, device=x.device)
    if _gpu(x):
        _native.ops().gemm_dense(x, w, out, swiglu, cfg)
    elif swiglu:
        ref.silu_mul(x @ w.t(), out)
    else:
        torch.matmul(x, w.t(), out=out)
    return out


def rms_norm(x, w, eps, out=None):
    out = torch.empty_like(x) if out is None else out
    if _gpu(x):
        _native.ops().rms_norm(x, w, eps, out)
    else:
        ref.rms_norm(x, w, eps, out)
    return out


def fused_add_rms_norm(x, residual, w, eps, out=None):
    """residual <- x + residual ; out <- rmsnorm(residual) * w  (out may alias x)."""
    out = torch.empty_like(x) if out is None else out
    if _gpu(x):
        _native.ops().fused_add_rms_norm(x, residual, w, eps, out)
    else:
        ref.fused_add_rms_norm(x, residual, w, eps, out)
    return out


def silu_mul(gate_up, out=None):
    F = gate_up.shape[1] // 2
    out = torch.empty((gate_up.shape[0], F), dtype=gate_up.dtype, device=gate_up.device) \
        if out is None else out
    if _gpu(gate_up):
        _native.ops().silu_mul(gate_up, out)
    else:
        ref.silu_mul(gate_up, out)
    return out


def embed(ids, table, out=None, vocab_start: int = 0):
    out = torch.empty((ids.numel(), table.shape[1]), dtype=table.dtype, device=table.device) \
        if out is None else out
    if _gpu(table):
        _native.ops().embed(ids, table, out, vocab_start)
    else:
        ref.embed(ids, table, out, vocab_start)
    return out


def rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv):
    if _gpu(qkv):
        _native.ops().rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv)
    else:
        ref.rope_kv(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv)


def attn_decode(q, k_cache, v_cache, block_tables, q_start, q_len, kv_len, work_seq, work_ct,
                out, part_o, part_ml, Hq, Hkv, scale, num_splits=1, tiles_per_item=1,
                tickets=None, reduce: bool = True):
    """Paged attention for decode / short-extend rows (see csrc/kernels/attn_decode.hip).
    A work item (work_seq[w], work_ct[w]) covers column tiles
    [work_ct*tiles_per_item, +tiles_per_item) of its sequence's q_len*G (query, head) pairs.
    With num_splits > 1, ``tickets`` (int32 zeros, >= work items * Hkv, reset by the kernel)
    makes it single-pass: the last split to finish merges the partials in-kernel.
    ``reduce=False`` (num_splits > 1, no tickets): the split partials are left in
    part_o / part_ml (merge them with :func:`attn_decode_merge`)."""
    if _gpu(q):
        _native.ops().attn_decode(q, k_cache, v_cache, block_tables, q_start, q_len, kv_len,
                                  work_seq, work_ct, out, part_o, part_ml, Hq, Hkv, scale,
                                  num_splits, tiles_per_item, tickets, reduce)
    else:
        ref.attn_prefill(q, k_cache, v_cache, block_tables, q_start, q_len, kv_len, None, None,
                         out, Hq, Hkv, scale)


# decode batches at least this large use the shared-prefix (cascade) attention path
# (0 = off, the default: measured neutral on the RFQ bench, profiles/r1_experiments_rejected.md §8)
SHARED_PREFIX_MIN_ROWS = int(os.environ.get("RFQ_SHARED_PREFIX_MIN_ROWS", "0"))


def attn_decode_shared(q, k_cache, v_cache, block_tables, q_start, q_len, kv_len, work_seq,
                       work_ct, out, ws_i32, pre_o, pre_ml, Hq, Hkv, scale, tiles_per_item=1,
                       run_meta=True):
    """attn_decode (one split) with the shared system-prompt pages attended once per 8
    rows instead of once per sequence (csrc/kernels/attn_decode.hip, cascade mode).
    run_meta=False reuses the prefix metadata an earlier layer of the step computed in
    ws_i32 (same block tables).  Workspaces: ws_i32 int32 >= 2 + nseq + rows, pre_o fp32
    >= rows*Hq*128, pre_ml fp32 >= rows*Hq*2."""
    if _gpu(q):
        _native.ops().attn_decode_shared(q, k_cache, v_cache, block_tables, q_start, q_len,
                                         kv_len, work_seq, work_ct, out, ws_i32, pre_o, pre_ml,
                                         Hq, Hkv, scale, tiles_per_item, run_meta)
    else:
        ref.attn_prefill(q, k_cache, v_cache, block_tables, q_start, q_len, kv_len, None, None,
                         out, Hq, Hkv, scale)


PREFILL_GROUPS = {2: 64, 4: 64, 8: 32}


def prefill_qblk(Hq: int, Hkv: int) -> int:
    """Queries per prefill work item: 128 or 256 (query, head) rows per workgroup (4 or
    8 waves, attn_prefill.hip) -> 64 queries at GQA group 4 (Llama-3-8B, Mixtral) and
    2, 32 at group 8 (Llama-3-70B).  Other groups have no prefill kernel instance:
    rejected here, when the model is built, not at the first prefill."""
    g = Hq // Hkv if Hkv else 0
    if Hkv <= 0 or Hq % Hkv or g not in PREFILL_GROUPS:
        raise ValueError(f"attn_prefill supports GQA groups {sorted(PREFILL_GROUPS)} "
                         f"(Hq / Hkv per rank); got Hq={Hq}, Hkv={Hkv}")
    return PREFILL_GROUPS[g]


# prefill grids with fewer (work item x kv head) workgroups than this split the 8 query
# heads of a kv head over two 4-wave workgroups (GQA group 8, e.g. the TP = 8 rank shard
# of Llama-3-70B: one kv head); 0 = never.  profiles/r3_prefill_head_split.md
PREFILL_HSPLIT_BELOW = int(os.environ.get("RFQ_PREFILL_HSPLIT_BELOW", "256"))


# RFQ_PREFILL_KVSPLIT=0: no split-KV on top of the head split
PREFILL_KVSPLIT = os.environ.get("RFQ_PREFILL_KVSPLIT", "1") != "0"


def prefill_split_ws(device):
    """(fp32 workspace, zeroed int32 tickets) of the split-KV prefill attention (the
    kernel leaves the tickets at zero); one per device, allocated on first use."""
    d = torch.device(device)
    key = ("prefill_split", d)
    ws = _NORM_COUNTERS.get(key)
    if ws is None:
        nf, nt = _native.ops().prefill_split_ws_sizes()
        ws = _NORM_COUNTERS[key] = (torch.empty(nf, dtype=torch.float32, device=d),
                                    torch.zeros(nt, dtype=torch.int32, device=d))
    return ws


# RFQ_PREFILL_SMALL: small-grid prefill form, 0 = auto, 1 = head split, 2 = 8-wave split-KV
PREFILL_SMALL_MODE = int(os.environ.get("RFQ_PREFILL_SMALL", "0"))


def attn_prefill(q, k_cache, v_cache, block_tables, seq_q_start, seq_q_len, seq_kv_len,
                 work_seq, work_qblk, out, Hq, Hkv, scale, qblk: int = 32,
                 hsplit_below: int | None = None, kvsplit: bool | None = None,
                 small_mode: int | None = None):
    """Causal paged prefill attention; the work list holds (sequence, query block of
    ``qblk`` queries) items (qblk * Hq / Hkv must be 128 or 256).  Small grids at GQA
    group 8 split the heads over two workgroups (``hsplit_below``) and, with
    ``kvsplit``, the key tiles of each item over two more (merged in-kernel)."""
    if _gpu(q):
        hs = PREFILL_HSPLIT_BELOW if hsplit_below is None else hsplit_below
        ws, tk = prefill_split_ws(q.device) if (PREFILL_KVSPLIT if kvsplit is None
                                                 else kvsplit) else (None, None)
        _native.ops().attn_prefill(q, k_cache, v_cache, block_tables, seq_q_start, seq_q_len,
                                   seq_kv_len, work_seq, work_qblk, out, Hq, Hkv, scale, qblk,
                                   hs, ws, tk,
                                   PREFILL_SMALL_MODE if small_mode is None else small_mode)
    else:
        ref.attn_prefill(q, k_cache, v_cache, block_tables, seq_q_start, seq_q_len, seq_kv_len,
                         work_seq, work_qblk, out, Hq, Hkv, scale)


def sample_partial(logits, v0, mask_table, mask_idx, temps, seeds, part_val, part_idx):
    """GPU-only first stage (per-shard (val, idx) partials)."""
    _native.ops().sample_partial(logits, v0, mask_table, mask_idx, temps, seeds, part_val,
                                 part_idx)


def sample_final(part_val, part_idx, out):
    _native.ops().sample_final(part_val, part_idx, out)


def sample(logits, mask_table, mask_idx, temps, seeds, v0=0, nsplit=8, out=None):
    """Single-device grammar-masked Gumbel-max sampling -> int32 token ids [B]."""
    B = logits.shape[0]
    if _gpu(logits):
        pv = torch.empty((1, B, nsplit), dtype=torch.float32, device=logits.device)
        pi = torch.empty((1, B, nsplit), dtype=torch.int32, device=logits.device)
        out = torch.empty(B, dtype=torch.int32, device=logits.device) if out is None else out
        sample_partial(logits, v0, mask_table, mask_idx, temps, seeds, pv[0], pi[0])
        sample_final(pv, pi, out)
        return out
    _, idx = ref.sample(logits, mask_table, mask_idx, temps, seeds, v0)
    if out is not None:
        out.copy_(idx)
        return out
    return idx


def moe_topk(router_logits, topk, renorm, weights, ids):
    if _gpu(router_logits):
        _native.ops().moe_topk(router_logits, topk, renorm, weights, ids)
    else:
        w, i = ref.moe_topk(router_logits, topk, renorm)
        weights.copy_(w)
        ids.copy_(i)


def moe_align(topk_ids, E, block_m, sorted_ids, inv_pos, expert_of_block, expert_offsets,
              num_blocks):
    _native.ops().moe_align(topk_ids, E, block_m, sorted_ids, inv_pos, expert_of_block,
                            expert_offsets, num_blocks)


def moe_gather(x, sorted_ids, topk, out):
    _native.ops().moe_gather(x, sorted_ids, topk, out)


def moe_grouped_gemm(x, w, out, expert_of_block, num_blocks):
    _native.ops().moe_grouped_gemm(x, w, out, expert_of_block, num_blocks)


def count_nonfinite(x, counter):
    """counter[0] += number of Inf / NaN entries of the 2-D bf16 ``x`` (no host sync;
    graph-capturable).  CPU: the same count with torch."""
    if _gpu(x):
        _native.ops().count_nonfinite(x, counter)
    else:
        counter[0] += int((~torch.isfinite(x.float())).sum())


def moe_gemm8_ok(w, swiglu: bool) -> bool:
    """Shapes the 8-wave 128x256 grouped GEMM (moe.hip moe_gemm8_kernel) takes."""
    return w.shape[2] % 64 == 0 and w.shape[1] % 256 == 0   # swiglu: F % 128


MOE_TILE_ROWS = int(os.environ.get("RFQ_MOE_TILE", "256"))


def moe_gemm8(x, w, out, expert_of_block, num_blocks, expert_offsets, swiglu: bool = False,
              tile: int | None = None):
    """Grouped GEMM over 128-row expert blocks (moe_align's segments: expert_offsets
    [E+1] padded row offsets); swiglu: w = [E, 2F, K] gate|up and out = silu(x Wg^T) *
    (x Wu^T) ([rows, F]), rounded like GEMM -> bf16 -> silu_mul.  tile: 256 = the
    256x256 kernel (pairs of an expert's blocks, half tiles skipped), 128 = 128x256."""
    _native.ops().moe_gemm8(x, w, out, expert_of_block, num_blocks, expert_offsets, swiglu,
                            tile or MOE_TILE_ROWS)


# RFQ_MOE_W4=0: the grouped expert GEMMs on gemm_dense's 8-wave ping-pong instead of the
# one-wave-per-SIMD gemm_w4 structure
MOE_W4 = os.environ.get("RFQ_MOE_W4", "1") != "0"


def moe_gemm_dense(x, w, out, expert_offsets, swiglu: bool = False, cfg: int | None = None):
    """Grouped GEMM over expert segments (moe_align with block 128): no host sync, fixed
    grid; swiglu: w = [E, 2F, K] gate|up and out = silu(x Wg^T) * (x Wu^T).  cfg bit 3
    (default with RFQ_MOE_W4, K % 128): the one-wave-per-SIMD 256 x 256 structure of
    gemm_w4.hip (GROUPED), else gemm_dense.hip's 8-wave ping-pong (GROUPED)."""
    if cfg is None:
        cfg = 8 if MOE_W4 and w.shape[2] % 128 == 0 else 0
    _native.ops().moe_gemm_dense(x, w, out, expert_offsets, swiglu, cfg)


def moe_w2_combine(x, w, y, yf, expert_offsets, inv_pos, weights, topk, out, cus: int):
    """Throughput-path w2 + weighted top-k combine in two launches (gemm_w4.hip GROUPED
    KS = 2 and moe.hip moe_combine_w2_kernel).  Both decide on the device from the expert
    offsets whether the grouped GEMM cuts each tile's K range in two (fp32 partial slabs
    in yf [2, >= rows, N]) or stores bf16 rows in y; cus <= 0 never splits."""
    _native.ops().moe_w2_combine(x, w, y, yf, expert_offsets, inv_pos, weights, topk, out, cus)


def moe_gemm_dense_ok(w, swiglu: bool) -> bool:
    N, K = w.shape[1], w.shape[2]
    return K % 64 == 0 and ((N // 2) % 128 == 0 if swiglu else N % 256 == 0)


def moe_route(x, router_w, topk, renorm, weights, ids):
    """Router logits (x . router_w^T, bf16-rounded) + softmax top-k in one kernel (GPU,
    small T); CPU: the same two steps in torch."""
    if _gpu(x):
        _native.ops().moe_route(x, router_w, topk, renorm, weights, ids)
    else:
        moe_topk(x @ router_w.t(), topk, renorm, weights, ids)


def moe_skinny(x, sorted_ids, topk, expert_offsets, w, out, gated, gather, max_rows):
    """Per-expert weight-streaming GEMM (small token counts); see gemm_skinny.hip."""
    _native.ops().moe_skinny(x, sorted_ids, topk, expert_offsets, w, out, gated, gather,
                             max_rows)


def moe_skinny_splitk(x, sorted_ids, topk, expert_offsets, w, yf, max_rows, splits):
    """Latency-path w2 with split-K: fp32 partial slabs yf[splits, rows, N]."""
    _native.ops().moe_skinny_splitk(x, sorted_ids, topk, expert_offsets, w, yf, max_rows, splits)


def moe_combine_splitk(yf, splits, inv_pos, weights, topk, out):
    _native.ops().moe_combine_splitk(yf, splits, inv_pos, weights, topk, out)


def moe_combine(y, inv_pos, weights, topk, out):
    _native.ops().moe_combine(y, inv_pos, weights, topk, out)


def reset_plans() -> None:
    """Forget every start-up plan (tests that build bare models after an engine: the
    plans are keyed by shape and may name a decode-tiled copy the new weights lack)."""
    for d in (_LINEAR_PLAN, _SILU_PLAN, _NORM_PLAN, _SWI_PLAN, _ROWS_BEST,
              _ROPE_PLAN, _SPLIT_PLAN):
        d.clear()
    _TUNED_MS.clear()
