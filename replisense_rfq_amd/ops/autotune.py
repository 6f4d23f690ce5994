"""Per-shape GEMM selection for the latency path: skinny MFMA kernel vs hipBLASLt.

Run once at engine start, before hipGraph capture, on the model's own weights:
for every projection shape (N, K) and every token count M the captured graphs
use (<= 64), time hipBLASLt and each skinny-kernel config over the real
per-layer weight list (32-80 distinct matrices, so every call streams from HBM
exactly as in a forward pass) and keep the fastest.  The plan is installed with
:func:`replisense_rfq_amd.ops.set_linear_plan` and read by :func:`ops.linear`.
"""
from __future__ import annotations

import logging
import os
import time

import torch

from . import (ROWS_BIT, ROWS_CFGS, ROWS_CFGS_PAIRED, SPLITK_BIT, SPLITK_CFGS, SPLITK_NT,
               SPLITK_TILED, _native, _wsel, gemm_dense_ok, gemm_w4_ok, rows_ok, set_rows_best,
               w4p_stream_k_applies,
               set_linear_plan, set_norm_plan, set_rope_plan, set_silu_plan,
               set_split_plan,
               set_swiglu_plan, silu_linear, silu_mul, splitk_fits, splitk_ws, tiled_of,
               tiled_only)

log = logging.getLogger("replisense_rfq_amd.ops")

# (name, M, N, K, one-call µs, chunk rows, split µs) of the last tune_split
SPLIT_REPORT: list = []

# tile configs (bits 0-1) on the contiguous-k / plain-load variant (bits 2-3 = 3)
CANDIDATES = (12, 13, 14, 15)


def _time(fn, ws, reps: int, graph: bool = True) -> float:
    """µs per call of fn(w) over the weight list, replayed from a captured hipGraph:
    the decode steps these plans serve run as graphs, so host launch cost must not
    enter the comparison (eager timing of 1-2 µs-scale kernels measures Python)."""
    fn(ws[0])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = None
    if graph and os.environ.get("RFQ_TUNE_GRAPHS", "1") != "0":
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
                for w in ws:
                    fn(w)
            torch.cuda.current_stream().wait_stream(s)
            g.replay()
            torch.cuda.synchronize()
        except RuntimeError as e:       # capture refused: fall back to eager timing
            log.warning("autotune: graph capture failed (%s); timing eagerly", e)
            g = None
    if g is None:
        # eager timing of one large GEMM takes a few ms at most: after the host gap of
        # the previous measurement the GPU clock is still ramping up, which read hipBLASLt
        # and the hand-written GEMM alike ~3x slow (gate|up at M = 4096: 2.5 ms here vs
        # 0.7 ms steady).  Keep the GPU busy for ~10 ms first.
        t_end = time.perf_counter() + 0.010
        while time.perf_counter() < t_end:
            for w in ws:
                fn(w)
            torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3 if g is not None else 1):     # min of 3 trials: one slow trial
        e0.record()                                # must not flip a plan entry
        for _ in range(reps):
            if g is not None:
                g.replay()
            else:
                for w in ws:
                    fn(w)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / (reps * len(ws)))
    return best


LATENCY_MARGIN = float(os.environ.get("RFQ_LATENCY_LIB_MARGIN", "1.05"))


def _tiled_group(ws: list[torch.Tensor]) -> bool:
    """Every layer's weight is stored in the decode-tiled layout only (in-place mode):
    no hipBLASLt or skinny-kernel candidate can read it."""
    return all(tiled_only(w) for w in ws)


def _splitk_cands(ws: list[torch.Tensor], base=SPLITK_CFGS) -> tuple:
    """Split-K GEMV cfgs to time: ``base`` on the row-major weights, or, when every layer
    has a decode-tiled copy (SPLITK_TILED), on the tiled copies with plain and with
    non-temporal weight loads (SPLITK_NT: +5-15 % on the tiled stream, a loss on the
    row-major one's half lines; profiles/r3_host_gaps_and_mall.md §3)."""
    tiled = all(tiled_of(w) is not None for w in ws)
    if not tiled:
        return tuple(base)
    # the row-major split-K cfgs are left out: the tiled stream beat them on every
    # 8B / 70B / TP=8 shape measured (start-up time stays ~2x, not 3x)
    return tuple(c | SPLITK_TILED for c in base) + tuple(c | SPLITK_TILED | SPLITK_NT
                                                         for c in base)


def tune_linear(groups: dict[str, list[torch.Tensor]], ms_by_group: dict[str, list[int]],
                reps: int = 2, margin: float = 1.03) -> dict:
    """groups: name -> per-layer weights [N, K]; ms_by_group: name -> token counts.
    ``margin`` > 1: a hand-written kernel within 3 % of hipBLASLt is kept (at M <= 64
    the library's small-M tiles measured at parity at best, and the latency-path graphs
    then launch only kernels this tree can tune and fuse); at M <= 16 (the decode /
    jump-forward steps of single requests) the tolerance is LATENCY_MARGIN."""
    ops = _native.ops()
    plan, report = {}, []
    for name, ws in groups.items():
        N, K = ws[0].shape
        if K % 128 or N % 16:
            continue
        for M in ms_by_group.get(name, []):
            if M > 64:
                continue
            x = torch.randn(M, K, device=ws[0].device, dtype=ws[0].dtype)
            out = torch.empty(M, N, device=x.device, dtype=x.dtype)
            if _tiled_group(ws):
                # in-place tiled weights: only the tiled split-K GEMV reads them (M > 16
                # runs in 16-row chunks of the M = 16 entry, ops._gemv_tiled)
                if M > 16:
                    continue
                part, tiles = splitk_ws(x.device)
                best, t_best = -1, float("inf")
                for c in _splitk_cands(ws):
                    if K // 128 < (2 << (c & 3)) or not splitk_fits(x.device, c, M, N, N // 16):
                        continue
                    t = _time(lambda w, c=c: ops.gemv_splitk(x, w, out, part, tiles, c), ws, reps)
                    if t < t_best:
                        best, t_best = c | SPLITK_BIT, t
                plan[(M, N, K)] = best
                report.append((name, M, N, K, 0.0, best, round(t_best, 1)))
                continue
            t_lib = _time(lambda w: torch.matmul(x, w.t(), out=out), ws, reps)
            best, t_best = -1, t_lib * (LATENCY_MARGIN if M <= 16 else margin)
            for c in CANDIDATES:
                if c & 1 and N % 32:
                    continue
                t = _time(lambda w, c=c: ops.skinny_gemm(x, w, out, c), ws, reps)
                if t < t_best:
                    best, t_best = c, t
            if M <= 16:
                # split-K GEMV (KS workgroups per 16-row tile, in-launch reduction): short
                # N or short K shapes that leave CUs idle with one workgroup per tile
                part, tiles = splitk_ws(x.device)
                for c in _splitk_cands(ws):
                    if K // 128 < (2 << (c & 3)) or not splitk_fits(x.device, c, M, N, N // 16):
                        continue
                    t = _time(lambda w, c=c: ops.gemv_splitk(x, _wsel(w, c), out, part, tiles, c),
                              ws, reps)
                    if t < t_best:
                        best, t_best = c | SPLITK_BIT, t
            if rows_ok(M, K, ws[0]):
                # row-streaming GEMV (one wave per row, full K): M <= 4
                rb, t_rb = -1, float("inf")
                for c in ROWS_CFGS:
                    t = _time(lambda w, c=c: ops.gemv_rows(x, w, out, c), ws, reps)
                    if t < t_rb:
                        rb, t_rb = c, t
                    if t < t_best:
                        best, t_best = c | ROWS_BIT, t
                set_rows_best({("plain", M, N, K): rb})
            plan[(M, N, K)] = best
            report.append((name, M, N, K, round(t_lib, 1), best, round(min(t_best, t_lib), 1)))
    return plan, report


def tune_silu_down(ws: list[torch.Tensor], ms: list[int], reps: int = 2, margin: float = 0.97):
    """down projection with its SwiGLU input: silu_mul + best plain GEMM vs the gated
    skinny kernel (one pass)."""
    from . import linear

    ops = _native.ops()
    N, F = ws[0].shape
    plan, report = {}, []
    if F % 128 or N % 16 or _tiled_group(ws):
        return plan, report
    for M in ms:
        if M > 64:
            continue
        gu = torch.randn(M, 2 * F, device=ws[0].device, dtype=ws[0].dtype)
        out = torch.empty(M, N, device=gu.device, dtype=gu.dtype)
        t_ref = _time(lambda w: linear(silu_mul(gu), w, out=out), ws, reps)
        best, t_best = -1, t_ref * margin
        for c in (16, 17, 18, 19):
            if c & 1 and N % 32:
                continue
            t = _time(lambda w, c=c: ops.skinny_gemm(gu, w, out, c), ws, reps)
            if t < t_best:
                best, t_best = c, t
        plan[(M, N, F)] = best
        report.append(("silu+down", M, N, F, round(t_ref, 1), best, round(min(t_best, t_ref), 1)))
    return plan, report


def tune_norm(ws: list[torch.Tensor], ms: list[int], norm_w: torch.Tensor, gated: bool,
              reps: int = 2, margin: float = 1.02, eps: float = 1e-5):
    """o / down projection followed by the residual-add RMSNorm: the planned GEMM path
    (linear or silu_linear) + fused_add_rms_norm vs the skinny kernel that runs the
    norm in its last workgroup (one launch instead of two).  ``margin`` > 1: a fused
    kernel within 2 % of the two-launch path is kept (one launch fewer per layer in
    the captured graph, and no library GEMM on the latency path)."""
    from . import (NORM_FUSE_MAX_M, SPLITK_BIT, fused_add_rms_norm, linear, norm_counter,
                   norm_partials, splitk_ws)

    ops = _native.ops()
    N, K = ws[0].shape
    plan, report = {}, []
    if K % 128 or N % 16 or N % 8 or N > 8192:
        return plan, report
    dev, dt = ws[0].device, ws[0].dtype
    counter, partials = norm_counter(dev), norm_partials(dev)
    part, tiles = splitk_ws(dev)
    for M in ms:
        if M > NORM_FUSE_MAX_M:
            continue
        x = torch.randn(M, 2 * K if gated else K, device=dev, dtype=dt)
        y = torch.empty(M, N, device=dev, dtype=dt)
        res = torch.randn(M, N, device=dev, dtype=dt)
        out = torch.empty(M, N, device=dev, dtype=dt)

        def ref(w):
            (silu_linear(x, w, out=y) if gated else linear(x, w, out=y))
            fused_add_rms_norm(y, res, norm_w, eps, out=out)

        t_ref = _time(ref, ws, reps)
        best, t_best = -1, t_ref * margin
        base = () if _tiled_group(ws) else ((16, 17, 18, 19) if gated else CANDIDATES)
        for c in base + tuple(b | 64 for b in base):       # | 64: two K slices per tile
            if c & 1 and N % 32:
                continue
            t = _time(lambda w, c=c: ops.skinny_gemm_norm(x, w, y, res, norm_w, eps, out,
                                                          counter, partials, c), ws, reps)
            if t < t_best:
                best, t_best = c, t
        # the split-K GEMV with the in-launch per-tile reduction + norm (plain x only;
        # tools/bench_gemv.py: KS 2-4, 4 waves, U 2-4 are its useful corner)
        for c in (_splitk_cands(ws, (8, 9, 12, 13, 4, 5, 0)) if not gated else ()):
            if (K // 128) < (2 << (c & 3)):
                continue
            t = _time(lambda w, c=c: ops.gemv_splitk_norm(x, _wsel(w, c), y, res, norm_w, eps,
                                                          out, counter, part, tiles, c), ws, reps)
            if t < t_best:
                best, t_best = c | SPLITK_BIT, t
        if best >= 0:
            plan[(M, N, K, gated)] = best
        report.append(("down+norm" if gated else "o+norm", M, N, K, round(t_ref, 1), best,
                       round(min(t_best, t_ref), 1)))
    return plan, report


def decode_splits_for(rows: int, hkv: int) -> int:
    """The split count the captured decode graphs use for ``rows`` decode rows
    (engine/runner.py ModelRunner._decode_splits with graph=True)."""
    s = 1
    while rows * hkv * s < 1024 and s < 16:
        s *= 2
    return s


def tune_swiglu(ws: list[torch.Tensor], ms: list[int], reps: int = 2, margin: float = 0.97):
    """gate|up projection + silu_mul (planned GEMM path) vs the skinny kernel with the
    SwiGLU epilogue (gemm_skinny.hip SWI; 4 or 8 waves)."""
    from . import NORM_FUSE_MAX_M, linear

    ops = _native.ops()
    N2, K = ws[0].shape
    F = N2 // 2
    plan, report = {}, []
    if K % 128 or F % 16:
        return plan, report
    dev, dt = ws[0].device, ws[0].dtype
    for M in ms:
        if M > NORM_FUSE_MAX_M:
            continue
        x = torch.randn(M, K, device=dev, dtype=dt)
        gu = torch.empty(M, N2, device=dev, dtype=dt)
        act = torch.empty(M, F, device=dev, dtype=dt)
        t_ref = _time(lambda w: silu_mul(linear(x, w, out=gu), out=act), ws, reps)
        best, t_best = -1, t_ref * margin
        for c in (() if _tiled_group(ws) else (0, 2)):
            t = _time(lambda w, c=c: ops.skinny_gemm_swiglu(x, w, act, c), ws, reps)
            if t < t_best:
                best, t_best = c, t
        part, tiles = splitk_ws(dev)
        for c in _splitk_cands(ws):
            if K // 128 < (2 << (c & 3)) or not splitk_fits(dev, c, M, N2, F // 16):
                continue
            t = _time(lambda w, c=c: ops.gemv_splitk_swiglu(x, _wsel(w, c), act, part, tiles, c),
                      ws, reps)
            if t < t_best:
                best, t_best = c | SPLITK_BIT, t
        if rows_ok(M, K, ws[0]):
            rb, t_rb = -1, float("inf")
            for c in ROWS_CFGS_PAIRED:
                t = _time(lambda w, c=c: ops.gemv_rows_swiglu(x, w, act, c), ws, reps)
                if t < t_rb:
                    rb, t_rb = c, t
                if t < t_best:
                    best, t_best = c | ROWS_BIT, t
            set_rows_best({("swiglu", M, F, K): rb})
        if best >= 0:
            plan[(M, F, K)] = best
        report.append(("gate_up+swiglu", M, N2, K, round(t_ref, 1), best,
                       round(min(t_best, t_ref), 1)))
    return plan, report


def tune_rope(ws: list[torch.Tensor], ms: list[int], cos_sin: torch.Tensor, hq: int, hkv: int,
              reps: int = 2, margin: float = 0.97):
    """QKV projection followed by rope_kv (planned GEMM + rope_kv.hip) vs the skinny
    kernel with the RoPE / KV-append epilogue (NT = 2 tiles, 4 or 8 waves)."""
    from . import ROPE_FUSE_MAX_M, linear, rope_kv

    ops = _native.ops()
    N, K = ws[0].shape
    plan, report = {}, []
    if K % 128 or N != (hq + 2 * hkv) * 128:
        return plan, report
    dev, dt = ws[0].device, ws[0].dtype
    for M in ms:
        if M > ROPE_FUSE_MAX_M:
            continue
        x = torch.randn(M, K, device=dev, dtype=dt)
        qkv = torch.empty(M, N, device=dev, dtype=dt)
        nb = M // 32 + 2
        kc = torch.zeros(nb, hkv, 32, 128, device=dev, dtype=dt)
        vc = torch.zeros_like(kc)
        pos = torch.arange(100, 100 + M, device=dev, dtype=torch.int32)
        slots = torch.arange(M, device=dev, dtype=torch.int32)

        def ref(w):
            linear(x, w, out=qkv)
            rope_kv(qkv, pos, cos_sin, slots, kc, vc, hq, hkv)

        t_ref = _time(ref, ws, reps)
        best, t_best = -1, t_ref * margin
        for c in (() if _tiled_group(ws) else (13, 15)):
            t = _time(lambda w, c=c: ops.skinny_gemm_rope(x, w, qkv, pos, cos_sin, slots, kc, vc,
                                                          hq, hkv, c), ws, reps)
            if t < t_best:
                best, t_best = c, t
        part, tiles = splitk_ws(dev)
        for c in _splitk_cands(ws):
            if K // 128 < (2 << (c & 3)) or not splitk_fits(dev, c, M, N, N // 32):
                continue
            t = _time(lambda w, c=c: ops.gemv_splitk_rope(x, _wsel(w, c), qkv, pos, cos_sin, slots,
                                                          kc, vc, hq, hkv, part, tiles, c),
                      ws, reps)
            if t < t_best:
                best, t_best = c | SPLITK_BIT, t
        if rows_ok(M, K, ws[0]):
            rb, t_rb = -1, float("inf")
            for c in ROWS_CFGS_PAIRED:
                t = _time(lambda w, c=c: ops.gemv_rows_rope(x, w, qkv, pos, cos_sin, slots, kc, vc,
                                                            hq, hkv, c), ws, reps)
                if t < t_rb:
                    rb, t_rb = c, t
                if t < t_best:
                    best, t_best = c | ROWS_BIT, t
            set_rows_best({("rope", M, N, K): rb})
        if best >= 0:
            plan[(M, N, K)] = best
        report.append(("qkv+rope", M, N, K, round(t_ref, 1), best, round(min(t_best, t_ref), 1)))
    return plan, report


def plan_splits(times: list[float], margin: float = 0.95, launch_us: float = 4.0) -> list:
    """Row-chunk plan from measured single-GEMM times.

    ``times[j]`` = µs of one hipBLASLt call with ``j`` quanta of rows (``times[0]``
    unused).  Returns ``table`` with ``table[j]`` = chunk sizes in quanta (largest
    first) whose summed times (+ ``launch_us`` per extra call) beat ``times[j]`` by
    ``margin``, or None where one call is best.  Exact DP over all partitions."""
    J = len(times) - 1
    best = [0.0] * (J + 1)
    choice = [0] * (J + 1)        # size of one chunk of the best partition of j
    for j in range(1, J + 1):
        best[j], choice[j] = times[j], j
        for c in range(1, j):
            t = times[c] + best[j - c] + launch_us
            if t < best[j]:
                best[j], choice[j] = t, c
    table: list = [None] * (J + 1)
    for j in range(1, J + 1):
        if choice[j] == j or best[j] > margin * times[j]:
            continue
        parts, r = [], j
        while r > 0:
            parts.append(choice[r])
            r -= choice[r]
        table[j] = tuple(sorted(parts, reverse=True))
    return table


LT_CANDIDATES = int(os.environ.get("RFQ_GEMM_LT_CANDIDATES", "6"))   # heuristic algorithms timed per (M bucket, N, K)
# RFQ_GEMM_DENSE=0 keeps every large-M projection on hipBLASLt
DENSE_ON = os.environ.get("RFQ_GEMM_DENSE", "1") != "0"
# 2: gemm_dense's 8-wave ping-pong; 13960 = 8 | 128 | 512 | 1024 | 4096 | 8192: gemm_w4
# (one wave per SIMD), DMA spread over the MFMA groups, 4 row tiles per L2 group, fragment
# reads early in each half, the weight image in three LDS slots, persistent over output
# tiles with the K-tile pipeline crossing tile boundaries (K % 256; otherwise the same
# kernel without persistence, 5768; 1672 without the third slot; profiles/r4_gemm_w4.md);
# 30344 = 13960 | 16384: the same with stream-K over its last rounds (timed only where
# the launcher would use it: ops.w4p_stream_k_applies; profiles/r5_gemm_stream_k.md)
DENSE_CFGS = tuple(int(c) for c in os.environ.get("RFQ_GEMM_DENSE_CFGS", "2,13960,30344").split(","))
DENSE_MARGIN = 0.99              # the hand-written kernel must win by 1 %


def plan_hybrid(t_lib: list, t_dense: list, tiles_n: int, quantum: int = 256,
                launch_us: float = 4.0, margin: float = DENSE_MARGIN, cus: int = 256) -> list:
    """Row split of a large-M GEMM between the hand-written persistent kernel and the
    library.  The hand-written kernel runs whole rounds of 256 x 256 tiles on the 256 CUs
    only when its row-tile count times ``tiles_n`` is a multiple of 256; its last, partly
    filled round is what the library's stream-K split avoids.  So for bucket j (j
    quanta of rows) try: the first m1 rows (a multiple of one full round) on the
    hand-written kernel, the rest on the library.  ``t_lib[j]`` / ``t_dense[j]``: µs of
    j quanta on each (index 0 unused; inf where not measured).  Returns ``hyb[j]`` = m1
    quanta, or 0 where one kernel alone is at least as fast (margin).  ``cus``: the
    persistent grid's workgroups per round = the device's CU count rounded down to a
    multiple of 8 (gemm_w4.hip launch_gemm_w4 sizes its grid the same way)."""
    import math

    J = len(t_lib) - 1
    cus = max(8, cus - cus % 8)
    round_tiles = cus // math.gcd(cus, tiles_n)          # row tiles per full round
    step = max(1, round_tiles * 256 // quantum)          # in quanta
    hyb = [0] * (J + 1)
    for j in range(1, J + 1):
        best = min(t_lib[j], t_dense[j])
        for m1 in range(step, j, step):
            t = t_dense[m1] + t_lib[j - m1] + launch_us
            if t < margin * best:
                best, hyb[j] = t, m1
    return hyb


def tune_split(groups: dict[str, list[torch.Tensor]], max_m: dict[str, int], quantum: int = 256,
               reps: int = 3) -> tuple[dict, list]:
    """For each projection and every multiple of ``quantum`` rows up to ``max_m[name]``:
    time torch.matmul (hipBLASLt's first heuristic choice) and the heuristic's top
    LT_CANDIDATES algorithms called directly (csrc/bindings/gemm_lt.cpp), keep the
    fastest per bucket, then derive the M-split plan over the best times (see
    ops.split_chunks / ops.linear)."""
    ops = _native.ops()
    lt_on = os.environ.get("RFQ_GEMM_LT", "0") == "1"     # measured neutral: off by default
    plan, report = {}, []
    for name, ws in groups.items():
        N, K = ws[0].shape
        J = max_m.get(name, 0) // quantum
        if J < 2 or (N, K) in plan or _tiled_group(ws):
            continue                 # in-place tiled weights: always the tiled dense GEMM
        w = ws[0]
        x = torch.randn(J * quantum, K, device=w.device, dtype=w.dtype)
        out = torch.empty(J * quantum, N, device=w.device, dtype=w.dtype)
        times, algos, n_lt = [0.0], [-1], 0
        for j in range(1, J + 1):
            m = j * quantum
            t_best = _time(lambda w_, m=m: torch.matmul(x[:m], w_.t(), out=out[:m]), [w], reps,
                           graph=False)
            a_best = -1
            if lt_on:
                for a in ops.lt_heuristic(m, N, K, LT_CANDIDATES):
                    if ops.lt_matmul(x[:m], w, out[:m], a) != 0:
                        continue                     # algorithm rejects this shape
                    t = _time(lambda w_, m=m, a=a: ops.lt_matmul(x[:m], w_, out[:m], a), [w],
                              reps, graph=False)
                    if t < 0.98 * t_best:
                        t_best, a_best = t, a
            n_lt += a_best >= 0
            times.append(t_best)
            algos.append(a_best)
        table = plan_splits(times)
        # the hand-written 256x256 MFMA GEMM (gemm_dense.hip) per bucket, against the
        # library's best (one call or the split plan); for gate|up the comparison is
        # GEMM + silu_mul vs the same kernel with the SwiGLU epilogue
        dense = [-1] * (J + 1)
        swi = [-1] * (J + 1)
        t_dense = [float("inf")] * (J + 1)         # best hand-written time per bucket
        c_dense = [-1] * (J + 1)                   # and its cfg
        t_lib_j = [float("inf")] * (J + 1)
        n_dense = n_swi = 0
        if DENSE_ON and gemm_dense_ok(quantum, N, K):
            act = torch.empty(J * quantum, N // 2, device=w.device, dtype=w.dtype) \
                if name == "gate_up" else None
            cus = torch.cuda.get_device_properties(w.device).multi_processor_count

            def skip(c, m):
                # K % 128, < 2 GiB operands; a stream-K cfg only where it changes the launch
                return (c & 8 and not gemm_w4_ok(m, N, K)) or \
                    (c & 16384 and not w4p_stream_k_applies(m, N, K, cus))
            for j in range(1, J + 1):
                m = j * quantum
                t_lib = times[j] if table[j] is None else \
                    sum(times[c] for c in table[j]) + 4.0 * (len(table[j]) - 1)
                best_c, t_best = -1, t_lib * DENSE_MARGIN
                t_lib_j[j] = t_lib
                for c in DENSE_CFGS:
                    if skip(c, m):
                        continue
                    t = _time(lambda w_, m=m, c=c: ops.gemm_dense(x[:m], w_, out[:m], False, c),
                              [w], reps, graph=False)
                    if t < t_dense[j]:
                        t_dense[j], c_dense[j] = t, c
                    if t < t_best:
                        best_c, t_best = c, t
                dense[j] = best_c
                n_dense += best_c >= 0
                if act is not None:
                    t_silu = _time(lambda w_, m=m: silu_mul(out[:m], act[:m]), [w], reps,
                                   graph=False)
                    # the plain GEMM the reference pays: the hand-written kernel only
                    # where it won above (t_best is t_lib * margin where it did not --
                    # using that would apply the margin twice)
                    t_ref = (t_best if best_c >= 0 else t_lib) + t_silu
                    bs, ts = -1, t_ref * DENSE_MARGIN
                    for c in DENSE_CFGS:
                        if skip(c, m):
                            continue
                        t = _time(lambda w_, m=m, c=c: ops.gemm_dense(x[:m], w_, act[:m], True, c),
                                  [w], reps, graph=False)
                        if t < ts:
                            bs, ts = c, t
                    swi[j] = bs
                    n_swi += bs >= 0
                    report.append(("swiglu:" + name, m, N, K, round(t_ref, 1),
                                   f"dense{bs}" if bs >= 0 else "lib", round(min(ts, t_ref), 1)))
                report.append(("dense:" + name, m, N, K, round(t_lib, 1),
                               f"dense{best_c}" if best_c >= 0 else "lib", round(t_best, 1)))
            del act
        # rows split between a whole number of the hand-written kernel's rounds and the
        # library (plain GEMMs; buckets where one kernel alone was not beaten stay so)
        hyb = [0] * (J + 1)
        if DENSE_ON and any(c >= 0 for c in c_dense) and os.environ.get("RFQ_GEMM_HYBRID", "1") != "0":
            cus = torch.cuda.get_device_properties(w.device).multi_processor_count
            hyb = plan_hybrid(t_lib_j, t_dense, N // 256, quantum, cus=cus)
            hyb = [(m1, c_dense[m1]) if m1 > 0 and c_dense[m1] >= 0 and dense[j] < 0 else 0
                   for j, m1 in enumerate(hyb)]
        n_hyb = sum(1 for h in hyb if h)
        plan[(N, K)] = (quantum, table, algos, dense, swi, hyb)
        report.append(("lt:" + name, J * quantum, N, K, J, f"{n_lt}/{J} buckets", 0.0))
        w4 = sum(1 for c in dense if c >= 0 and c & 8)
        w4s = sum(1 for c in swi if c >= 0 and c & 8)
        sk = sum(1 for c in dense if c >= 0 and c & 16384)
        sks = sum(1 for c in swi if c >= 0 and c & 16384)
        report.append(("dense:" + name, J * quantum, N, K, J,
                       f"{n_dense}/{J} buckets (w4 {w4}, stream-K {sk}), hybrid {n_hyb}, "
                       f"swiglu {n_swi}/{J} (w4 {w4s}, stream-K {sks})", 0.0))
        for j, parts in enumerate(table):
            if parts is not None:
                t_split = sum(times[c] for c in parts)
                report.append(("split:" + name, j * quantum, N, K, round(times[j], 1),
                               "+".join(str(c * quantum) for c in parts), round(t_split, 1)))
        del x, out
    return plan, report


def _rotation(ws: list[torch.Tensor], min_bytes: int = 1 << 30) -> list[torch.Tensor]:
    """The leading layers' weights of a projection that add up to >= ``min_bytes``
    (at least two): a timing that rotates through them streams every call from HBM
    (4x the 256 MB Infinity Cache), and a 70B layer's 168-470 MB projections do not
    need all 80 layers for that (the start-up plans' timings replay every weight of the
    list per repetition)."""
    out, nb = [], 0
    for w in ws:
        out.append(w)
        nb += w.numel() * w.element_size()
        if nb >= min_bytes and len(out) >= 2:
            break
    return out


def tune_model(model, ms: list[int], lm_ms: list[int], max_tokens: int = 0,
               max_seqs: int = 0) -> list:
    """Tune every projection of a DecoderLM and install the plan."""
    w = model.w
    groups = {"qkv": [l["qkv"] for l in w["layers"]], "o": [l["o"] for l in w["layers"]]}
    if "gate_up" in w["layers"][0]:
        groups["gate_up"] = [l["gate_up"] for l in w["layers"]]
        groups["down"] = [l["down"] for l in w["layers"]]
    groups["lm_head"] = [w["lm_head"]] * 4
    groups = {k: _rotation(v) for k, v in groups.items()}
    msg = {k: ms for k in groups}
    msg["lm_head"] = lm_ms
    plan, report = tune_linear(groups, msg)
    set_linear_plan(plan, sorted(set(ms) | set(lm_ms)))
    if "down" in groups:                       # after the plain plan: the reference path uses it
        splan, sreport = tune_silu_down(groups["down"], ms)
        set_silu_plan(splan)
        report += sreport
    if os.environ.get("RFQ_FUSE_ROPE", "1") != "0" and getattr(model, "cos_sin", None) is not None:
        rplan, rreport = tune_rope(groups["qkv"], ms, model.cos_sin, model.hq, model.hkv)
        set_rope_plan(rplan)
        report += rreport
    if "gate_up" in groups and os.environ.get("RFQ_FUSE_SWIGLU", "1") != "0":
        # column-parallel gate|up: the SwiGLU epilogue needs no collective, so the
        # plan applies at any TP degree (the shard's own F = ffn / TP)
        wplan, wreport = tune_swiglu(groups["gate_up"], ms)
        set_swiglu_plan(wplan)
        report += wreport
    tp = getattr(model, "tp", None)
    if os.environ.get("RFQ_FUSE_NORM", "1") != "0" and not (tp is not None and tp.enabled):
        # TP = 1 only: with TP an all-reduce sits between the projection and the norm
        nw = w["layers"][0]["mlp_norm"]
        nplan, nreport = tune_norm(groups["o"], ms, nw, gated=False)
        if "down" in groups:
            p2, r2 = tune_norm(groups["down"], ms, nw, gated=True)
            nplan.update(p2)
            nreport += r2
            # the down projection on the SwiGLU output of the fused gate|up kernel
            p3, r3 = tune_norm(groups["down"], ms, nw, gated=False)
            nplan.update(p3)
            nreport += [("down(act)+norm",) + tuple(r[1:]) for r in r3]
        set_norm_plan(nplan)
        report += nreport
    if max_tokens > 0:
        mm = {k: max_tokens for k in groups}
        mm["lm_head"] = max_seqs
        xplan, xreport = tune_split(groups, mm)
        set_split_plan(xplan)
        SPLIT_REPORT[:] = xreport
        for r in xreport:
            log.info("gemm split %-14s M=%-5d N=%-6d K=%-6d lib %.1fus -> %s %.1fus", *r)
    for r in report:
        sel = "lib" if r[5] < 0 else (
            f"rows{r[5] & 15}" if r[5] & ROWS_BIT else
            (f"splitk{r[5] & 15}" + ("t" if r[5] & SPLITK_TILED else "")
             + ("n" if r[5] & SPLITK_NT else ""))
            if r[5] & SPLITK_BIT else f"skinny{r[5]}")
        log.info("gemm plan %-8s M=%-3d N=%-6d K=%-6d hipblaslt %.1fus -> %s %.1fus",
                 r[0], r[1], r[2], r[3], r[4], sel, r[6])
    return report
