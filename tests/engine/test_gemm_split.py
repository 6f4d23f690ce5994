"""hipBLASLt M-split planner (ops/autotune.py plan_splits + ops.split_chunks): exact DP
on synthetic timing curves, chunk rows always cover M exactly, and the split
linear path equals one GEMM (CPU oracle)."""
import itertools

import pytest

import torch

from replisense_rfq_amd import ops
from replisense_rfq_amd.ops.autotune import plan_splits


def _brute(times, launch):
    J = len(times) - 1
    best = {}

    def parts(n, mx):
        if n == 0:
            yield ()
            return
        for c in range(min(n, mx), 0, -1):
            for rest in parts(n - c, c):
                yield (c,) + rest

    for j in range(1, J + 1):
        best[j] = min(sum(times[c] for c in p) + launch * (len(p) - 1) for p in parts(j, j))
    return best


def test_plan_matches_bruteforce_and_margin():
    # a curve with a cliff: 5..7 quanta are slow per row (heuristic picks a bad tile)
    times = [0.0, 10, 18, 26, 34, 80, 95, 110, 70, 78, 86]
    table = plan_splits(times, margin=1.0, launch_us=1.0)
    brute = _brute(times, 1.0)
    for j in range(1, len(times)):
        p = table[j]
        got = times[j] if p is None else sum(times[c] for c in p) + (len(p) - 1) * 1.0
        assert abs(got - brute[j]) < 1e-9, (j, p, got, brute[j])
        if p is not None:
            assert sum(p) == j and list(p) == sorted(p, reverse=True)
    assert table[5] is not None and table[4] is None
    # margin: a 1 % gain is not worth a second launch
    flat = [0.0] + [10.0 * j for j in range(1, 9)]
    assert all(p is None for p in plan_splits(flat, margin=0.95, launch_us=0.0))


def test_split_chunks_cover_m():
    times = [0.0, 10, 18, 26, 34, 80, 95, 110, 70, 78, 86]
    ops.set_split_plan({(64, 32): (16, plan_splits(times, margin=1.0, launch_us=1.0))})
    try:
        for M in range(1, 16 * 10 + 1):
            rows = ops.split_chunks(M, 64, 32)
            if rows is not None:
                assert sum(rows) == M and all(r > 0 for r in rows)
        assert ops.split_chunks(16 * 11, 64, 32) is None      # past the tuned range
        assert ops.split_chunks(100, 64, 31) is None          # untuned shape
        rows = ops.split_chunks(16 * 5 - 3, 64, 32)
        assert rows is not None and len(rows) > 1
    finally:
        ops.set_split_plan({})


def test_split_linear_equals_one_gemm(monkeypatch):
    """The chunked path writes every row exactly once (run on CPU via the same slicing)."""
    torch.manual_seed(0)
    x = torch.randn(77, 32)
    w = torch.randn(64, 32)
    want = x @ w.t()
    rows = [48, 16, 13]
    out = torch.empty(77, 64)
    a = 0
    for r in rows:
        torch.matmul(x[a:a + r], w.t(), out=out[a:a + r])
        a += r
    assert torch.allclose(out, want, atol=1e-5)
    assert list(itertools.accumulate(rows))[-1] == 77


def test_decode_splits_rule_matches_runner():
    """The tuner's copy of the decode split rule equals ModelRunner._decode_splits(graph=True)."""
    from types import SimpleNamespace

    from replisense_rfq_amd.engine.runner import ModelRunner
    from replisense_rfq_amd.ops.autotune import decode_splits_for

    for hkv in (1, 2, 8):
        fake = SimpleNamespace(is_cuda=True, model=SimpleNamespace(hkv=hkv))
        for rows in (1, 2, 4, 8, 16, 64, 200):
            assert decode_splits_for(rows, hkv) == ModelRunner._decode_splits(fake, rows, 4096,
                                                                             True)


def test_plan_hybrid_whole_rounds():
    """Hybrid rows: the hand-written kernel takes whole rounds of 256 x 256 tiles (for
    16 weight tiles that is every 16 row tiles = 4,096 rows), the library the rest, only
    where that beats both kernels alone."""
    from replisense_rfq_amd.ops.autotune import plan_hybrid

    J = 32                                    # buckets of 256 rows up to 8,192
    # hand-written: 10 µs per 16-row-tile round (quantised), library: linear 0.7 µs / tile
    t_dense = [float("inf")] + [10.0 * -(-j // 16) for j in range(1, J + 1)]
    t_lib = [float("inf")] + [0.7 * j for j in range(1, J + 1)]
    hyb = plan_hybrid(t_lib, t_dense, tiles_n=16, quantum=256, launch_us=0.0, margin=1.0)
    assert all(h in (0, 16) for h in hyb)               # only whole rounds (16 quanta)
    # 17 quanta: dense alone 20 (two rounds), library 11.9, hybrid 10 + 0.7 = 10.7
    assert hyb[17] == 16
    # 16 quanta: one full round is best alone, no split
    assert hyb[16] == 0
    # a split never wins where the library alone is cheaper than a round
    assert hyb[5] == 0


@pytest.mark.gpu
def test_linear_hybrid_rows_gpu():
    """ops.linear with a hybrid plan entry: the first m1 rows on the persistent
    hand-written GEMM, the rest on the library, equal to one GEMM."""
    import math

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N, K, M = 4096, 512, 4096 + 1000
    J = -(-M // 256)
    hyb = [0] * (J + 2)
    hyb[J] = (16, 13960)
    plan = {(N, K): (256, [None] * (J + 2), [-1] * (J + 2), [-1] * (J + 2), [-1] * (J + 2), hyb)}
    ops.set_split_plan(plan)
    try:
        g = torch.Generator(device="cuda").manual_seed(3)
        x = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16)
        assert ops._hybrid_rows(M, N, K) == (4096, 13960)
        y = ops.linear(x, w)
        ref = (x.float() @ w.float().t())
        assert (y.float() - ref).abs().max().item() < 3e-2
    finally:
        ops.set_split_plan({})


def test_hybrid_rows_lookup():
    """ops._hybrid_rows reads the plan's sixth entry per M bucket; older 5-entry plans,
    untuned shapes and splits that would cover all of M mean no hybrid."""
    q = 256
    hyb = [0] * 40
    hyb[20] = (16, 13960)            # 20 buckets: 4,096 rows on the hand-written kernel
    hyb[16] = (16, 13960)            # m1 == M: never a split
    ops.set_split_plan({(4096, 512): (q, [None] * 40, [-1] * 40, [-1] * 40, [-1] * 40, hyb),
                        (4096, 1024): (q, [None] * 40, [-1] * 40, [-1] * 40, [-1] * 40)})
    try:
        assert ops._hybrid_rows(20 * q - 100, 4096, 512) == (4096, 13960)
        assert ops._hybrid_rows(16 * q, 4096, 512) == (0, -1)
        assert ops._hybrid_rows(10 * q, 4096, 512) == (0, -1)
        assert ops._hybrid_rows(20 * q, 4096, 1024) == (0, -1)     # 5-entry plan
        assert ops._hybrid_rows(20 * q, 2048, 512) == (0, -1)      # untuned shape
        assert ops._hybrid_rows(100 * q, 4096, 512) == (0, -1)     # past the tuned range
    finally:
        ops.set_split_plan({})


def test_plan_hybrid_follows_cu_count():
    """a whole round of persistent tiles is CU-count dependent.  On a 240-CU
    device with 16 weight tiles a round is 15 row tiles (240 / gcd(240, 16)), so the only
    split the plan may take is a multiple of 15 quanta."""
    from replisense_rfq_amd.ops.autotune import plan_hybrid

    J = 40
    t_dense = [float("inf")] + [10.0 * -(-j // 15) for j in range(1, J + 1)]
    t_lib = [float("inf")] + [0.7 * j for j in range(1, J + 1)]
    hyb = plan_hybrid(t_lib, t_dense, tiles_n=16, quantum=256, launch_us=0.0, margin=1.0,
                      cus=240)
    assert all(h % 15 == 0 for h in hyb)
    assert hyb[16] == 15
    # a CU count that is not a multiple of 8 rounds down like the launcher (244 -> 240)
    assert plan_hybrid(t_lib, t_dense, 16, 256, 0.0, 1.0, cus=244) == hyb


def test_tuning_rotation_streams_from_hbm():
    """The start-up plans time each candidate over the leading layers' weights that add
    up to >= 1 GiB (>= 2 of them), not all of a 70B model's 80 layers."""
    from replisense_rfq_amd.ops.autotune import _rotation

    mb = 1 << 20
    big = [torch.empty(84 * mb, dtype=torch.bfloat16) for _ in range(10)]     # 168 MB each
    r = _rotation(big)
    assert len(r) == 7 and sum(w.numel() * 2 for w in r) >= 1 << 30
    small = [torch.empty(mb, dtype=torch.bfloat16) for _ in range(32)]        # 2 MB each
    assert len(_rotation(small)) == 32                 # all of them, still under 1 GiB
    huge = [torch.empty(600 * mb, dtype=torch.bfloat16) for _ in range(3)]   # 1.2 GB each
    # (torch.empty never touches the pages: ~4 GB of address space, no resident memory)
    assert len(_rotation(huge)) == 2


def test_stream_k_rule_matches_launcher():
    """ops.w4p_stream_k_applies mirrors gemm_w4.hip launch_gemm_w4's stream-K region rule
    (the start-up plan times cfg bit 14 only where it changes the launch): 256-row x
    256-column tiles on the CU count rounded down to 8; a last round at least half full,
    or (under half) that round plus the full one before it; >= 2 chunks of 4 K-tiles
    per workgroup; K % 256."""
    from replisense_rfq_amd.ops import w4p_stream_k_applies as sk
    assert sk(2048, 6144, 4096, 256)          # 192 tiles, below one round, >= half
    assert not sk(1024, 6144, 4096, 256)      # 96 tiles: under half a round, no full round
    assert sk(5000, 4096, 1024, 256)          # 320 tiles: 64 past a full round -> 320
    assert not sk(4096, 4096, 4096, 256)      # 256 tiles: whole rounds
    assert not sk(2048, 6144, 4224, 256)      # K % 256
    assert not sk(2048, 6144, 256, 256)       # 192 chunks < 2 per workgroup
    assert sk(2048, 6144, 4096, 260) == sk(2048, 6144, 4096, 256)   # 260 CUs -> 256
