"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference."""
import math

import pytest
import torch

from replisense_rfq_amd import ops
from replisense_rfq_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _close(a, b, atol, rtol=0.0, what=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"{what}: max err {err} > {lim}"


@pytest.mark.parametrize("rows,d", [(1, 4096), (7, 8192), (300, 4096), (3, 1024)])
def test_rms_norm(gpu, rows, d):
    torch.manual_seed(0)
    x = torch.randn(rows, d, device=gpu, dtype=BF)
    w = (1 + 0.1 * torch.randn(d, device=gpu)).to(BF)
    out = ops.rms_norm(x, w, 1e-5)
    exp = torch.empty_like(x)
    ref.rms_norm(x, w, 1e-5, exp)
    _close(out, exp, 2e-2, 1e-2, "rms_norm")


@pytest.mark.parametrize("rows,d", [(1, 4096), (33, 8192)])
def test_fused_add_rms_norm(gpu, rows, d):
    torch.manual_seed(1)
    x = torch.randn(rows, d, device=gpu, dtype=BF)
    res = torch.randn(rows, d, device=gpu, dtype=BF)
    w = torch.randn(d, device=gpu).to(BF)
    r1, r2 = res.clone(), res.clone()
    out = ops.fused_add_rms_norm(x, r1, w, 1e-5)
    exp = torch.empty_like(x)
    ref.fused_add_rms_norm(x, r2, w, 1e-5, exp)
    assert torch.equal(r1, r2), "residual sum must be bit-exact"
    _close(out, exp, 3e-2, 1e-2, "fused_add_rms_norm")
    # in-place (out aliases x)
    x2, r3 = x.clone(), res.clone()
    ops.fused_add_rms_norm(x2, r3, w, 1e-5, out=x2)
    _close(x2, exp, 3e-2, 1e-2, "fused_add_rms_norm inplace")


def test_silu_mul_and_embed(gpu):
    torch.manual_seed(2)
    # full width, a TP=8 shard (row slice narrower than one workgroup), and a
    # row-strided view of a wider buffer
    for rows, F, pad in ((37, 14336, 0), (70000, 1792, 0), (5, 1800, 24)):
        gu = torch.randn(rows, 2 * F + pad, device=gpu, dtype=BF)[:, :2 * F]
        out = ops.silu_mul(gu)
        exp = torch.empty_like(out)
        ref.silu_mul(gu, exp)
        _close(out, exp, 1e-2, 1e-2, f"silu_mul rows={rows} F={F}")
    table = torch.randn(1000, 4096, device=gpu, dtype=BF)
    ids = torch.randint(0, 1000, (19,), device=gpu, dtype=torch.int32)
    assert torch.equal(ops.embed(ids, table), table[ids.long()])
    # vocab-parallel shard [500, 1000)
    shard = table[500:].contiguous()
    got = ops.embed(ids, shard, vocab_start=500)
    exp = torch.where((ids >= 500)[:, None], table[ids.long()], torch.zeros_like(table[ids.long()]))
    assert torch.equal(got, exp)


def _paged_cache(nblocks, Hkv, device, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    k = torch.randn(nblocks, Hkv, 32, 128, generator=g).to(device=device, dtype=BF)
    v = torch.randn(nblocks, Hkv, 32, 128, generator=g).to(device=device, dtype=BF)
    return k, v


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])
def test_rope_kv(gpu, Hq, Hkv):
    torch.manual_seed(3)
    T = 37
    cs = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * 128, device=gpu, dtype=BF)
    pos = torch.randint(0, 4000, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(64 * 32, device=gpu)[:T].int()
    slots[5] = -1
    k1, v1 = _paged_cache(64, Hkv, gpu)
    k2, v2 = k1.clone(), v1.clone()
    q1, q2 = qkv.clone(), qkv.clone()
    ops.rope_kv(q1, pos, cs, slots, k1, v1, Hq, Hkv)
    ref.rope_kv(q2, pos, cs, slots, k2, v2, Hq, Hkv)
    _close(q1, q2, 2e-2, 0, "rope q")
    _close(k1, k2, 2e-2, 0, "rope k cache")
    assert torch.equal(v1, v2)


def _block_tables(lens, nblocks, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    maxb = max((l + 31) // 32 for l in lens)
    perm = torch.randperm(nblocks, generator=g)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32)
    i = 0
    for b, l in enumerate(lens):
        nb = (l + 31) // 32
        bt[b, :nb] = perm[i:i + nb]
        i += nb
    return bt.to(device)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8)])
@pytest.mark.parametrize("splits,single", [(1, False), (4, False), (4, True), (16, True)])
@pytest.mark.parametrize("tiles", [1, 2])
def test_attn_decode(gpu, Hq, Hkv, splits, single, tiles):
    """Decode rows (q=1) and short extend rows (q>1, causal inside the extend); a work
    item covers `tiles` 16-column tiles of a sequence.  single: split partials merged
    in-kernel by the last split wave (ticket buffer), three launches in a row so the
    tickets must have been reset, compared bit-for-bit with the two-launch merge."""
    torch.manual_seed(4)
    G = Hq // Hkv
    cases = [(1, 1), (1, 31), (1, 32), (1, 33), (1, 700), (5, 129), (9, 2049), (3, 3), (1, 64)]
    qlens = [c[0] for c in cases]
    kvlens = [c[1] for c in cases]
    k, v = _paged_cache(512, Hkv, gpu, seed=5)
    bt = _block_tables(kvlens, 512, gpu)
    T = sum(qlens)
    qs = [sum(qlens[:i]) for i in range(len(qlens))]
    ws, wct = [], []
    for i, ql in enumerate(qlens):
        for ct in range(((ql * G + 15) // 16 + tiles - 1) // tiles):
            ws.append(i)
            wct.append(ct)
    ws.append(-1)          # a padding work item must be ignored
    wct.append(0)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=gpu)  # noqa: E731
    q = torch.randn(T, Hq * 128, device=gpu, dtype=BF)
    out = torch.empty(T, Hq * 128, device=gpu, dtype=BF)
    po = torch.empty(T * Hq * splits * 128, device=gpu)
    pm = torch.empty(T * Hq * splits * 2, device=gpu)
    scale = 1 / math.sqrt(128)
    ops.attn_decode(q, k, v, bt, i32(qs), i32(qlens), i32(kvlens), i32(ws), i32(wct), out, po,
                    pm, Hq, Hkv, scale, splits, tiles)
    if single:
        tickets = torch.zeros(len(ws) * Hkv, dtype=torch.int32, device=gpu)
        for it in range(3):
            out1 = torch.full_like(out, float("nan"))
            ops.attn_decode(q, k, v, bt, i32(qs), i32(qlens), i32(kvlens), i32(ws), i32(wct),
                            out1, po, pm, Hq, Hkv, scale, splits, tiles, tickets)
            torch.cuda.synchronize()
            assert int(tickets.abs().sum()) == 0, "tickets not reset"
            # same partials, same merge order and arithmetic up to f32 rounding of the weights
            _close(out1, out, 8e-3, 0, f"single-pass it={it}")
    exp = torch.zeros(T, Hq * 128, dtype=BF)
    ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), torch.tensor(qs), torch.tensor(qlens),
                     torch.tensor(kvlens), None, None, exp, Hq, Hkv, scale)
    _close(out, exp, 2e-2, 0, f"attn_decode Hq={Hq} splits={splits} tiles={tiles}")


@pytest.mark.parametrize("Hq,Hkv,tiles", [(32, 8, 1), (32, 8, 2), (8, 1, 1)])
@pytest.mark.parametrize("share", [True, False])
def test_attn_decode_shared_prefix(gpu, Hq, Hkv, tiles, share):
    """Cascade decode attention == per-sequence attention: sequences whose leading pages
    equal sequence 0's (>= 4 pages, and before their queries) get the shared pages from
    the 8-rows-per-wave prefix pass; others (2 shared pages, too short, unrelated,
    padding) attend in full."""
    torch.manual_seed(11)
    G = Hq // Hkv
    nblocks = 2048
    k, v = _paged_cache(nblocks, Hkv, gpu, seed=12)
    rng = torch.Generator().manual_seed(13)
    perm = torch.randperm(nblocks - 1, generator=rng).tolist()
    common = perm[:12]
    nxt = 12
    cases = [(1, 400, 12)] + [(1, int(torch.randint(230, 900, (1,), generator=rng)), 7 + i % 4)
                               for i in range(30)]
    cases += [(5, 300, 9), (1, 500, 2), (1, 333, 0), (1, 100, 12), (9, 240, 12), (1, 1, -1)]
    maxb = max((kv + 31) // 32 for _, kv, _ in cases)
    bt = torch.full((len(cases), maxb), nblocks - 1, dtype=torch.int32)
    for i, (ql, kvl, sh) in enumerate(cases):
        nb = (kvl + 31) // 32
        for j in range(nb):
            if share and j < sh:
                bt[i, j] = common[j]
            elif sh >= 0:
                bt[i, j] = perm[nxt]
                nxt += 1
    qlens = [c[0] for c in cases]
    kvlens = [c[1] for c in cases]
    T = sum(qlens)
    qs = [sum(qlens[:i]) for i in range(len(qlens))]
    ws, wct = [], []
    for i, ql in enumerate(qlens[:-1]):
        for ct in range(((ql * G + 15) // 16 + tiles - 1) // tiles):
            ws.append(i)
            wct.append(ct)
    ws.append(-1)
    wct.append(0)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=gpu)  # noqa: E731
    q = torch.randn(T, Hq * 128, device=gpu, dtype=BF)
    bt = bt.to(gpu)
    args = (q, k, v, bt, i32(qs), i32(qlens), i32(kvlens), i32(ws), i32(wct))
    scale = 1 / math.sqrt(128)
    out = torch.zeros(T, Hq * 128, device=gpu, dtype=BF)
    wsi = torch.full((2 + len(cases) + T,), -7, dtype=torch.int32, device=gpu)
    pre_o = torch.empty(T * Hq * 128, device=gpu)
    pre_ml = torch.empty(T * Hq * 2, device=gpu)
    ops.attn_decode_shared(*args, out, wsi, pre_o, pre_ml, Hq, Hkv, scale, tiles, True)
    torch.cuda.synchronize()
    meta = wsi.cpu()
    if share:
        assert meta[0].item() == 7 * 32
        flags = meta[2:2 + len(cases)].tolist()
        assert flags[:32] == [1] * 32 and flags[32:] == [0, 0, 0, 1, 0]
        assert meta[1].item() == 31 + 5 + 9
    else:
        assert meta[0].item() == 0 and meta[1].item() == 0
    exp = torch.zeros(T, Hq * 128, dtype=BF)
    ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), torch.tensor(qs), torch.tensor(qlens),
                     torch.tensor(kvlens), None, None, exp, Hq, Hkv, scale)
    _close(out[:T - 1], exp[:T - 1], 2e-2, 0, f"attn_decode_shared Hq={Hq} share={share}")
    # a later layer of the same step reuses the metadata
    out2 = torch.zeros_like(out)
    ops.attn_decode_shared(*args, out2, wsi, pre_o, pre_ml, Hq, Hkv, scale, tiles, False)
    torch.testing.assert_close(out2[:T - 1], out[:T - 1], rtol=0, atol=0)


@pytest.mark.parametrize("Hq,Hkv,q_len,kv_len", [(8, 1, 2496, 2912), (8, 1, 2048, 2048),
                                                 (8, 1, 700, 3000), (64, 8, 400, 800),
                                                 (64, 8, 512, 512)])
def test_attn_prefill_balanced_split(gpu, Hq, Hkv, q_len, kv_len):
    """One long prompt at the TP=8 rank shape (Hq 8 / Hkv 1) and a short one at 70B TP=1
    (64 / 8: 13-16 items x 8 kv heads), with and without a cached prefix: the auto
    small-grid form and the balanced split-KV form (small_mode 3: up to 4 splits per
    item, fewer for the light ones) against the fp32 reference; each form runs twice
    (tickets reset) and the tickets end at zero."""
    torch.manual_seed(11)
    qblk = 32
    pages = (kv_len + 31) // 32
    k, v = _paged_cache(pages + 8, Hkv, gpu, seed=12)
    bt = _block_tables([kv_len], pages + 8, gpu, seed=13)
    q = torch.randn(q_len, Hq * 128, device=gpu, dtype=BF)
    nqb = (q_len + qblk - 1) // qblk
    i32 = dict(dtype=torch.int32, device=gpu)
    qs, ql, kvl = (torch.tensor([x], **i32) for x in (0, q_len, kv_len))
    ws, wq = torch.zeros(nqb, **i32), torch.arange(nqb, **i32)
    scale = 1 / math.sqrt(128)
    exp = torch.zeros(q_len, Hq * 128, dtype=BF)
    ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), qs.cpu(), ql.cpu(), kvl.cpu(), None,
                     None, exp, Hq, Hkv, scale)
    out = torch.zeros(q_len, Hq * 128, device=gpu, dtype=BF)
    for sm in (0, 3, 3, 2):
        out.zero_()
        ops.attn_prefill(q, k, v, bt, qs, ql, kvl, ws, wq, out, Hq, Hkv, scale, qblk,
                         hsplit_below=4096, kvsplit=True, small_mode=sm)
        _close(out, exp, 2e-2, 0, f"attn_prefill balanced q={q_len} kv={kv_len} mode={sm}")
    if ops.native_available():
        torch.cuda.synchronize()
        assert int(ops.prefill_split_ws(gpu)[1].abs().sum()) == 0, "split tickets not reset"


def test_attn_prefill_balanced_multi_sequence(gpu):
    """A chunked-prefill step at the rank shape with several prompts (fresh, prefix hit,
    chunk continuation, 1-token extend): 100 work items, so auto takes the balanced task
    list over a work list that is not one causal ramp."""
    torch.manual_seed(21)
    Hq, Hkv, qblk = 8, 1, 32
    cases = [(800, 800), (640, 1056), (1, 300), (900, 1700), (831, 2000)]
    qlens = [c[0] for c in cases]
    kvlens = [c[1] for c in cases]
    nblocks = sum((l + 31) // 32 for l in kvlens) + 16
    k, v = _paged_cache(nblocks, Hkv, gpu, seed=22)
    bt = _block_tables(kvlens, nblocks, gpu, seed=23)
    T = sum(qlens)
    starts = torch.tensor([sum(qlens[:i]) for i in range(len(qlens))], dtype=torch.int32)
    q = torch.randn(T, Hq * 128, device=gpu, dtype=BF)
    ws, wq = [], []
    for s_, ql in enumerate(qlens):
        for j in range((ql + qblk - 1) // qblk):
            ws.append(s_)
            wq.append(j)
    assert 64 < len(ws) <= 128
    args = [torch.tensor(a, dtype=torch.int32, device=gpu) for a in (qlens, kvlens, ws, wq)]
    scale = 1 / math.sqrt(128)
    exp = torch.zeros(T, Hq * 128, dtype=BF)
    ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), starts, args[0].cpu(), args[1].cpu(),
                     None, None, exp, Hq, Hkv, scale)
    out = torch.zeros(T, Hq * 128, device=gpu, dtype=BF)
    for sm in (0, 0, 2):
        out.zero_()
        ops.attn_prefill(q, k, v, bt, starts.to(gpu), args[0], args[1], args[2], args[3], out,
                         Hq, Hkv, scale, qblk, hsplit_below=4096, kvsplit=True, small_mode=sm)
        _close(out, exp, 2e-2, 0, f"attn_prefill multi-sequence mode={sm}")
    if ops.native_available():
        torch.cuda.synchronize()
        assert int(ops.prefill_split_ws(gpu)[1].abs().sum()) == 0, "split tickets not reset"


@pytest.mark.parametrize("Hq,Hkv,qblk,spike", [(32, 8, 32, False), (32, 8, 64, False),
                                               (8, 1, 32, False), (64, 8, 32, False),
                                               (32, 8, 64, True)])
def test_attn_prefill(gpu, Hq, Hkv, qblk, spike):
    """spike: a few late keys get a large norm so a row's running max jumps past the
    defer-max threshold mid-stream (forces the rescale branch, guide rule 26)."""
    torch.manual_seed(6)
    # (q_len, kv_len): fresh prompt, prefix-cache hit, 1-token extend, chunk
    cases = [(300, 300), (77, 542), (1, 65), (64, 64), (33, 1000)]
    qlens = [c[0] for c in cases]
    kvlens = [c[1] for c in cases]
    k, v = _paged_cache(512, Hkv, gpu, seed=7)
    if spike:
        k[::7, :, 5] *= 40.0                   # every 7th page: one key row 40x larger
    bt = _block_tables(kvlens, 512, gpu, seed=1)
    T = sum(qlens)
    starts = torch.tensor([sum(qlens[:i]) for i in range(len(qlens))], dtype=torch.int32)
    q = torch.randn(T, Hq * 128, device=gpu, dtype=BF)
    ws, wq = [], []
    for s, ql in enumerate(qlens):
        for j in range((ql + qblk - 1) // qblk):
            ws.append(s)
            wq.append(j)
    args = [torch.tensor(a, dtype=torch.int32, device=gpu) for a in (qlens, kvlens, ws, wq)]
    out = torch.zeros(T, Hq * 128, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(128)
    exp = torch.zeros(T, Hq * 128, dtype=BF)
    ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), starts, args[0].cpu(), args[1].cpu(),
                     None, None, exp, Hq, Hkv, scale)
    # hsplit_below 0: one workgroup per (item, kv head); 4096: GQA group 8 split over two
    # 4-wave workgroups (the small-grid form)
    # kvsplit: the head-split form's items of >= 4 key tiles split over two workgroups
    # (merged in-kernel; run twice, so the tickets must have been reset); small_mode 2:
    # the 8-wave form with the key tiles split 2-4 ways (8-wave shapes only); small_mode 3:
    # the 8-wave form with a per-item split count from the work list (balanced)
    for hs, kvs, sm in ((0, False, 0), (4096, False, 1), (4096, True, 1), (4096, True, 1),
                        (4096, True, 2), (4096, True, 2), (4096, True, 0), (4096, True, 3),
                        (4096, True, 3)):
        out.zero_()
        ops.attn_prefill(q, k, v, bt, starts.to(gpu), args[0], args[1], args[2], args[3], out,
                         Hq, Hkv, scale, qblk, hsplit_below=hs, kvsplit=kvs, small_mode=sm)
        _close(out, exp, 2e-2, 0,
               f"attn_prefill Hq={Hq} qblk={qblk} hsplit={hs} kvsplit={kvs} small_mode={sm}")
    if ops.native_available():
        torch.cuda.synchronize()
        assert int(ops.prefill_split_ws(gpu)[1].abs().sum()) == 0, "split tickets not reset"


def test_sampler_masks_and_gumbel(gpu):
    torch.manual_seed(8)
    B, V = 6, 128256
    logits = torch.randn(B, V, device=gpu, dtype=BF) * 3
    W = (V + 31) // 32
    mt = torch.zeros(3, W, dtype=torch.int64)
    mt[0] = 0xFFFFFFFF                                # everything allowed
    allowed = torch.tensor([5, 77, 1000, 128255])
    for a in allowed.tolist():                        # mask 1: four tokens
        mt[1, a >> 5] |= 1 << (a & 31)
    mt[2, 3] = 1 << 7                                 # mask 2: single token 103
    mt = (mt & 0xFFFFFFFF).to(torch.int64)
    mt = torch.where(mt >= 2 ** 31, mt - 2 ** 32, mt).to(torch.int32).to(gpu)
    midx = torch.tensor([0, 1, 2, -1, 1, 0], dtype=torch.int32, device=gpu)
    temps = torch.tensor([0.0, 0.0, 0.1, 0.1, 0.1, 1.0], device=gpu)
    seeds = torch.tensor([1, 2, 3, 4, 5, 6], dtype=torch.int64, device=gpu)
    got = ops.sample(logits, mt, midx, temps, seeds).cpu()
    _, exp = ref.sample(logits.cpu(), mt.cpu(), midx.cpu(), temps.cpu(), seeds.cpu())
    assert got.tolist() == exp.tolist()
    assert int(got[0]) == int(torch.argmax(logits[0].float()))
    assert int(got[1]) in allowed.tolist() and int(got[2]) == 103


@pytest.mark.parametrize("T", [1, 3, 17, 64, 200])
def test_moe_pipeline(gpu, T):
    """T <= 64 takes the per-expert skinny path (gather + fused SwiGLU), larger T the
    128-row grouped GEMM path; both against the fp32 torch oracle."""
    torch.manual_seed(9 + T)
    d, F, E, k = 512, 384, 8, 2
    x = (torch.randn(T, d, device=gpu) * 0.5).to(BF)
    router = (torch.randn(E, d, device=gpu) * 0.05).to(BF)
    w13 = (torch.randn(E, 2 * F, d, device=gpu) / math.sqrt(d)).to(BF)
    w2 = (torch.randn(E, d, F, device=gpu) / math.sqrt(F)).to(BF)
    from replisense_rfq_amd.models.moe import MoEBuffers, moe_mlp

    bufs = MoEBuffers.allocate(T, k, E, d, F, gpu)
    out = moe_mlp(x, router, w13, w2, k, bufs)
    logits = (x @ router.t()).cpu()
    exp = ref.moe_forward(x.cpu(), w13.cpu(), w2.cpu(), logits, k)
    _close(out, exp, 3e-2, 2e-2, f"moe T={T}")


@pytest.mark.parametrize("rows,cols", [(1, 128256), (37, 16032), (5, 1003)])
def test_count_nonfinite(gpu, rows, cols):
    """check.hip: Inf / NaN entries counted (tail columns included), finite extremes not;
    the counter accumulates across launches."""
    # rows 16-byte aligned (the kernel's vector loads); cols need not be a multiple of 8
    stride = (cols + 7) // 8 * 8
    x = (torch.randn(rows, stride, device=gpu) * 1e4).to(BF)
    x[:, cols:] = float("nan")                    # outside the view: must not be counted
    x = x[:, :cols]
    x[0, 0] = float("inf")
    x[rows - 1, cols - 1] = float("nan")
    x[rows // 2, cols // 2] = float("-inf")
    x[0, 1] = torch.finfo(torch.bfloat16).max
    cnt = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.count_nonfinite(x, cnt)
    ops.count_nonfinite(x, cnt)
    exp = int((~torch.isfinite(x.float())).sum())
    assert exp == 3 and int(cnt[0]) == 2 * exp


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("N,K", [(512, 512), (768, 384), (1024, 1024)])
def test_moe_gemm8(gpu, swiglu, N, K, tile):
    """8-wave grouped GEMM over 128-row expert blocks (padding blocks -1 and blocks
    past num_blocks untouched) == per-block fp32 GEMM; swiglu == GEMM -> bf16 ->
    silu_mul (act.hip rounding)."""
    torch.manual_seed(N + K + swiglu)
    # segments as moe_align lays them out: expert-sorted, padded rows at the end; expert 1
    # has one block, expert 3 three (a full and a half 256-row tile)
    E, nb = 4, 9
    x = torch.randn(nb * 128, K, device=gpu, dtype=BF)
    w = (torch.randn(E, N, K, device=gpu) / math.sqrt(K)).to(BF)
    eob = torch.tensor([0, 0, 1, 2, 2, 3, 3, 3, -1], dtype=torch.int32, device=gpu)
    offs = torch.tensor([0, 256, 384, 640, 1024], dtype=torch.int32, device=gpu)
    num = torch.tensor([8], dtype=torch.int32, device=gpu)       # block 8 not computed
    n_out = N // 2 if swiglu else N
    out = torch.full((nb * 128, n_out), float("nan"), device=gpu, dtype=BF)
    ops.moe_gemm8(x, w, out, eob, num, offs, swiglu, tile)
    for b in range(nb):
        rows = slice(128 * b, 128 * b + 128)
        e = int(eob[b])
        if b >= 8 or e < 0:
            assert torch.isnan(out[rows].float()).all(), f"block {b} written"
            continue
        h = (x[rows].float() @ w[e].float().t())
        if swiglu:
            act = torch.empty(128, n_out, dtype=BF)
            ref.silu_mul(h.to(BF).cpu(), act)
            _close(out[rows], act.float(), 3e-2, 2e-2, f"gemm8 swiglu block {b}")
        else:
            _close(out[rows], h, 2e-2, 1e-2, f"gemm8 block {b}")


@pytest.mark.parametrize("M", [1, 5, 16, 17, 40, 64])
@pytest.mark.parametrize("N,K", [(512, 4096), (256, 14336), (1024, 3584)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3])
def test_skinny_gemm(gpu, M, N, K, cfg):
    torch.manual_seed(M * 7 + cfg)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(BF)
    out = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm(x, w, out, cfg)
    exp = x.float() @ w.float().t()
    _close(out, exp, 1e-2, 1e-2, f"skinny_gemm M={M} cfg={cfg}")


def test_skinny_gemm_strided_rows(gpu):
    """x / out as row-slices of wider buffers (the runner's packed activations)."""
    torch.manual_seed(3)
    big = torch.randn(8, 4096 + 256, device=gpu, dtype=BF)
    x = big[:, :4096]
    w = (torch.randn(1024, 4096, device=gpu) * 0.02).to(BF)
    obuf = torch.zeros(8, 1024 + 64, device=gpu, dtype=BF)
    out = obuf[:, :1024]
    ops.linear(x, w, out=out)
    _close(out, x.float() @ w.float().t(), 1e-2, 1e-2, "linear strided")
    assert torch.all(obuf[:, 1024:] == 0)


@pytest.mark.parametrize("M", [1, 7, 16, 33])
@pytest.mark.parametrize("cfg", [16, 17, 18, 19])
def test_skinny_gemm_gated_swiglu(gpu, M, cfg):
    """Gated-X skinny GEMM == silu_mul (act.hip semantics) followed by the GEMM."""
    torch.manual_seed(M + cfg)
    F, N = 1024, 512
    gu = torch.randn(M, 2 * F, device=gpu, dtype=BF)
    w = (torch.randn(N, F, device=gpu) * 0.03).to(BF)
    out = torch.empty(M, N, device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm(gu, w, out, cfg)
    act = torch.empty(M, F, dtype=BF)
    ref.silu_mul(gu.cpu(), act)
    _close(out, act.float() @ w.float().cpu().t(), 2e-2, 1e-2, f"gated skinny M={M} cfg={cfg}")


@pytest.mark.parametrize("M", [1, 5, 16])
@pytest.mark.parametrize("gated,cfg", [(False, 12), (False, 13), (False, 14), (False, 15),
                                       (True, 16), (True, 19), (False, 12 | 64), (False, 15 | 64),
                                       (True, 16 | 64), (True, 18 | 64)])
def test_skinny_gemm_fused_add_norm(gpu, M, gated, cfg):
    """skinny GEMM + last-workgroup residual-add RMSNorm == skinny GEMM followed by
    fused_add_rms_norm; three launches in a row (the ticket counter must reset)."""
    torch.manual_seed(M * 31 + cfg)
    N, K = 4096, 1024
    x = torch.randn(M, 2 * K if gated else K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.03).to(BF)
    nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(BF)
    counter = torch.zeros(4, dtype=torch.int32, device=gpu)
    partials = torch.empty(2 * M * N, device=gpu)
    res = torch.randn(M, N, device=gpu, dtype=BF)
    res_ref = res.clone()
    for it in range(3):
        y = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
        out = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
        torch.ops.rfq_amd.skinny_gemm_norm(x, w, y, res, nw, 1e-5, out, counter, partials, cfg)
        y_ref = torch.empty(M, N, device=gpu, dtype=BF)
        torch.ops.rfq_amd.skinny_gemm(x, w, y_ref, cfg & 63)
        res_cpu, out_ref = res_ref.cpu(), torch.empty(M, N, dtype=BF)
        ref.fused_add_rms_norm(y_ref.cpu(), res_cpu, nw.cpu(), 1e-5, out_ref)
        res_ref = res_cpu.to(gpu)
        if cfg & 64:     # split-K sums fp32 slices in another order: within one bf16 ulp
            _close(res, res_ref, 3e-2, 1e-2, f"split-K residual it={it}")
            res_ref = res.clone()
        else:
            assert torch.equal(y, y_ref), f"GEMM part differs (iteration {it})"
            assert torch.equal(res, res_ref), f"residual differs (iteration {it})"
        _close(out, out_ref, 3e-2, 1e-2, f"fused norm M={M} cfg={cfg} it={it}")
    torch.cuda.synchronize()
    assert int(counter[0]) == 0, "ticket counter not reset"


@pytest.mark.parametrize("splits", [0, 2, 4])
@pytest.mark.parametrize("T", [1, 3, 37])
def test_moe_latency_path_w2_splitk(gpu, T, splits, monkeypatch):
    """Latency-path MoE (route -> align -> gated w13 -> w2 -> combine) with the w2
    split into 0/2/4 K slices (fp32 partials summed in the combine) == the oracle."""
    from replisense_rfq_amd.models import moe as M

    monkeypatch.setattr(M, "W2_SPLITS", splits)
    torch.manual_seed(70 + T)
    d, F, E, k = 512, 1024, 8, 2
    x = (torch.randn(T, d, device=gpu) * 0.5).to(BF)
    router = (torch.randn(E, d, device=gpu) * 0.05).to(BF)
    w13 = (torch.randn(E, 2 * F, d, device=gpu) / math.sqrt(d)).to(BF)
    w2 = (torch.randn(E, d, F, device=gpu) / math.sqrt(F)).to(BF)
    bufs = M.MoEBuffers.allocate(T, k, E, d, F, gpu)
    assert (bufs.yf is not None) == (splits > 1)
    out = M.moe_mlp(x, router, w13, w2, k, bufs)
    logits = (x @ router.t()).cpu()
    exp = ref.moe_forward(x.cpu(), w13.cpu(), w2.cpu(), logits, k)
    _close(out, exp, 3e-2, 2e-2, f"moe latency path T={T} splits={splits}")


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (5, 8, 2), (64, 8, 2), (3, 16, 4)])
def test_moe_route_matches_gemm_topk(gpu, T, E, k):
    """Fused router GEMV + top-k == bf16 router GEMM followed by the top-k oracle
    (same experts; weights within bf16-logit rounding)."""
    torch.manual_seed(T * 7 + E)
    d = 4096
    x = torch.randn(T, d, device=gpu, dtype=BF)
    router = (torch.randn(E, d, device=gpu) * 0.05).to(BF)
    w = torch.empty(T, k, device=gpu)
    ids = torch.empty(T, k, device=gpu, dtype=torch.int32)
    ops.moe_route(x, router, k, True, w, ids)
    logits = (x.float() @ router.float().t()).to(BF)
    w_e, i_e = ref.moe_topk(logits.cpu(), k, True)
    # rows whose k-th and (k+1)-th logits are within summation-order rounding may
    # legitimately pick either expert: compare the others
    srt = logits.float().cpu().sort(1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]) > 0.1 if k < E else torch.ones(T, dtype=torch.bool)
    assert clear.any()
    got, exp = ids.cpu().long().sort(1).values, i_e.long().sort(1).values
    assert torch.equal(got[clear], exp[clear])
    _close(w.cpu()[clear].sort(1).values, w_e.float()[clear].sort(1).values, 2e-2, 0,
           "moe_route weights")


@pytest.mark.parametrize("M", [200, 512, 1000])
def test_lt_matmul_every_heuristic_algo(gpu, M):
    """Direct hipBLASLt calls (gemm_lt.cpp) with each of the heuristic's top algorithms
    == fp32 x w^T, including a row-strided output slice; an out-of-range index fails
    with a non-zero status instead of launching."""
    torch.manual_seed(M)
    N, K = 1536, 1024
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.03).to(BF)
    exp = x.float() @ w.float().t()
    algos = torch.ops.rfq_amd.lt_heuristic(M, N, K, 6)
    assert len(algos) >= 1
    buf = torch.zeros(M, N + 64, device=gpu, dtype=BF)
    for a in algos:
        out = buf[:, :N]
        out.fill_(float("nan"))
        assert torch.ops.rfq_amd.lt_matmul(x, w, out, a) == 0
        _close(out, exp, 2e-2, 1e-2, f"lt_matmul algo {a}")
        assert torch.all(buf[:, N:] == 0)
    assert torch.ops.rfq_amd.lt_matmul(x, w, buf[:, :N], 10 ** 6) != 0


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("cfg", [13, 15])
def test_skinny_gemm_rope_kv(gpu, M, cfg):
    """QKV skinny GEMM with the RoPE + paged-KV-append epilogue == fp32 GEMM followed by
    the rope_kv oracle (q columns of the output, k/v pages of the cache); padding rows
    (slot -1) write nothing."""
    torch.manual_seed(M * 13 + cfg)
    Hq, Hkv, K = 8, 2, 512
    N = (Hq + 2 * Hkv) * 128
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.05).to(BF)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(4 * 32, device=gpu)[:M].to(torch.int32)
    if M > 1:
        slots[-1] = -1
    kc = torch.zeros(4, Hkv, 32, 128, device=gpu, dtype=BF)
    vc = torch.zeros_like(kc)
    qkv = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm_rope(x, w, qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, cfg)
    exp = (x.float() @ w.float().t()).cpu()
    kc_e, vc_e = torch.zeros(kc.shape), torch.zeros(vc.shape)
    ref.rope_kv(exp, pos.cpu(), cos_sin.cpu(), slots.cpu(), kc_e, vc_e, Hq, Hkv)
    q = Hq * 128
    _close(qkv[:, :q], exp[:, :q], 2e-2, 1e-2, f"rope q M={M} cfg={cfg}")
    _close(kc, kc_e, 2e-2, 1e-2, f"rope k cache M={M} cfg={cfg}")
    _close(vc, vc_e, 2e-2, 1e-2, f"v cache M={M} cfg={cfg}")


@pytest.mark.parametrize("T", [3, 40, 100, 200])
@pytest.mark.parametrize("mode", ["dense", "gemm8"])
def test_moe_expert_parallel_partial(gpu, T, mode, monkeypatch):
    """Expert parallelism: a rank holding experts [2, 6) of 8 computes exactly the
    partial sum of its experts (remote pairs -> dummy segment, weight 0) on every
    path: skinny (T <= 64), the dense-structure grouped GEMMs (T > 64, the default)
    and round 2's gemm8 grouped kernels (forced by refusing the dense ones)."""
    from replisense_rfq_amd.models import moe as M

    if mode == "gemm8":
        monkeypatch.setattr(M.ops, "moe_gemm_dense_ok", lambda w, swiglu: False)
    grouped = mode
    torch.manual_seed(40 + T)
    d, F, E, k, e0, el = 512, 384, 8, 2, 2, 4
    x = (torch.randn(T, d, device=gpu) * 0.5).to(BF)
    router = (torch.randn(E, d, device=gpu) * 0.05).to(BF)
    w13 = (torch.randn(E, 2 * F, d, device=gpu) / math.sqrt(d)).to(BF)
    w2 = (torch.randn(E, d, F, device=gpu) / math.sqrt(F)).to(BF)
    bufs = M.MoEBuffers.allocate(T, k, E, d, F, gpu)
    out = M.moe_mlp(x, router, w13[e0:e0 + el].contiguous(), w2[e0:e0 + el].contiguous(), k, bufs,
                    expert_offset=e0)
    logits = (x @ router.t()).cpu()
    exp = ref.moe_forward(x.cpu(), w13[e0:e0 + el].cpu(), w2[e0:e0 + el].cpu(), logits, k, e0)
    _close(out, exp, 3e-2, 2e-2, f"moe EP T={T} grouped={grouped}")


def test_linear_m_split_plan(gpu):
    """hipBLASLt row-chunk plan (ops.autotune.tune_split): a measured plan on a real
    shape, then ops.linear through a forced multi-chunk split == one GEMM."""
    from replisense_rfq_amd.ops.autotune import plan_splits, tune_split

    torch.manual_seed(11)
    w = (torch.randn(512, 1024, device=gpu) * 0.03).to(BF)
    plan, _ = tune_split({"t": [w]}, {"t": 1024}, quantum=128, reps=1)
    q, table, algos = plan[(512, 1024)][:3]
    assert q == 128 and len(table) == 9 and len(algos) == 9
    forced = plan_splits([0.0] + [1.0] * 8 + [100.0], margin=1.0, launch_us=0.0)
    try:
        # forced multi-chunk split, each chunk on its bucket's measured algorithm
        ops.set_split_plan({(512, 1024): (128, forced, algos + [-1])})
        M = 128 * 8 + 77
        rows = ops.split_chunks(M, 512, 1024)
        assert rows is not None and len(rows) > 1 and sum(rows) == M
        x = torch.randn(M, 1024, device=gpu, dtype=BF)
        out = ops.linear(x, w)
        _close(out, x.float() @ w.float().t(), 1e-2, 1e-2, "split linear")
        # the measured plan itself, every M in the tuned range
        ops.set_split_plan(plan)
        for M in (65, 128, 300, 777, 1024):
            xm = x[:M]
            _close(ops.linear(xm, w), xm.float() @ w.float().t(), 1e-2, 1e-2, f"lt plan M={M}")
    finally:
        ops.set_split_plan({})


@pytest.mark.parametrize("M,cfg", [(1, 12), (4, 15), (16, 13), (1, 12 | 64)])
def test_skinny_norm_handoff_stress(gpu, M, cfg):
    """The NormEpi hand-off (sc1 tile stores drained by every wave, relaxed agent
    ticket, sc1 loads in the last workgroup -- cdna_hip_programming.md §6
    Guideline 16, "every load sc1" form) over many launches, with a second stream
    keeping other CUs busy (uneven load): the residual written by the last
    workgroup must equal bf16(y + residual) of the unfused GEMM bit for bit every
    time; a stale Y read would break it."""
    torch.manual_seed(M + cfg)
    N, K = 4096, 4096
    w = (torch.randn(N, K, device=gpu) * 0.02).to(BF)
    nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(BF)
    counter = torch.zeros(4, dtype=torch.int32, device=gpu)
    partials = torch.empty(2 * M * N, device=gpu)
    load_a = torch.randn(4096, 4096, device=gpu, dtype=BF)
    side = torch.cuda.Stream()
    bad = 0
    for it in range(300):
        x = torch.randn(M, K, device=gpu, dtype=BF)
        res = torch.randn(M, N, device=gpu, dtype=BF)
        res0 = res.clone()
        y = torch.empty(M, N, device=gpu, dtype=BF)
        out = torch.empty(M, N, device=gpu, dtype=BF)
        if it % 3 == 0:
            with torch.cuda.stream(side):
                load_a @ load_a                          # concurrent work on other CUs
        torch.ops.rfq_amd.skinny_gemm_norm(x, w, y, res, nw, 1e-5, out, counter, partials, cfg)
        y_ref = torch.empty(M, N, device=gpu, dtype=BF)
        torch.ops.rfq_amd.skinny_gemm(x, w, y_ref, cfg & 63)
        if cfg & 64:                                      # split-K: fp32 slices summed
            want = (y_ref.float() + res0.float()).to(BF)
            bad += int(((res.float() - want.float()).abs() > 0.05 * want.float().abs() + 0.05)
                       .any())
        else:
            bad += int(not torch.equal(res, (y_ref.float() + res0.float()).to(BF)))
    torch.cuda.synchronize()
    assert bad == 0, f"{bad} of 300 launches read a stale tile"
    assert int(counter[0]) == 0


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("cfg", [0, 2])
def test_skinny_gemm_swiglu(gpu, M, cfg):
    """gate|up GEMM with the SwiGLU epilogue == the same tile's skinny GEMM followed
    by silu_mul, bit for bit (same wave split: cfg 0 <-> 13, cfg 2 <-> 15)."""
    torch.manual_seed(M + cfg)
    F, K = 1024, 2048
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(2 * F, K, device=gpu) * 0.03).to(BF)
    out = torch.empty(M, F, device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm_swiglu(x, w, out, cfg)
    gu = torch.empty(M, 2 * F, device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm(x, w, gu, 13 if cfg == 0 else 15)
    want = torch.empty(M, F, device=gpu, dtype=BF)
    torch.ops.rfq_amd.silu_mul(gu, want)
    assert torch.equal(out, want)
    # and against the fp32 torch reference of the op
    g, u = (x.float() @ w.float().t()).split(F, dim=1)
    _close(out, torch.nn.functional.silu(g) * u, 3e-2, 2e-2, f"swiglu M={M}")


@pytest.mark.parametrize("M", [1, 5, 16])
@pytest.mark.parametrize("cfg", [0, 1, 8, 9, 12, 13])
@pytest.mark.parametrize("N,K", [(4096, 4096), (1024, 14336)])
def test_gemv_splitk(gpu, M, cfg, N, K):
    """Split-K GEMV with the in-launch per-tile reduction vs an fp32 torch matmul;
    the norm variant vs skinny GEMM + fused_add_rms_norm; repeated launches (tile
    tickets and the norm counter must be left at zero)."""
    torch.manual_seed(M * 7 + cfg)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(BF)
    part = torch.empty(16 * 16 * 16384, device=gpu)
    tiles = torch.zeros(1024, dtype=torch.int32, device=gpu)
    y = torch.empty(M, N, device=gpu, dtype=BF)
    ref_y = x.float() @ w.float().t()
    for it in range(3):
        torch.ops.rfq_amd.gemv_splitk(x, w, y, part, tiles, cfg)
        _close(y, ref_y, 2e-2, 1e-2, f"gemv_splitk cfg={cfg} it={it}")
    nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(BF)
    counter = torch.zeros(4, dtype=torch.int32, device=gpu)
    res = torch.randn(M, N, device=gpu, dtype=BF)
    for it in range(3):
        res0 = res.clone()
        out = torch.empty(M, N, device=gpu, dtype=BF)
        torch.ops.rfq_amd.gemv_splitk_norm(x, w, y, res, nw, 1e-5, out, counter, part, tiles, cfg)
        want_res = (y.float() + res0.float()).to(BF)
        assert torch.equal(res, want_res), f"residual it={it}"
        r = want_res.float()
        want = r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
        _close(out, want, 3e-2, 2e-2, f"gemv_splitk_norm cfg={cfg} it={it}")
    torch.cuda.synchronize()
    assert int(tiles.abs().sum()) == 0 and int(counter[0]) == 0


@pytest.mark.parametrize("M", [1, 3, 16])
@pytest.mark.parametrize("cfg", [0, 2, 9, 13, 14])
@pytest.mark.parametrize("F,K", [(3584, 8192), (512, 1024)])
def test_gemv_splitk_swiglu(gpu, M, cfg, F, K):
    """Split-K gate|up GEMV with the SwiGLU epilogue (TP=8 70B shard shape: F 3584,
    K 8192) vs the fp32 torch op rounded like the unfused path (GEMM -> bf16 ->
    silu_mul); repeated launches leave the tile tickets at zero."""
    torch.manual_seed(M * 11 + cfg + F)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(2 * F, K, device=gpu) / math.sqrt(K)).to(BF)
    part, tiles = ops.splitk_ws(gpu)
    out = torch.empty(M, F, device=gpu, dtype=BF)
    r = x.float() @ w.float().t()
    gg, u = r[:, :F].to(BF).float(), r[:, F:].to(BF).float()
    want = (gg * torch.sigmoid(gg)).to(BF).float() * u
    for it in range(3):
        torch.ops.rfq_amd.gemv_splitk_swiglu(x, w, out, part, tiles, cfg)
        _close(out, want, 2e-2, 1e-2, f"gemv_splitk_swiglu cfg={cfg} it={it}")
    torch.cuda.synchronize()
    assert int(tiles.abs().sum()) == 0


@pytest.mark.parametrize("M", [1, 4, 16])
@pytest.mark.parametrize("cfg", [0, 2, 9, 13])
@pytest.mark.parametrize("Hq,Hkv,K", [(8, 1, 8192), (8, 2, 1024)])
def test_gemv_splitk_rope_kv(gpu, M, cfg, Hq, Hkv, K):
    """Split-K QKV GEMV with the RoPE + paged-KV-append epilogue (TP=8 70B shard:
    Hq 8, Hkv 1, K 8192) == fp32 GEMM followed by the rope_kv oracle; padding rows
    (slot -1) write nothing; tickets left at zero."""
    torch.manual_seed(M * 17 + cfg + Hkv)
    N = (Hq + 2 * Hkv) * 128
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(4 * 32, device=gpu)[:M].to(torch.int32)
    if M > 1:
        slots[-1] = -1
    kc = torch.zeros(4, Hkv, 32, 128, device=gpu, dtype=BF)
    vc = torch.zeros_like(kc)
    qkv = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    part, tiles = ops.splitk_ws(gpu)
    torch.ops.rfq_amd.gemv_splitk_rope(x, w, qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, part,
                                       tiles, cfg)
    exp = (x.float() @ w.float().t()).cpu()
    kc_e, vc_e = torch.zeros(kc.shape), torch.zeros(vc.shape)
    ref.rope_kv(exp, pos.cpu(), cos_sin.cpu(), slots.cpu(), kc_e, vc_e, Hq, Hkv)
    q = Hq * 128
    _close(qkv[:, :q], exp[:, :q], 2e-2, 1e-2, f"splitk rope q M={M} cfg={cfg}")
    _close(kc, kc_e, 2e-2, 1e-2, f"splitk rope k cache M={M} cfg={cfg}")
    _close(vc, vc_e, 2e-2, 1e-2, f"splitk v cache M={M} cfg={cfg}")
    torch.cuda.synchronize()
    assert int(tiles.abs().sum()) == 0


@pytest.mark.parametrize("M", [1, 5, 16])
@pytest.mark.parametrize("cfg", [0, 5, 10, 14, 0 | 32 | 64, 5 | 64, 10 | 32 | 64, 14 | 64])
def test_gemv_splitk_tiled_layout(gpu, M, cfg):
    """Split-K GEMV on the decode-tiled weight layout (ops.tile_weight, cfg bit 16), also
    with non-temporal loads (32) and the persistent grid (64): the same loads in a
    different memory order / work order, so every epilogue (plain, norm, SwiGLU, RoPE +
    KV append) is bit-identical to the row-major kernel, which the fp32 oracles above
    cover; plus the plain result vs fp32 torch."""
    torch.manual_seed(M * 29 + cfg)
    T = ops.SPLITK_TILED
    part, tiles = ops.splitk_ws(gpu)
    N, K = 1024, 2048
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    wt = ops.tile_weight(w)
    assert torch.equal(ops.untile_weight(wt), w)
    y0, y1 = (torch.empty(M, N, device=gpu, dtype=BF) for _ in range(2))
    torch.ops.rfq_amd.gemv_splitk(x, w, y0, part, tiles, cfg)
    torch.ops.rfq_amd.gemv_splitk(x, wt, y1, part, tiles, cfg | T)
    assert torch.equal(y0, y1)
    _close(y1, x.float() @ w.float().t(), 2e-2, 1e-2, f"tiled gemv cfg={cfg}")
    # residual-add RMSNorm epilogue
    nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(BF)
    res = torch.randn(M, N, device=gpu, dtype=BF)
    outs = []
    for ww, c in ((w, cfg), (wt, cfg | T)):
        r = res.clone()
        o = torch.empty(M, N, device=gpu, dtype=BF)
        torch.ops.rfq_amd.gemv_splitk_norm(x, ww, y0, r, nw, 1e-5, o, ops.norm_counter(gpu),
                                           part, tiles, c)
        outs.append((r, o))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # SwiGLU epilogue (gate rows [0, F), up rows [F, 2F))
    F = N // 2
    a0, a1 = (torch.empty(M, F, device=gpu, dtype=BF) for _ in range(2))
    torch.ops.rfq_amd.gemv_splitk_swiglu(x, w, a0, part, tiles, cfg)
    torch.ops.rfq_amd.gemv_splitk_swiglu(x, wt, a1, part, tiles, cfg | T)
    assert torch.equal(a0, a1)
    # RoPE + paged KV append (Hq 6, Hkv 1: N = 1024)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(4 * 32, device=gpu)[:M].to(torch.int32)
    got = []
    for ww, c in ((w, cfg), (wt, cfg | T)):
        kc = torch.zeros(4, 1, 32, 128, device=gpu, dtype=BF)
        vc = torch.zeros_like(kc)
        q = torch.zeros((M, N), device=gpu, dtype=BF)
        torch.ops.rfq_amd.gemv_splitk_rope(x, ww, q, pos, cos_sin, slots, kc, vc, 6, 1, part,
                                           tiles, c)
        got.append((q[:, :768], kc, vc))
    for u, v in zip(*got):
        assert torch.equal(u, v)
    torch.cuda.synchronize()
    assert int(tiles.abs().sum()) == 0


@pytest.mark.parametrize("M", [1, 7, 16, 40])
@pytest.mark.parametrize("cfg", [12, 13, 14, 15])
@pytest.mark.parametrize("N,K", [(8192, 1024), (512, 384), (1024, 3584)])
def test_skinny_gemm_short_k_tail(gpu, M, cfg, N, K):
    """Skinny GEMM on K ranges shorter than one unrolled step per wave (the TP=8 o
    projection, K = 1024) and ragged tails (K = 3584: 28 k-steps over 4 / 8 waves):
    the tail path issues every load before its MFMAs; vs the fp32 torch matmul."""
    if K % 128:
        pytest.skip("K % 128")
    torch.manual_seed(M + cfg + K)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    y = torch.empty(M, N, device=gpu, dtype=BF)
    torch.ops.rfq_amd.skinny_gemm(x, w, y, cfg)
    _close(y, x.float() @ w.float().t(), 2e-2, 1e-2, f"skinny tail M={M} cfg={cfg} K={K}")


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 8, 8 | 128, 8 | 128 | 512 | 1024, 8 | 128 | 512 | 1024 | 2048,
                                 8 | 128 | 512 | 1024 | 4096, 8 | 128 | 512 | 1024 | 4096 | 8192])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (100, 512, 128), (256, 768, 1024),
                                   (300, 1280, 8192), (513, 4096, 576), (2048, 1024, 4096),
                                   (777, 2048, 512), (256, 512, 256), (4000, 4608, 512)])
def test_gemm_dense(gpu, M, N, K, swiglu, cfg):
    """The 256x256 8-wave MFMA GEMM (gemm_dense.hip) and the one-wave-per-SIMD kernel
    (cfg 8, gemm_w4.hip: K % 128 == 0) against the fp32 oracle, asymmetric operands, row
    tails (M % 256 != 0), one-tile and many-tile K loops (K 128 / 256: only the w4
    kernel's 4-step tail; 512: one steady iteration); swiglu vs the unfused GEMM ->
    bf16 -> silu_mul rounding.  4000 x 4608: 288 output tiles (256 of them with a
    partial row tile), so the persistent form (cfg bit 13) runs two tiles on 32
    workgroups with the K-tile pipeline crossing the tile boundary."""
    if cfg & 8 and K % 128:
        pytest.skip("the w4 kernel needs K % 128 == 0")
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    x = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(BF)
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / math.sqrt(K)).to(BF)
    out = ops.gemm_dense(x, w, swiglu=swiglu, cfg=cfg)
    r = x.float() @ w.float().t()
    if swiglu:
        F = N // 2
        gg, u = r[:, :F].to(BF).float(), r[:, F:].to(BF).float()
        r = (gg * torch.sigmoid(gg)).to(BF).float() * u
    _close(out, r, atol=2e-2, rtol=2e-2, what=f"gemm_dense M{M} N{N} K{K} swiglu={swiglu}")


@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("M,N,K", [(2048, 6144, 4096), (3000, 4096, 2048), (5000, 4096, 1024),
                                   (4000, 4608, 512), (7000, 4096, 1024)])
def test_gemm_w4p_stream_k(gpu, M, N, K, swiglu):
    """Stream-K form of the persistent gemm_w4p (cfg bit 14): the last rounds' tiles cut
    into runs of 4-K-tile chunks, partial tiles published as fp32 slabs and added by the
    tile's owner.  Shapes: the whole grid below one round (192 tiles), a half-full last
    round, a last round under half full (+ the full round before it), and 2-chunk runs
    (K 512: every unit 4 K-tiles long).  Three launches each (the flags must be reset by
    the owners), against the fp32 oracle and the non-stream-K kernel."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + swiglu)
    x = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(BF)
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / math.sqrt(K)).to(BF)
    base = ops.gemm_dense(x, w, swiglu=swiglu, cfg=13960)
    r = x.float() @ w.float().t()
    if swiglu:
        F = N // 2
        gg, u = r[:, :F].to(BF).float(), r[:, F:].to(BF).float()
        r = (gg * torch.sigmoid(gg)).to(BF).float() * u
    for it in range(3):
        out = ops.gemm_dense(x, w, swiglu=swiglu, cfg=13960 | 16384)
        _close(out, r, atol=2e-2, rtol=2e-2, what=f"gemm_w4p stream-K M{M} N{N} K{K} it{it}")
        # same products, only the fp32 summation order of split tiles differs
        assert (out.float() - base.float()).abs().max().item() <= 2e-2 * r.abs().max().item()


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 8, 8 | 128 | 512 | 1024 | 2048, 8 | 128 | 512 | 1024 | 4096,
                                 8 | 128 | 512 | 1024 | 4096 | 8192])
def test_gemm_dense_identity_asymmetric(gpu, cfg):
    """A = I with an asymmetric B catches a transposed C write (§3)."""
    K = 256
    x = torch.eye(K, device="cuda", dtype=BF)
    w = (torch.arange(512 * K, device="cuda", dtype=torch.float32).reshape(512, K) % 97 - 48).to(BF)
    out = ops.gemm_dense(x, w, cfg=cfg)
    assert torch.equal(out.float(), w.float().t()[:K])


@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("M,N,K", [(1, 256, 128), (100, 512, 256), (513, 1280, 1024),
                                   (300, 4096, 8192)])
def test_gemm_dense_tiled_weight(gpu, M, N, K, swiglu):
    """gemm_dense reading the decode-tiled weight layout (cfg bit 4 -> 2 | 4): same LDS
    image, so bit-identical to the row-major kernel of the same schedule (cfg 2)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + swiglu)
    x = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(BF)
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / math.sqrt(K)).to(BF)
    a = ops.gemm_dense(x, w, swiglu=swiglu, cfg=2)
    b = ops.gemm_dense(x, ops.tile_weight(w), swiglu=swiglu, cfg=2 | 4)
    assert torch.equal(a, b)


def test_gemm_dense_strided_rows(gpu):
    x = torch.randn(300, 1024 + 64, device="cuda", dtype=BF)[:, :1024]
    w = (torch.randn(512, 1024, device="cuda") / 32).to(BF)
    out = torch.empty(300, 512 + 256, device="cuda", dtype=BF)[:, :512]
    ops.gemm_dense(x, w, out=out)
    _close(out, x.float() @ w.float().t(), atol=2e-2, rtol=2e-2, what="strided")


@pytest.mark.parametrize("T", [65, 300, 1000])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("cfg", [0, 8])
@pytest.mark.parametrize("d,F", [(256, 384), (512, 512)])
def test_moe_gemm_dense(gpu, T, swiglu, cfg, d, F):
    """The grouped forms of the dense MFMA GEMMs (cfg 0: gemm_dense's 8-wave ping-pong,
    8: gemm_w4's one wave per SIMD) over moe_align's 128-row expert segments (odd block
    counts, empty experts) against the per-expert fp32 oracle, at two model widths;
    padding rows of an expert with an odd block count must not spill into the next
    expert."""
    from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers

    E, k = 8, 2
    g = torch.Generator(device="cuda").manual_seed(T)
    N = 2 * F if swiglu else d
    K = d if swiglu else F
    w = ((torch.rand(E, N, K, device="cuda", generator=g) * 2 - 1) / math.sqrt(K)).to(BF)
    bufs = MoEBuffers.allocate(T, k, E, max(d, K), F, "cuda")
    logits = torch.randn(T, E, device="cuda", generator=g).to(BF)
    logits[:, 3] = -30.0                                  # expert 3 gets no rows
    n = T * k
    cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
    wts, ids = bufs.weights[:T], bufs.ids[:T]
    ops.moe_topk(logits, k, True, wts, ids)
    ops.moe_align(ids, E, BLOCK_M, bufs.sorted_ids[:cap], bufs.inv_pos[:n],
                  bufs.expert_of_block[:cap // BLOCK_M], bufs.expert_offsets, bufs.num_blocks)
    xs = (torch.rand(cap, K, device="cuda", generator=g) * 2 - 1).to(BF)
    out = torch.full((cap, F if swiglu else N), 7.0, device="cuda", dtype=BF)
    ops.moe_gemm_dense(xs, w, out, bufs.expert_offsets, swiglu, cfg)
    off = bufs.expert_offsets.tolist()
    assert off[4] == off[3]
    for e in range(E):
        a, b = off[e], off[e + 1]
        if b <= a:
            continue
        r = xs[a:b].float() @ w[e].float().t()
        if swiglu:
            gg, u = r[:, :F].to(BF).float(), r[:, F:].to(BF).float()
            r = (gg * torch.sigmoid(gg)).to(BF).float() * u
        _close(out[a:b], r, atol=2e-2, rtol=2e-2, what=f"expert {e} rows {a}:{b}")
    if off[E] < cap:                                       # rows past the live segments
        assert bool((out[off[E]:].float() == 7.0).all())


@pytest.mark.parametrize("T", [65, 300, 1000])
@pytest.mark.parametrize("mode", ["never", "split", "full_rounds"])
def test_moe_w2_combine_split_rule(gpu, T, mode):
    """Throughput-path w2 + top-k combine (ops.moe_w2_combine): the grouped GEMM and the
    combine take the split-K decision on the device from the expert offsets and the CU
    count.  `cus` is chosen per case so each branch runs: 0 = never split; twice the live
    tile count = the last round at most half full -> two fp32 K slices; exactly the tile
    count = whole rounds -> one bf16 store.  Every branch must equal the fp32 oracle of
    act . w2^T combined with the top-k weights (empty expert, odd block counts)."""
    from replisense_rfq_amd.models.moe import BLOCK_M, MoEBuffers

    E, k, d, F = 8, 2, 512, 1024
    g = torch.Generator(device="cuda").manual_seed(T + 11)
    w2 = ((torch.rand(E, d, F, device="cuda", generator=g) * 2 - 1) / math.sqrt(F)).to(BF)
    bufs = MoEBuffers.allocate(T, k, E, d, F, "cuda")
    logits = torch.randn(T, E, device="cuda", generator=g).to(BF)
    logits[:, 5] = -30.0                                  # expert 5 gets no rows
    n = T * k
    cap = (n + E * (BLOCK_M - 1) + BLOCK_M - 1) // BLOCK_M * BLOCK_M
    wts, ids = bufs.weights[:T], bufs.ids[:T]
    ops.moe_topk(logits, k, True, wts, ids)
    ops.moe_align(ids, E, BLOCK_M, bufs.sorted_ids[:cap], bufs.inv_pos[:n],
                  bufs.expert_of_block[:cap // BLOCK_M], bufs.expert_offsets, bufs.num_blocks)
    act = (torch.rand(cap, F, device="cuda", generator=g) * 2 - 1).to(BF)
    off = bufs.expert_offsets.tolist()
    tiles = sum(((off[e + 1] - off[e]) // BLOCK_M + 1) // 2 for e in range(E)) * (d // 256)
    cus = {"never": 0, "split": 2 * tiles, "full_rounds": tiles}[mode]
    y = torch.full((cap, d), 7.0, device="cuda", dtype=BF)
    yf = torch.full((2, cap + 128, d), 7.0, device="cuda", dtype=torch.float32)
    out = torch.empty(T, d, device="cuda", dtype=BF)
    ops.moe_w2_combine(act, w2, y, yf, bufs.expert_offsets, bufs.inv_pos[:n], wts, k, out, cus)
    yr = torch.zeros(cap, d, device="cuda")
    for e in range(E):
        a, b = off[e], off[e + 1]
        if b > a:
            yr[a:b] = act[a:b].float() @ w2[e].float().t()
    pos = bufs.inv_pos[:n].long().view(T, k)
    ref = (yr[pos] * wts.float().unsqueeze(-1)).sum(1)
    _close(out, ref, atol=2e-2, rtol=2e-2, what=f"w2 combine {mode}")
    wrote_slabs = bool((yf[:, :off[E]] != 7.0).any())
    assert wrote_slabs == (mode == "split"), (mode, wrote_slabs)
    assert bool((y[:off[E]] != 7.0).any()) == (mode != "split")


ROWS_CFGS_PLAIN = (0 | 4, 0 | 8, 0 | 12, 1 | 4, 1 | 8, 2 | 0, 2 | 4, 3 | 0)   # (RW, CU) pairs


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("cfg", ROWS_CFGS_PLAIN)
@pytest.mark.parametrize("N,K", [(1280, 8192), (8192, 1024), (1000, 3584)])
def test_gemv_rows(gpu, M, cfg, N, K):
    """Row-streaming GEMV (gemv_rows.hip, M <= 4, one wave per RW rows over the full K,
    v_dot2c_f32_bf16) == fp32 torch; N not a multiple of RW (1000) and K / 512 not a
    multiple of the in-flight chunk count (3584 = 7 x 512) cover the tails."""
    torch.manual_seed(M * 31 + cfg + N)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    y = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows(x, w, y, cfg)
    _close(y, x.float() @ w.float().t(), 2e-2, 1e-2, f"gemv_rows M={M} cfg={cfg} N={N} K={K}")


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("cfg", [4, 8, 12])
def test_gemv_rows_strided_x(gpu, M, cfg):
    """x as a row-strided view of a wider buffer (ldx > K): the X buffer resource spans
    M rows of the stride, rows past M read zeros."""
    torch.manual_seed(M + cfg)
    K, N = 2048, 512
    xb = torch.randn(M, K + 64, device=gpu, dtype=BF)
    x = xb[:, :K]
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    y = torch.empty(M, N, device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows(x, w, y, cfg)
    _close(y, x.float() @ w.float().t(), 2e-2, 1e-2, f"gemv_rows strided M={M}")


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("cfg", [4, 8, 12, 68, 72, 76])
@pytest.mark.parametrize("F,K", [(3584, 8192), (1792, 4096)])
def test_gemv_rows_swiglu(gpu, M, cfg, F, K):
    """gate|up GEMV with the SwiGLU epilogue (waves 2j / 2j+1 pair through LDS) ==
    silu_mul of the fp32 GEMM, rounded like act.hip."""
    torch.manual_seed(M * 7 + cfg + F)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(2 * F, K, device=gpu) / math.sqrt(K)).to(BF)
    out = torch.full((M, F), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows_swiglu(x, w, out, cfg)
    gu = (x.float() @ w.float().t()).to(BF)
    exp = torch.empty(M, F, dtype=BF, device=gpu)
    ref.silu_mul(gu, exp)
    _close(out, exp, 2e-2, 1e-2, f"gemv_rows_swiglu M={M} cfg={cfg}")


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("cfg", [4, 8, 12, 68, 72, 76])
@pytest.mark.parametrize("Hq,Hkv,K", [(8, 1, 8192), (32, 8, 4096)])
def test_gemv_rows_rope_kv(gpu, M, cfg, Hq, Hkv, K):
    """QKV GEMV with the RoPE + paged-KV-append epilogue (waves 2j / 2j+1 = rotate-half
    partners) == fp32 GEMM + rope_kv oracle; padding rows (slot -1) write nothing."""
    torch.manual_seed(M * 13 + cfg + Hq)
    N = (Hq + 2 * Hkv) * 128
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(4 * 32, device=gpu)[:M].to(torch.int32)
    if M > 1:
        slots[-1] = -1
    kc = torch.zeros(4, Hkv, 32, 128, device=gpu, dtype=BF)
    vc = torch.zeros_like(kc)
    qkv = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows_rope(x, w, qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, cfg)
    exp = (x.float() @ w.float().t()).cpu()
    kc_e, vc_e = torch.zeros(kc.shape), torch.zeros(vc.shape)
    ref.rope_kv(exp, pos.cpu(), cos_sin.cpu(), slots.cpu(), kc_e, vc_e, Hq, Hkv)
    q = Hq * 128
    _close(qkv[:, :q], exp[:, :q], 2e-2, 1e-2, f"rows rope q M={M} cfg={cfg}")
    _close(kc, kc_e, 2e-2, 1e-2, f"rows rope k cache M={M} cfg={cfg}")
    _close(vc, vc_e, 2e-2, 1e-2, f"rows rope v cache M={M} cfg={cfg}")


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("cfg", [4, 8, 72])
def test_gemv_rows_folded_norm(gpu, M, cfg):
    """Folded-norm forms of the row-streaming GEMV (models/llama.py _forward_fold):
    SwiGLU / RoPE over the UN-normalised residual x with the RMSNorm weight folded into
    w's columns (cfg bit 4) == the fp32 oracle of rmsnorm(x) g . w^T; the plain form's
    residual add (cfg bit 5) == bf16(bf16(x w^T) + residual)."""
    torch.manual_seed(M * 3 + cfg)
    K, F, eps = 4096, 1792, 1e-5
    x = (3 * torch.randn(M, K, device=gpu)).to(BF)
    g = (1 + 0.1 * torch.randn(K, device=gpu)).to(BF)
    w = (torch.randn(2 * F, K, device=gpu) / math.sqrt(K)).to(BF)
    wf = (w.float() * g.float()[None, :]).to(BF)                 # DecoderLM.fold_norms
    xn = torch.empty_like(x)
    ref.rms_norm(x, g, eps, xn)
    # SwiGLU
    act = torch.full((M, F), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows_swiglu(x, wf, act, cfg | 16, eps)
    gu = (xn.float() @ w.float().t()).to(BF)
    exp = torch.empty(M, F, dtype=BF, device=gpu)
    ref.silu_mul(gu, exp)
    _close(act, exp, 3e-2, 2e-2, f"folded swiglu M={M}")
    # RoPE + KV append
    Hq, Hkv = 8, 2
    N = (Hq + 2 * Hkv) * 128
    wq = (torch.randn(N, K, device=gpu) / math.sqrt(K)).to(BF)
    wqf = (wq.float() * g.float()[None, :]).to(BF)
    cos_sin = ref.rope_cos_sin(4096, 128, 500000.0, device=gpu)
    pos = torch.randint(0, 4000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(64, device=gpu)[:M].to(torch.int32)
    kc = torch.zeros(2, Hkv, 32, 128, device=gpu, dtype=BF)
    vc = torch.zeros_like(kc)
    qkv = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
    torch.ops.rfq_amd.gemv_rows_rope(x, wqf, qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv, cfg | 16,
                                     eps)
    e = (xn.float() @ wq.float().t()).cpu()
    kc_e, vc_e = torch.zeros(kc.shape), torch.zeros(vc.shape)
    ref.rope_kv(e, pos.cpu(), cos_sin.cpu(), slots.cpu(), kc_e, vc_e, Hq, Hkv)
    _close(qkv[:, :Hq * 128], e[:, :Hq * 128], 3e-2, 2e-2, f"folded rope q M={M}")
    _close(kc, kc_e, 3e-2, 2e-2, f"folded rope k M={M}")
    _close(vc, vc_e, 3e-2, 2e-2, f"folded rope v M={M}")
    # residual add
    wo = (torch.randn(K, 1024, device=gpu) / math.sqrt(1024)).to(BF)
    a = torch.randn(M, 1024, device=gpu, dtype=BF)
    res = torch.randn(M, K, device=gpu, dtype=BF)
    r2 = res.clone()
    torch.ops.rfq_amd.gemv_rows(a, wo, r2, ((cfg & 15) | 1) | 32)
    y = (a.float() @ wo.float().t()).to(BF)
    _close(r2, (y.float() + res.float()).to(BF), 2e-2, 1e-2, f"residual add M={M}")


def test_linear_zero_rows_with_rows_plan(gpu):
    """A chunked-prefill step whose chunk ends no prompt selects zero logits rows: the LM
    head's linear must return an empty result even when the start-up plan put the M = 1
    bucket on the row-streaming GEMV (which takes 1 <= M <= 4 only) -- the 70B phase's
    multi-page PDF set failed there before."""
    ops.reset_plans()
    N, K = 1024, 512
    w = (torch.randn(N, K, device="cuda") / 16).to(BF)
    ops.set_linear_plan({(1, N, K): ops.ROWS_BIT | 9}, [1])
    try:
        x = torch.empty(0, K, device="cuda", dtype=BF)
        assert ops.linear(x, w).shape == (0, N)
        x1 = torch.randn(1, K, device="cuda").to(BF)
        _close(ops.linear(x1, w), x1.float() @ w.float().t(), atol=2e-2, rtol=2e-2, what="M=1 rows")
    finally:
        ops.reset_plans()
