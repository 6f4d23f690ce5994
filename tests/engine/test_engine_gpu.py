"""GPU engine: model numerics vs the CPU torch-oracle path, eager vs hipGraph decode,
grammar-valid output end to end."""
import json

import pytest
import torch

from replisense_rfq_amd.engine.engine import LLMEngine
from replisense_rfq_amd.models.config import get_config
from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta
from replisense_rfq_amd.service.prompt import build_messages
from replisense_rfq_amd.service.schema import RFQResponse
from replisense_rfq_amd.utils import synth
from replisense_rfq_amd.utils.config import EngineConfig

pytestmark = pytest.mark.gpu


def _meta(T, device, nblocks):
    g = torch.Generator().manual_seed(1234)
    ids = torch.randint(0, 1000, (T,), dtype=torch.int32, generator=g)
    pos = torch.arange(T, dtype=torch.int32)
    bt = torch.arange((T + 31) // 32, dtype=torch.int32)[None]
    m = dict(input_ids=ids, positions=pos, slot_mapping=pos.clone(), num_decode=0,
             num_prefill_tokens=T, pf_block_tables=bt,
             pf_q_start=torch.tensor([0], dtype=torch.int32),
             pf_q_len=torch.tensor([T], dtype=torch.int32),
             pf_kv_len=torch.tensor([T], dtype=torch.int32),
             work_seq=torch.zeros((T + 31) // 32, dtype=torch.int32),
             work_qblk=torch.arange((T + 31) // 32, dtype=torch.int32),
             logits_idx=torch.tensor([T - 1], dtype=torch.int64))
    return ForwardMeta(**{k: (v.to(device) if isinstance(v, torch.Tensor) else v)
                          for k, v in m.items()})


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_model_forward_matches_cpu_oracle(gpu, name):
    from replisense_rfq_amd import ops

    ops.reset_plans()            # bare models: no plan of an earlier engine applies
    torch.manual_seed(0)
    cfg = get_config(name)
    m_gpu = DecoderLM(cfg, gpu, seed=3)
    w_cpu = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in m_gpu.w.items()}
    w_cpu["layers"] = [type(l)({k: t.cpu() for k, t in l.items()}) for l in m_gpu.w["layers"]]
    m_cpu = DecoderLM(cfg, "cpu", weights=w_cpu)
    nb = 8
    shape = (cfg.n_layers, nb, m_gpu.hkv, 32, 128)
    for m in (m_gpu, m_cpu):
        dev = m.device
        m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16, device=dev),
                          torch.zeros(shape, dtype=torch.bfloat16, device=dev))
    T = 150
    lg = m_gpu.forward(_meta(T, gpu, nb)).float().cpu()
    lc = m_cpu.forward(_meta(T, "cpu", nb)).float()
    torch.manual_seed(0)
    rel = (lg - lc).norm() / lc.norm()
    assert rel < 0.05, rel


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_sequence_parallel_layout_matches_forward(gpu, name):
    """The SP forward (row-sharded residual stream; RS/AG degenerate to copies at
    W=1) drives the same HIP kernels through its out= views and buffers and must
    give the same logits as the plain forward on the GPU.  The W=2 collectives are
    covered by tests/distributed/test_tp_gloo.py."""
    cfg = get_config(name)
    m = DecoderLM(cfg, gpu, seed=3)
    shape = (cfg.n_layers, 8, m.hkv, 32, 128)
    m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16, device=gpu),
                      torch.zeros(shape, dtype=torch.bfloat16, device=gpu))
    T = 150
    a = m.forward(_meta(T, gpu, 8)).float()
    b = m._forward_sp(_meta(T, gpu, 8)).float()
    rel = (a - b).norm() / a.norm()
    assert rel < 1e-2, rel


def _engine(graphs: bool, model="tiny-llama"):
    cfg = EngineConfig(model=model, max_num_seqs=16, use_graphs=graphs, max_kv_blocks=4096,
                       graph_buckets=(1, 2, 4, 8, 16), decode_hints=True)
    return LLMEngine(cfg)


def test_engine_generates_valid_rfq_json(gpu):
    eng = _engine(True)
    tok = eng.tokenizer
    prompts = [tok.chat_ids(build_messages(synth.make_rfq(i).text)) for i in range(6)]
    seqs = eng.generate(prompts)
    for s in seqs:
        assert s.finish_reason == "stop"
        RFQResponse(**json.loads(eng.decode_text(s)))
    st = eng.stats()
    assert st["graph_steps"] > 0, st
    # second wave hits the shared system+template prefix
    seqs2 = eng.generate(prompts[:2])
    assert all(s.prefix_hit_tokens >= 400 for s in seqs2), [s.prefix_hit_tokens for s in seqs2]


def test_graph_replay_matches_eager_forward(gpu):
    """A captured decode forward replays to bit-identical logits (same kernels, same
    shapes) and picks up new metadata written into its static input buffers."""
    cfg = get_config("tiny-llama")
    m = DecoderLM(cfg, gpu, seed=5)
    nb, B = 64, 8
    shape = (cfg.n_layers, nb, m.hkv, 32, 128)
    g0 = torch.Generator(device="cpu").manual_seed(0)
    m.attach_kv_cache(torch.randn(shape, generator=g0).to(gpu, torch.bfloat16),
                      torch.randn(shape, generator=g0).to(gpu, torch.bfloat16))
    i32 = dict(dtype=torch.int32, device=gpu)
    st = dict(ids=torch.zeros(B, **i32), pos=torch.zeros(B, **i32),
              slots=torch.zeros(B, **i32), bt=torch.zeros(B, 8, **i32), ctx=torch.ones(B, **i32))
    ar = torch.arange(B, **i32)
    one = torch.ones(B, **i32)
    zero = torch.zeros(B, **i32)

    def meta():
        return ForwardMeta(input_ids=st["ids"], positions=st["pos"], slot_mapping=st["slots"],
                           num_decode=B, dec_block_tables=st["bt"], dec_q_start=ar,
                           dec_q_len=one, dec_kv_len=st["ctx"], dec_work_seq=ar,
                           dec_work_ct=zero, decode_splits=4)

    def fill(seed):
        g = torch.Generator().manual_seed(seed)
        st["ids"].copy_(torch.randint(0, 5000, (B,), generator=g))
        ctx = torch.randint(1, 200, (B,), generator=g)
        st["ctx"].copy_(ctx)
        st["pos"].copy_(ctx - 1)
        bt = torch.arange(B * 8).view(B, 8) % (nb - 1)
        st["bt"].copy_(bt)
        st["slots"].copy_(bt[torch.arange(B), (ctx - 1) // 32] * 32 + (ctx - 1) % 32)

    fill(1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.forward(meta())
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = m.forward(meta())
    for seed in (2, 3):
        fill(seed)
        graph.replay()
        got = out.clone()
        fill(seed)
        exp = m.forward(meta())
        assert torch.equal(got, exp)


def test_engine_graphs_on_and_off_both_valid(gpu):
    for graphs in (False, True):
        eng = _engine(graphs)
        tok = eng.tokenizer
        prompts = [tok.chat_ids(build_messages(synth.make_rfq(10 + i).text)) for i in range(4)]
        for s in eng.generate(prompts):
            RFQResponse(**json.loads(eng.decode_text(s)))
        assert (eng.stats()["graph_steps"] > 0) == graphs
        del eng
        torch.cuda.empty_cache()


def test_mixtral_engine(gpu):
    eng = _engine(True, model="tiny-mixtral")
    tok = eng.tokenizer
    prompts = [tok.chat_ids(build_messages(synth.make_rfq(i).text)) for i in range(3)]
    for s in eng.generate(prompts):
        RFQResponse(**json.loads(eng.decode_text(s)))


def test_inplace_tiled_forward_matches_cpu_oracle(gpu):
    """In-place decode-tiled projections (the layout 70B at TP 1-2 keeps, no row-major
    copy): every GEMM on them runs a tiled-layout kernel -- split-K GEMVs (M <= 16, in
    16-row chunks up to 64) and the dense MFMA GEMM (larger M) -- vs the CPU oracle on
    the row-major weights, at prefill, chunked and decode-sized batches."""
    from replisense_rfq_amd import ops

    cfg = get_config("tiny-llama")
    m_gpu = DecoderLM(cfg, gpu, seed=5)
    w_cpu = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in m_gpu.w.items()}
    w_cpu["layers"] = [type(l)({k: t.cpu() for k, t in l.items()}) for l in m_gpu.w["layers"]]
    m_gpu.tile_decode_weights("inplace")
    assert m_gpu.tiled_inplace
    assert all(ops.tiled_only(m_gpu.w["layers"][0][k]) for k in DecoderLM.TILED_PROJ)
    m_cpu = DecoderLM(cfg, "cpu", weights=w_cpu)
    nb = 8
    shape = (cfg.n_layers, nb, m_gpu.hkv, 32, 128)
    for T in (150, 40, 5):
        for m in (m_gpu, m_cpu):
            dev = m.device
            m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16, device=dev),
                              torch.zeros(shape, dtype=torch.bfloat16, device=dev))
        lg = m_gpu.forward(_meta(T, gpu, nb)).float().cpu()
        lc = m_cpu.forward(_meta(T, "cpu", nb)).float()
        rel = (lg - lc).norm() / lc.norm()
        assert rel < 0.05, (T, rel)


def test_engine_inplace_tiled_valid(gpu, monkeypatch):
    """The engine with in-place tiled weights: start-up plans restricted to tiled
    kernels, graph-captured decode, valid RFQ JSON."""
    monkeypatch.setenv("RFQ_TILED_WEIGHTS", "inplace")
    eng = _engine(True)
    assert eng.model.tiled_inplace
    tok = eng.tokenizer
    prompts = [tok.chat_ids(build_messages(synth.make_rfq(30 + i).text)) for i in range(4)]
    for s in eng.generate(prompts):
        RFQResponse(**json.loads(eng.decode_text(s)))
    assert eng.stats()["graph_steps"] > 0
    del eng
    torch.cuda.empty_cache()


def test_mixed_tiled_plan_forward_matches_cpu_oracle(gpu, monkeypatch):
    """auto with a copy budget that holds only the smallest projections: qkv and o get
    tiled copies, down and gate|up are tiled in place; the mixed model still matches
    the CPU oracle at prefill- and decode-sized batches."""
    from replisense_rfq_amd import ops

    cfg = get_config("tiny-llama")
    m_gpu = DecoderLM(cfg, gpu, seed=9)
    w_cpu = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in m_gpu.w.items()}
    w_cpu["layers"] = [type(l)({k: t.cpu() for k, t in l.items()}) for l in m_gpu.w["layers"]]
    # budget = min(0.25 total, 0.40 free) = 2.7 MB: o (1.05 MB) + qkv (1.57 MB) fit
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda *a, **k: (6_750_000, 10_800_000))
    m_gpu.tile_decode_weights("auto")
    assert m_gpu.tiled_plan == {"qkv": "copy", "o": "copy", "gate_up": "inplace",
                                "down": "inplace"}, m_gpu.tiled_plan
    lw = m_gpu.w["layers"][0]
    assert ops.tiled_of(lw["qkv"]) is not None and not ops.tiled_only(lw["qkv"])
    assert ops.tiled_only(lw["down"]) and ops.tiled_only(lw["gate_up"])
    m_cpu = DecoderLM(cfg, "cpu", weights=w_cpu)
    nb = 8
    shape = (cfg.n_layers, nb, m_gpu.hkv, 32, 128)
    for T in (150, 40, 5):
        for m in (m_gpu, m_cpu):
            dev = m.device
            m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16, device=dev),
                              torch.zeros(shape, dtype=torch.bfloat16, device=dev))
        lg = m_gpu.forward(_meta(T, gpu, nb)).float().cpu()
        lc = m_cpu.forward(_meta(T, "cpu", nb)).float()
        rel = (lg - lc).norm() / lc.norm()
        assert rel < 0.05, (T, rel)


def test_chunked_prefill_steps_without_logits(gpu, monkeypatch):
    """Long prompts split into prefill chunks whose steps select no logits rows (the
    70B phase's multi-page PDF set, 1,024-token chunks): the LM head gets zero rows and
    the runner must still wait for such a step before the next one is packed into the same
    pinned staging buffer (an empty readback does not synchronise; without the wait the
    previous step's upload could read the next payload).  Every step is checked to have
    finished before the next upload, and the documents must decode to valid JSON twice
    over with identical tokens."""
    from replisense_rfq_amd.engine import runner as runner_mod

    waits = []
    orig = runner_mod.ModelRunner._run

    def _run(self, header, payload):
        out = orig(self, header, payload)
        waits.append(torch.cuda.current_stream().query())   # the step has drained
        return out

    monkeypatch.setattr(runner_mod.ModelRunner, "_run", _run)
    texts = []
    for _ in range(2):
        eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_kv_blocks=2048,
                                     max_batched_tokens=96, graph_buckets=(1, 2, 4),
                                     decode_hints=True))
        tok = eng.tokenizer
        prompts = [tok.chat_ids(build_messages(synth.make_long_rfq(i).text)) for i in range(2)]
        assert all(len(p) > 3 * 96 for p in prompts)
        seqs = eng.generate(prompts)
        for s in seqs:
            assert s.finish_reason == "stop"
            RFQResponse(**json.loads(eng.decode_text(s)))
        texts.append([eng.decode_text(s) for s in seqs])
        del eng
    assert texts[0] == texts[1]
    assert waits and all(waits)
