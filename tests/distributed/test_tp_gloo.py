"""Tensor parallelism on CPU over gloo: sharded forward == TP=1 forward, and the TP
engine (rank-0 scheduler + metadata broadcast + vocab-parallel sampler) produces
valid RFQ JSON.  World sizes 2, 4 and 8; ``tiny-llama70`` has Llama-3-70B's per-rank
attention shape at TP=8 (8 q heads, one kv head, GQA group 8)."""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _forward_worker(rank, world, port, q, sp=False, model=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(max(1, 8 // world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from replisense_rfq_amd.models.config import get_config
    from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta
    from replisense_rfq_amd.models.weights import init_weights, shard_weights
    from replisense_rfq_amd.parallel.tp import SINGLE, TPContext

    cfg = get_config(model) if model else \
        get_config("tiny-llama").__class__(**{**get_config("tiny-llama").to_dict(),
                                              "n_kv_heads": 2, "name": "tiny-tp"})
    full = init_weights(cfg, SINGLE, "cpu", seed=11)
    tp = TPContext(rank=rank, world=world, group=dist.group.WORLD)
    m = DecoderLM(cfg, "cpu", tp=tp, weights=shard_weights(full, cfg, tp))
    m.sp_min_tokens = 1 if sp else 0
    T, nb = (39 if sp else 40), 4  # 39: SP pads the last rank's row shard (any world)
    shape = (cfg.n_layers, nb, m.hkv, 32, 128)
    m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16), torch.zeros(shape, dtype=torch.bfloat16))
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 5000, (T,), generator=g, dtype=torch.int32)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    meta = ForwardMeta(input_ids=ids, positions=torch.arange(T, dtype=torch.int32),
                       slot_mapping=torch.arange(T, dtype=torch.int32), num_decode=0,
                       num_prefill_tokens=T, pf_block_tables=i32([[0, 1]]), pf_q_start=i32([0]),
                       pf_q_len=i32([T]), pf_kv_len=i32([T]), work_seq=i32([0, 0]),
                       work_qblk=i32([0, 1]), logits_idx=torch.tensor([T - 1]))
    part = m.forward(meta).float()
    parts = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(parts, part)
    if rank == 0:
        ref = DecoderLM(cfg, "cpu", weights=full)
        shape1 = (cfg.n_layers, nb, ref.hkv, 32, 128)
        ref.attach_kv_cache(torch.zeros(shape1, dtype=torch.bfloat16),
                            torch.zeros(shape1, dtype=torch.bfloat16))
        exp = ref.forward(meta).float()
        got = torch.cat(parts, -1)
        q.put(float((got - exp).norm() / exp.norm()))
    dist.destroy_process_group()


def _engine_worker(rank, world, port, q, control="shm", model="tiny-llama-tp"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), RFQ_TP_CONTROL=control)
    torch.set_num_threads(max(1, 8 // world))
    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.parallel.tp import init_distributed
    from replisense_rfq_amd.service.prompt import build_messages
    from replisense_rfq_amd.utils import synth
    from replisense_rfq_amd.utils.config import EngineConfig

    tp = init_distributed("gloo")
    eng = LLMEngine(EngineConfig(model=model, device="cpu", max_num_seqs=4,
                                 decode_hints=True), tp=tp)
    assert (eng.runner.ring is not None) == (control == "shm")
    if tp.rank == 0:
        prompts = [eng.tokenizer.chat_ids(build_messages(synth.make_rfq(i).text)) for i in range(2)]
        seqs = eng.generate(prompts)
        eng.shutdown()
        q.put([eng.decode_text(s) for s in seqs])
    else:
        eng.worker_loop()
    dist.destroy_process_group()


def _moe_forward_worker(rank, world, port, q, ep, sp=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from replisense_rfq_amd.models.config import get_config
    from replisense_rfq_amd.models.llama import DecoderLM, ForwardMeta
    from replisense_rfq_amd.models.weights import init_weights, shard_weights
    from replisense_rfq_amd.parallel.tp import SINGLE, TPContext

    base = get_config("tiny-mixtral")
    cfg = base.__class__(**{**base.to_dict(), "n_heads": 8, "n_kv_heads": 2, "name": "tiny-mx-tp"})
    full = init_weights(cfg, SINGLE, "cpu", seed=5)
    tp = TPContext(rank=rank, world=world, group=dist.group.WORLD)
    m = DecoderLM(cfg, "cpu", tp=tp, weights=shard_weights(full, cfg, tp, moe_ep=ep), moe_ep=ep)
    m.sp_min_tokens = 1 if sp else 0
    T, nb = (23 if sp else 24), 2
    shape = (cfg.n_layers, nb, m.hkv, 32, 128)
    m.attach_kv_cache(torch.zeros(shape, dtype=torch.bfloat16),
                      torch.zeros(shape, dtype=torch.bfloat16))
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, 5000, (T,), generator=g, dtype=torch.int32)
    i32 = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    meta = ForwardMeta(input_ids=ids, positions=torch.arange(T, dtype=torch.int32),
                       slot_mapping=torch.arange(T, dtype=torch.int32), num_decode=0,
                       num_prefill_tokens=T, pf_block_tables=i32([[0]]), pf_q_start=i32([0]),
                       pf_q_len=i32([T]), pf_kv_len=i32([T]), work_seq=i32([0]),
                       work_qblk=i32([0]), logits_idx=torch.tensor([T - 1]))
    part = m.forward(meta).float()
    parts = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(parts, part)
    if rank == 0:
        ref = DecoderLM(cfg, "cpu", weights=full)
        shape1 = (cfg.n_layers, nb, ref.hkv, 32, 128)
        ref.attach_kv_cache(torch.zeros(shape1, dtype=torch.bfloat16),
                            torch.zeros(shape1, dtype=torch.bfloat16))
        exp = ref.forward(meta).float()
        got = torch.cat(parts, -1)
        q.put(float((got - exp).norm() / exp.norm()))
    dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ep,sp", [(False, False), (True, False), (True, True)])
def test_tp2_mixtral_forward_matches_tp1(ep, sp):
    """Mixtral MoE under TP=2: FFN-split experts (ep=False) or whole experts per
    rank (expert parallelism, ep=True) both reproduce the single-device logits,
    also with the sequence-parallel residual stream (sp=True)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    mp.start_processes(_moe_forward_worker, args=(2, port, q, ep, sp), nprocs=2,
                       start_method="spawn")
    assert q.get(timeout=10) < 0.02


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sp", [False, True])
def test_tp2_forward_matches_tp1(sp):
    """Llama TP=2 logits == TP=1; sp=True runs the Megatron sequence-parallel
    forward (reduce-scatter / all-gather of token rows, padded odd T)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    mp.start_processes(_forward_worker, args=(2, port, q, sp), nprocs=2,
                       start_method="spawn")
    assert q.get(timeout=10) < 0.02


@pytest.mark.timeout(600)
@pytest.mark.parametrize("control", ["shm", "rccl"])
def test_tp2_engine_valid_json(control):
    """TP=2 engine; step metadata over the shared-memory control plane or the
    collective broadcast."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    mp.start_processes(_engine_worker, args=(2, port, q, control), nprocs=2,
                       start_method="spawn")
    from replisense_rfq_amd.service.schema import RFQResponse

    for text in q.get(timeout=10):
        RFQResponse(**json.loads(text))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,sp", [(4, False), (8, False), (8, True)])
def test_tp_70b_shape_forward_matches_tp1(world, sp):
    """Llama-3-70B's TP=8 per-rank layout (Hq_local=8, Hkv_local=1, G=8) and TP=4
    (Hkv_local=2): sharded logits == single-device logits, also with the
    sequence-parallel residual stream split 8 ways (odd T padded)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    mp.start_processes(_forward_worker, args=(world, port, q, sp, "tiny-llama70"), nprocs=world,
                       start_method="spawn")
    assert q.get(timeout=10) < 0.02


@pytest.mark.timeout(900)
def test_tp8_engine_vocab_parallel_sampler():
    """The 8-rank TP engine on the 70B-shaped model: rank-0 scheduler, shared-memory
    control plane to 7 followers, vocab sharded 8 ways (each rank samples its 16,032-
    token shard; the (value, index) partials are all-gathered) -> valid RFQ JSON."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    mp.start_processes(_engine_worker, args=(8, port, q, "shm", "tiny-llama70"), nprocs=8,
                       start_method="spawn")
    from replisense_rfq_amd.service.schema import RFQResponse

    texts = q.get(timeout=10)
    for text in texts:
        RFQResponse(**json.loads(text))
