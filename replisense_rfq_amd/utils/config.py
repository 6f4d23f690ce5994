"""Typed engine/service configuration from environment + CLI.

Reference env vars are kept with their defaults (MAX_FILE_SIZE_MB=10,
ALLOWED_ORIGINS=*, PORT=8000, ENVIRONMENT=development, LOG_LEVEL=info —
app/main.py:37,85,414-416); GROQ_API_KEY is no longer required because inference
is on-node.  Engine knobs are RFQ_* variables.
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field, fields


def _env(name, default, cast=str):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "on", "yes")
    return cast(v)


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    weights_path: str = ""               # HF-layout safetensors dir/file; "" = seeded random init
    tokenizer_path: str = ""             # tokenizer.json; default: <weights_path>/tokenizer.json
    tp: int = 1
    dp: int = 1
    device: str = "auto"                 # auto -> cuda if available else cpu
    seed: int = 0
    kv_fraction: float = 0.85            # of free HBM for the paged KV pool (bench.py default)
    max_kv_blocks: int = 0               # 0 = from kv_fraction
    block_size: int = 32                 # tokens per KV page (kernel tile)
    # sequences in flight per replica.  The service default bounds latency: 160 in flight
    # serves 58-60 docs/s at loaded p50 2.6 s / p99 3.8 s on one MI355X (the bench's
    # latency_bounded_depth phase), where the throughput headline's 1,536 (bench.py
    # --max-num-seqs, RFQ_MAX_BATCH=1536) gives ~109 docs/s but makes a saturated server
    # hold every request ~14 s (profiles/r3_depth_sweep.md)
    max_num_seqs: int = 160
    max_batched_tokens: int = 16384      # prefill chunk budget per step
    max_model_len: int = 8192            # llama3-70b-8192 context
    graph_buckets: tuple = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384,
                            448, 512, 640, 768, 896, 1024)
    use_graphs: bool = True
    grammar: bool = True
    jump_forward: bool = True
    prefix_cache: bool = True
    temperature: float = 0.1             # rfq_agent.py:66
    max_tokens: int = 1200               # rfq_agent.py:67
    request_timeout_s: float = 30.0      # rfq_agent.py:69
    step_timeout_s: float = 120.0        # watchdog
    moe_parallel: str = "tp"             # tp: FFN-split experts | ep: whole experts per rank
    decode_tiles: int = 2                # column tiles per decode attention work item
    tune_gemm: bool = True               # per-shape skinny-vs-hipBLASLt plan at start-up
    gemm_split: bool = True              # + hipBLASLt row-chunk plan for large steps
    custom_allreduce: bool = True        # TP>1 on GPU: xGMI one-/two-shot kernels (self-tested)
    trace: bool = False                  # per-request JSON spans
    warm_prefix: bool = True             # prefill + pin the shared prompt template at start-up
    check_finite: bool = False           # debug: count Inf/NaN logits every step, fail the step
    decode_hints: bool = False           # bench-only: SYNTHETIC grammar profile + min_items for
                                         # random-init weights (service/hints.py); off = reference

    @classmethod
    def from_env(cls, **overrides) -> "EngineConfig":
        c = cls(
            model=_env("RFQ_MODEL", cls.model),
            weights_path=_env("RFQ_WEIGHTS", cls.weights_path),
            tokenizer_path=_env("RFQ_TOKENIZER", cls.tokenizer_path),
            tp=_env("RFQ_TP", cls.tp, int),
            dp=_env("RFQ_DP", cls.dp, int),
            device=_env("RFQ_DEVICE", cls.device),
            seed=_env("RFQ_SEED", cls.seed, int),
            kv_fraction=_env("RFQ_KV_FRACTION", cls.kv_fraction, float),
            max_num_seqs=_env("RFQ_MAX_BATCH", cls.max_num_seqs, int),
            max_batched_tokens=_env("RFQ_PREFILL_CHUNK", cls.max_batched_tokens, int),
            use_graphs=_env("RFQ_GRAPHS", cls.use_graphs, bool),
            grammar=_env("RFQ_GRAMMAR", cls.grammar, bool),
            jump_forward=_env("RFQ_JUMP_FORWARD", cls.jump_forward, bool),
            prefix_cache=_env("RFQ_PREFIX_CACHE", cls.prefix_cache, bool),
            custom_allreduce=_env("RFQ_CUSTOM_AR", cls.custom_allreduce, bool),
            tune_gemm=_env("RFQ_TUNE_GEMM", cls.tune_gemm, bool),
            gemm_split=_env("RFQ_GEMM_SPLIT", cls.gemm_split, bool),
            decode_tiles=_env("RFQ_DECODE_TILES", cls.decode_tiles, int),
            moe_parallel=_env("RFQ_MOE_PARALLEL", cls.moe_parallel),
            trace=_env("RFQ_TRACE", cls.trace, bool),
            warm_prefix=_env("RFQ_WARM_PREFIX", cls.warm_prefix, bool),
            check_finite=_env("RFQ_CHECK_FINITE", cls.check_finite, bool),
            decode_hints=_env("RFQ_DECODE_HINTS", cls.decode_hints, bool),
            request_timeout_s=_env("RFQ_REQUEST_TIMEOUT_S", cls.request_timeout_s, float),
        )
        gb = os.environ.get("RFQ_GRAPH_BUCKETS")
        if gb:
            c.graph_buckets = tuple(int(x) for x in gb.split(","))
        for k, v in overrides.items():
            if v is not None:
                setattr(c, k, v)
        return c

    def to_dict(self):
        return asdict(self)


@dataclass
class ServiceConfig:
    max_file_size_mb: int = field(default_factory=lambda: _env("MAX_FILE_SIZE_MB", 10, int))
    allowed_origins: str = field(default_factory=lambda: _env("ALLOWED_ORIGINS", "*"))
    port: int = field(default_factory=lambda: _env("PORT", 8000, int))
    environment: str = field(default_factory=lambda: _env("ENVIRONMENT", "development"))
    log_level: str = field(default_factory=lambda: _env("LOG_LEVEL", "info"))
    backend: str = field(default_factory=lambda: _env("RFQ_BACKEND", "engine"))  # engine|mock


def field_names(cls) -> list[str]:
    return [f.name for f in fields(cls)]
