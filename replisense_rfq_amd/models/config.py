"""Model configurations (random-init weights of the real architectures).

The reference calls ``llama3-70b-8192`` remotely (rfq_agent.py:62); BASELINE.json
names Llama-3-8B TP=1, Llama-3-70B TP=8 and Mixtral-8x7B as the configurations to
serve on-node.  Dimensions are the public model-card values.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int = 128256
    hidden: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    n_experts: int = 0          # >0 => sparse MoE MLP (Mixtral)
    moe_topk: int = 2
    init_std: float = 0.02
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128009)

    @property
    def is_moe(self) -> bool:
        return self.n_experts > 0

    @property
    def group(self) -> int:
        return self.n_heads // self.n_kv_heads

    def params(self) -> int:
        d, L = self.hidden, self.n_layers
        attn = d * (self.n_heads + 2 * self.n_kv_heads) * self.head_dim + self.n_heads * self.head_dim * d
        mlp = 3 * d * self.ffn * max(1, self.n_experts) + (d * self.n_experts if self.is_moe else 0)
        return L * (attn + mlp + 2 * d) + 2 * self.vocab_size * d + d

    def kv_bytes_per_token(self, tp: int = 1, dtype_bytes: int = 2) -> int:
        return 2 * self.n_layers * max(1, self.n_kv_heads // tp) * self.head_dim * dtype_bytes

    def to_dict(self):
        return asdict(self)


LLAMA3_8B = ModelConfig("llama3-8b")
LLAMA3_70B = ModelConfig("llama3-70b", hidden=8192, n_layers=80, n_heads=64, n_kv_heads=8,
                         ffn=28672)
MIXTRAL_8X7B = ModelConfig("mixtral-8x7b", vocab_size=32000, hidden=4096, n_layers=32,
                           n_heads=32, n_kv_heads=8, ffn=14336, rope_theta=1e6,
                           max_position=32768, n_experts=8, moe_topk=2, bos_id=1, eos_ids=(2,))
# Small same-family configs for tests / smoke runs (head_dim stays 128: the kernels'
# tile shape).  Vocab stays at the tokenizer's size so the real grammar masks apply.
TINY_LLAMA = ModelConfig("tiny-llama", hidden=512, n_layers=2, n_heads=4, n_kv_heads=1,
                         ffn=1024, max_position=8192)
TINY_LLAMA_TP = ModelConfig("tiny-llama-tp", hidden=512, n_layers=2, n_heads=8, n_kv_heads=2,
                            ffn=1024, max_position=8192)
# Llama-3-70B's per-rank attention shape at TP=8 (Hq=64, Hkv=8 -> 8 q heads and ONE kv
# head per rank, GQA group 8) on a 2-layer, 512-wide body: the CPU/gloo rehearsal of
# BASELINE config 4 (tests/distributed/test_tp_gloo.py, test_bench_cli.py).
TINY_LLAMA70 = ModelConfig("tiny-llama70", hidden=512, n_layers=2, n_heads=64, n_kv_heads=8,
                           ffn=1024, max_position=8192)
TINY_MIXTRAL = replace(MIXTRAL_8X7B, name="tiny-mixtral", hidden=512, n_layers=2, n_heads=4,
                       n_kv_heads=1, ffn=512, vocab_size=32000)

CONFIGS = {c.name: c for c in (LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, TINY_LLAMA, TINY_LLAMA_TP,
                                TINY_LLAMA70, TINY_MIXTRAL)}
ALIASES = {"llama3-70b-8192": "llama3-70b", "8b": "llama3-8b", "70b": "llama3-70b",
           "mixtral": "mixtral-8x7b"}


def get_config(name: str) -> ModelConfig:
    name = ALIASES.get(name, name)
    if name not in CONFIGS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(CONFIGS)}")
    return CONFIGS[name]
