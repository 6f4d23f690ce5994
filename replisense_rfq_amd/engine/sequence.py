"""Per-request decoding state owned by the scheduler thread."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field

_ids = itertools.count()


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


@dataclass
class SamplingParams:
    temperature: float = 0.1
    max_tokens: int = 1200
    seed: int = 0
    grammar: bool = True
    min_items: int = 0      # bench-only schema hint: minimum line_items the output must contain
    profile: int = 0        # grammar profile: 0 reference (service default), 1 synthetic
                            # (bench-only caps for random-init weights; grammar/compiler.py)


@dataclass
class Sequence:
    prompt: list[int]
    params: SamplingParams
    req_id: int = field(default_factory=lambda: next(_ids))
    tokens: list[int] = field(default_factory=list)       # prompt + generated (incl. forced)
    num_cached: int = 0                                  # tokens whose KV is in the cache
    blocks: list[int] = field(default_factory=list)
    block_hashes: list[int] = field(default_factory=list)  # prompt full-block hashes
    num_registered: int = 0                              # prompt blocks published to the prefix cache
    prefix_hit_tokens: int = 0
    gstate: tuple | None = None                          # grammar automaton state
    mask_idx: int = -1
    status: Status = Status.WAITING
    finish_reason: str | None = None
    num_sampled: int = 0                                 # tokens chosen by the sampler
    num_forced: int = 0                                  # tokens appended by jump-forward
    # timing (perf_counter seconds)
    t_arrival: float = field(default_factory=time.perf_counter)
    t_first_sched: float = 0.0
    t_prefill_done: float = 0.0
    t_first_token: float = 0.0
    t_finish: float = 0.0
    callback: object = None                              # called once with the Sequence

    def __post_init__(self):
        if not self.tokens:
            self.tokens = list(self.prompt)

    @property
    def prompt_len(self) -> int:
        return len(self.prompt)

    @property
    def num_generated(self) -> int:
        return len(self.tokens) - len(self.prompt)

    @property
    def pending(self) -> int:
        return len(self.tokens) - self.num_cached

    @property
    def in_prefill(self) -> bool:
        return self.num_cached < self.prompt_len

    @property
    def output_ids(self) -> list[int]:
        return self.tokens[len(self.prompt):]

    def span(self) -> dict:
        """Per-request trace span."""
        t0 = self.t_arrival
        return {
            "req": self.req_id, "prompt_tokens": self.prompt_len,
            "prefix_hit_tokens": self.prefix_hit_tokens,
            "completion_tokens": self.num_generated, "sampled": self.num_sampled,
            "jump_forward": self.num_forced,
            "queue_ms": round(1e3 * (self.t_first_sched - t0), 3) if self.t_first_sched else None,
            "prefill_ms": round(1e3 * (self.t_prefill_done - self.t_first_sched), 3)
            if self.t_prefill_done else None,
            "ttft_ms": round(1e3 * (self.t_first_token - t0), 3) if self.t_first_token else None,
            "e2e_ms": round(1e3 * (self.t_finish - t0), 3) if self.t_finish else None,
            "finish": self.finish_reason,
        }
