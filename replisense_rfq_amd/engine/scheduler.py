"""Continuous-batching scheduler (single owner of all sequence / KV state).

Every step packs ONE mixed batch (SURVEY.md §3.2 target, §5.7):

  decode rows   running sequences with exactly one token to feed (q = 1) — these
                are the hipGraph-captured rows when the step has nothing else;
  extend rows   (a) prompt prefill, chunked to the step token budget, starting
                    after the prefix-cache hit, and
                (b) grammar jump-forward: a sampled token plus the forced schema
                    tokens that follow it are fed together (q = 1 + k), so the
                    ~54 % schema-forced characters cost no extra decode steps.

Admission is FCFS under ``max_num_seqs`` and the KV block budget; if a running
sequence cannot grow its block table the most recently admitted sequence is
preempted (blocks released, recomputed later).
"""
from __future__ import annotations

import collections
import time
from dataclasses import dataclass, field

from ..utils.config import EngineConfig
from .kv_cache import KVCache
from .sequence import Sequence, Status


@dataclass
class StepPlan:
    decode: list[Sequence] = field(default_factory=list)
    extend: list[tuple[Sequence, int]] = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return len(self.decode) + sum(q for _, q in self.extend)

    @property
    def empty(self) -> bool:
        return not self.decode and not self.extend


class Scheduler:
    def __init__(self, cfg: EngineConfig, kv: KVCache):
        self.cfg = cfg
        self.kv = kv
        self.waiting: collections.deque[Sequence] = collections.deque()
        self.running: list[Sequence] = []
        self.num_preempted = 0

    def add(self, seq: Sequence) -> None:
        self.waiting.append(seq)

    @property
    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    def _q_for(self, s: Sequence, budget: int) -> int:
        if s.in_prefill or self.cfg.jump_forward:
            return min(s.pending, budget)
        return 1

    def schedule(self) -> StepPlan:
        plan = StepPlan()
        budget = self.cfg.max_batched_tokens
        # 1) running sequences: decode rows first (cheap), then extends
        keep: list[Sequence] = []
        for s in list(self.running):
            if s.status is not Status.RUNNING:      # preempted earlier in this loop
                continue
            if s.pending <= 0:
                keep.append(s)
                continue
            q = self._q_for(s, max(1, budget)) if not (s.pending == 1 and not s.in_prefill) else 1
            if q > 1 and budget <= 1:
                keep.append(s)          # out of token budget this step; decode next step
                continue
            while not self.kv.grow(s, s.num_cached + q):
                victim = self._preempt_victim(exclude=s)
                if victim is None:
                    break
                self._preempt(victim)
                if victim in keep:
                    keep.remove(victim)
            if self.kv.blocks_needed(s, s.num_cached + q):
                self._preempt(s)
                continue
            keep.append(s)
            if q == 1 and not s.in_prefill:
                plan.decode.append(s)
            else:
                plan.extend.append((s, q))
            budget -= q
        self.running = [s for s in keep if s.status is Status.RUNNING]
        # 2) admit waiting sequences into the remaining budget
        now = time.perf_counter()
        while self.waiting and budget > 0 and len(self.running) < self.cfg.max_num_seqs:
            s = self.waiting[0]
            if not s.blocks:
                self.kv.admit(s)
            q = min(s.pending, budget)
            if not self.kv.grow(s, s.num_cached + q):
                break
            self.waiting.popleft()
            s.status = Status.RUNNING
            if not s.t_first_sched:
                s.t_first_sched = now
            self.running.append(s)
            plan.extend.append((s, q))
            budget -= q
        return plan

    def _preempt_victim(self, exclude: Sequence):
        """Newest running sequence not yet placed in this step's plan (those come
        after `exclude` in admission order); None -> preempt `exclude` itself."""
        idx = self.running.index(exclude) if exclude in self.running else -1
        for s in reversed(self.running[idx + 1:]):
            if s.status is Status.RUNNING and s.blocks:
                return s
        return None

    def _preempt(self, s: Sequence) -> None:
        """Recompute-style preemption: drop KV, keep tokens, requeue at the front."""
        self.kv.free(s)
        s.num_cached = 0
        s.num_registered = 0
        s.status = Status.WAITING
        if s in self.running:
            self.running.remove(s)
        self.waiting.appendleft(s)
        self.num_preempted += 1

    def finish(self, s: Sequence, reason: str) -> None:
        s.status = Status.FINISHED
        s.finish_reason = reason
        s.t_finish = time.perf_counter()
        self.kv.free(s)
        if s in self.running:
            self.running.remove(s)
