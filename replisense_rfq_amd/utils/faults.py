"""Fault injection for the failure-detection paths.

The reference has no failure handling beyond retry + fallback JSON
(rfq_agent.py:26-39,186-200).  The on-node engine adds failure modes of its own
(a step that raises, a step that stalls, a dead DP replica); these hooks let the
tests drive each one deterministically.

``RFQ_FAULT`` is a comma-separated list of ``kind:arg`` entries:

  step_raise:N      raise RuntimeError on engine step N (0-based)
  step_sleep:N:MS   sleep MS milliseconds inside step N (watchdog tests)
  replica_exit:N    a DP replica process exits after serving N requests
  car_error:N       engine step N fails as if the custom all-reduce had counted a
                    flag timeout (only on an engine configured with the custom
                    all-reduce; the replica then restarts on RCCL)
"""
from __future__ import annotations

import os
import time


class InjectedFault(RuntimeError):
    pass


class CustomAllReduceError(RuntimeError):
    """A custom all-reduce flag timed out during a step: its sums may be stale.
    Fatal for the whole TP replica (engine/router.py restarts it on RCCL)."""


class FaultInjector:
    def __init__(self, spec: str | None = None):
        spec = os.environ.get("RFQ_FAULT", "") if spec is None else spec
        self.rules: list[tuple[str, list[int]]] = []
        for part in filter(None, (p.strip() for p in spec.split(","))):
            kind, *args = part.split(":")
            self.rules.append((kind, [int(a) for a in args]))

    @property
    def active(self) -> bool:
        return bool(self.rules)

    def on_step(self, step: int, custom_allreduce: bool = False) -> None:
        for i, (kind, args) in enumerate(self.rules):
            if kind == "step_raise" and args and args[0] == step:
                del self.rules[i]                    # each fault fires once
                raise InjectedFault(f"injected fault at step {step}")
            if kind == "car_error" and args and args[0] == step and custom_allreduce:
                del self.rules[i]
                raise CustomAllReduceError(f"custom all-reduce: injected flag timeout at "
                                           f"step {step}")
            if kind == "step_sleep" and len(args) == 2 and args[0] == step:
                time.sleep(args[1] / 1000.0)

    def replica_exit_after(self) -> int | None:
        for kind, args in self.rules:
            if kind == "replica_exit" and args:
                return args[0]
        return None


NONE = FaultInjector("")
