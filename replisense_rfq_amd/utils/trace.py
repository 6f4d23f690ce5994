"""Tracing hooks.

Three layers, all off by default:
  * roctx ranges around the engine's schedule / execute / post phases and the
    model's per-layer ops (``RFQ_TRACE=1``) — ``torch.cuda.nvtx`` is backed by
    roctx on ROCm builds, so the ranges show up in ``rocprofv3 --marker-trace``
    timelines next to the HIP kernels;
  * per-request spans (queue / prefill / decode / total) on every Sequence,
    summarised by ``/metrics``;
  * per-kernel timing from ``tools/profile.sh`` (rocprofv3 --kernel-trace --stats).
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get("RFQ_TRACE", "").lower() in ("1", "true", "on", "yes")


def enable(flag: bool = True) -> None:
    global _ENABLED
    _ENABLED = flag


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    import torch

    if not torch.cuda.is_available():
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
