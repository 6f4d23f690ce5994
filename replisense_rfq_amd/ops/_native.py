"""Loader for the in-tree gfx950 op library (``replisense_rfq_amd/_C.so``).

On a machine with a GPU the HIP path is mandatory: if the library is missing or
fails to load, :func:`require` raises instead of silently falling back to eager
PyTorch (the round-end audit records which native objects a GPU process loaded).
On a CPU-only host (this build container, CI) the ops dispatch to the torch
reference implementations in :mod:`replisense_rfq_amd.ops.reference`, which are
also the numerics oracles of the kernel tests.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

# RFQ_C_SO: an alternative build of the same library (A/B tools only, never the default)
_LIB = Path(os.environ.get("RFQ_C_SO") or Path(__file__).resolve().parent.parent / "_C.so")
_lock = threading.Lock()
_loaded = False
_error: Exception | None = None


def lib_path() -> Path:
    return _LIB


def _try_load() -> bool:
    global _loaded, _error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not _LIB.exists() and os.environ.get("RFQ_AUTOBUILD", "1") == "1":
            try:
                from .. import _build

                _build.build_kernels()
            except Exception as e:  # pragma: no cover - build errors surface below
                _error = e
        try:
            torch.ops.load_library(str(_LIB))
            _loaded = True
        except Exception as e:
            _error = e
    return _loaded


def available() -> bool:
    return _try_load()


def require() -> None:
    """Load the op library or raise — used by every GPU code path."""
    if not _try_load():
        raise RuntimeError(
            f"replisense_rfq_amd native op library unavailable ({_LIB}): {_error!r}. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950).")


def ops():
    require()
    return torch.ops.rfq_amd
