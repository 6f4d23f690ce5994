"""Custom xGMI all-reduce (csrc/comm/custom_ar.hip) for TP messages up to the
staging capacity: one-shot for decode-size messages, two-shot (reduce-scatter +
all-gather, ~2n bytes per rank over all links) above 512 KiB on more than 2 ranks.

Setup: every rank of the TP group allocates one uncached region (signal flags +
staging buffer), exports it with hipIpcGetMemHandle, all-gathers the handles
over the group's process group and opens its peers' regions (dmabuf IPC:
``HSA_ENABLE_IPC_MODE_LEGACY=0``).  A call stages the local tensor, exchanges
per-block flags with system-scope release/acquire and sums every rank's copy in
one kernel — capturable in a hipGraph because the flag counters live in device
memory.  Messages above the staging capacity go to RCCL.

The kernel's spins are bounded; :meth:`CustomAllReduce.errors` reads the
timeout counter so a broken peer path is detected instead of hanging the GPU.
The model runner reads it after every step (one 4-byte copy behind the step's
existing sync) and fails the step on a non-zero count (engine/runner.py); the
router then restarts the TP replica on RCCL (engine/router.py).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops import _native

# RFQ_CAR_NORM=0: keep the all-reduce and the residual-add RMSNorm as two launches
FUSE_NORM = os.environ.get("RFQ_CAR_NORM", "1") != "0"
# fused all-reduce + norm form: 0 = push (one xGMI hop, double-buffered slots) for
# decode rows, staged above; 1 = always the staged one-shot (flag, remote read, end flag)
CAR_NORM_ALGO = 1 if os.environ.get("RFQ_CAR_PUSH", "1") == "0" else 0


class CustomAllReduce:
    def __init__(self, rank: int, world: int, group=None, capacity_bytes: int = 8 << 20):
        if world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI hop)")
        ops = _native.ops()
        self.rank, self.world, self.group = rank, world, group
        self.capacity = capacity_bytes
        self.bases, self._opened = [], []
        self.calls = 0
        # ``ok`` is False when this rank could not allocate, export or open a region.
        # The group's collectives below still run on every rank (no rank leaves the
        # set-up early and strands its peers); TPContext.enable_custom_allreduce then
        # agrees on RCCL for the whole group.
        self.ok = True
        self.ptr = 0
        handle = b""
        try:
            self.ptr = ops.car_alloc(capacity_bytes)
            handle = ops.car_ipc_handle(self.ptr).numpy().tobytes()
        except RuntimeError:
            self.ok = False
        handles = [None] * world
        dist.all_gather_object(handles, handle, group=group)
        if self.ok and all(handles):
            try:
                for r in range(world):
                    if r == rank:
                        self.bases.append(self.ptr)
                    else:
                        p = ops.car_ipc_open(torch.frombuffer(bytearray(handles[r]),
                                                              dtype=torch.uint8))
                        self.bases.append(p)
                        self._opened.append(p)
            except RuntimeError:
                self.ok = False
        else:
            self.ok = False
        dist.barrier(group=group)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()
                and t.numel() % 8 == 0 and t.numel() * 2 <= self.capacity)

    def all_reduce_(self, t: torch.Tensor, algo: int = 0) -> torch.Tensor:
        """In-place sum over the group; algo 0 = size-based choice, 1 = one-shot,
        2 = two-shot."""
        torch.ops.rfq_amd.car_allreduce(t, t, self.bases, self.rank, self.capacity, algo)
        self.calls += 1
        return t

    # rows handled by the fused all-reduce + residual-add RMSNorm kernel (one
    # workgroup per row; the signal area has 64 per-block flag slots)
    NORM_MAX_ROWS = 64

    def eligible_norm(self, t: torch.Tensor, residual: torch.Tensor, out: torch.Tensor) -> bool:
        return (FUSE_NORM and self.eligible(t) and t.dim() == 2
                and 1 <= t.shape[0] <= self.NORM_MAX_ROWS and t.shape[1] <= 16384
                and residual.shape == t.shape and out.shape == t.shape
                and residual.stride(1) == 1 and out.stride(1) == 1
                and residual.stride(0) % 8 == 0 and out.stride(0) % 8 == 0
                and all(x.data_ptr() % 16 == 0 for x in (t, residual, out)))

    def all_reduce_add_norm_(self, t: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                             eps: float, out: torch.Tensor, algo: int | None = None
                             ) -> torch.Tensor:
        """residual <- bf16(sum over the group of t + residual); out <- rmsnorm(residual)
        * w, in one launch (bit-identical to all_reduce_ + fused_add_rms_norm; t itself
        is left holding this rank's partial).  Decode rows (<= 16) use the push form:
        every rank writes its row into the peers' double-buffered slots and raises one
        flag, so a call is one xGMI hop with no end barrier (custom_ar.hip)."""
        torch.ops.rfq_amd.car_allreduce_add_norm(t, residual, w, eps, out, self.bases,
                                                 self.rank, self.capacity,
                                                 CAR_NORM_ALGO if algo is None else algo)
        self.calls += 1
        return out

    def errors(self) -> int:
        return int(_native.ops().car_error(self.ptr))

    def error_info(self) -> str:
        """The first flag timeout this region recorded: which protocol phase, block and
        peer never answered within the kernel's 2 s bound ("" if none)."""
        v = int(_native.ops().car_error_info(self.ptr))
        if not v & 0x80000000:
            return ""
        phase = {1: "start", 2: "mid", 3: "end", 4: "push"}.get((v >> 24) & 0x7F, "?")
        return f"{phase} flag of peer {v & 0xFF} at block {(v >> 8) & 0xFFFF} timed out"

    def close(self) -> None:
        ops = _native.ops()
        for p in self._opened:
            ops.car_ipc_close(p)
        self._opened = []
        if self.ptr:
            ops.car_free(self.ptr)
            self.ptr = 0
