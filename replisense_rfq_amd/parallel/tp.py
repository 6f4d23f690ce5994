"""Tensor parallelism over RCCL/xGMI (Megatron column/row split).

SURVEY.md §2.3 / §2.5: per decoder layer the QKV and gate|up projections are
column-parallel (each rank owns Hq/TP query heads, Hkv/TP kv heads and FFN/TP
columns), the O and down projections are row-parallel and followed by ONE
all-reduce each (C1, C2); the LM head is vocab-parallel and the sampler reduces
(value, index) partials with an all-gather (C3).  Embeddings are replicated (no
collective).  One process per GPU; ``torch.distributed`` backend ``"nccl"`` is
RCCL on ROCm and its collectives are capturable inside hipGraphs.

On a CPU host the same code runs over ``gloo`` (tests use world_size 2-4).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class TPContext:
    rank: int = 0
    world: int = 1
    group: object = None
    car: object = None            # CustomAllReduce (RFQ_CUSTOM_AR, on by default)
    car_status: str = ""          # why the custom all-reduce is (not) in use
    emulated = False              # EmulatedTP: every collective is a local no-op

    @property
    def enabled(self) -> bool:
        return self.world > 1

    def shard(self, n: int) -> tuple[int, int]:
        """[start, end) of this rank's slice of a dimension of size n (n % world == 0)."""
        if n % self.world:
            raise ValueError(f"dimension {n} not divisible by TP={self.world}")
        s = n // self.world
        return self.rank * s, (self.rank + 1) * s

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            if self.car is not None and self.car.eligible(t):
                return self.car.all_reduce_(t)
            dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_add_norm_(self, t: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                             eps: float, out: torch.Tensor) -> torch.Tensor:
        """Row-parallel projection epilogue of a decoder layer: all-reduce ``t``, then
        residual += t and out = rmsnorm(residual) * w.  Decode-size messages on the
        custom xGMI path run both in ONE kernel (custom_ar.hip
        car_oneshot_add_norm_kernel); everything else is all_reduce_ + the fused norm."""
        if self.world > 1 and self.car is not None and self.car.eligible_norm(t, residual, out):
            return self.car.all_reduce_add_norm_(t, residual, w, eps, out)
        from .. import ops

        self.all_reduce_(t)
        return ops.fused_add_rms_norm(t, residual, w, eps, out=out)

    def enable_custom_allreduce(self, capacity_bytes: int = 8 << 20) -> bool:
        """Switch all-reduces up to ``capacity_bytes`` to the xGMI one-/two-shot kernels
        (GPU groups only).  A start-up self-test runs both algorithms against the known
        sum; unless every rank passes with no flag timeouts the group stays on RCCL."""
        if self.world <= 1 or not torch.cuda.is_available() or self.car is not None:
            return self.car is not None
        from .custom_ar import CustomAllReduce

        car = CustomAllReduce(self.rank, self.world, self.group, capacity_bytes)
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"

        def everyone(ok: bool) -> bool:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
            return int(flag.item()) == 1

        # a rank that could not set up its region votes RCCL before any kernel runs
        if not everyone(car.ok):
            car.close()
            self.car_status = "set-up failed" + ("" if car.ok else " on this rank")
            return False
        why = []
        try:
            want = float(sum(range(1, self.world + 1)))
            for algo, n in ((1, 4096), (2, 1 << 19)):
                x = torch.full((n,), float(self.rank + 1), dtype=torch.bfloat16, device="cuda")
                car.all_reduce_(x, algo)
                if not bool((x.float() == want).all().item()):
                    why.append(f"algo {algo} sum")
            t = torch.full((2, 4096), float(self.rank + 1), dtype=torch.bfloat16, device="cuda")
            r, o = torch.zeros_like(t), torch.empty_like(t)
            if car.eligible_norm(t, r, o):       # the fused decode epilogue, same vote
                # three calls: the push form alternates its slot / flag parity per call
                ones = torch.ones(4096, dtype=torch.bfloat16, device="cuda")
                for k in range(3):
                    t.fill_(float(self.rank + 1 + k))
                    r.zero_()
                    car.all_reduce_add_norm_(t, r, ones, 1e-5, o)
                    if not bool((r.float() == want + k * self.world).all().item()):
                        why.append(f"add-norm residual (call {k})")
                        break
            if car.errors():
                why.append(f"{car.errors()} flag timeouts ({car.error_info()})")
        except RuntimeError as e:
            why.append(f"{type(e).__name__}: {str(e)[:120]}")
        if not everyone(not why):
            car.close()
            self.car_status = "self-test failed" + (f" on this rank: {'; '.join(why)}"
                                                    if why else " on a peer")
            return False
        self.car_status = "ok"
        self.car = car
        return True

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out: [world, *inp.shape]"""
        if self.world > 1:
            # rank-major rows: each of the world chunks of dim 0 has exactly inp's
            # shape (gloo checks that; RCCL only checks the element count)
            flat = out.flatten(0, 1) if inp.dim() >= 1 else out
            dist.all_gather_into_tensor(flat, inp.contiguous(), group=self.group)
        else:
            out[0].copy_(inp)
        return out

    def reduce_scatter_rows(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """Sequence-parallel hand-off: sum ``inp`` [W*n, d] over ranks, keep rows
        [rank*n, (rank+1)*n) in ``out`` [n, d].  One RCCL reduce-scatter moves half an
        all-reduce's bytes per rank over the xGMI ring."""
        if self.world > 1:
            dist.reduce_scatter_tensor(out, inp, group=self.group)
        else:
            out.copy_(inp)
        return out

    def all_gather_rows(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out [W*n, d] <- concat over ranks of inp [n, d] (rank order)."""
        if self.world > 1:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        else:
            out.copy_(inp)
        return out

    def broadcast_obj(self, obj, src: int = 0):
        if self.world == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)


SINGLE = TPContext()


class EmulatedTP(TPContext):
    """One rank of a TP group, alone on one GPU, with every collective a local no-op.

    Builds the rank's exact shard (column / row / vocab-parallel weight shapes, local
    heads, KV heads and FFN columns) so one GPU can time what one rank of the real
    group computes per step -- the evidence for BASELINE config 4 (Llama-3-70B TP=8)
    on a single MI355X (tools/tp8_rank_emulation.py).  The all-reduce epilogue keeps
    its local work (residual add + RMSNorm); the all-reduce itself, whose xGMI cost
    is priced separately, is skipped, and the sampler's partial all-gather copies this
    rank's partials into every slot."""

    emulated = True

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def all_reduce_add_norm_(self, t, residual, w, eps, out):
        from .. import ops

        return ops.fused_add_rms_norm(t, residual, w, eps, out=out)

    def enable_custom_allreduce(self, capacity_bytes: int = 8 << 20) -> bool:
        self.car_status = "emulated (collectives skipped)"
        return False

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        out.copy_(inp.unsqueeze(0).expand_as(out))
        return out

    def reduce_scatter_rows(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        n = out.shape[0]
        out.copy_(inp[self.rank * n:(self.rank + 1) * n])
        return out

    def all_gather_rows(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        out.copy_(inp.repeat(self.world, 1))
        return out

    def broadcast_obj(self, obj, src: int = 0):
        return obj

    def barrier(self):
        return None


def init_distributed(backend: str | None = None, timeout_s: float = 600.0) -> TPContext:
    """Initialise the default process group from torchrun env vars (RANK/WORLD_SIZE/...).

    Returns a TPContext spanning the whole world.  Idempotent.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world == 1:
        return TPContext()
    if not dist.is_initialized():
        if backend is None:
            # RFQ_DIST_BACKEND=gloo: a rehearsal of N ranks sharing one GPU (RCCL
            # refuses two ranks on one device); production multi-GPU runs use RCCL
            backend = os.environ.get("RFQ_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", rank))
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s),
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s))
    return TPContext(rank=dist.get_rank(), world=dist.get_world_size(), group=dist.group.WORLD)


def split_groups(tp: int) -> tuple[TPContext, int, int]:
    """Partition the world into world/tp tensor-parallel groups (DP replicas x TP).

    Returns (tp_context, dp_rank, dp_world).  Must be called by every rank.
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if tp == 1:
        return TPContext(), rank, world
    if world % tp:
        raise ValueError(f"world {world} not divisible by tp {tp}")
    mine = None
    for g in range(world // tp):
        ranks = list(range(g * tp, (g + 1) * tp))
        grp = dist.new_group(ranks)
        if rank in ranks:
            mine = TPContext(rank=rank - g * tp, world=tp, group=grp)
    return mine, rank // tp, world // tp
