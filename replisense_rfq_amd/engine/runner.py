"""Model runner: packed step (from the native EngineCore) -> one H2D metadata
upload -> forward -> grammar-masked sampling -> one D2H of the sampled ids.

A step's rows are laid out in two sections:

  A  decode rows (q = 1) and short grammar jump-forward extends (q <= EXT_MAX):
     paged split-K MFMA attention (csrc/kernels/attn_decode.hip), one work item
     per (sequence, 16-column tile of q*G (query, head) pairs);
  B  prompt prefill chunks: varlen causal flash attention (attn_prefill.hip).

* All step metadata (token ids, positions, KV slots, block tables, per-sequence
  q/kv lengths, work lists, logits rows, grammar mask rows, temperatures, seeds)
  is packed into ONE pinned int32 buffer and copied with one async H2D.
* Steps without a prefill section replay a hipGraph (torch.cuda.CUDAGraph on
  ROCm) captured for a (sequence bucket NB, token bucket TB) pair; the graph
  holds the whole forward + sampler and reads its metadata from a static device
  buffer in the same layout, so the H2D copy is the only extra work.  Because
  jump-forward extends live in section A, decode steps that also append forced
  schema tokens stay on the graph path.
* With tensor parallelism rank 0 owns the scheduler; it broadcasts the packed
  buffer (header + payload) to the TP workers, which run the identical forward;
  the vocab-parallel sampler all-gathers (value, index) partials (C3).
"""
from __future__ import annotations

import os
import time
import numpy as np
import torch

from .. import ops
from ..models.llama import DecoderLM, ForwardMeta
from ..parallel.tp import TPContext
from ..utils.faults import CustomAllReduceError
from .kv_cache import KVCache

(H_T, H_TA, H_NA, H_WA, H_NB, H_WB, H_S, H_MAXB, H_GNB, H_GTB, H_SPLITS, H_PAYLOAD,
 H_STOP, H_TILES) = range(14)
HEADER = 16
SAMPLE_SPLITS = 8
EXT_MAX = 32                 # extends up to this many tokens use the decode kernel
TOKEN_MULTS = (1, 2, 3, 4, 6, 8)
MAX_GRAPH_TOKENS = 4096
_STEP_LOG = os.environ.get("RFQ_STEP_LOG", "")


def _seed64(req_seed: int, pos: int) -> int:
    x = (req_seed * 0x9E3779B97F4A7C15 + pos * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB)
    x &= (1 << 64) - 1
    x ^= x >> 31
    return x - (1 << 64) if x >= (1 << 63) else x


def _layout(T, NA, WA, NB, WB, S, maxb):
    """(name, length) of every int32 array in the payload, in order."""
    return [("seeds", 2 * S), ("ids", T), ("pos", T), ("slots", T),
            ("a_bt", NA * maxb), ("a_qs", NA), ("a_ql", NA), ("a_kvl", NA), ("a_ws", WA),
            ("a_wct", WA), ("b_bt", NB * maxb), ("b_qs", NB), ("b_ql", NB), ("b_kvl", NB),
            ("b_ws", WB), ("b_wq", WB), ("lidx", S), ("midx", S), ("temps", S)]


class ModelRunner:
    def __init__(self, model: DecoderLM, kv: KVCache, cfg, mask_table: np.ndarray | None,
                 tp: TPContext):
        self.model = model
        self.kv = kv
        self.cfg = cfg
        self.tp = tp
        self.device = model.device
        self.is_cuda = self.device.type == "cuda"
        self.G = model.hq // model.hkv
        self.mask_table = (torch.from_numpy(np.ascontiguousarray(mask_table)).to(self.device)
                           if mask_table is not None else
                           torch.zeros((1, (model.cfg.vocab_size + 31) // 32), dtype=torch.int32,
                                       device=self.device))
        self.max_blocks = (cfg.max_model_len + kv.block_size - 1) // kv.block_size
        self.graphs: dict[tuple, object] = {}
        self._pinned = None
        self._dev = None
        self._stage_t = None                 # pinned staging tensor the core packs into
        self._stage = None                   # its numpy view
        self._header = np.zeros(HEADER, np.int32)
        self.decode_tiles = int(getattr(cfg, "decode_tiles", 1))
        # validated on every device (a config the GPU kernels cannot run fails at start-up)
        qblk = ops.prefill_qblk(model.hq, model.hkv)
        self.prefill_qblk = qblk if self.is_cuda else 32
        self.ring = None
        # SURVEY.md §5.2 debug check: Inf/NaN logits are counted on device inside the step
        # (captured into the decode graphs too) and read back with the sampled tokens
        self.check_finite = bool(getattr(cfg, "check_finite", False))
        self._nonfinite = torch.zeros(1, dtype=torch.int32, device=self.device)
        # bounded in-launch waits (stream-K slabs, persistent decode stages) count their
        # timeouts in host-mapped words (csrc/kernels/kerr.hip); allocated here, before
        # any graph capture, and compared after every step's token readback
        self._kerr0 = ops.kernel_errors()[:2] if self.is_cuda else [0, 0]
        if tp.enabled:
            self._setup_control_plane()
        # host-side split of a step: pack (scheduler), launch (upload + forward + sampler
        # enqueue), overlap (busy_hook), wait (device drain + token readback)
        self.stats = {"steps": 0, "graph_steps": 0, "tokens": 0, "forward_s": 0.0,
                      "pack_s": 0.0, "launch_s": 0.0, "overlap_s": 0.0, "wait_s": 0.0}
        # host work to run while the step executes on the device (after the launch,
        # before the token readback), e.g. admitting new requests into the core: the
        # core is between schedule_and_pack and post then, and add() only appends to
        # the waiting queue, so the admitted requests are scheduled from the next step
        self.busy_hook = None

    def _decode_splits(self, NA: int, max_ctx: int, graph: bool) -> int:
        if NA == 0 or not self.is_cuda:
            return 1
        wg = NA * self.model.hkv
        s = 1
        while wg * s < 1024 and s < 16:
            s *= 2
        if not graph:
            s = max(1, min(s, (max_ctx + 255) // 256))
        return s

    # ------------------------------------------------------------- unpacking
    @staticmethod
    def _views(buf: torch.Tensor, h) -> dict:
        T, TA, NA, WA, NB, WB, S, maxb = (int(h[i]) for i in (H_T, H_TA, H_NA, H_WA, H_NB, H_WB,
                                                              H_S, H_MAXB))
        out, o = {}, 0
        for name, n in _layout(T, NA, WA, NB, WB, S, maxb):
            out[name] = buf[o:o + n]
            o += n
        out["a_bt"] = out["a_bt"].view(NA, maxb)
        out["b_bt"] = out["b_bt"].view(NB, maxb)
        out["seeds"] = out["seeds"].view(torch.int64)
        out["temps"] = out["temps"].view(torch.float32)
        out["lidx"] = out["lidx"]
        return out

    def _meta(self, v, h) -> ForwardMeta:
        T, TA = int(h[H_T]), int(h[H_TA])
        return ForwardMeta(
            input_ids=v["ids"], positions=v["pos"], slot_mapping=v["slots"], num_decode=TA,
            dec_block_tables=v["a_bt"], dec_q_start=v["a_qs"], dec_q_len=v["a_ql"],
            dec_kv_len=v["a_kvl"], dec_work_seq=v["a_ws"], dec_work_ct=v["a_wct"],
            num_prefill_tokens=T - TA, pf_block_tables=v["b_bt"], pf_q_start=v["b_qs"],
            pf_q_len=v["b_ql"], pf_kv_len=v["b_kvl"], work_seq=v["b_ws"], work_qblk=v["b_wq"],
            logits_idx=v["lidx"], decode_splits=int(h[H_SPLITS]),
            decode_tiles=max(1, int(h[H_TILES])), prefill_qblk=self.prefill_qblk)

    def _staging(self, words: int) -> np.ndarray:
        if self._stage is None or self._stage.size < words:
            if self.is_cuda:
                self._stage_t = torch.empty(words, dtype=torch.int32, pin_memory=True)
                self._stage = self._stage_t.numpy()
            else:
                self._stage = np.zeros(words, np.int32)
        return self._stage

    def _upload(self, payload: np.ndarray, dst: torch.Tensor | None = None) -> torch.Tensor:
        n = payload.size
        if not self.is_cuda:
            return torch.from_numpy(payload.copy())
        if self._dev is None or self._dev.numel() < n:
            self._dev = torch.empty(max(n, 1 << 20), dtype=torch.int32, device=self.device)
        staged = (self._stage is not None and n > 0
                  and payload.ctypes.data == self._stage.ctypes.data)
        if staged:
            src = self._stage_t[:n]
        else:
            if self._pinned is None or self._pinned.numel() < n:
                self._pinned = torch.empty(max(n, 1 << 20), dtype=torch.int32, pin_memory=True)
            self._pinned[:n].numpy()[:] = payload
            src = self._pinned[:n]
        dst = self._dev if dst is None else dst
        dst[:n].copy_(src, non_blocking=True)
        return dst[:n]

    # ---------------------------------------------------------------- execute
    def execute(self, core, now: float):
        """Rank-0 entry: the native core schedules and packs the step straight into
        the pinned staging buffer; run it and return the sampled id per logits row
        (None when there is nothing to run)."""
        t0 = time.perf_counter()
        buf = self._staging(core.payload_bound())
        n = core.schedule_and_pack(self._header, buf, now)
        self.stats["pack_s"] += time.perf_counter() - t0
        if n == 0:
            return None
        header, payload = self._header, buf[:n]
        if self.tp.enabled:
            self._broadcast(header, payload)
        return self._run(header, payload)

    def _setup_control_plane(self, capacity: int = 64 << 20) -> None:
        """TP step metadata over a host shared-memory channel (csrc/runtime/shm_ring.cpp)
        when every rank of the group is on this node; RCCL broadcast otherwise
        (``RFQ_TP_CONTROL=rccl``)."""
        import os
        import socket
        import uuid

        from .. import runtime

        mode = os.environ.get("RFQ_TP_CONTROL", "shm")
        host = socket.gethostname()
        same = all(h == host for h in self._gather_hosts(host))
        if mode != "shm" or not same:
            return
        rt = runtime.load()
        if self.tp.rank == 0:
            name = f"rfq_tp_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            self.ring = rt.ShmRing(name, capacity, self.tp.world - 1, True, -1)
            self.tp.broadcast_obj(name)
        else:
            name = self.tp.broadcast_obj(None)
            self.ring = rt.ShmRing(name, capacity, self.tp.world - 1, False, self.tp.rank - 1)
        self.tp.barrier()

    def _gather_hosts(self, host: str) -> list:
        out = [None] * self.tp.world
        torch.distributed.all_gather_object(out, host, group=self.tp.group)
        return out

    def _broadcast(self, header, payload):
        if self.ring is not None:
            msg = np.concatenate([header.astype(np.int32), payload.astype(np.int32, copy=False)])
            if not self.ring.publish(msg, 120.0):
                raise RuntimeError("TP control plane: a worker stopped acknowledging steps")
            return
        dev = self.device if self.is_cuda else "cpu"
        h = torch.from_numpy(header.copy()).to(dev)
        torch.distributed.broadcast(h, src=0, group=self.tp.group)
        if payload.size:
            p = torch.from_numpy(payload.copy()).to(dev)
            torch.distributed.broadcast(p, src=0, group=self.tp.group)

    def worker_step(self) -> bool:
        """TP ranks > 0: receive one step from rank 0 and run it.  False = stop."""
        if self.ring is not None:
            msg = None
            while msg is None:                   # idle server: keep waiting for rank 0
                msg = self.ring.receive(1.0)
            header = msg[:HEADER]
            if header[H_STOP]:
                return False
            self._run(header, msg[HEADER:HEADER + int(header[H_PAYLOAD])])
            return True
        dev = self.device if self.is_cuda else "cpu"
        h = torch.empty(HEADER, dtype=torch.int32, device=dev)
        torch.distributed.broadcast(h, src=0, group=self.tp.group)
        header = h.cpu().numpy()
        if header[H_STOP]:
            return False
        n = int(header[H_PAYLOAD])
        p = torch.empty(n, dtype=torch.int32, device=dev)
        if n:
            torch.distributed.broadcast(p, src=0, group=self.tp.group)
        self._run(header, p.cpu().numpy())
        return True

    def stop_workers(self):
        if self.tp.enabled:
            h = np.zeros(HEADER, np.int32)
            h[H_STOP] = 1
            self._broadcast(h, np.zeros(0, np.int32))

    def _run(self, header: np.ndarray, payload: np.ndarray) -> np.ndarray:
        t0 = time.perf_counter()
        key = (int(header[H_GNB]), int(header[H_GTB]))
        if _STEP_LOG:
            # debugging aid (RFQ_STEP_LOG=path): each step's shape, flushed before launch
            with open(_STEP_LOG, "a") as f:
                f.write(" ".join(f"{k}={int(header[i])}" for k, i in (
                    ("T", H_T), ("TA", H_TA), ("NA", H_NA), ("NB", H_NB), ("S", H_S),
                    ("maxb", H_MAXB), ("gnb", H_GNB), ("gtb", H_GTB), ("splits", H_SPLITS)))
                        + "\n")
        if key[0]:
            g, gbuf, out = self.graphs[key]
            self._upload(payload, gbuf)
            g.replay()
        else:
            buf = self._upload(payload)
            v = self._views(buf, header)
            logits = self.model.forward(self._meta(v, header))
            out = self._sample(logits, v["midx"], v["temps"], v["seeds"])
        t1 = time.perf_counter()
        hook_err = None
        if self.busy_hook is not None:
            try:
                self.busy_hook()
            except Exception as e:  # noqa: BLE001 - re-raised once the step has drained
                hook_err = e
        t2 = time.perf_counter()
        if out.is_cuda and out.numel() == 0:
            # a step with no logits rows (a prefill chunk that ends no prompt): copying an
            # empty tensor does not wait for the stream, and the next step is packed into
            # the same pinned staging buffer this step's payload is still being uploaded
            # from -- wait for the step, as the token readback does for every other step
            torch.cuda.current_stream(self.device).synchronize()
        toks = out.cpu().numpy() if out.is_cuda else out.numpy()
        self.stats["launch_s"] += t1 - t0
        self.stats["overlap_s"] += t2 - t1
        self.stats["wait_s"] += time.perf_counter() - t2
        if hook_err is not None:
            # the device work of this step is finished (readback above), so the caller
            # sees the hook's failure with no kernel of the step still in flight
            raise hook_err
        if self.check_finite:
            bad = int(self._nonfinite[0])
            if bad:
                self._nonfinite.zero_()
                raise RuntimeError(f"non-finite logits: {bad} Inf/NaN entries in step "
                                   f"{self.stats['steps']} (TP rank {self.tp.rank})")
        if self.is_cuda:
            kerr = ops.kernel_errors()
            if kerr[:2] != self._kerr0:
                # a hand-off inside a launch gave up after its bounded wait: this step's
                # outputs may hold unpublished partial sums.  Fatal, like the custom
                # all-reduce's flag timeout below.
                self._kerr0 = kerr[:2]
                raise RuntimeError(f"in-launch hand-off timeout (stream-K {kerr[0]}, persistent "
                                   f"decode {kerr[1]}, first at {kerr[2] - 1:#x}) on TP rank "
                                   f"{self.tp.rank}; results of this step are unreliable")
        car = self.tp.car
        if car is not None and car.errors():
            # a peer's flag never arrived inside the kernel's bounded spin: the sums of
            # this step may be stale.  The error counter is never reset: the replica
            # is done.  On a TP follower this ends the process; TP rank 0's router
            # worker fails its requests and exits (router.py), and the router
            # restarts the whole group with RCCL all-reduces.
            raise CustomAllReduceError(f"custom all-reduce: {car.errors()} flag timeouts on TP rank "
                               f"{self.tp.rank}; results of this step are unreliable")
        self.stats["steps"] += 1
        self.stats["graph_steps"] += bool(key[0])
        self.stats["tokens"] += int(header[H_T])
        self.stats["forward_s"] += time.perf_counter() - t0
        return toks

    def _sample(self, logits, midx, temps, seeds, out=None):
        S = logits.shape[0]
        if self.check_finite:
            ops.count_nonfinite(logits, self._nonfinite)
        if not logits.is_cuda:
            mt = self.mask_table.cpu()
            vals, idx = ops.reference.sample(logits, mt, midx, temps, seeds, self.model.vocab_start)
            if self.tp.enabled:
                allv = [torch.empty_like(vals) for _ in range(self.tp.world)]
                alli = [torch.empty_like(idx) for _ in range(self.tp.world)]
                torch.distributed.all_gather(allv, vals, group=self.tp.group)
                torch.distributed.all_gather(alli, idx, group=self.tp.group)
                best = torch.stack(allv).argmax(0)
                idx = torch.stack(alli).gather(0, best[None])[0]
            return idx
        pv = torch.empty((1, S, SAMPLE_SPLITS), dtype=torch.float32, device=self.device)
        pi = torch.empty((1, S, SAMPLE_SPLITS), dtype=torch.int32, device=self.device)
        out = torch.empty(S, dtype=torch.int32, device=self.device) if out is None else out
        ops.sample_partial(logits, self.model.vocab_start, self.mask_table, midx, temps, seeds,
                           pv[0], pi[0])
        if self.tp.enabled:
            gv = torch.empty((self.tp.world, S, SAMPLE_SPLITS), dtype=torch.float32,
                             device=self.device)
            gi = torch.empty((self.tp.world, S, SAMPLE_SPLITS), dtype=torch.int32,
                             device=self.device)
            self.tp.all_gather_into(gv, pv[0])
            self.tp.all_gather_into(gi, pi[0])
            ops.sample_final(gv, gi, out)
        else:
            ops.sample_final(pv, pi, out)
        return out

    # ----------------------------------------------------------------- graphs
    def capture_graphs(self, buckets, max_tokens: int = MAX_GRAPH_TOKENS) -> float:
        """Capture forward+sample graphs for (NB, TB) buckets, largest first."""
        if not self.is_cuda or not self.cfg.use_graphs:
            return 0.0
        t0 = time.perf_counter()
        keys = [(nb, nb * m) for nb in sorted(buckets) for m in TOKEN_MULTS
                if nb * m <= max(max_tokens, nb if max_tokens >= MAX_GRAPH_TOKENS else 0)]
        maxb = self.max_blocks
        pool = torch.cuda.graph_pool_handle()
        for nb, tb in sorted(keys, key=lambda k: (-k[1], -k[0])):
            header = np.zeros(HEADER, np.int32)
            header[[H_T, H_TA, H_NA, H_WA, H_NB, H_WB, H_S, H_MAXB, H_SPLITS]] = \
                [tb, tb, nb, tb, 0, 0, nb, maxb, self._decode_splits(nb, 0, graph=True)]
            header[H_TILES] = self.decode_tiles
            n = sum(k for _, k in _layout(tb, nb, tb, 0, 0, nb, maxb))
            gbuf = torch.zeros(n, dtype=torch.int32, device=self.device)
            v = self._views(gbuf, header)
            # a harmless padding state for the capture run: no sequences, no KV writes
            v["slots"].fill_(-1)
            v["a_ws"].fill_(-1)
            v["a_kvl"].fill_(1)
            v["midx"].fill_(-1)
            v["a_bt"].fill_(self.kv.scratch_block)
            meta = self._meta(v, header)
            out = torch.zeros(nb, dtype=torch.int32, device=self.device)

            def body():
                logits = self.model.forward(meta)
                self._sample(logits, v["midx"], v["temps"], v["seeds"], out=out)

            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()          # warm-up (allocator + hipBLASLt heuristics)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                body()
            self.graphs[(nb, tb)] = (g, gbuf, out)
        torch.cuda.synchronize()
        return time.perf_counter() - t0
