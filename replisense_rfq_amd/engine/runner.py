"""Model runner: StepPlan -> one H2D metadata upload -> forward -> grammar-masked
sampling -> one D2H of the sampled ids.

* All step metadata (token ids, positions, KV slots, block tables, context
  lengths, prefill work lists, logits rows, grammar mask rows, temperatures,
  seeds) is packed into ONE pinned int32 buffer and copied with one async H2D.
* Pure-decode steps whose batch fits a captured bucket replay a hipGraph
  (torch.cuda.CUDAGraph on ROCm) holding the whole forward + sampler: ~L*12
  kernel launches become one graph launch (SURVEY.md north star: "hipGraph-
  captured decode steps shown in rocprof").
* With tensor parallelism rank 0 owns the scheduler; it broadcasts the packed
  buffer (header + payload) to the TP workers, which run the identical forward;
  the vocab-parallel sampler all-gathers (value, index) partials (C3).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np
import torch

from .. import ops
from ..models.llama import DecoderLM, ForwardMeta
from ..parallel.tp import TPContext
from .kv_cache import KVCache
from .scheduler import StepPlan

H_T, H_D, H_P, H_W, H_S, H_MAXB, H_GRAPH, H_SPLITS, H_PAYLOAD, H_STOP = range(10)
HEADER = 16
SAMPLE_SPLITS = 8


def _seed64(req_seed: int, pos: int) -> int:
    x = (req_seed * 0x9E3779B97F4A7C15 + pos * 0xBF58476D1CE4E5B9 + 0x94D049BB133111EB)
    x &= (1 << 64) - 1
    x ^= x >> 31
    return x - (1 << 64) if x >= (1 << 63) else x


@dataclass
class Packed:
    header: np.ndarray
    payload: np.ndarray            # int32
    rows: list                     # (seq, samples?) per logits row (rank 0 only)


class ModelRunner:
    def __init__(self, model: DecoderLM, kv: KVCache, cfg, mask_table: np.ndarray | None,
                 tp: TPContext):
        self.model = model
        self.kv = kv
        self.cfg = cfg
        self.tp = tp
        self.device = model.device
        self.is_cuda = self.device.type == "cuda"
        self.mask_table = (torch.from_numpy(np.ascontiguousarray(mask_table)).to(self.device)
                           if mask_table is not None else
                           torch.zeros((1, (model.cfg.vocab_size + 31) // 32), dtype=torch.int32,
                                       device=self.device))
        self.max_blocks = (cfg.max_model_len + kv.block_size - 1) // kv.block_size
        self.graphs: dict[int, tuple] = {}
        self.graph_pool = None
        self._pinned = None
        self.stats = {"steps": 0, "graph_steps": 0, "tokens": 0, "forward_s": 0.0}

    # ---------------------------------------------------------------- packing
    def pack(self, plan: StepPlan) -> Packed:
        kv, bs = self.kv, self.kv.block_size
        dec, ext = plan.decode, plan.extend
        D = len(dec)
        T = D + sum(q for _, q in ext)
        P = len(ext)
        ids = np.empty(T, np.int32)
        pos = np.empty(T, np.int32)
        slots = np.empty(T, np.int32)
        maxb = max([len(s.blocks) for s in dec] + [len(s.blocks) for s, _ in ext] + [1])
        graph_b = 0
        if (self.is_cuda and self.cfg.use_graphs and P == 0 and D > 0 and self.graphs):
            graph_b = next((b for b in sorted(self.graphs) if b >= D), 0)
        if graph_b:
            maxb = self.max_blocks
        dbt = np.full((D, maxb), kv.scratch_block, np.int32)
        dctx = np.empty(D, np.int32)
        rows = []
        for i, s in enumerate(dec):
            p = s.num_cached
            ids[i], pos[i], slots[i] = s.tokens[p], p, kv.slot(s, p)
            dbt[i, : len(s.blocks)] = s.blocks
            dctx[i] = p + 1
            rows.append((s, s.pending == 1))
        pbt = np.full((P, maxb), kv.scratch_block, np.int32)
        pqs, pql, pkv = np.empty(P, np.int32), np.empty(P, np.int32), np.empty(P, np.int32)
        ws, wq = [], []
        t = D
        ext_rows = []
        for j, (s, q) in enumerate(ext):
            p0 = s.num_cached
            ids[t:t + q] = s.tokens[p0:p0 + q]
            pos[t:t + q] = np.arange(p0, p0 + q)
            blk = np.asarray(s.blocks, np.int64)
            pp = np.arange(p0, p0 + q)
            slots[t:t + q] = blk[pp // bs] * bs + pp % bs
            pbt[j, : len(s.blocks)] = s.blocks
            pqs[j], pql[j], pkv[j] = t - D, q, p0 + q
            nb = (q + 31) // 32
            ws += [j] * nb
            wq += list(range(nb))
            if p0 + q == len(s.tokens):
                ext_rows.append((t + q - 1, s))
            t += q
        # logits rows: all decode rows (graph computes them anyway), then finishing extends
        lidx = list(range(D)) + [r for r, _ in ext_rows]
        rows += [(s, True) for _, s in ext_rows]
        S = len(lidx)
        midx = np.empty(S, np.int32)
        temps = np.empty(S, np.float32)
        seeds = np.empty(S, np.int64)
        for k, (s, _) in enumerate(rows):
            midx[k] = s.mask_idx if s.params.grammar else -1
            temps[k] = s.params.temperature
            seeds[k] = _seed64(s.params.seed ^ (s.req_id * 0x632BE5AB), len(s.tokens))
        splits = self._decode_splits(D, int(dctx.max()) if D else 0, graph_b)
        # int64 seeds first so their view stays 8-byte aligned
        parts = [seeds.view(np.int32), ids, pos, slots, dbt.reshape(-1), dctx, pbt.reshape(-1),
                 pqs, pql, pkv, np.asarray(ws, np.int32), np.asarray(wq, np.int32),
                 np.asarray(lidx, np.int32), midx, temps.view(np.int32)]
        payload = np.concatenate(parts) if parts else np.zeros(0, np.int32)
        header = np.zeros(HEADER, np.int32)
        header[[H_T, H_D, H_P, H_W, H_S, H_MAXB, H_GRAPH, H_SPLITS, H_PAYLOAD]] = \
            [T, D, P, len(ws), S, maxb, graph_b, splits, payload.size]
        return Packed(header, payload, rows)

    def _decode_splits(self, D: int, max_ctx: int, graph_b: int) -> int:
        if D == 0 or not self.is_cuda:
            return 1
        n = graph_b or D
        wg = n * self.model.hkv
        s = 1
        while wg * s < 1024 and s < 16:
            s *= 2
        if not graph_b:
            s = max(1, min(s, (max_ctx + 255) // 256))
        return s

    # ------------------------------------------------------------- unpacking
    @staticmethod
    def _views(buf: torch.Tensor, h: np.ndarray):
        T, D, P, W, S, maxb = (int(h[i]) for i in (H_T, H_D, H_P, H_W, H_S, H_MAXB))
        sizes = [2 * S, T, T, T, D * maxb, D, P * maxb, P, P, P, W, W, S, S, S]
        out, o = [], 0
        for n in sizes:
            out.append(buf[o:o + n])
            o += n
        (seeds, ids, pos, slots, dbt, dctx, pbt, pqs, pql, pkv, ws, wq, lidx, midx, temps) = out
        return dict(ids=ids, pos=pos, slots=slots, dbt=dbt.view(D, maxb), dctx=dctx,
                    pbt=pbt.view(P, maxb), pqs=pqs, pql=pql, pkv=pkv, ws=ws, wq=wq,
                    lidx=lidx.long(), midx=midx, temps=temps.view(torch.float32),
                    seeds=seeds.view(torch.int64))

    def _upload(self, header: np.ndarray, payload: np.ndarray) -> torch.Tensor:
        n = payload.size
        if not self.is_cuda:
            return torch.from_numpy(payload.copy())
        if self._pinned is None or self._pinned.numel() < n:
            self._pinned = torch.empty(max(n, 1 << 20), dtype=torch.int32, pin_memory=True)
            self._dev = torch.empty(max(n, 1 << 20), dtype=torch.int32, device=self.device)
        self._pinned[:n].numpy()[:] = payload
        self._dev[:n].copy_(self._pinned[:n], non_blocking=True)
        return self._dev[:n]

    # ---------------------------------------------------------------- execute
    def execute(self, plan: StepPlan) -> tuple[list, np.ndarray]:
        """Rank-0 entry: run one step, return (rows, sampled ids per logits row)."""
        pk = self.pack(plan)
        if self.tp.enabled:
            self._broadcast(pk.header, pk.payload)
        toks = self._run(pk.header, pk.payload)
        return pk.rows, toks

    def _broadcast(self, header, payload):
        h = torch.from_numpy(header).to(self.device)
        self.tp.group and torch.distributed.broadcast(h, src=0, group=self.tp.group)
        if payload.size:
            p = torch.from_numpy(payload).to(self.device)
            torch.distributed.broadcast(p, src=0, group=self.tp.group)

    def worker_step(self) -> bool:
        """TP ranks > 0: receive one step from rank 0 and run it.  False = stop."""
        h = torch.empty(HEADER, dtype=torch.int32, device=self.device)
        torch.distributed.broadcast(h, src=0, group=self.tp.group)
        header = h.cpu().numpy()
        if header[H_STOP]:
            return False
        n = int(header[H_PAYLOAD])
        p = torch.empty(n, dtype=torch.int32, device=self.device)
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
        graph_b = int(header[H_GRAPH])
        if graph_b:
            out = self._run_graph(header, payload, graph_b)
        else:
            buf = self._upload(header, payload)
            v = self._views(buf, header)
            meta = self._meta(v, header)
            logits = self.model.forward(meta)
            out = self._sample(logits, v["midx"], v["temps"], v["seeds"])
        toks = out.cpu().numpy() if out.is_cuda else out.numpy()
        self.stats["steps"] += 1
        self.stats["graph_steps"] += bool(graph_b)
        self.stats["tokens"] += int(header[H_T])
        self.stats["forward_s"] += time.perf_counter() - t0
        return toks[: int(header[H_S])]

    def _meta(self, v, header) -> ForwardMeta:
        D, P = int(header[H_D]), int(header[H_P])
        T = int(header[H_T])
        return ForwardMeta(
            input_ids=v["ids"], positions=v["pos"], slot_mapping=v["slots"], num_decode=D,
            dec_block_tables=v["dbt"], dec_context_lens=v["dctx"], num_prefill_tokens=T - D,
            pf_block_tables=v["pbt"], pf_q_start=v["pqs"], pf_q_len=v["pql"],
            pf_kv_len=v["pkv"], work_seq=v["ws"], work_qblk=v["wq"], logits_idx=v["lidx"],
            decode_splits=int(header[H_SPLITS]))

    def _sample(self, logits, midx, temps, seeds, out=None, parts=None):
        S = logits.shape[0]
        if not logits.is_cuda:
            mt = self.mask_table.cpu()
            vals, idx = ops.reference.sample(logits, mt, midx, temps, seeds, self.model.vocab_start)
            if self.tp.enabled:
                allv = [torch.empty_like(vals) for _ in range(self.tp.world)]
                alli = [torch.empty_like(idx) for _ in range(self.tp.world)]
                torch.distributed.all_gather(allv, vals, group=self.tp.group)
                torch.distributed.all_gather(alli, idx, group=self.tp.group)
                V = torch.stack(allv)
                I = torch.stack(alli)
                best = V.argmax(0)
                idx = I.gather(0, best[None])[0]
            return idx
        if parts is None:
            pv = torch.empty((1, S, SAMPLE_SPLITS), dtype=torch.float32, device=self.device)
            pi = torch.empty((1, S, SAMPLE_SPLITS), dtype=torch.int32, device=self.device)
        else:
            pv, pi = parts
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
    def capture_graphs(self, buckets) -> float:
        """Capture decode+sample graphs for each batch bucket (largest first)."""
        if not self.is_cuda or not self.cfg.use_graphs:
            return 0.0
        t0 = time.perf_counter()
        Bmax = max(buckets)
        mb = self.max_blocks
        dev = self.device
        i32 = dict(dtype=torch.int32, device=dev)
        st = dict(ids=torch.zeros(Bmax, **i32), pos=torch.zeros(Bmax, **i32),
                  slots=torch.full((Bmax,), -1, **i32),
                  dbt=torch.full((Bmax, mb), self.kv.scratch_block, **i32),
                  dctx=torch.ones(Bmax, **i32), midx=torch.full((Bmax,), -1, **i32),
                  temps=torch.zeros(Bmax, dtype=torch.float32, device=dev),
                  seeds=torch.zeros(Bmax, dtype=torch.int64, device=dev),
                  out=torch.zeros(Bmax, **i32))
        self._gstatic = st
        self._gparts = (torch.empty((1, Bmax, SAMPLE_SPLITS), dtype=torch.float32, device=dev),
                        torch.empty((1, Bmax, SAMPLE_SPLITS), dtype=torch.int32, device=dev))
        pool = torch.cuda.graph_pool_handle()
        for B in sorted(buckets, reverse=True):
            splits = self._decode_splits(B, 0, B)
            meta = ForwardMeta(input_ids=st["ids"][:B], positions=st["pos"][:B],
                               slot_mapping=st["slots"][:B], num_decode=B,
                               dec_block_tables=st["dbt"][:B], dec_context_lens=st["dctx"][:B],
                               logits_idx=None, decode_splits=splits)
            parts = (self._gparts[0][:, :B], self._gparts[1][:, :B])

            def body():
                logits = self.model.forward(meta)
                self._sample(logits, st["midx"][:B], st["temps"][:B], st["seeds"][:B],
                             out=st["out"][:B], parts=parts)

            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                body()          # warm-up (allocator + hipBLASLt heuristics)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                body()
            self.graphs[B] = (g, splits)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def _run_graph(self, header, payload, B):
        v = self._views(torch.from_numpy(payload), header)
        D = int(header[H_D])
        st = self._gstatic
        # stage on host, one H2D per static buffer slice (rows >= D are padding)
        host = np.zeros(0, np.int32)
        ids = np.zeros(B, np.int32); ids[:D] = v["ids"].numpy()
        pos = np.zeros(B, np.int32); pos[:D] = v["pos"].numpy()
        slots = np.full(B, -1, np.int32); slots[:D] = v["slots"].numpy()
        dctx = np.ones(B, np.int32); dctx[:D] = v["dctx"].numpy()
        midx = np.full(B, -1, np.int32); midx[:D] = v["midx"].numpy()[:D]
        temps = np.zeros(B, np.float32); temps[:D] = v["temps"].numpy()[:D]
        seeds = np.zeros(B, np.int64); seeds[:D] = v["seeds"].numpy()[:D]
        dbt = np.full((B, self.max_blocks), self.kv.scratch_block, np.int32)
        dbt[:D] = v["dbt"].numpy()
        host = np.concatenate([seeds.view(np.int32), ids, pos, slots, dctx, midx,
                               temps.view(np.int32), dbt.reshape(-1)])
        buf = self._upload(header, host)
        st["seeds"][:B].copy_(buf[: 2 * B].view(torch.int64))
        o = 2 * B
        for name, n in (("ids", B), ("pos", B), ("slots", B), ("dctx", B), ("midx", B)):
            st[name][:B].copy_(buf[o:o + n])
            o += n
        st["temps"][:B].copy_(buf[o:o + B].view(torch.float32)); o += B
        st["dbt"][:B].copy_(buf[o:o + B * self.max_blocks].view(B, self.max_blocks))
        g, _ = self.graphs[B]
        g.replay()
        return st["out"][:D]
