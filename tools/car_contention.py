"""Custom all-reduce with W rank processes sharing ONE GPU: per-call latency and flag
timeouts, with or without the launching process itself holding a GPU context.

Root-causing the round-2 world-8 self-test fallback (profiles/r3_custom_ar_world8.md):
the kernel's grid is tiny (1-8 blocks per rank in the engine's self-test, <= 64 in
the GPU test), so all ranks' workgroups fit on the chip at once; what does not fit
is the number of GPU *processes*: the amdgpu HWS runs at most ``hws_max_conc_proc``
processes' queues at a time (printed below when readable), and a rank whose queues
are not mapped cannot raise the flags its peers spin on.  A pytest run holds one
context in the parent (the ``gpu`` fixture), so the world-8 test puts 9 processes on
the device.  This tool measures the one-shot call latency for W ranks, with the
parent holding a context (--parent-gpu) or not.

Usage: python tools/car_contention.py --world 8 [--parent-gpu] [--calls 200]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, calls, reps, q):
    import torch
    import torch.distributed as dist

    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        from replisense_rfq_amd.parallel.custom_ar import CustomAllReduce

        car = CustomAllReduce(rank, world, None, capacity_bytes=4 << 20)
        x = torch.full((8192,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
        car.all_reduce_(x, 1)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
            for _ in range(calls):
                car.all_reduce_(x, 1)
        torch.cuda.current_stream().wait_stream(s)
        us = []
        for _ in range(reps):
            dist.barrier()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            us.append((time.perf_counter() - t0) * 1e6 / calls)
        dist.barrier()
        q.put((rank, us, car.errors(), car.error_info()))
        car.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), -1, ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--parent-gpu", action="store_true")
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    info = {}
    for k in ("hws_max_conc_proc", "sched_policy", "mes"):
        try:
            with open(f"/sys/module/amdgpu/parameters/{k}") as f:
                info[k] = f.read().strip()
        except OSError:
            info[k] = None
    hold = None
    if a.parent_gpu:
        import torch

        hold = torch.ones(1, device="cuda")          # the parent now owns a GPU context
        torch.cuda.synchronize()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, a.world, port, a.calls, a.reps, q))
             for r in range(a.world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(a.world))
    for p in procs:
        p.join(timeout=60)
    per_rank = {r: (round(statistics.median(us), 1) if isinstance(us, list) else us)
                for r, us, _, _ in res}
    out = {"world": a.world, "gpu_processes": a.world + (1 if hold is not None else 0),
           "amdgpu": info, "us_per_call_median_by_rank": per_rank,
           "us_per_call_max": max(max(us) for _, us, _, _ in res if isinstance(us, list)),
           "timeouts": sum(max(0, e) for _, _, e, _ in res),
           "timeout_info": [i for _, _, _, i in res if i]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
