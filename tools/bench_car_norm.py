"""Fused all-reduce + residual-add RMSNorm vs the two-launch epilogue, per call.

    python tools/bench_car_norm.py [world] [rows ...]

`world` ranks share GPU 0 (separate processes, IPC regions, gloo for set-up), so
the peer reads stay on one device: this prices the launch and flag-protocol
cost that fusion removes, not xGMI bandwidth.  Each variant is captured 200
times back to back in one hipGraph (as in a decode graph) and the replay is
timed with events; rank 0 prints µs per call.
"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N_CALLS = 200


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _time_graph(fn, dist):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N_CALLS):
            fn()
    ts = []
    for _ in range(5):
        dist.barrier()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / N_CALLS)
    return min(ts)


def _worker(rank, world, port, rows_list, q):
    import torch.distributed as dist

    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    from replisense_rfq_amd import ops
    from replisense_rfq_amd.parallel.custom_ar import CustomAllReduce

    car = CustomAllReduce(rank, world, None, capacity_bytes=4 << 20)
    out = []
    for rows in rows_list:
        d = 8192
        t = torch.randn(rows, d, device="cuda").to(torch.bfloat16)
        r = torch.zeros_like(t)
        o = torch.empty_like(t)
        w = torch.ones(d, device="cuda", dtype=torch.bfloat16)

        def two():
            car.all_reduce_(t, 1)
            ops.fused_add_rms_norm(t, r, w, 1e-5, out=o)

        def staged():
            car.all_reduce_add_norm_(t, r, w, 1e-5, o, algo=1)

        def push():
            car.all_reduce_add_norm_(t, r, w, 1e-5, o, algo=2)

        out.append((rows, _time_graph(two, dist), _time_graph(staged, dist),
                    _time_graph(push, dist) if rows <= 16 else float("nan")))
    q.put((rank, out, car.errors()))
    dist.barrier()
    car.close()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rows_list = [int(x) for x in sys.argv[2:]] or [1, 4, 8, 16, 32]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, rows_list, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda r: r[0])
    print(f"world {world} (ranks share one GPU), d 8192, us per call; flag timeouts "
          f"{[e for _, _, e in res]}")
    print("| rows | all-reduce + add-norm (2 launches) | fused staged (flag, remote read, "
          "end flag) | fused push (one hop, parity slots) |")
    print("|---|---|---|---|")
    for rows, two, one, push in res[0][1]:
        print(f"| {rows} | {two:.2f} | {one:.2f} | {push:.2f} |")


if __name__ == "__main__":
    main()
