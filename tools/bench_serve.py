"""HTTP-level benchmark: the FastAPI service with the on-node engine behind it.

Starts ``python -m replisense_rfq_amd.api.serve`` (RFQ_BACKEND=engine) in its own
process group, waits for /health, then measures
  * p50 / p90 end-to-end ``POST /parse-text/`` latency, one request at a time
    (the reference's metric: its p50 Groq server time was 0.883 s), and
  * RFQ docs/s with ``--clients`` concurrent HTTP clients (continuous batching
    behind one uvicorn worker).
Synthetic RFQ documents with the reference's length distribution; random-init
weights.  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _wait_healthy(url: str, proc, timeout: float) -> None:
    import httpx

    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode}")
        try:
            if httpx.get(url + "/health", timeout=2.0).status_code == 200:
                return
        except Exception:
            pass
        time.sleep(1.0)
    raise TimeoutError("server did not become healthy")


async def _latency(url: str, docs: list[str]) -> list[float]:
    import httpx

    out = []
    async with httpx.AsyncClient(timeout=120.0) as c:
        for d in docs:
            t0 = time.perf_counter()
            r = await c.post(url + "/parse-text/", json={"text": d})
            r.raise_for_status()
            assert r.json()["success"] is True
            out.append(time.perf_counter() - t0)
    return out


async def _throughput_aio(url: str, docs: list, clients: int) -> tuple[int, int, int]:
    """One client process: ``clients`` concurrent keep-alive connections (aiohttp)."""
    import aiohttp

    queue: asyncio.Queue = asyncio.Queue()
    for d in docs:
        queue.put_nowait(d)
    ok = bad = retries = 0

    async def worker(sess):
        nonlocal ok, bad, retries
        while True:
            try:
                d = queue.get_nowait()
            except asyncio.QueueEmpty:
                return
            status, body = None, {}
            for _ in range(3):                       # transport hiccups are retried, not
                try:                                 # counted as extraction failures
                    if isinstance(d, tuple):         # (filename, bytes): POST /upload/
                        form = aiohttp.FormData()
                        form.add_field("file", d[1], filename=d[0])
                        async with sess.post(url + "/upload/", data=form) as r:
                            status, body = r.status, await r.json()
                    else:
                        async with sess.post(url + "/parse-text/", json={"text": d}) as r:
                            status, body = r.status, await r.json()
                    break
                except (aiohttp.ClientError, asyncio.TimeoutError):
                    retries += 1
            data = body.get("data", {}) if status == 200 else {}
            if data.get("success") and "validation warnings" not in data.get("message", ""):
                ok += 1
            else:
                bad += 1

    conn = aiohttp.TCPConnector(limit=clients, limit_per_host=clients)
    async with aiohttp.ClientSession(connector=conn,
                                     timeout=aiohttp.ClientTimeout(total=600)) as sess:
        await asyncio.gather(*(worker(sess) for _ in range(clients)))
    return ok, bad, retries


def _client_proc(url, docs, clients, start_evt, out_q):
    start_evt.wait()
    out_q.put(asyncio.run(_throughput_aio(url, docs, clients)))


def _throughput(url: str, docs: list, clients: int, procs: int = 4) -> tuple[float, int, int]:
    """Closed-loop load from ``procs`` client processes (``clients`` connections in
    total): one Python HTTP client process saturates its own CPU long before the
    server does (httpx: ~23 ms of client CPU per request at 512 connections)."""
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    procs = max(1, min(procs, clients))
    start_evt, out_q = ctx.Event(), ctx.Queue()
    ps = [ctx.Process(target=_client_proc,
                      args=(url, docs[i::procs], clients // procs + (i < clients % procs),
                            start_evt, out_q), daemon=True) for i in range(procs)]
    for p in ps:
        p.start()
    time.sleep(1.0)                               # let every client process import
    t0 = time.perf_counter()
    start_evt.set()
    res = [out_q.get() for _ in ps]
    dt = time.perf_counter() - t0
    for p in ps:
        p.join()
    _throughput.retries = sum(r[2] for r in res)
    return dt, sum(r[0] for r in res), sum(r[1] for r in res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--port", type=int, default=8765)
    ap.add_argument("--clients", type=int, default=512)
    ap.add_argument("--requests", type=int, default=2048)
    ap.add_argument("--latency-requests", type=int, default=10)
    ap.add_argument("--max-batch", type=int, default=1024)
    ap.add_argument("--startup-timeout", type=float, default=600.0)
    ap.add_argument("--mode", choices=("text", "upload"), default="text",
                    help="upload: PDF/XLSX/DOCX attachments through POST /upload/ "
                         "(parsing on the server, RFQ_PARSER_PROCS workers)")
    ap.add_argument("--parser-procs", type=int, default=8)
    ap.add_argument("--client-procs", type=int, default=4)
    a = ap.parse_args()

    from replisense_rfq_amd.utils import synth

    url = f"http://127.0.0.1:{a.port}"
    env = dict(os.environ, RFQ_BACKEND="engine", RFQ_MODEL=a.model, ENVIRONMENT="production",
               RFQ_PARSER_PROCS=str(a.parser_procs),
               RFQ_MAX_BATCH=str(a.max_batch), LOG_LEVEL="warning", PYTHONUNBUFFERED="1",
               # random-init weights: the bench-only decoding hints (service/hints.py)
               RFQ_DECODE_HINTS=os.environ.get("RFQ_DECODE_HINTS", "1"))
    log = open(os.path.join(ROOT, "gpurun_out", "bench_serve_server.log")
               if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else os.devnull, "w")
    proc = subprocess.Popen([sys.executable, "-m", "replisense_rfq_amd.api.serve", "--host",
                             "127.0.0.1", "--port", str(a.port)], cwd=ROOT, env=env,
                            stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        t0 = time.time()
        _wait_healthy(url, proc, a.startup_timeout)
        startup = time.time() - t0
        warm = [synth.make_rfq(900_000 + i).text for i in range(4)]
        asyncio.run(_latency(url, warm))
        lat = asyncio.run(_latency(url, [synth.make_rfq(800_000 + i).text
                                         for i in range(a.latency_requests)]))
        if a.mode == "upload":
            from replisense_rfq_amd.utils import docgen

            fmts = ("pdf", "xlsx", "docx")
            docs = []
            for i in range(a.requests):
                f = fmts[i % 3]
                docs.append((f"rfq_{i}.{f}",
                             docgen.rfq_attachment(synth.make_rfq(700_000 + i), f)))
        else:
            docs = [synth.make_rfq(700_000 + i).text for i in range(a.requests)]
        dt, ok, bad = _throughput(url, docs, a.clients, a.client_procs)
        try:
            import httpx

            m = httpx.get(url + "/metrics", timeout=10.0).json().get("data", {})
            eng = m.get("engine") or m.get("router") or {}
        except Exception:                      # metrics are diagnostics only
            eng = {}
        q = statistics.quantiles(lat, n=10) if len(lat) >= 2 else [lat[0]] * 9
        print(json.dumps({
            "metric": "http_rfq_docs_per_sec", "mode": a.mode,
            "value": round(a.requests / dt, 3),
            "unit": "docs/s", "model": a.model, "clients": a.clients, "requests": a.requests,
            "valid": ok, "invalid": bad, "transport_retries": getattr(_throughput, "retries", 0),
            "p50_parse_text_http_s": round(statistics.median(lat), 4),
            "p90_parse_text_http_s": round(q[8], 4),
            "baseline_p50_s": 0.883, "server_startup_s": round(startup, 1),
            "engine": {k: eng[k] for k in ("steps", "graph_steps", "preempted", "blocks",
                                           "forward_s", "execute_s", "post_s", "running", "replicas",
                                           "outstanding")
                       if k in eng},
            "data": "synthetic RFQ documents, random-init weights"}), flush=True)
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=30)
        except Exception:
            os.killpg(proc.pid, signal.SIGKILL)


if __name__ == "__main__":
    main()
