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


async def _throughput(url: str, docs: list, clients: int) -> tuple[float, int, int]:
    import httpx

    queue: asyncio.Queue = asyncio.Queue()
    for d in docs:
        queue.put_nowait(d)
    ok = bad = 0
    retries = [0]
    limits = httpx.Limits(max_connections=clients, max_keepalive_connections=clients)

    async def worker(c):
        nonlocal ok, bad
        while True:
            try:
                d = queue.get_nowait()
            except asyncio.QueueEmpty:
                return
            r = None
            for _ in range(3):                       # transport hiccups are retried, not
                try:                                 # counted as extraction failures
                    if isinstance(d, tuple):         # (filename, bytes): POST /upload/
                        r = await c.post(url + "/upload/", files={"file": d})
                    else:
                        r = await c.post(url + "/parse-text/", json={"text": d})
                    break
                except httpx.TransportError:
                    retries[0] += 1
            data = r.json().get("data", {}) if r is not None and r.status_code == 200 else {}
            if data.get("success") and "validation warnings" not in data.get("message", ""):
                ok += 1
            else:
                bad += 1

    async with httpx.AsyncClient(timeout=600.0, limits=limits) as c:
        t0 = time.perf_counter()
        await asyncio.gather(*(worker(c) for _ in range(clients)))
        dt = time.perf_counter() - t0
    _throughput.retries = retries[0]
    return dt, ok, bad


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
    a = ap.parse_args()

    from replisense_rfq_amd.utils import synth

    url = f"http://127.0.0.1:{a.port}"
    env = dict(os.environ, RFQ_BACKEND="engine", RFQ_MODEL=a.model, ENVIRONMENT="production",
               RFQ_PARSER_PROCS=str(a.parser_procs),
               RFQ_MAX_BATCH=str(a.max_batch), LOG_LEVEL="warning", PYTHONUNBUFFERED="1")
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
        dt, ok, bad = asyncio.run(_throughput(url, docs, a.clients))
        q = statistics.quantiles(lat, n=10) if len(lat) >= 2 else [lat[0]] * 9
        print(json.dumps({
            "metric": "http_rfq_docs_per_sec", "mode": a.mode,
            "value": round(a.requests / dt, 3),
            "unit": "docs/s", "model": a.model, "clients": a.clients, "requests": a.requests,
            "valid": ok, "invalid": bad, "transport_retries": getattr(_throughput, "retries", 0),
            "p50_parse_text_http_s": round(statistics.median(lat), 4),
            "p90_parse_text_http_s": round(q[8], 4),
            "baseline_p50_s": 0.883, "server_startup_s": round(startup, 1),
            "data": "synthetic RFQ documents, random-init weights"}), flush=True)
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=30)
        except Exception:
            os.killpg(proc.pid, signal.SIGKILL)


if __name__ == "__main__":
    main()
