"""End-to-end over real HTTP: uvicorn serving the app in a subprocess, concurrent
clients.  CPU: deterministic mock backend.  GPU: the on-node engine (tiny model)
through the same server, checking every response validates."""
import concurrent.futures as cf
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _serve(env_extra):
    import httpx

    port = _port()
    env = dict(os.environ, ENVIRONMENT="production", LOG_LEVEL="warning", **env_extra)
    proc = subprocess.Popen([sys.executable, "-m", "replisense_rfq_amd.api.serve", "--host",
                             "127.0.0.1", "--port", str(port)], cwd=ROOT, env=env,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True)
    url = f"http://127.0.0.1:{port}"
    t0 = time.time()
    while time.time() - t0 < 300:
        if proc.poll() is not None:
            raise RuntimeError("server exited")
        try:
            if httpx.get(url + "/health", timeout=2).status_code == 200:
                return proc, url
        except Exception:
            pass
        time.sleep(0.5)
    os.killpg(proc.pid, signal.SIGKILL)
    raise TimeoutError("server not healthy")


def _stop(proc):
    os.killpg(proc.pid, signal.SIGTERM)
    try:
        proc.wait(timeout=30)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, signal.SIGKILL)


def _exercise(url, n=16, validate=True):
    import httpx

    from replisense_rfq_amd.service.schema import RFQResponse
    from replisense_rfq_amd.utils import docgen, synth

    def one(i):
        r = httpx.post(url + "/parse-text/", json={"text": synth.make_rfq(i).text}, timeout=300)
        assert r.status_code == 200 and "X-Process-Time" in r.headers
        body = r.json()
        assert body["success"] is True and body["message"] == "Successfully processed text input"
        data = body["data"]
        assert data["parsing_info"]["input_type"] == "direct_text"
        if validate:
            RFQResponse(**{k: v for k, v in data.items() if k != "parsing_info"})
        return data

    with cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(one, range(n)))
    # multipart upload through the real server
    doc = synth.make_rfq(3, style="formal")
    pdf = docgen.write_pdf(doc.text.splitlines())
    r = httpx.post(url + "/upload/", files={"file": ("rfq.pdf", pdf, "application/pdf")},
                   timeout=300)
    assert r.status_code == 200, r.text
    assert r.json()["data"]["parsing_info"]["original_filename"] == "rfq.pdf"
    r = httpx.get(url + "/metrics", timeout=10)
    assert r.status_code == 200
    return outs


def test_http_mock_backend():
    proc, url = _serve({"RFQ_BACKEND": "mock"})
    try:
        _exercise(url)
    finally:
        _stop(proc)


@pytest.mark.gpu
def test_http_engine_backend(gpu):
    """The in-process layout (RFQ_ENGINE_PROCESS=0; the GPU default is the engine in
    its own process, below): REFERENCE grammar profile, no decoding hints (random
    weights then fill strings until the token-budget close-out): every response is
    the reference's success envelope (validated or fallback dict)."""
    proc, url = _serve({"RFQ_BACKEND": "engine", "RFQ_MODEL": "tiny-llama", "RFQ_MAX_BATCH": "16",
                        "RFQ_KV_FRACTION": "0.05", "RFQ_ENGINE_PROCESS": "0"})
    try:
        outs = _exercise(url, n=12, validate=False)
        assert all(o["success"] for o in outs)
    finally:
        _stop(proc)


@pytest.mark.gpu
def test_http_engine_process_router(gpu):
    """The router spawn path on the GPU, the service default there: the engine in its
    own process (RFQ_ENGINE_PROCESS=auto), pinned through HIP_VISIBLE_DEVICES."""
    proc, url = _serve({"RFQ_BACKEND": "engine", "RFQ_MODEL": "tiny-llama", "RFQ_MAX_BATCH": "16",
                        "RFQ_KV_FRACTION": "0.05", "RFQ_DECODE_HINTS": "1"})
    try:
        outs = _exercise(url, n=8)
        assert all(o["success"] for o in outs)
    finally:
        _stop(proc)


def test_http_tensor_parallel_replica_cpu():
    """RFQ_TP=2 through the served API: the router spawns one TP group (rank 0 = the
    engine loop, rank 1 = follower) joined over gloo; /parse-text/ and /upload/
    return the reference envelopes.  (On GPUs the same path uses RCCL; SURVEY.md
    §2.3, BASELINE config 4.)"""
    proc, url = _serve({"RFQ_BACKEND": "engine", "RFQ_MODEL": "tiny-llama-tp", "RFQ_TP": "2",
                        "RFQ_DEVICE": "cpu", "RFQ_MAX_BATCH": "4", "RFQ_DECODE_HINTS": "1",
                        "RFQ_GRAPHS": "0", "OMP_NUM_THREADS": "2"})
    try:
        import httpx

        outs = _exercise(url, n=3)
        assert all(o["success"] for o in outs)
        m = httpx.get(url + "/metrics", timeout=10).json()
        assert m["data"]["router"]["tp"] == 2 and m["data"]["router"]["ready"] == 1
    finally:
        _stop(proc)
