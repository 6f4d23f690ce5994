"""The bench.py driver contract, rehearsed on CPU with gloo: torchrun launch, one
JSON line from rank 0 with the required keys, TP and DP layouts, self-launch of
N ranks from ``--gpus N`` and the driver's exact step flags inside a time budget
(the GPU box runs the same script over RCCL)."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}
SMALL = ["--docs-per-step", "2", "--max-num-seqs", "2", "--latency-runs", "2"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, timeout=600, threads=2, **extra_env):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), **extra_env)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    return out


@pytest.mark.parametrize("tp,par", [(2, "dp1-tp2"), (1, "dp2")])
def test_bench_torchrun_gloo(tp, par):
    model = "tiny-llama-tp" if tp > 1 else "tiny-llama"
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                str(_port()), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                "--model", model, "--tp", str(tp)] + SMALL)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == par
    assert out["per_doc"]["valid"] == 1.0 and out["p50_parse_text_latency_s"] > 0


@pytest.mark.timeout(900)
def test_bench_tp8_gloo():
    """`bench.py --gpus 8 --tp 8` -- the driver's 70B layout (one TP=8 replica) -- on 8
    gloo ranks with the 70B-shaped tiny model (per-rank Hq=8, Hkv=1)."""
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                str(_port()), "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama70", "--tp", "8"] + SMALL, timeout=800, threads=1)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp1-tp8"
    assert out["per_doc"]["valid"] == 1.0 and out["p50_parse_text_latency_s"] > 0


def test_bench_tp_latency_phase_gloo():
    """After the DP docs/s window the N ranks re-form as ONE TP group and serve
    single requests (what the driver's 8-GPU run does with Llama-3-70B at TP=8):
    the result rides in the same JSON line, the timed fields are untouched."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama", "--tp-latency-model", "tiny-llama-tp",
                "--tp-latency-runs", "2", "--tp-docs", "4", "--tp-in-flight", "2",
                "--pdf-set", "1"] + SMALL)
    assert out["config"]["parallelism"] == "dp2"
    tpl = out["tp_latency"]
    # BASELINE config 4's prefill-heavy documents on the TP group too
    assert tpl["pdf_set"]["docs"] == 1 and tpl["pdf_set"]["valid"] == 1.0, tpl.get("pdf_set")
    assert tpl["status"] == "ok", tpl
    assert tpl["model"] == "tiny-llama-tp" and tpl["parallelism"] == "tp2"
    assert tpl["runs"] == 2 and tpl["p50_parse_text_latency_s"] > 0
    # the fixed latency set of the one-GPU 70B phase: the reference's recorded prompts
    assert tpl["latency_set"].startswith("reference prompts")
    assert [r["row"] for r in tpl["per_row"]] == [1, 2] and tpl["sampled_steps_p50"] > 0
    assert tpl["p50_at_reference_steps_s"] > 0
    assert tpl["docs"] == 4 and tpl["docs_per_s"] > 0 and tpl["per_doc"]["valid"] == 1.0


def test_bench_tp_latency_watchdog():
    """A TP phase that overruns its budget still yields the JSON line (phase marked
    timeout) and a zero exit on every rank."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama", "--tp-latency-model", "tiny-llama-tp",
                "--tp-latency-budget", "0.05"] + SMALL)
    assert out["tp_latency"]["status"].startswith("timeout"), out["tp_latency"]
    assert out["value"] > 0


def test_bench_tp_latency_error_reported():
    """A TP phase that raises (here: an unknown model) is reported in the JSON line;
    the timed fields stand and every rank exits 0."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama", "--tp-latency-model", "no-such-model"] + SMALL)
    assert out["tp_latency"]["status"].startswith("error"), out["tp_latency"]
    assert out["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_tp_latency_phase_one_gpu():
    """The TP phase on the GPU path (HIP kernels at the TP shard shapes, the custom
    IPC all-reduce inside the engine, the vocab-parallel sampler's all-gather): two
    ranks share one MI355X over gloo (RCCL refuses two ranks per device).  The
    pytest process itself never initialises the GPU (device_count only)."""
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    env_extra = {"RFQ_DIST_BACKEND": "gloo"}
    os.environ.update(env_extra)
    try:
        out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                    "--model", "tiny-llama", "--kv-fraction", "0.05", "--no-graphs",
                    "--tp-latency-model", "tiny-llama-tp", "--tp-latency-runs", "2",
                    "--tp-docs", "8", "--tp-in-flight", "4"] + SMALL,
                   timeout=380)
    finally:
        for k in env_extra:
            os.environ.pop(k, None)
    tpl = out["tp_latency"]
    assert tpl["status"] == "ok", tpl
    assert tpl["custom_allreduce"] is True and tpl["p50_parse_text_latency_s"] > 0
    assert tpl["docs_per_s"] > 0 and tpl["per_doc"]["valid"] == 1.0
    assert out["per_doc"]["valid"] == 1.0


def test_bench_tp_latency_auto_off():
    """'auto' only turns the phase on for the driver's 8-GPU run of the 8B bench."""
    sys.path.insert(0, ROOT)
    import bench

    class A:
        tp_latency_model, tp, model, latency_runs = "auto", 1, "llama3-8b", 15
    assert bench._tp_latency_model(A, 8) == "llama3-70b"
    assert bench._tp_latency_model(A, 4) is None and bench._tp_latency_model(A, 1) is None
    A.tp = 8
    assert bench._tp_latency_model(A, 8) is None


def test_bench_self_launch():
    """`bench.py --gpus 2` outside torchrun starts 2 ranks itself (never a silent
    1-GPU run labelled whole-node)."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                "--model", "tiny-llama"] + SMALL)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["engine"]["docs_completed_in_window_rank0"] >= 4


def test_bench_driver_flags_time_budget():
    """The driver's exact step flags (`--gpus 1 --steps 20 --warmup 5`) on the tiny
    model: a step is a fixed slice of completed documents, so the whole run is
    bounded and the reported time covers exactly the timed steps."""
    t0 = time.perf_counter()
    out = _run([sys.executable, "bench.py", "--gpus", "1", "--steps", "20", "--warmup", "5",
                "--model", "tiny-llama", "--docs-per-step", "2", "--max-num-seqs", "4",
                "--latency-runs", "2"], timeout=600)
    wall = time.perf_counter() - t0
    # ~80 s alone; the bound only has to catch an unbounded step (the round-1 failure
    # mode: 25 steps of 3,072 documents), with room for a CI host running the suite
    # under pytest-xdist
    assert wall < 590, wall
    assert out["steps"] == 20 and out["warmup"] == 5
    assert out["ms_per_step"] * 20 / 1e3 < wall
    assert out["engine"]["docs_completed_in_window_rank0"] >= 40
    assert out["per_doc"]["valid"] == 1.0
    # latency under load of the timed window's documents, the
    # service's deadline, the shaped-workload label, no docs/s baseline to divide by
    lat = out["loaded_latency_s"]
    assert {"p50", "p90", "p99", "max", "mean", "n"} <= set(lat)
    assert 0 < lat["p50"] <= lat["p90"] <= lat["p99"] <= lat["max"]
    assert lat["n"] == out["engine"]["docs_completed_in_window_rank0"]
    assert out["loaded_ttft_s"]["p50"] <= lat["p50"]
    assert out["latency_slo_s"] == 30.0 and isinstance(out["slo_met_p99"], bool)
    assert out["config"]["profile"] == "synthetic" and out["config"]["in_flight_per_replica"] == 4
    assert out["vs_baseline"] is None
    # host-side split of the timed window (scheduler, launch, device wait, post)
    host = out["engine"]["host_s"]
    assert {"pack_s", "launch_s", "overlap_s", "wait_s", "post_s", "execute_s"} <= set(host)
    assert out["config"]["admit"] == "during step" and host["overlap_s"] > 0
    assert all(v >= 0 for v in host.values())
    assert host["execute_s"] <= out["ms_per_step"] * 20 / 1e3 + 1.0


def test_bench_extra_phases_cpu():
    """after the timed window the 1-GPU run serves BASELINE config 3
    over real HTTP (/upload/ of generated pdf/xlsx/docx through uvicorn), config 5
    (the MoE model over a parsed pdf/xlsx stream) and the 70B-architecture latency
    phase, all in the same JSON line (tiny models of the same architectures here)."""
    out = _run([sys.executable, "bench.py", "--gpus", "1", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama", "--docs-per-step", "2", "--max-num-seqs", "4",
                "--latency-runs", "1", "--phases", "http_open,http,depth,mixtral,70b",
                "--depth-in-flight", "2", "--depth-docs", "2",
                "--http-open-rate", "3", "--http-open-warm", "2", "--http-open-measure", "4",
                "--http-idle-requests", "3", "--http-docs", "6",
                "--http-clients", "3", "--mixtral-model", "tiny-mixtral",
                "--mixtral-in-flight", "4", "--mixtral-warm", "2", "--mixtral-docs", "4",
                "--big-model", "tiny-llama70", "--big-latency-runs", "2",
                # the default budget is sized for the GPU; tiny CPU models on a loaded
                # test host need more for the five phases
                "--phase-budget", "700"], timeout=900,
               # the service's 30 s generation deadline (rfq_agent.py:69) is for a GPU
               # engine; a tiny CPU model on a loaded test host can take longer
               RFQ_REQUEST_TIMEOUT_S="600")
    ph = out["phases"]
    o = ph["http_open_loop"]
    assert o["status"] == "ok", o
    assert o["offered_rate"] == 3 and o["requests"] > 0, o
    # requests a loaded CPU host leaves in flight at the phase deadline are counted
    # apart ("unfinished"); a failure is a service-side error or a broken connection
    assert o["failed"] == 0, (o.get("failed_by"), o.get("failed_s"), o.get("http_latency_s"))
    assert o["requests"] >= o["failed"] + o["unfinished"]
    assert o["burst_depth"] == 3 and o["engine_depth"] is not None
    assert o["layout"] == "api process + engine process" and o["responses"] >= o["docs"]
    # every request that ended inside the run came back valid; on a loaded CPU host the
    # tiny model's responses can all land after the 4 s window, so the in-window docs/s
    # is checked only when responses fell inside it
    assert o["requests"] - o["failed"] - o["unfinished"] > 0, o
    if o["responses"]:
        assert o["docs_per_s"] > 0 and o["valid"] == 1.0 and o["http_vs_engine"] > 0, o
    assert o["http_latency_s"] is None or o["http_latency_s"]["p50"] > 0
    assert o["failed_by"] == {}, o
    # the metric's p50 /parse-text/ comes from HTTP responses
    idle = o["idle"]
    assert idle["requests"] == 3 and idle["valid"] == 3, idle
    assert idle["client_p50_s"] > 0 and idle["x_process_time_p50_s"] > 0
    assert idle["client_p50_s"] >= idle["x_process_time_p50_s"] * 0.9
    assert out["p50_parse_text_latency_s"] == idle["client_p50_s"]
    assert out["p50_parse_text_source"].startswith("HTTP POST /parse-text/")
    assert out["p50_x_process_time_s"] == idle["x_process_time_p50_s"]
    assert out["p50_engine_latency_s"] > 0
    dp = ph["latency_bounded_depth"]
    assert dp["status"] == "ok" and dp["in_flight"] == 2 and dp["docs"] >= 2, dp
    assert dp["docs_per_s"] > 0 and dp["loaded_latency_s"]["p50"] > 0 and dp["valid"] == 1.0
    h = ph["http_upload"]
    assert h["status"] == "ok" and h["docs"] == 6 and h["valid"] == 1.0, h
    assert h["docs_per_s"] > 0 and h["http_latency_s"]["n"] == 6
    m = ph["mixtral"]
    assert m["status"] == "ok" and m["model"] == "tiny-mixtral", m
    assert m["docs"] >= 4 and m["formats"] == ["pdf", "xlsx"] and m["per_doc"]["valid"] == 1.0
    assert m["loaded_latency_s"]["p50"] > 0
    b = ph["llama3_70b"]
    assert b["status"] == "ok" and b["runs"] == 2 and b["p50_parse_text_latency_s"] > 0, b
    # the fixed latency set is the reference's recorded prompts
    assert b["latency_set"].startswith("reference prompts")
    assert [r["row"] for r in b["per_row"]] == [1, 2] and all(r["sampled"] > 0 for r in b["per_row"])
    assert b["p50_at_reference_steps_s"] > 0
    assert out["value"] > 0 and out["steps"] == 1


def test_bench_phases_auto_only_on_one_gpu_8b():
    sys.path.insert(0, ROOT)
    import bench

    class A:
        phases, tp, model = "auto", 1, "llama3-8b"
    assert bench._phase_list(A, 1) == ["http_open", "http", "depth", "mixtral", "70b"]
    assert bench._phase_list(A, 8) == [] and bench._phase_list(A, 2) == []
    A.model = "tiny-llama"
    assert bench._phase_list(A, 1) == []
    A.phases = "none"
    assert bench._phase_list(A, 1) == []


def test_http_phase_releases_the_engine():
    """The 1-GPU run frees the 8B engine after the HTTP phase before it builds Mixtral
    (an engine kept alive by the API's module globals ran the next phase out of HBM)."""
    import gc
    import weakref

    sys.path.insert(0, ROOT)
    from replisense_rfq_amd.benchmarks.phases import http_upload_phase
    from replisense_rfq_amd.engine.engine import LLMEngine
    from replisense_rfq_amd.utils.config import EngineConfig

    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", max_num_seqs=4))
    res = http_upload_phase(eng, n_docs=2, clients=2, client_procs=1, parse_procs=1,
                            budget_s=120)
    assert res["status"] == "ok", res
    wr = weakref.ref(eng)
    del eng
    import time

    t_end = time.time() + 10.0        # the server / parser threads wind down asynchronously
    while True:
        gc.collect()
        if wr() is None or time.time() > t_end:
            break
        time.sleep(0.2)
    assert wr() is None, [type(r).__name__ for r in gc.get_referrers(wr())]


@pytest.mark.timeout(1200)
def test_bench_default_gpus8_flow_gloo():
    """the driver's 8-GPU flow -- `bench.py --gpus 8` self-launching
    8 ranks, DP=8 replicas for the docs/s window, then ONE TP=8 group for the
    latency phase -- on gloo with tiny models of the same architectures.  The JSON
    line carries the DP docs/s, the tp_latency block with car_status, the
    in-window post-processing counts and the affinity report."""
    out = _run([sys.executable, "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "0",
                "--model", "tiny-llama", "--tp-latency-model", "tiny-llama70",
                "--tp-latency-runs", "1", "--tp-docs", "2", "--tp-in-flight", "2",
                "--docs-per-step", "1", "--max-num-seqs", "2", "--latency-runs", "1"],
               timeout=1150, threads=1)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["value"] > 0 and out["config"]["global_batch"] == 8
    assert out["postprocess"]["validated"] >= 1 and out["postprocess"]["failed"] == 0
    assert out["config"]["counted"] == "validated in window"
    tpl = out["tp_latency"]
    assert tpl["status"] == "ok", tpl
    assert tpl["parallelism"] == "tp8" and tpl["p50_parse_text_latency_s"] > 0
    assert isinstance(tpl["car_status"], str) and tpl["car_status"]
    assert "status" in out["engine"]["affinity"]


def test_bench_tp_latency_car_fallback():
    """A custom all-reduce flag timeout in the TP phase (injected on rank 0: RFQ_FAULT
    car_error fires only while the custom all-reduce is configured) re-forms the group
    on RCCL-path all-reduces and measures again: the phase still reports its numbers,
    says why it fell back, and the DP docs/s fields stand."""
    os.environ["RFQ_FAULT"] = "car_error:3"
    try:
        out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                    "--model", "tiny-llama", "--tp-latency-model", "tiny-llama-tp",
                    "--tp-latency-runs", "2", "--tp-docs", "2", "--tp-in-flight", "2"] + SMALL)
    finally:
        os.environ.pop("RFQ_FAULT", None)
    tpl = out["tp_latency"]
    assert tpl["status"] == "ok", tpl
    assert "injected flag timeout" in tpl["car_fallback"], tpl
    assert tpl["custom_allreduce"] is False and "re-formed on RCCL" in tpl["car_status"]
    assert tpl["runs"] == 2 and tpl["p50_parse_text_latency_s"] > 0
    assert tpl["docs"] == 2 and tpl["per_doc"]["valid"] == 1.0
    assert out["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_bench_tp_latency_car_fallback_one_gpu():
    """The RCCL fallback on the GPU path: two ranks share one MI355X over gloo with the
    custom IPC all-reduce live; an injected flag timeout on rank 0 makes every rank close
    its custom all-reduce region and rebuild the TP engine without it."""
    import torch

    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    env_extra = {"RFQ_DIST_BACKEND": "gloo", "RFQ_FAULT": "car_error:3"}
    os.environ.update(env_extra)
    try:
        out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0",
                    "--model", "tiny-llama", "--kv-fraction", "0.05", "--no-graphs",
                    "--tp-latency-model", "tiny-llama-tp", "--tp-latency-runs", "2",
                    "--tp-docs", "4", "--tp-in-flight", "2"] + SMALL,
                   timeout=380)
    finally:
        for k in env_extra:
            os.environ.pop(k, None)
    tpl = out["tp_latency"]
    assert tpl["status"] == "ok", tpl
    assert "injected flag timeout" in tpl["car_fallback"], tpl
    assert tpl["custom_allreduce"] is False and tpl["p50_parse_text_latency_s"] > 0
    assert tpl["per_doc"]["valid"] == 1.0
