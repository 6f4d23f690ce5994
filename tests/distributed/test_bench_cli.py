"""The bench.py driver contract, rehearsed on CPU with gloo: torchrun launch, one
JSON line from rank 0 with the required keys, TP and DP layouts (the GPU box
runs the same script over RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("tp,par", [(2, "dp1-tp2"), (1, "dp2")])
def test_bench_torchrun_gloo(tp, par):
    model = "tiny-llama-tp" if tp > 1 else "tiny-llama"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py",
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--model", model, "--tp", str(tp),
           "--docs-per-step", "2", "--max-num-seqs", "2", "--latency-runs", "2"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == par
    assert out["per_doc"]["valid"] == 1.0 and out["p50_parse_text_latency_s"] > 0
