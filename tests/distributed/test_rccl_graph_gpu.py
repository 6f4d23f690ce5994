"""RCCL collectives captured inside a hipGraph (what the TP decode graphs do with
the vocab-parallel sampler's all-gather and the row-parallel all-reduce above the
custom kernel's size cap).  RCCL refuses two ranks on one device, so this runs a
one-rank RCCL group in a child process: it checks the capture mechanism of this
torch/RCCL stack, and the graph replays the collective with fresh inputs."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r"""
import datetime, os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ["RFQ_ROOT"])
from replisense_rfq_amd.parallel.tp import TPContext
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, timeout=datetime.timedelta(seconds=60),
                        device_id=torch.device("cuda", 0))
tp = TPContext(rank=0, world=1, group=dist.group.WORLD)
x = torch.zeros(4, 16, device="cuda")
g_out = torch.empty(1, 4, 16, device="cuda")
s = torch.zeros(1 << 20, dtype=torch.bfloat16, device="cuda")
def body():
    dist.all_gather_into_tensor(g_out.flatten(0, 1), x)
    dist.all_reduce(s)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    body()
torch.cuda.current_stream().wait_stream(side)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
for k in range(3):
    x.fill_(float(k + 1)); s.fill_(float(k + 2))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(g_out[0], x), (k, g_out[0, 0, 0].item())
    assert float(s[0]) == float(k + 2)
dist.destroy_process_group()
print("RCCL_GRAPH_OK")
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(180)
def test_rccl_collectives_in_hipgraph():
    import torch

    if torch.cuda.device_count() < 1:       # no GPU init in the pytest process
        pytest.skip("no GPU")
    env = dict(os.environ, RFQ_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True,
                       timeout=150, env=env)
    assert r.returncode == 0 and "RCCL_GRAPH_OK" in r.stdout, r.stderr[-3000:]
