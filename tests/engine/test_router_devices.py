"""DPRouter replica device mapping (an operator's HIP_VISIBLE_DEVICES and
cfg.device = "cuda:N" must survive the engine-process layout)."""
from types import SimpleNamespace

import pytest

from replisense_rfq_amd.engine.router import DPRouter


def _router(device="cuda", n=1, dpr=1):
    r = DPRouter.__new__(DPRouter)
    r.cfg = SimpleNamespace(device=device)
    r.n, r.dpr = n, dpr
    return r


@pytest.fixture
def clean_env(monkeypatch):
    for k in ("RFQ_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_default_is_identity(clean_env):
    assert _router()._devices(0) == "0"
    r = _router(n=4, dpr=2)
    assert [r._devices(i) for i in range(4)] == ["0,1", "2,3", "4,5", "6,7"]


def test_inherits_hip_visible_devices(clean_env):
    clean_env.setenv("HIP_VISIBLE_DEVICES", "3")
    assert _router()._devices(0) == "3"
    clean_env.setenv("HIP_VISIBLE_DEVICES", "4,5,6,7")
    r = _router(n=2, dpr=2)
    assert [r._devices(i) for i in range(2)] == ["4,5", "6,7"]


def test_cuda_index_selects_logical_device(clean_env):
    assert _router("cuda:1")._devices(0) == "1"
    clean_env.setenv("HIP_VISIBLE_DEVICES", "2,5")
    assert _router("cuda:1")._devices(0) == "5"


def test_rfq_devices_wins_and_bounds_checked(clean_env):
    clean_env.setenv("HIP_VISIBLE_DEVICES", "2,5")
    clean_env.setenv("RFQ_DEVICES", "7,6")
    assert _router()._devices(0) == "7"
    with pytest.raises(ValueError):
        _router(n=3)._devices(2)


def test_cpu_has_no_devices(clean_env):
    assert _router("cpu")._devices(0) == ""
