"""NUMA pinning of rank processes (utils/affinity.py) on a synthetic sysfs tree:
2 NUMA nodes x 4 GPUs, KFD CPU agents interleaved, visibility filters."""
import os

from replisense_rfq_amd.utils import affinity as af


def _tree(tmp_path, gpus_per_node=4, cores=16):
    kfd, pci = tmp_path / "kfd", tmp_path / "pci"
    n = 0
    for numa in range(2):
        d = kfd / str(n)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count 16\nsimd_count 0\n")
        n += 1
        for g in range(gpus_per_node):
            bus = 0x10 * (numa * gpus_per_node + g + 1)
            d = kfd / str(n)
            d.mkdir(parents=True)
            (d / "properties").write_text(
                f"simd_count 1024\ndomain 0\nlocation_id {bus << 8}\n")
            n += 1
            p = pci / ("0000:%02x:00.0" % bus)
            p.mkdir(parents=True)
            (p / "numa_node").write_text(f"{numa}\n")
            lo = numa * cores
            (p / "local_cpulist").write_text(f"{lo}-{lo + cores - 1}\n")
    return str(kfd), str(pci)


def test_parse_cpulist():
    assert af.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]


def test_eight_gpus_two_sockets(tmp_path, monkeypatch):
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    kfd, pci = _tree(tmp_path)
    assert len(af.gpu_agents(kfd)) == 8
    plans = [af.plan_affinity(r, kfd, pci) for r in range(8)]
    assert [p["numa_node"] for p in plans] == [0] * 4 + [1] * 4
    assert plans[0]["cpus"] == [0, 1, 2, 3] and plans[7]["cpus"] == [28, 29, 30, 31]
    seen = [c for p in plans for c in p["cpus"]]
    assert sorted(seen) == list(range(32))            # disjoint, covering every core
    assert af.plan_affinity(8, kfd, pci) is None


def test_visible_devices_filter(tmp_path, monkeypatch):
    kfd, pci = _tree(tmp_path)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    p = af.plan_affinity(0, kfd, pci)
    assert p["numa_node"] == 1 and p["gpus_on_node"] == 1 and p["cpus"] == list(range(16, 32))


def test_pin_without_topology_is_a_noop(monkeypatch):
    before = os.sched_getaffinity(0)
    monkeypatch.setattr(af, "KFD_NODES", "/nonexistent")
    monkeypatch.setattr(af, "plan_affinity", lambda r: None)
    assert af.pin_to_gpu(0)["status"] == "no topology"
    assert os.sched_getaffinity(0) == before
    monkeypatch.setenv("RFQ_PIN_NUMA", "0")
    assert af.pin_to_gpu(0)["status"] == "off"


def test_restore_affinity_undoes_pinning(monkeypatch):
    """processes that inherit the engine's NUMA pinning but are no part of the
    engine (API server, load generators) put the original mask back."""
    import os

    from replisense_rfq_amd.utils import affinity

    if not hasattr(os, "sched_setaffinity"):
        return
    orig = os.sched_getaffinity(0)
    monkeypatch.setenv(affinity.ORIG_ENV, ",".join(str(c) for c in sorted(orig)))
    try:
        os.sched_setaffinity(0, {min(orig)})
        assert affinity.restore_affinity()
        assert os.sched_getaffinity(0) == orig
    finally:
        os.sched_setaffinity(0, orig)
    monkeypatch.delenv(affinity.ORIG_ENV)
    assert not affinity.restore_affinity()
