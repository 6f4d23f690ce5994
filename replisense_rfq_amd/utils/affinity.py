"""Pin a rank process to the CPU cores next to its GPU.

One process per GPU: on an 8-GPU MI355X node the eight rank processes (and the
prompt-producer and post-processing processes each one spawns) all run Python step
loops whose host gaps land straight on the GPU timeline (``engine.host_s``).  Left
to the scheduler they migrate across sockets, pay remote-NUMA memory latency on
every pinned-host copy, and several can pile onto one socket while the other idles.

``pin_to_gpu(local_rank)`` runs BEFORE anything touches HIP (it reads only sysfs):

  * the GPU agents come from the KFD topology (``/sys/class/kfd/kfd/topology/nodes``,
    nodes with SIMDs), in node order -- the order the ROCm runtime enumerates them --
    filtered by ``ROCR_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES``;
  * each agent's PCI function (``domain`` + ``location_id``) gives its NUMA node
    and ``local_cpulist`` (``/sys/bus/pci/devices/<bdf>/``);
  * the GPUs that share a NUMA node split that node's cores into equal, disjoint
    slices; this rank takes its GPU's slice.

Children started afterwards (spawned producer / post processes) inherit the mask.
The result (cores, NUMA node) is reported in the bench JSON; every failure (no KFD,
no sysfs, a container without those CPUs) leaves the affinity untouched.
``RFQ_PIN_NUMA=0`` turns it off.
"""
from __future__ import annotations

import os

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
PCI_DEVICES = "/sys/bus/pci/devices"


def parse_cpulist(text: str) -> list[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: list[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _props(path: str) -> dict:
    d = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.strip().partition(" ")
                if v.strip().lstrip("-").isdigit():
                    d[k] = int(v)
    except OSError:
        pass
    return d


def gpu_agents(kfd_nodes: str = KFD_NODES) -> list[dict]:
    """GPU agents in KFD node order: [{'node', 'bdf'}]."""
    agents = []
    try:
        nodes = sorted(int(n) for n in os.listdir(kfd_nodes) if n.isdigit())
    except OSError:
        return agents
    for n in nodes:
        p = _props(os.path.join(kfd_nodes, str(n), "properties"))
        if p.get("simd_count", 0) <= 0:
            continue                                   # a CPU agent
        loc = p.get("location_id", 0)
        bdf = "%04x:%02x:%02x.%x" % (p.get("domain", 0), (loc >> 8) & 0xFF,
                                     (loc >> 3) & 0x1F, loc & 0x7)
        agents.append({"node": n, "bdf": bdf})
    return agents


def _visible(agents: list[dict]) -> list[dict]:
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var, "").strip()
        if v:
            try:
                idx = [int(x) for x in v.split(",") if x.strip()]
            except ValueError:
                return agents                          # UUID form: keep the full list
            agents = [agents[i] for i in idx if 0 <= i < len(agents)]
    return agents


def _pci_info(bdf: str, pci_devices: str = PCI_DEVICES) -> tuple[int, list[int]]:
    base = os.path.join(pci_devices, bdf)
    try:
        numa = int(open(os.path.join(base, "numa_node")).read().strip())
    except (OSError, ValueError):
        numa = -1
    try:
        cpus = parse_cpulist(open(os.path.join(base, "local_cpulist")).read())
    except (OSError, ValueError):
        cpus = []
    return numa, cpus


def plan_affinity(local_rank: int, kfd_nodes: str = KFD_NODES,
                  pci_devices: str = PCI_DEVICES) -> dict | None:
    """The cores this rank should run on: its GPU's NUMA-local cores, split evenly
    among the visible GPUs of the same NUMA node.  None if it cannot be determined."""
    all_agents = gpu_agents(kfd_nodes)
    agents = _visible(all_agents)
    if not agents or local_rank >= len(agents):
        return None
    info = [_pci_info(a["bdf"], pci_devices) for a in agents]
    numa, cpus = info[local_rank]
    if not cpus:
        return None
    peers = [i for i, (n, c) in enumerate(info) if n == numa and c == cpus]
    k, n = peers.index(local_rank), len(peers)
    per = max(1, len(cpus) // n)
    mine = cpus[k * per:(k + 1) * per] if k < n - 1 else cpus[k * per:]
    return {"gpu_bdf": agents[local_rank]["bdf"], "numa_node": numa,
            "cpus": mine or cpus, "node_cpus": len(cpus), "gpus_on_node": n}


ORIG_ENV = "RFQ_ORIG_AFFINITY"


def restore_affinity() -> bool:
    """Undo pin_to_gpu's NUMA pinning in a process that inherited it but is no part of
    the engine (HTTP API server, client / load-generator processes).  True if reset."""
    orig = os.environ.get(ORIG_ENV)
    if not orig or not hasattr(os, "sched_setaffinity"):
        return False
    try:
        os.sched_setaffinity(0, {int(c) for c in orig.split(",") if c})
    except OSError:
        return False
    return True


def pin_to_gpu(local_rank: int) -> dict:
    """Apply :func:`plan_affinity` to this process (call before any HIP call).
    Returns what was done, for the bench JSON."""
    if os.environ.get("RFQ_PIN_NUMA", "1") == "0":
        return {"status": "off"}
    if not hasattr(os, "sched_setaffinity"):
        return {"status": "unsupported"}
    plan = plan_affinity(local_rank)
    if plan is None:
        return {"status": "no topology"}
    allowed = os.sched_getaffinity(0)
    cpus = [c for c in plan["cpus"] if c in allowed]
    if not cpus:
        return {"status": "cores not in this container's cpuset", "numa_node": plan["numa_node"]}
    try:
        os.sched_setaffinity(0, cpus)
    except OSError as e:
        return {"status": f"failed: {e}"}
    # children that are not part of the engine (API server, load generators) put the
    # original mask back with restore_affinity(): they must not compete with the engine
    # for its few pinned cores
    os.environ.setdefault(ORIG_ENV, ",".join(str(c) for c in sorted(allowed)))
    return {"status": "pinned", "numa_node": plan["numa_node"], "cores": len(cpus),
            "first_core": cpus[0], "gpus_on_node": plan["gpus_on_node"]}
