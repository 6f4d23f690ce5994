"""hipGraph evidence from a rocprofv3 ``--hip-trace --kernel-trace`` run.

Usage: python tools/graph_trace_summary.py <prof dir> [window_s]

Joins the HIP API trace with the kernel trace on ``Correlation_Id``: every kernel
dispatched by a ``hipGraphLaunch`` carries that call's correlation id, every
eagerly launched kernel carries its own ``hipLaunchKernel``/``hipExtModuleLaunchKernel``
id.  Over the last ``window_s`` seconds (the single-request latency runs at the
end of ``bench.py``) it reports

* hipGraphLaunch calls and the kernels each one dispatched (= one decode step),
* kernels launched eagerly (prefill steps, one-off copies),
* the HIP API calls the host made per graph-launched step,

so "decode runs as hipGraphs" is read off the trace, not asserted.
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys
from collections import Counter, defaultdict


def _one(d, pat):
    hits = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return hits[0] if hits else None


def _rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def main(d: str, window_s: float = 3.0) -> int:
    kpath, apath = _one(d, "*kernel_trace.csv"), _one(d, "*hip_api_trace.csv")
    if not kpath or not apath:
        print(f"need kernel_trace.csv and hip_api_trace.csv under {d}")
        return 1
    api = {}
    api_rows = []
    for r in _rows(apath):
        cid = int(r["Correlation_Id"])
        fn = r["Function"]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        api[cid] = fn
        api_rows.append((t0, t1, fn))
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Correlation_Id"]),
             r["Kernel_Name"]) for r in _rows(kpath)]
    kern.sort()
    t_end = kern[-1][1]
    lo = t_end - int(window_s * 1e9)
    win = [k for k in kern if k[0] >= lo]
    by_launch = defaultdict(list)
    for s, e, cid, name in win:
        by_launch[cid].append((s, e, name))
    graph_ids = [c for c in by_launch if api.get(c, "").startswith("hipGraphLaunch")]
    eager = Counter(api.get(c, "?") for c in by_launch if c not in set(graph_ids))
    per_graph = [len(by_launch[c]) for c in graph_ids]
    span = [max(e for _, e, _ in by_launch[c]) - min(s for s, _, _ in by_launch[c])
            for c in graph_ids]
    n_graph_k = sum(per_graph)
    api_win = Counter(fn for t0, _, fn in api_rows if t0 >= lo)
    print(f"# hipGraph launch evidence (last {window_s:.1f} s of the trace)\n")
    print(f"- kernels in window: {len(win)}")
    print(f"- hipGraphLaunch calls: {len(graph_ids)}; kernels they dispatched: {n_graph_k} "
          f"({100.0 * n_graph_k / max(1, len(win)):.1f} % of the window's kernels)")
    if per_graph:
        print(f"- kernels per graph launch: median {statistics.median(per_graph):.0f}, "
              f"min {min(per_graph)}, max {max(per_graph)}")
        print(f"- GPU span per graph launch (first kernel start -> last kernel end): "
              f"median {statistics.median(span) / 1e3:.1f} us")
    print(f"- eagerly launched kernels by API: {dict(eager.most_common(8))}")
    print("\n## HIP API calls in the window\n")
    print("| function | calls |")
    print("|---|---|")
    for fn, n in api_win.most_common(15):
        print(f"| `{fn}` | {n} |")
    if graph_ids:
        first = by_launch[graph_ids[len(graph_ids) // 2]]
        names = Counter(n.split("(")[0][:70] for _, _, n in first)
        print("\n## Kernels of one graph-launched decode step\n")
        print("| kernel | count |")
        print("|---|---|")
        for n, c in names.most_common(20):
            print(f"| `{n}` | {c} |")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 3.0))
