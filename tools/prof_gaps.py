"""Busy/idle breakdown of the tail of a rocprofv3 kernel trace.

Usage: python tools/prof_gaps.py <prof dir> [window_s]

Takes the dispatches of the last ``window_s`` seconds of the trace (default 3 s: the
single-request latency runs at the end of ``bench.py``), and reports wall time, the
union of kernel intervals (GPU busy), the idle gaps between consecutive kernels, and
per-kernel totals inside that window.  Used for the latency-path profile, where
inter-kernel gaps are a visible share of a ~4 ms decode step.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def _short(n):
    if n is None:
        return "-"
    n = n.split("(")[0]
    return n if len(n) <= 60 else n[:57] + "..."


def main(d, window_s=3.0):
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not traces:
        print("no kernel_trace.csv under", d)
        return
    ev = []
    with open(traces[0]) as f:
        for r in csv.DictReader(f):
            s = int(_col(r, "Start_Timestamp", "BeginNs", "Start"))
            e = int(_col(r, "End_Timestamp", "EndNs", "End"))
            ev.append((s, e, _col(r, "Kernel_Name", "KernelName", "Name")))
    ev.sort()
    t_end = max(e for _, e, _ in ev)
    lo = t_end - int(window_s * 1e9)
    ev = [x for x in ev if x[0] >= lo]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    where = defaultdict(lambda: [0, 0])       # (kernel before, kernel after) of big gaps
    prev_n = None
    per = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        per[n][0] += 1
        per[n][1] += e - s
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            if s - cur_e >= 20_000:
                k = (_short(prev_n), _short(n))
                where[k][0] += 1
                where[k][1] += s - cur_e
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_n = n
    busy += cur_e - cur_s
    wall = ev[-1][1] - ev[0][0]
    gaps.sort()
    small = [g for g in gaps if g < 20_000]
    big = [g for g in gaps if g >= 20_000]
    print(f"window {window_s:.1f} s: {len(ev)} dispatches, wall {wall / 1e6:.1f} ms, "
          f"GPU busy {busy / 1e6:.1f} ms ({100 * busy / wall:.1f} %)")
    if small:
        print(f"gaps < 20 us (between kernels of a step): {len(small)} summing "
              f"{sum(small) / 1e6:.1f} ms, median {small[len(small) // 2] / 1e3:.2f} us")
    print(f"gaps >= 20 us (host waits between steps): {len(big)} summing {sum(big) / 1e6:.1f} ms")
    if where:
        print("\n| big gap after | before | count | total ms |\n|---|---|---|---|")
        for (a, b), (c, t) in sorted(where.items(), key=lambda kv: -kv[1][1])[:8]:
            print(f"| `{a}` | `{b}` | {c} | {t / 1e6:.1f} |")
    print("\n| kernel | calls | total ms | avg us | % of busy |\n|---|---|---|---|---|")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:25]:
        nm = n if len(n) <= 90 else n[:87] + "..."
        print(f"| `{nm}` | {c} | {t / 1e6:.2f} | {t / c / 1e3:.1f} | {100 * t / busy:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof",
         float(sys.argv[2]) if len(sys.argv) > 2 else 3.0)
