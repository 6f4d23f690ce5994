"""Per-kernel time over the last ``window_s`` seconds of a rocprofv3 --kernel-trace run
(e.g. the timed single-request runs at the end of a tool, after start-up tuning and
graph capture), as a markdown table; with ``steps`` the per-step time of each kernel.

Usage: python tools/trace_window_stats.py <prof dir> <window_s> [steps]
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def main(d: str, window_s: float, steps: int = 0) -> int:
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        print(f"no kernel_trace.csv under {d}")
        return 1
    rows = []
    with open(paths[0], newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    end = max(r[1] for r in rows)
    lo = end - int(window_s * 1e9)
    win = [r for r in rows if r[0] >= lo]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[n][0] += 1
        agg[n][1] += e - s
    busy = sum(v[1] for v in agg.values())
    span = max(r[1] for r in win) - min(r[0] for r in win)
    print(f"window {window_s:.2f} s: {len(win)} dispatches, kernel time {busy / 1e6:.2f} ms, "
          f"span {span / 1e6:.2f} ms (GPU busy {100 * busy / max(1, span):.1f} %)"
          + (f", {steps} steps" if steps else ""))
    print()
    hdr = "| kernel | calls | total ms | avg us | % |" + (" us per step |" if steps else "")
    print(hdr)
    print("|---|---|---|---|---|" + ("---|" if steps else ""))
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        name = n if len(n) <= 90 else n[:87] + "..."
        line = f"| `{name}` | {c} | {t / 1e6:.2f} | {t / c / 1e3:.1f} | {100 * t / busy:.1f} |"
        if steps:
            line += f" {t / 1e3 / steps:.1f} |"
        print(line)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 0))
