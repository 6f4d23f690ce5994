"""GPU busy fraction and inter-kernel gaps from a rocprofv3 kernel_trace.csv,
over the last `--window` seconds of the run (e.g. the single-request latency
phase of bench.py)."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window", type=float, default=3.0)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t_end = rows[-1][1]
    lo = t_end - int(a.window * 1e9)
    win = [r for r in rows if r[0] >= lo]
    busy = 0
    cur_s, cur_e = win[0][0], win[0][1]
    gaps = []
    for s, e, _ in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = win[-1][1] - win[0][0]
    gaps.sort()
    big = [g for g in gaps if g > 20_000]
    print(f"kernels={len(win)} span_ms={span / 1e6:.1f} busy={busy / span:.3f} "
          f"gaps={len(gaps)} median_gap_us={gaps[len(gaps) // 2] / 1e3 if gaps else 0:.1f} "
          f"gaps>20us={len(big)} sum_big_ms={sum(big) / 1e6:.1f}")


if __name__ == "__main__":
    main()
