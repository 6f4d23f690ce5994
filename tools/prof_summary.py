"""Summarise rocprofv3 --kernel-trace --stats CSVs into a markdown table."""
import csv
import glob
import os
import sys


def main(d):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        print("no kernel_stats.csv under", d)
        return
    rows = list(csv.DictReader(open(stats[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
        name = r["Name"]
        if len(name) > 90:
            name = name[:87] + "..."
        t = float(r["TotalDurationNs"])
        print(f"| `{name}` | {r['Calls']} | {t / 1e6:.2f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{100 * t / tot:.1f} |")
    print(f"\nTotal GPU kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} "
          f"dispatches")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
