"""Run one kernel configuration repeatedly for a rocprofv3 --pmc pass, or summarise
the counters of such a pass.

  python tools/prof_one_kernel.py run prefill B S Hq Hkv      # the profiled program
  python tools/prof_one_kernel.py sum <prof dir> <kernel substring>
"""
import csv
import glob
import math
import os
import sys
from collections import defaultdict


def run(kind, *a):
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from tools import bench_prefill

    if kind == "prefill":
        B, S, Hq, Hkv = (int(x) for x in a)
        bench_prefill.run(B, S, Hq, Hkv, iters=5)
    torch.cuda.synchronize()


def summarise(d, sub):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        print("no counter_collection.csv under", d)
        return
    tot = defaultdict(float)
    n = defaultdict(int)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if sub not in r.get("Kernel_Name", ""):
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    for k in sorted(tot):
        print(f"{k:32s} {tot[k]:16.0f}  (dispatch rows {n[k]})")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*sys.argv[2:])
    else:
        summarise(sys.argv[2], sys.argv[3])
