#!/bin/bash
# PMC counters of the engine form, one layer of gate|up (8B): full, and with no weight
# stream and no consumer compute (protocol only)
set -o pipefail
mkdir -p gpurun_out/pmc_eng
cd /tmp
R=$GRAFT_REPO_ROOT
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for f in 16 112; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_eng/f$f -o run --output-format csv -- python3 $R/tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --iters 20 --modes raw:8 --flags $f > $R/gpurun_out/pmc_eng/f$f.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for tag in ("f16", "f112"):
    files = glob.glob(f"gpurun_out/pmc_eng/{tag}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "decode_engine" in k:
                agg[k[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
                n[k[:40]] += 1
    for k, d in agg.items():
        print(tag, k, {c: round(v / max(1, n[k] / 8)) for c, v in d.items()})
PY
