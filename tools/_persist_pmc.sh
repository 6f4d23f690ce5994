#!/bin/bash
# PMC counters of one persistent GEMV stage vs its row-streaming launch (1 layer, 8B gate|up)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp
R=$GRAFT_REPO_ROOT
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
for m in raw:8 rows:gu; do
  tag=${m/:/_}
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmc/$tag -o run --output-format csv -- python3 $R/tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --iters 20 --modes $m > $R/gpurun_out/pmc/$tag.log 2>&1 || exit 1
done
cd $R
python3 - <<'PY'
import csv, glob, collections
for tag in ("raw_8", "rows_gu"):
    files = glob.glob(f"gpurun_out/pmc/{tag}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if "decode_persist" in k or "gemv_rows" in k:
                agg[k[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
                n[k[:60]] += 1
    for k, d in agg.items():
        print(tag, k, {c: round(v / max(1, n[k] / 8)) for c, v in d.items()})
PY
