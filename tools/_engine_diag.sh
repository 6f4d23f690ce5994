#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for f in 0 64; do
  timeout -k 10 60 python -u tools/diag_engine.py 8 $f > gpurun_out/diag_eng_f$f.json 2>&1 || { tail -5 gpurun_out/diag_eng_f$f.json; exit 1; }
done
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --modes raw:8 --flags 528 --iters 200 > gpurun_out/eng_sleep.jsonl 2>&1
python3 - <<'PY'
import json, numpy as np
for f in (0, 64):
    d = json.loads([l for l in open(f"gpurun_out/diag_eng_f{f}.json") if l.startswith("{")][-1])
    iss = [(b - a) for a, b in zip(d["issue_start"], d["issued"]) if a is not None and b is not None]
    st = [x for x in d["issue_start"] if x is not None]
    print(f, "issue16 mean", round(float(np.mean(iss)), 3) if iss else None, "slot gap", round(float(np.mean(np.diff(st))), 3) if len(st) > 1 else None,
          "end", d["wave_end"], "epi", d["epilogue"], "clock", d["clock_mhz"])
PY
grep '^{' gpurun_out/eng_sleep.jsonl
