#!/bin/bash
# engine form: correctness, CU-0 timeline, gate|up alone and the whole step (8B, 70B rank)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_decode_persist_gpu.py -k engine > gpurun_out/eng_tests.log 2>&1 || { tail -30 gpurun_out/eng_tests.log; exit 1; }
tail -2 gpurun_out/eng_tests.log
timeout -k 10 60 python -u tools/diag_engine.py 8 0 > gpurun_out/diag_eng_f0.json 2>&1 || { tail -5 gpurun_out/diag_eng_f0.json; exit 1; }
python3 - <<'PY'
import json, numpy as np
d = json.loads([l for l in open("gpurun_out/diag_eng_f0.json") if l.startswith("{")][-1])
iss = [(b - a) for a, b in zip(d["issue_start"], d["issued"]) if a is not None and b is not None]
st = [x for x in d["issue_start"] if x is not None]
print("issue16", round(float(np.mean(iss)), 3), "slot gap", round(float(np.mean(np.diff(st))), 3), "end", d["wave_end"], "clock", d["clock_mhz"])
PY
O=gpurun_out/eng_round.jsonl
: > $O
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --modes raw:8,rows:gu --flags 16 --iters 200 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes raw:8,raw:31 --flags 16 --iters 20 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes 0,engine --iters 30 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python -u tools/bench_persist.py --shape 70b --ctx 1024 --modes 0,engine --iters 30 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep '^{' $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['layers'], d['mode'], d['flags'], d.get('us_per_layer'), d.get('ms_per_step'), d.get('rel_vs_first'), d.get('kernel_errors'))"
