#!/bin/bash
# engine form with two loader waves (flags bit 7): gate|up alone, the layer, the step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
O=gpurun_out/eng_nl2.jsonl
: > $O
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --modes raw:8 --flags 144 --iters 200 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes raw:8,raw:31,raw:16,raw:1,raw:4,raw:2 --flags 144 --iters 20 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes raw:16,raw:1,raw:4,raw:2 --flags 16 --iters 20 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 200 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes engine --flags 128 --iters 30 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep '^{' $O | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['layers'], d['mode'], d['flags'], d.get('us_per_layer'), d.get('ms_per_step'), d.get('rel_vs_first'), d.get('kernel_errors'))"
