#!/bin/bash
# engine form timing pieces (8B, ctx 1024): gate|up alone (1 and 32 layers) and the whole
# layer, one or two loader waves, consumers' compute or the loader's stream switched off
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
O=gpurun_out/eng_parts2.jsonl
: > $O
for f in 16 112; do
  timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --layers 1 --modes raw:8 --flags $f --iters 200 >> $O 2>&1 || { tail -20 $O; exit 1; }
  timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes raw:8,raw:31 --flags $f --iters 20 >> $O 2>&1 || { tail -20 $O; exit 1; }
done
timeout -k 10 120 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes 0,engine --iters 20 >> $O 2>&1 || { tail -20 $O; exit 1; }
grep '^{' $O
timeout -k 10 60 python -u tools/diag_engine.py 8 0 > gpurun_out/diag_eng_0.json 2>&1 || { tail -5 gpurun_out/diag_eng_0.json; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/diag_eng_0.json'))
print('issued', d['issued'][:12]); print('published', d['published'][:12]); print('consumed', d['consumed'][:12]); print('end', d['wave_end'], 'epi', d['epilogue'])"
