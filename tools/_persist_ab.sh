#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 200 python -u tools/bench_persist.py --shape 8b --ctx 1024"
for f in 0 8; do
  $B --modes raw:8,raw:16,raw:4 --layers 1 --iters 200 --flags $f >> gpurun_out/ab_1l.jsonl 2>> gpurun_out/ab.err || exit 1
  $B --modes all,raw:24 --flags $f >> gpurun_out/ab_32l.jsonl 2>> gpurun_out/ab.err || exit 1
done
cat gpurun_out/ab_1l.jsonl gpurun_out/ab_32l.jsonl
