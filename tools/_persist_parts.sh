#!/bin/bash
# persistent decode: serialized case walk, the GPU tests, then component timings
set -o pipefail
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 200 python -u tools/diag_persist.py tiny all > gpurun_out/diag.log 2>&1 || { tail -5 gpurun_out/diag.log; exit 1; }
echo diag-ok
timeout -k 10 420 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_decode_persist_gpu.py > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 1; }
tail -2 gpurun_out/persist_tests.log
B="timeout -k 10 300 python -u tools/bench_persist.py --shape 8b --ctx 1024"
$B --modes 0,all,ao,raw:31,raw:4,raw:6,raw:8,raw:16,raw:24 > gpurun_out/parts_8b.jsonl 2> gpurun_out/parts_8b.err || exit 1
$B --modes raw:8,raw:16,raw:4,rows:gu,rows:down,rows:o --layers 1 --iters 200 > gpurun_out/parts_8b_1l.jsonl 2>> gpurun_out/parts_8b.err || exit 1
timeout -k 10 300 python -u tools/bench_persist.py --shape tp8 --ctx 1024 --modes 0,all,ao > gpurun_out/parts_tp8.jsonl 2>> gpurun_out/parts_8b.err || exit 1
cat gpurun_out/parts_*.jsonl
