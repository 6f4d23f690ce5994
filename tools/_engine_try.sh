#!/bin/bash
# engine form of the persistent decode layers: first a 2-layer bench (hang / fault check),
# then the GPU tests, then the whole-step A/B at 8B and the 70B TP=8 rank shape
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/bench_persist.py --shape 8b --ctx 1024 --layers 2 --modes 0,engine --iters 10 > gpurun_out/eng_try.jsonl 2>&1 || { tail -20 gpurun_out/eng_try.jsonl; exit 1; }
cat gpurun_out/eng_try.jsonl | grep '^{'
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/kernels/test_decode_persist_gpu.py -k engine > gpurun_out/eng_tests.log 2>&1 || { tail -40 gpurun_out/eng_tests.log; exit 1; }
tail -5 gpurun_out/eng_tests.log
timeout -k 10 200 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes 0,all,engine --iters 30 > gpurun_out/eng_8b.jsonl 2>&1 || { tail -20 gpurun_out/eng_8b.jsonl; exit 1; }
grep '^{' gpurun_out/eng_8b.jsonl
timeout -k 10 200 python -u tools/bench_persist.py --shape 70b --ctx 1024 --modes 0,engine --iters 30 > gpurun_out/eng_70b.jsonl 2>&1 || { tail -20 gpurun_out/eng_70b.jsonl; exit 1; }
grep '^{' gpurun_out/eng_70b.jsonl
