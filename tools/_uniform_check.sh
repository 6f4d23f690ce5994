#!/bin/bash
# after the wave-uniform control-word fixes: attention oracle tests, batch-1 attention
# latency, the persistent forms' whole-step A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "attn_decode" tests/kernels/test_decode_persist_gpu.py > gpurun_out/uni_tests.log 2>&1 || { tail -30 gpurun_out/uni_tests.log; exit 1; }
tail -2 gpurun_out/uni_tests.log
LAT_SP=1 timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/attn_lat_uni.jsonl 2> gpurun_out/attn_lat_uni.err || exit 1
cat gpurun_out/attn_lat_uni.jsonl
timeout -k 10 300 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes 0,all,ao,engine --iters 30 > gpurun_out/uni_persist.jsonl 2>&1 || { tail -20 gpurun_out/uni_persist.jsonl; exit 1; }
grep '^{' gpurun_out/uni_persist.jsonl
