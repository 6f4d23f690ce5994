#!/bin/bash
# after the items rule: prefill tests, 70B TP=1 short prompts and the rank PDF shape in auto
set -o pipefail
mkdir -p gpurun_out/bal
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/kernels/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/bal/tests_rule.log 2>&1 || exit $?
SHAPES=1x400x64x8,1x512x64x8,1x300x64x8 timeout -k 10 120 python -u tools/bench_prefill.py \
  > gpurun_out/bal/rule_70b.jsonl 2>/dev/null || exit $?
PREFIX=416 SHAPES=1x2912x8x1,1x4096x8x1,2x2048x8x1 timeout -k 10 120 python -u tools/bench_prefill.py \
  > gpurun_out/bal/rule_rank.jsonl 2>/dev/null || exit $?
echo done
