#!/bin/bash
# balanced prefill with the own item's metadata from the enumeration: tests, stamps, timings
set -o pipefail
mkdir -p gpurun_out/bal
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/kernels/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/bal/tests_meta.log 2>&1 || exit $?
SHAPES=1x2912x8x1,1x4096x8x1 SMALL=3 timeout -k 10 120 python -u tools/prefill_timing.py \
  > gpurun_out/bal/timing_meta.jsonl 2>/dev/null || exit $?
PREFIX=416 SHAPES=1x2912x8x1,1x4096x8x1,2x2048x8x1 timeout -k 10 120 python -u tools/bench_prefill.py \
  > gpurun_out/bal/meta_rank.jsonl 2>/dev/null || exit $?
SHAPES=1x2912x8x1,1x4096x8x1,2x2048x8x1 timeout -k 10 120 python -u tools/bench_prefill.py \
  > gpurun_out/bal/meta_rank_p0.jsonl 2>/dev/null || exit $?
echo done
