#!/bin/bash
# balanced split-KV prefill (small_mode 3) vs auto: tests, phase stamps, rank-shape timings
set -o pipefail
mkdir -p gpurun_out/bal
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/kernels/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/bal/tests.log 2>&1 || exit $?
SHAPES=1x2912x8x1,1x4096x8x1 SMALL=0,3 RAW=1 timeout -k 10 120 python -u tools/prefill_timing.py \
  > gpurun_out/bal/timing.jsonl 2>/dev/null || exit $?
for sm in 0 3; do
  for P in 0 416; do
    SMALL=$sm PREFIX=$P SHAPES=1x2912x8x1,1x2048x8x1,1x1440x8x1,1x4096x8x1,2x2048x8x1,1x1024x8x1 \
      timeout -k 10 120 python -u tools/bench_prefill.py > gpurun_out/bal/sm${sm}_p${P}.jsonl 2>/dev/null || exit $?
  done
done
echo done
