#!/bin/bash
# auto small-grid prefill with the balanced form: tests, rank-shape timings, rank emulation
set -o pipefail
mkdir -p gpurun_out/bal
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/kernels/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/bal/tests_auto.log 2>&1 || exit $?
for P in 0 416; do
  PREFIX=$P SHAPES=1x2912x8x1,1x2048x8x1,1x1440x8x1,1x4096x8x1,2x2048x8x1,1x1024x8x1,1x2912x64x8,1x2912x32x8 \
    timeout -k 10 120 python -u tools/bench_prefill.py > gpurun_out/bal/auto_p${P}.jsonl 2>/dev/null || exit $?
done
timeout -k 10 700 python -u tools/tp8_rank_emulation.py --ar-us 6,7.7,8,10 --steps-p50 160 --pdf-set 12 --md gpurun_out/bal/emul.md \
  > gpurun_out/bal/emul.log 2>&1 || exit $?
echo done
