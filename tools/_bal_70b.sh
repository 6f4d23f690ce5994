#!/bin/bash
# balanced prefill at 70B TP=1 short prompts (auto = balanced vs mode 2 = the old 2-way
# split), then the full GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out/bal
for sm in 0 2; do
  SMALL=$sm SHAPES=1x400x64x8,1x512x64x8,1x300x64x8 timeout -k 10 120 python -u tools/bench_prefill.py \
    > gpurun_out/bal/70b_sm${sm}_p0.jsonl 2>/dev/null || exit $?
  SMALL=$sm PREFIX=400 SHAPES=1x800x64x8,1x900x64x8 timeout -k 10 120 python -u tools/bench_prefill.py \
    > gpurun_out/bal/70b_sm${sm}_p400.jsonl 2>/dev/null || exit $?
done
bash tools/_final_tests.sh
