#!/bin/bash
# row-streaming GEMV with the predicated last iteration: oracle tests (rows, folded path,
# persistent forms that mirror its accumulation order), per-cfg times, whole 8B step
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_kernels_gpu.py tests/engine/test_fold_norms.py tests/kernels/test_decode_persist_gpu.py -k "rows or fold or persist or engine" > gpurun_out/rows_tests.log 2>&1 || { tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -2 gpurun_out/rows_tests.log
timeout -k 10 400 python -u tools/bench_gemv_rows.py --model 8b 1 > gpurun_out/rows_8b.jsonl 2>&1 || { tail -10 gpurun_out/rows_8b.jsonl; exit 1; }
timeout -k 10 400 python -u tools/bench_gemv_rows.py --model 70b 1 > gpurun_out/rows_70b.jsonl 2>&1 || { tail -10 gpurun_out/rows_70b.jsonl; exit 1; }
timeout -k 10 200 python -u tools/bench_persist.py --shape 8b --ctx 1024 --modes 0,rows:down,rows:o,rows:qkv,rows:gu --iters 30 > gpurun_out/rows_step.jsonl 2>&1 || { tail -10 gpurun_out/rows_step.jsonl; exit 1; }
grep '^{' gpurun_out/rows_step.jsonl
