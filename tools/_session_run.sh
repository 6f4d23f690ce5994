set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "splitk_merge or attn_decode" > gpurun_out/t_merge.log 2>&1 || { tail -30 gpurun_out/t_merge.log; exit 1; }
tail -2 gpurun_out/t_merge.log
timeout -k 10 400 python -u tools/bench_attn_merge_o.py > gpurun_out/merge_o.jsonl 2> gpurun_out/merge_o.err
cat gpurun_out/merge_o.jsonl
