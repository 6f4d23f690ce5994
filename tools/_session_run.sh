set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "wg_merge" > gpurun_out/t_wg.log 2>&1
tail -2 gpurun_out/t_wg.log
LAT_W8=1 timeout -k 10 500 python -u tools/bench_attn.py > gpurun_out/attn_w8.jsonl 2> gpurun_out/attn_w8.err
cat gpurun_out/attn_w8.jsonl
