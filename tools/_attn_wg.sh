set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "attn_decode" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1
LAT_WG=1 timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/attn_wg.jsonl 2> gpurun_out/attn_wg.err
