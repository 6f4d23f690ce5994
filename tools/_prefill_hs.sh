set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "attn_prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_prefill.log 2>&1
timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_kv4.jsonl 2> gpurun_out/prefill_kv4.err
KVSPLIT=0 timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_kv0.jsonl 2> gpurun_out/prefill_kv0.err
timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_kv4b.jsonl 2> gpurun_out/prefill_kv4b.err
