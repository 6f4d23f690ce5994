set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "attn_prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_prefill.log 2>&1
timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_auto.jsonl 2> gpurun_out/prefill_auto.err
RFQ_PREFILL_SMALL=1 timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_hs.jsonl 2> gpurun_out/prefill_hs.err
RFQ_PREFILL_SMALL=2 timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_kv8.jsonl 2> gpurun_out/prefill_kv8.err
