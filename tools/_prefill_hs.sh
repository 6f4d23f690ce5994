set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "attn_prefill" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_prefill.log 2>&1
timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_f1.jsonl 2> gpurun_out/prefill_f1.err
KVSPLIT=0 timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_f0.jsonl 2> gpurun_out/prefill_f0.err
HSPLIT=0 timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_fh0.jsonl 2> gpurun_out/prefill_fh0.err
timeout -k 10 300 python -u tools/bench_prefill.py > gpurun_out/prefill_f1b.jsonl 2> gpurun_out/prefill_f1b.err
