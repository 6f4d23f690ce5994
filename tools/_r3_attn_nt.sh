set -e
RFQ_ATTN_NT=1 timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "test_attn_decode" > gpurun_out/attn_nt_tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_attn_nt0.json 2> gpurun_out/bench_attn_nt0.err
RFQ_ATTN_NT=1 timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_attn_nt1.json 2> gpurun_out/bench_attn_nt1.err
