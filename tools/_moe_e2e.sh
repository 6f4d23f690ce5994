set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "moe" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_moe.log 2>&1
timeout -k 10 200 python -u tools/bench_moe_dense.py 128 256 384 > gpurun_out/bmoed_small.log 2>&1
timeout -k 10 700 python -u bench.py --model mixtral-8x7b --max-num-seqs 3072 --docs-per-step 512 --steps 3 --warmup 1 --latency-runs 3 --phases none > gpurun_out/mix3072.json 2> gpurun_out/mix3072.err
