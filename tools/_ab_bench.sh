set -e
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_dense.json 2> gpurun_out/bench_dense.err
RFQ_GEMM_DENSE=0 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_lib.json 2> gpurun_out/bench_lib.err
