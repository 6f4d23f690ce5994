set -e
RFQ_BENCH_PRODUCER=thread timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_prod_thread.json 2> gpurun_out/bench_prod_thread.err
RFQ_BENCH_PRODUCER=process timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_prod_process.json 2> gpurun_out/bench_prod_process.err
