set -e
timeout -k 10 400 python -u bench.py --steps 6 --warmup 3 --latency-runs 0 --phases none > gpurun_out/bench_gil.json 2> gpurun_out/bench_gil.err
