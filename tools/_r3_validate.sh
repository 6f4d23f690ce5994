# full GPU test suite, smoke, then the driver's 1-GPU bench command (default flags)
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 1000 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3v.json 2> gpurun_out/bench_r3v.err
