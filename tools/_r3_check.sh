set -e
start=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests_s=$(( $(date +%s) - start ))" > gpurun_out/check.wall
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
start=$(date +%s)
timeout -k 10 700 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err
echo "bench_wall_s=$(( $(date +%s) - start ))" >> gpurun_out/check.wall
