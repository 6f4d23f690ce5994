set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r6.log 2>&1 || { tail -30 gpurun_out/gputests_r6.log; exit 1; }
tail -3 gpurun_out/gputests_r6.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r6a.json 2> gpurun_out/bench_r6a.err || { tail -30 gpurun_out/bench_r6a.err; exit 1; }
tail -c 3000 gpurun_out/bench_r6a.json
