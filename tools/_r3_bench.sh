set -e
start=$(date +%s)
timeout -k 10 1100 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r3v.json 2> gpurun_out/bench_r3v.err
echo "wall_s=$(( $(date +%s) - start ))" > gpurun_out/bench_r3v.wall
