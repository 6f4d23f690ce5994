set -e
timeout -k 10 300 python -u tools/bench_gemm_dense.py --ms 4096 --shapes gate_up,o,down --cfgs 2,18,34,50,66,98 --out gpurun_out/gemm_abl.md > gpurun_out/babl.log 2>&1
timeout -k 10 700 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
