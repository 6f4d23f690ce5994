set -e
timeout -k 10 500 python -u tools/bench_gemv_tiled.py > gpurun_out/gemv_tiled_nt.jsonl 2> gpurun_out/gemv_tiled_nt.err
