set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tiled" > gpurun_out/persist_tests.log 2>&1
timeout -k 10 600 python -u tools/bench_gemv_tiled.py > gpurun_out/gemv_persist.jsonl 2> gpurun_out/gemv_persist.err
