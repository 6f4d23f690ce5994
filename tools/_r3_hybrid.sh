set -e
timeout -k 10 400 python -u -m pytest tests/engine/test_engine_gpu.py tests/kernels/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "inplace or tiled or mixed" > gpurun_out/hybrid_tests.log 2>&1
timeout -k 10 500 python -u tools/phase_70b.py 5 > gpurun_out/p70_hybrid.json 2> gpurun_out/p70_hybrid.err
