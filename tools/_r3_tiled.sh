set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tiled_layout or gemv_splitk" > gpurun_out/tiled_tests.log 2>&1
timeout -k 10 400 python -u tools/bench_gemv_tiled.py > gpurun_out/gemv_tiled.jsonl 2> gpurun_out/gemv_tiled.err
bash tools/_lat8b.sh
timeout -k 10 400 python -u tools/tp8_rank_emulation.py --md gpurun_out/tp8_proj.md > gpurun_out/tp8.json 2> gpurun_out/tp8.err
