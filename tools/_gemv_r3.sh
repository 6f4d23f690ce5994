set -e
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k "gemv_splitk or skinny" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gemv.log 2>&1
timeout -k 10 300 python -u tools/bench_decode_gemv.py --model tp8 1 4 > gpurun_out/gemv_tp8.jsonl 2> gpurun_out/gemv_tp8.err
timeout -k 10 300 python -u tools/bench_decode_gemv.py --model 8b 1 4 > gpurun_out/gemv_8b.jsonl 2> gpurun_out/gemv_8b.err
timeout -k 10 400 python -u tools/tp8_rank_emulation.py --md gpurun_out/tp8_proj2.md > gpurun_out/tp8_2.json 2> gpurun_out/tp8_2.err
