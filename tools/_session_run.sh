set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "gemm_dense" > gpurun_out/t_gemm.log 2>&1 || { tail -40 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 600 python -u tools/bench_gemm_dense.py --cfg 8 --cfgs 2,8,24,40,72,120 --ms 4096 --shapes gate_up,down --rounds 3 --out gpurun_out/gemm_w4_abl.md > gpurun_out/gemm_w4_abl.jsonl 2> gpurun_out/gemm_w4_abl.err
cat gpurun_out/gemm_w4_abl.jsonl
