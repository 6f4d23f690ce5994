set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/kernels/test_kernels_gpu.py -k gemm_dense -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gd.log 2>&1
timeout -k 10 400 python -u tools/bench_gemm_dense.py --ms 2048,4096,7168 > gpurun_out/bgd.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_gd1 -- python3 $R/tools/prof_one_kernel.py run gemm 4096 28672 4096 0 2 > $R/gpurun_out/pmc_gd1.log 2>&1
