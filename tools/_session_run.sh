set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pf2
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "attn_prefill" > gpurun_out/pf2/t_pf.log 2>&1 || { tail -30 gpurun_out/pf2/t_pf.log; exit 1; }
tail -1 gpurun_out/pf2/t_pf.log
SMALL=0,2 SHAPES=1x2048x8x1,1x1024x8x1 timeout -k 10 300 python -u tools/prefill_timing.py > gpurun_out/pf2/timing.jsonl 2> gpurun_out/pf2/timing.err
cat gpurun_out/pf2/timing.jsonl | cut -c1-400
for m in 1 2; do
SMALL=$m SHAPES=1x2048x8x1,1x1024x8x1,1x512x8x1,1x4096x8x1,4x2048x32x8 timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/pf2/prof$m -o run -- python -u tools/bench_prefill.py > gpurun_out/pf2/prof$m.log 2>&1
cat gpurun_out/pf2/prof$m.log | grep '^{'
done
