set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "gemm_dense" > gpurun_out/t_gemm.log 2>&1 || { tail -40 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
# 648 spread group 4; 640 unspread group 4; 760 MFMA only (group 4); 712 spread no waits group 4
timeout -k 10 600 python -u tools/bench_gemm_dense.py --cfg 648 --cfgs 2,648,640,712,760 --ms 2048,4096,7168 --shapes gate_up,down,qkv,o,gate_up+swiglu --rounds 3 --out gpurun_out/gemm_w4_ord.md > gpurun_out/gemm_w4_ord.jsonl 2> gpurun_out/gemm_w4_ord.err
python - <<'PY'
import json
for l in open('gpurun_out/gemm_w4_ord.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['shape'], d['M'], d['us'])
PY
