set -euo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "gemm_dense" > gpurun_out/t_gemm.log 2>&1 || { tail -40 gpurun_out/t_gemm.log; exit 1; }
tail -1 gpurun_out/t_gemm.log
timeout -k 10 600 python -u tools/bench_gemm_dense.py --cfg 3720 --cfgs 2,1672,3720 --ms 2048,4096,7168 --shapes gate_up,down,qkv,o,gate_up+swiglu --rounds 3 --out gpurun_out/gemm_w4_mf32.md > gpurun_out/gemm_w4_mf32.jsonl 2> gpurun_out/gemm_w4_mf32.err
python - <<'PY'
import json
for l in open('gpurun_out/gemm_w4_mf32.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['shape'], d['M'], d['us'], d['ok'])
PY
