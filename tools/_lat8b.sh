set -e
timeout -k 10 400 python -u -c "
import logging, runpy, sys
logging.basicConfig(level=logging.INFO)
sys.argv = ['bench.py', '--steps', '1', '--warmup', '0', '--docs-per-step', '1', '--max-num-seqs', '64', '--latency-runs', '15', '--phases', 'none'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')
" "$@" > gpurun_out/lat8b.json 2> gpurun_out/lat8b.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/lat8b.json").read().strip().splitlines()[-1])
print(json.dumps({"single_stream": d["single_stream"], "p50": d["p50_parse_text_latency_s"]}))
PY
grep "gemm plan" gpurun_out/lat8b.err > gpurun_out/lat8b_plan.txt || true
