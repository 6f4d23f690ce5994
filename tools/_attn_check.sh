#!/bin/bash
# decode attention with interleaved split pages: oracle tests, batch-1 latency, and the
# 8B bench's decode shape on the calibrated caps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/kernels/test_kernels_gpu.py -k "attn_decode" tests/kernels/test_decode_persist_gpu.py > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
LAT_SP=1 timeout -k 10 300 python -u tools/bench_attn.py > gpurun_out/attn_lat_ilv.jsonl 2> gpurun_out/attn_lat.err || exit 1
cat gpurun_out/attn_lat_ilv.jsonl
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --phases none --latency-runs 0 > gpurun_out/calib_default.json 2> gpurun_out/calib_default.err || exit 1
python3 -c "
import json
d=json.loads(open('gpurun_out/calib_default.json').read().strip().splitlines()[-1])
print(d['value'], json.dumps(d.get('per_doc')))
"
