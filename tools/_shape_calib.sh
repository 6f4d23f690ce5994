#!/bin/bash
# decode-shape calibration of the SYNTHETIC grammar profile against the engine itself
# (VERDICT r5 item 4): per_doc of a short throughput window per (item cap, cap scale)
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-3:1.0 3:0.8 3:0.7 3:0.6}; do
  it=${cfg%%:*}; sc=${cfg##*:}
  RFQ_SYNTH_MAX_ITEMS=$it RFQ_SYNTH_CAP_SCALE=$sc timeout -k 10 300 python -u bench.py --steps 3 \
    --warmup 1 --phases none --latency-runs 0 > gpurun_out/calib_${it}_$sc.json \
    2> gpurun_out/calib_${it}_$sc.err || { tail -5 gpurun_out/calib_${it}_$sc.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/calib_${it}_$sc.json').read().strip().splitlines()[-1])
print('$it', '$sc', d['value'], json.dumps(d.get('per_doc')))
"
done
