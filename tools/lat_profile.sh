#!/bin/bash
# Latency-path profile on the GPU box: rocprofv3 kernel trace of the single-request
# runs at the end of a short bench, reduced on the box to busy/gap/per-kernel tables
# (tools/prof_gaps.py) so the raw trace never leaves it.  Usage:
#   bash tools/lat_profile.sh <out dir> [extra bench args]
set -u
OUT=${1:-gpurun_out/prof_lat}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT" -o run -- python3 bench.py --steps 1 --warmup 0 --docs-per-step 1 \
  --max-num-seqs 64 --latency-runs 8 "$@" > "$OUT/bench.log" 2>&1
rc=$?
tail -1 "$OUT/bench.log" | cut -c1-600
python3 tools/prof_gaps.py "$OUT" ${WINDOW_S:-3} > "$OUT.md" || true
find "$OUT" -name '*kernel_trace.csv' -delete
exit $rc
