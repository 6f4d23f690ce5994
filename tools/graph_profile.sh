#!/bin/bash
# hipGraph evidence for the decode path: rocprofv3 HIP-API + kernel trace of the
# single-request runs at the end of a short bench, reduced on the box by
# tools/graph_trace_summary.py (kernels joined to the hipGraphLaunch that
# dispatched them).  No PMC counters in this run.  Usage on the GPU box:
#   bash tools/graph_profile.sh <out dir> [extra bench args]
set -u
OUT=${1:-gpurun_out/prof_graph}; shift || true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p "$OUT"
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --hip-trace --kernel-trace --stats \
  --output-format csv -d "$OUT" -o run -- python3 bench.py --steps 1 --warmup 0 \
  --docs-per-step 1 --max-num-seqs 64 --latency-runs 4 "$@" > "$OUT/bench.log" 2>&1
rc=$?
tail -1 "$OUT/bench.log" | cut -c1-400
python3 tools/graph_trace_summary.py "$OUT" ${WINDOW_S:-2} > "$OUT.md" || true
cat "$OUT.md"
find "$OUT" -name '*_trace.csv' -delete
exit $rc
