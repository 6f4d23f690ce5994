#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (hipGraph-launched decode
# steps show up as graph-launched kernels).  Usage on the GPU box:
#   bash tools/profile.sh [bench args...]
# Output: gpurun_out/prof/ (raw) and a markdown summary on stdout.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 ${PROF_TIMEOUT:-900} rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$OUT" -o run -- python3 bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?
tail -2 "$OUT/bench.log"
python3 tools/prof_summary.py "$OUT" || true
# the raw per-dispatch trace can exceed gpurun's 64 MiB copy-back limit
[ "${KEEP_TRACE:-0}" = "1" ] || find "$OUT" -name '*kernel_trace.csv' -delete
exit $rc
