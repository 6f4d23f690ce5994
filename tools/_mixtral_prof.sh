#!/bin/bash
# Mixtral 8x7B phase (768 in flight, mixed PDF / XLSX) under rocprofv3 --kernel-trace
# --stats: class shares of a steady-state window
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/prof_mix
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/gpurun_out/prof_mix" -o run -- python3 "$R/tools/phase_mixtral.py" ${MIX_DOCS:-1024} ${MIX_WARM:-512}) \
    > gpurun_out/prof_mix.log 2>&1 || { tail -20 gpurun_out/prof_mix.log; exit 1; }
grep '^{' gpurun_out/prof_mix.log | tail -1 > gpurun_out/mix_phase.json || true
python3 tools/trace_window_stats.py gpurun_out/prof_mix ${MIX_WIN:-8} > gpurun_out/mix_window.md
find gpurun_out/prof_mix -name '*_trace.csv' -delete
head -45 gpurun_out/mix_window.md
cat gpurun_out/mix_phase.json | head -c 1500
