set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_tput3 -o run -- python3 $R/bench.py --steps 4 --warmup 2 --latency-runs 0 --phases none > $R/gpurun_out/prof_tput3.log 2>&1
cd $R
python3 tools/prof_gaps.py gpurun_out/prof_tput3 6 > gpurun_out/tput3_gaps.md
python3 tools/prof_summary.py gpurun_out/prof_tput3 > gpurun_out/tput3_stats.md || true
find gpurun_out/prof_tput3 -name '*_trace.csv' -delete
