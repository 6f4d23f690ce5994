set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_tput2 -o run -- python3 $R/bench.py --steps 4 --warmup 2 --latency-runs 0 --phases none > $R/gpurun_out/prof_tput2.log 2>&1
cd $R
python3 tools/prof_gaps.py gpurun_out/prof_tput2 6 > gpurun_out/tput2_gaps.md
python3 tools/prof_summary.py gpurun_out/prof_tput2 > gpurun_out/tput2_stats.md || true
find gpurun_out/prof_tput2 -name '*_trace.csv' -delete
