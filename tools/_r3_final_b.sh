set -e
R=$GRAFT_REPO_ROOT
PROF_TIMEOUT=400 bash tools/lat_profile.sh gpurun_out/prof_lat --phases none
timeout -k 10 400 python -u tools/tp8_rank_emulation.py --md gpurun_out/tp8_proj.md > gpurun_out/tp8.json 2> gpurun_out/tp8.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tp8 -o run -- python3 $R/tools/tp8_rank_emulation.py --runs 3 --decode-tokens 100 > $R/gpurun_out/prof_tp8.log 2>&1
cd $R
python3 tools/trace_window_stats.py gpurun_out/prof_tp8 1.5 > gpurun_out/tp8_window.md
find gpurun_out/prof_tp8 -name '*_trace.csv' -delete
