set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/car_contention.py --world 8 > gpurun_out/car_w8.json 2> gpurun_out/car_w8.err
timeout -k 10 120 python -u tools/car_contention.py --world 8 --parent-gpu > gpurun_out/car_w8p.json 2> gpurun_out/car_w8p.err
timeout -k 10 120 python -u tools/car_contention.py --world 7 --parent-gpu > gpurun_out/car_w7p.json 2> gpurun_out/car_w7p.err
timeout -k 10 400 python -u tools/tp8_rank_emulation.py --md gpurun_out/tp8_proj.md > gpurun_out/tp8.json 2> gpurun_out/tp8.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_tp8 -o run -- python3 $R/tools/tp8_rank_emulation.py --runs 3 --decode-tokens 100 > $R/gpurun_out/prof_tp8.log 2>&1
cd $R
python3 tools/trace_window_stats.py gpurun_out/prof_tp8 1.5 > gpurun_out/tp8_window.md
find gpurun_out/prof_tp8 -name '*_trace.csv' -delete
